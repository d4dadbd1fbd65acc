"""Pipelined host I/O (fcx_compress_stream / fcx_decompress_stream, SURVEY.md
§8(f) row 2): shard boundaries must not change the byte stream (records are per
block, shards are whole blocks), so a multi-shard stream equals the reference's
file body; the GPU decoder streams it back.  CLI end to end on the GPU."""
import hashlib
import io
import os
import subprocess

import pytest

import inputs
import my_compress_amd as mc
import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "my_compress_amd", "bin", "my_compress")


@pytest.mark.parametrize("n,block,shard", [(9_500_000, 65536, 1 << 20), (3_000_001, 4096, 1_000_000),
                                           (5 << 20, 1 << 20, 2 << 20), (777, 65536, 1 << 20)])
def test_multi_shard_stream_equals_reference(cuda, n, block, shard):
    data = inputs.mosaic(n ^ block, n)
    ctx = mc.Context(0, block, shard)
    try:
        sink = io.BytesIO()
        tin, tout, nb = ctx.compress_stream(io.BytesIO(data), sink, shard)
    finally:
        ctx.close()
    want = oracle.compress_file(data, block)
    assert tin == n and nb == (n + block - 1) // block
    assert mc.write_header(tin, nb) + sink.getvalue() == want
    d = mc.DContext(0)
    try:
        out = io.BytesIO()
        total, got, recs = d.decompress_stream(io.BytesIO(want), out)
    finally:
        d.close()
    # the reference decoder's bytes: incompressible small blocks (all-literal flags
    # = a single-symbol flags stream, decoded as zeros) come back empty, as in
    # my_decompress_file_lz77 itself
    ref = oracle.decompress_file(want, n + 16)
    assert (total, got, recs) == (n & 0xFFFFFFFF, len(ref), nb)
    assert out.getvalue() == ref


def test_cli_gpu_round_trip(cuda, tmp_path):
    data = inputs.generate("text", 21, 40 << 20)
    (tmp_path / "plain").write_bytes(data)
    r = subprocess.run([CLI, "-i", "plain", "-c", "lz77", "-b", "65536"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    blob = (tmp_path / "out").read_bytes()
    assert blob[:10] == mc.write_header(len(data), (len(data) + 65535) // 65536)
    ctx = mc.Context(0, 65536, len(data))
    try:
        assert blob[10:] == ctx.compress_host(data)
    finally:
        ctx.close()
    r = subprocess.run([CLI, "-i", "out", "-o", "back"], cwd=tmp_path, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "SUCCESS" in r.stdout, r.stdout + r.stderr
    assert "host" not in r.stderr   # decoded on the GPU
    assert (tmp_path / "back").read_bytes() == data


@pytest.mark.slow
def test_cli_multi_shard_file(cuda, tmp_path):
    """a 600 MiB file crosses the CLI's 256 MiB shards: three pipeline steps"""
    n = 600 << 20
    path = tmp_path / "big"
    with open(path, "wb") as f:
        for i in range(6):
            f.write(inputs.generate("text" if i % 2 else "runs", 40 + i, 100 << 20))
    r = subprocess.run([CLI, "-i", "big", "-o", "big.fcx", "-c", "lz77"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([CLI, "-i", "big.fcx", "-o", "back"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0 and "SUCCESS" in r.stdout, r.stdout + r.stderr
    h = lambda p: hashlib.sha256(open(p, "rb").read()).hexdigest()
    assert os.path.getsize(tmp_path / "back") == n
    assert h(tmp_path / "back") == h(path)
