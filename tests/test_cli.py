"""The my_compress CLI (main(), my_compress.cpp:3726-4213): same flags, default
output ./out, same byte stream.  Decompress runs on the host decoder (CPU test);
compress runs on the GPU (gpu test) and fails loudly without one."""
import hashlib
import os
import subprocess

import pytest

import inputs
import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "my_compress_amd", "bin", "my_compress")


def gpu_present() -> bool:
    """asks the product library (its own HIP runtime), not torch: torch bundles another
    HIP runtime, which may report no device once libfcx has initialised in-process"""
    import ctypes

    import my_compress_amd as mc

    h = ctypes.c_void_p()
    if mc.lib().fcx_dctx_create(ctypes.byref(h), 0) != 0:
        return False
    mc.lib().fcx_dctx_destroy(h)
    return True


def run(args, cwd):
    return subprocess.run([CLI] + args, cwd=cwd, capture_output=True, text=True, timeout=600)


def test_cli_decompresses_reference_streams(tmp_path, golden):
    for case in golden["cases"]:
        if case["name"] not in ("text_s7_300000_b4096", "mosaic_s1_b65536", "kat30", "tiny_17"):
            continue
        data = inputs.make(case)
        blob = oracle.compress_file(data, case["block"])
        (tmp_path / "in.fcx").write_bytes(blob)
        r = run(["-i", "in.fcx", "-o", "plain"], tmp_path)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "SUCCESS" in r.stdout
        assert (tmp_path / "plain").read_bytes() == data


def test_cli_decoder_quirks_match_reference_decoder(tmp_path, golden):
    """files whose reference decode is not the input (one-symbol sub-streams decode
    as zeros, my_compress.cpp:930-984; early stop at 2336-2339): the CLI writes the
    reference decoder's bytes and, like main() (4198-4201), reports FAIL on the size"""
    for case in golden["cases"]:
        if case["dec_is_input"] or case["in_bytes"] > 1 << 20:
            continue
        blob = oracle.compress_file(inputs.make(case), case["block"])
        (tmp_path / "in.fcx").write_bytes(blob)
        r = run(["-i", "in.fcx", "-o", "plain"], tmp_path)
        out = (tmp_path / "plain").read_bytes()
        assert hashlib.sha256(out).hexdigest() == case["dec_sha256"], case["name"]
        size_ok = case["dec_bytes"] == case["in_bytes"]
        assert ("SUCCESS" in r.stdout) == size_ok, (case["name"], r.stdout)


def test_cli_rejects_foreign_stream(tmp_path):
    (tmp_path / "junk").write_bytes(b"NOTFCX" * 10)
    assert run(["-i", "junk", "-o", "x"], tmp_path).returncode != 0


def test_cli_lz78_fails_loudly_without_gpu(tmp_path):
    if gpu_present():
        pytest.skip("GPU present")
    (tmp_path / "plain").write_bytes(b"hello hello")
    r = run(["-i", "plain", "-o", "x", "-c", "lz78"], tmp_path)
    assert r.returncode != 0 and ("HIP" in r.stderr or "GPU" in r.stderr)
    (tmp_path / "x8").write_bytes(oracle.lz78_compress_file(b"hello hello", 1 << 20))
    r = run(["-i", "x8", "-o", "y"], tmp_path)
    assert r.returncode != 0


@pytest.mark.gpu
def test_cli_lz78_matches_oracle_and_round_trips(tmp_path):
    data = inputs.mosaic(41, (2 << 20) + 4321)
    (tmp_path / "plain").write_bytes(data)
    r = run(["-i", "plain", "-o", "c8", "-c", "lz78"], tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert (tmp_path / "c8").read_bytes() == oracle.lz78_compress_file(data, 1 << 20)
    r = run(["-i", "c8", "-o", "back"], tmp_path)
    assert r.returncode == 0 and "SUCCESS" in r.stdout, r.stdout + r.stderr
    assert (tmp_path / "back").read_bytes() == oracle.lz78_decompress_file((tmp_path / "c8").read_bytes(), len(data) + 64)


@pytest.mark.gpu
def test_cli_lz78_small_blocks_round_trip(tmp_path):
    """-c lz78 -b 4096 on ~3 MiB (770 blocks): the decompress buffer follows the header's
    total, not 1 MiB per block"""
    data = inputs.mosaic(43, (3 << 20) + 17)
    (tmp_path / "plain").write_bytes(data)
    r = run(["-i", "plain", "-o", "c8", "-c", "lz78", "-b", "4096"], tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert (tmp_path / "c8").read_bytes() == oracle.lz78_compress_file(data, 4096)
    r = run(["-i", "c8", "-o", "back"], tmp_path)   # FAIL on size is the reference's verdict when
    assert "decompress total bytes" in r.stdout, r.stderr   # blocks end in 0x00 (3701-3703)
    assert (tmp_path / "back").read_bytes() == oracle.lz78_decompress_file((tmp_path / "c8").read_bytes(), len(data) + 64 * 800)


def test_cli_compress_fails_loudly_without_gpu(tmp_path):
    if gpu_present():
        pytest.skip("GPU present")
    (tmp_path / "plain").write_bytes(b"hello hello hello hello")
    r = run(["-i", "plain", "-o", "x", "-c", "lz77"], tmp_path)
    assert r.returncode != 0
    assert "GPU" in r.stderr or "HIP" in r.stderr


@pytest.mark.gpu
def test_cli_compress_matches_reference(tmp_path, golden):
    for case in golden["cases"]:
        if case["name"] not in ("text_s1_1048576_b1048576", "text_plus_partial", "A_x100000", "mosaic_s2_b1048576"):
            continue
        data = inputs.make(case)
        (tmp_path / "plain").write_bytes(data)
        args = ["-i", "plain", "-c", "lz77"]
        if case["block"] != 1 << 20:
            args += ["-b", str(case["block"])]
        r = run(args, tmp_path)   # default output ./out (my_compress.cpp:4040-4042)
        assert r.returncode == 0, r.stderr
        out = (tmp_path / "out").read_bytes()
        assert hashlib.sha256(out).hexdigest() == case["out_sha256"], case["name"]
        r = run(["-i", "out", "-o", "back"], tmp_path)
        assert r.returncode == 0
        if case["name"] != "A_x100000":   # single-symbol chars stream decodes as zeros (reference behaviour)
            assert (tmp_path / "back").read_bytes() == data
