"""The C++ multi-GPU path (fcx_dist_*, RCCL) on the one GPU of the test box: a
communicator of one rank exercises the size exchange, both concatenation forms and
the per-device compress threads; the result must be byte-identical to the
single-device path and to the reference (golden.json).  The N > 1 exchange itself
runs at the driver's 8-GPU scaling bench (torch.distributed over RCCL) and in the
gloo tests of test_dist.py."""
import hashlib
import os
import subprocess

import pytest

import inputs
import my_compress_amd as mc
import oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "my_compress_amd", "bin", "my_compress")


def test_local_dist_compress_matches_reference(golden):
    d = mc.Dist.local([0])
    try:
        assert d.size() == (1, 1)
        for case in golden["cases"]:
            if case["in_bytes"] > (1 << 20) + 20000:
                continue
            data = inputs.make(case)
            nb = (len(data) + case["block"] - 1) // case["block"]
            got = mc.write_header(len(data), nb) + d.compress_host(data, case["block"])
            assert hashlib.sha256(got).hexdigest() == case["out_sha256"], case["name"]
        # several rounds (round_bytes smaller than the input): records continue in block order
        data = inputs.mosaic(77, 3 * 65536 + 1234)
        assert mc.write_header(len(data), 4) + d.compress_host(data, 65536, round_bytes=65536) == \
            oracle.compress_file(data, 65536)
    finally:
        d.close()


def test_rank_concat_gather_and_allgather(cuda):
    import torch

    d = mc.Dist.rank(1, 0, mc.dist_unique_id(), 0)
    try:
        seg = torch.arange(0, 100000, dtype=torch.int64, device=cuda).to(torch.uint8)
        out = torch.zeros(200000, dtype=torch.uint8, device=cuda)
        st = torch.cuda.current_stream().cuda_stream
        for mode in (mc.DIST_GATHER, mc.DIST_ALLGATHER):
            out.zero_()
            n = d.concat(seg.data_ptr(), seg.numel(), out.data_ptr(), out.numel(), mode, st)
            assert n == seg.numel() and torch.equal(out[:n], seg)
        # in place: the segment already at offset 0 of the output buffer
        out[:seg.numel()].copy_(seg)
        assert d.concat(out.data_ptr(), seg.numel(), out.data_ptr(), out.numel(), mc.DIST_GATHER, st) == seg.numel()
        assert torch.equal(out[:seg.numel()], seg)
        with pytest.raises(mc.FcxError):   # capacity
            d.concat(seg.data_ptr(), seg.numel(), out.data_ptr(), 1000, mc.DIST_GATHER, st)
        # the capacity verdict is taken after the exchange by every rank alike:
        # the communicator is not left with a half-posted send and the next concat works
        out.zero_()
        assert d.concat(seg.data_ptr(), seg.numel(), out.data_ptr(), out.numel(), mc.DIST_ALLGATHER, st) == seg.numel()
        assert torch.equal(out[:seg.numel()], seg)
    finally:
        d.close()


def test_cli_gpus_flag_matches_single_device(tmp_path, golden):
    case = [c for c in golden["cases"] if c["name"] == "text_plus_partial"][0]
    data = inputs.make(case)
    (tmp_path / "plain").write_bytes(data)
    r = subprocess.run([CLI, "-i", "plain", "-o", "one", "-c", "lz77", "-b", str(case["block"])], cwd=tmp_path,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([CLI, "-i", "plain", "-o", "dist", "-c", "lz77", "-b", str(case["block"]), "-g", "1"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    assert "(1 GPUs)" in r.stdout
    one, dist = (tmp_path / "one").read_bytes(), (tmp_path / "dist").read_bytes()
    assert one == dist
    assert hashlib.sha256(dist).hexdigest() == case["out_sha256"]


def test_rank_compress_gather_one_rank(cuda):
    """fcx_dist_compress_gather on a one-rank communicator: the compress + exchange step of the
    strong-scaling bench (no peers: rank 0's own range, every nsub) equals the reference file"""
    import torch

    d = mc.Dist.rank(1, 0, mc.dist_unique_id(), 0)
    ctx = mc.Context(0, 65536, 1 << 20)
    try:
        data = inputs.make({"type": "mosaic", "seed": 31, "n": 700001})
        want = oracle.compress_file(data, 65536)
        d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(cuda)
        cap = mc.shard_bound(len(data), 65536)
        out = torch.zeros(cap, dtype=torch.uint8, device=cuda)
        st = torch.cuda.current_stream().cuda_stream
        for nsub in (1, 4, 64):
            out.zero_()
            n = d.compress_gather(ctx, d_in.data_ptr(), len(data), [len(data)], nsub, out.data_ptr(), cap, st)
            assert mc.write_header(len(data), 11) + out[:n].cpu().numpy().tobytes() == want
        with pytest.raises(mc.FcxError):   # rank_bytes[rank] must be this rank's n
            d.compress_gather(ctx, d_in.data_ptr(), len(data), [len(data) - 1], 1, out.data_ptr(), cap, st)
        with pytest.raises(mc.FcxError):   # nsub out of range
            d.compress_gather(ctx, d_in.data_ptr(), len(data), [len(data)], 65, out.data_ptr(), cap, st)
    finally:
        ctx.close()
        d.close()
