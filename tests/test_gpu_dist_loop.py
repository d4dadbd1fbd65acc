"""The C++ multi-rank protocols at N > 1 on the one GPU of the test box.

fcx_dist_compress_gather (the strong-scaling step bench.py runs at N > 1), fcx_dist_concat
and fcx_dist_compress_host run unchanged over the loopback transport (include/fcx.h):
thread ranks of this process, each with its own fcx_dist handle, fcx_ctx and stream, and a
matched send/recv pair is a device-to-device copy.  The RCCL transport only differs below
the seam (group start/end, send/recv, all-gather, broadcast).  Every assembled stream is
compared with the reference's file (oracle.compress_file, pinned to the reference in
test_oracle.py; HL-rand against its SURVEY digest); the reference writes the blocks to one
file in block order (my_compress.cpp:4110-4114)."""
import hashlib
import threading

import pytest

import inputs
import my_compress_amd as mc
import oracle
from my_compress_amd import dist as fdist

pytestmark = pytest.mark.gpu


def run_ranks(n, fn, timeout=110):
    """fn(r) on n host threads (ctypes releases the GIL inside the C calls); returns (results,
    errors) per rank.  A thread still alive after `timeout` s is a hang: the test fails."""
    res, errs = [None] * n, [None] * n

    def work(r):
        try:
            res[r] = fn(r)
        except Exception as e:   # (FcxError is what the protocol raises)
            errs[r] = e

    ths = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(n)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout)
    assert not any(t.is_alive() for t in ths), "a thread rank hung"
    return res, errs


class Job:
    """n thread ranks over one loopback hub: per rank a Dist handle and a stream"""

    def __init__(self, n, cuda, timeout_ms=30000):
        import torch

        hub = mc.Loop(n, cuda.index, timeout_ms)
        self.dists = [mc.Dist.loop(hub, r) for r in range(n)]
        hub.close()   # (the handles keep the hub)
        self.streams = [torch.cuda.Stream(cuda) for _ in range(n)]
        self.n, self.cuda = n, cuda

    def close(self):
        for d in self.dists:
            d.close()

    def gather(self, data: bytes, block: int, share0: int, nsub: int, caps=None, fail=None):
        """one fcx_dist_compress_gather step over `data`; returns (results, errors, rank 0's
        output tensor).  caps: per-rank capacity overrides; fail: {rank: piece} injected failures"""
        import torch

        n, cuda = self.n, self.cuda
        ranges = [fdist.byte_range(len(data), block, r, n, share0) for r in range(n)]
        rb = [b - a for a, b in ranges]
        d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(cuda) if data else \
            torch.zeros(1, dtype=torch.uint8, device=cuda)
        ctxs = [mc.Context(cuda.index, block, max(b, block)) for b in rb]
        cap = [mc.shard_bound(len(data), block) if r == 0 else mc.dist_gather_bound(rb[r], block, nsub)
               for r in range(n)]
        for r, c in (caps or {}).items():
            cap[r] = c
        outs = [torch.empty(max(c, 16), dtype=torch.uint8, device=cuda) for c in cap]
        for r in range(n):
            self.dists[r].debug_fail((fail or {}).get(r, -1))
        torch.cuda.synchronize(cuda)
        try:
            res, errs = run_ranks(n, lambda r: self.dists[r].compress_gather(
                ctxs[r], d_in.data_ptr() + ranges[r][0], rb[r], rb, nsub, outs[r].data_ptr(), cap[r],
                self.streams[r].cuda_stream))
        finally:
            for c in ctxs:
                c.close()
            for d in self.dists:
                d.debug_fail(-1)
        return res, errs, outs[0]


CASES = [   # (input spec, block, share0 ppm (None = the step model's), nsub)
    ({"type": "mosaic", "seed": 31, "n": 700001}, 65536, 0, 1),          # even split
    ({"type": "mosaic", "seed": 31, "n": 700001}, 65536, 500000, 4),
    ({"type": "mosaic", "seed": 32, "n": 700001}, 65536, 900000, 64),    # near-empty peers, 64 pieces
    ({"type": "gen", "kind": "text", "seed": 5, "n": 3 << 20}, 65536, None, 4),
    ({"type": "gen", "kind": "rand", "seed": 1, "n": 5000}, 4096, 1000000, 4),   # every peer empty
    ({"type": "mosaic", "seed": 33, "n": 257 * 4096 + 7}, 4096, 250000, 16),
]


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_loop_compress_gather_matches_reference(nranks, cuda):
    """rank 0 ends with every rank's records in block order, equal to the reference's file;
    a peer's total is the bytes it sent and the totals add up"""
    job = Job(nranks, cuda)
    try:
        assert job.dists[0].transport() == "loopback" and job.dists[0].size() == (nranks, 1)
        for spec, block, share0, nsub in CASES:
            data = inputs.make(spec)
            if share0 is None:
                share0 = fdist.gather_share_ppm(nranks, "text", nsub=nsub)
            res, errs, out0 = job.gather(data, block, share0, nsub)
            assert errs == [None] * nranks, (spec, share0, nsub, errs)
            want = oracle.compress_file(data, block)
            nb = (len(data) + block - 1) // block
            got = mc.write_header(len(data), nb) + out0[:res[0]].cpu().numpy().tobytes()
            assert got == want, (spec, share0, nsub)
            lo, hi = fdist.byte_range(len(data), block, 0, nranks, share0)
            own = len(oracle.compress_file(data[lo:hi], block)) - 10 if hi > lo else 0
            assert own + sum(res[1:]) == res[0]
    finally:
        job.close()


def test_loop_compress_gather_failures_fail_every_rank(cuda):
    """an injected failure anywhere fails every rank (rank 0 sends the job's verdict) with no
    hang, and the same handles then run a correct step"""
    n, block, nsub = 3, 65536, 4
    data = inputs.make({"type": "mosaic", "seed": 41, "n": 24 * 65536 + 99})
    want = oracle.compress_file(data, block)
    lo0, hi0 = fdist.byte_range(len(data), block, 0, n, 500000)
    own0 = len(oracle.compress_file(data[lo0:hi0], block)) - 10   # rank 0's own records
    job = Job(n, cuda)
    try:
        for caps, fail, why in [
            ({2: 1 << 16}, None, "peer capacity: fails before its first piece is queued"),
            (None, {1: 2}, "peer piece 2 fails after pieces 0-1 are queued"),
            (None, {2: 0}, "peer fails in its first piece"),
            ({0: own0 + 16}, None, "rank 0: room for its own segment only"),
        ]:
            res, errs, _ = job.gather(data, block, 500000, nsub, caps=caps, fail=fail)
            assert all(isinstance(e, mc.FcxError) for e in errs), (why, errs)
            res, errs, out0 = job.gather(data, block, 500000, nsub)
            assert errs == [None] * n, (why, errs)
            assert mc.write_header(len(data), 25) + out0[:res[0]].cpu().numpy().tobytes() == want, why
    finally:
        job.close()


def test_loop_hl_rand_n8_digest(cuda):
    """HL-rand (1 GiB of rand seed 4 at 1 MiB blocks) through the N = 8 step with the step
    model's rank-0 share: the reference's file digest"""
    import torch

    n = 1 << 30
    cfg = [c for c in inputs.SURVEY_DIGESTS.values() if c["kind"] == "rand" and c["n"] == n and c["block"] == 1 << 20]
    want_sha, want_bytes = cfg[0]["out"], cfg[0]["bytes"]
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    inputs.generate_into("rand", 4, host.data_ptr(), n)
    d_in = host.to(cuda)
    del host
    block, nsub, N = 1 << 20, 4, 8
    share0 = fdist.gather_share_ppm(N, "rand", nsub=nsub)
    ranges = [fdist.byte_range(n, block, r, N, share0) for r in range(N)]
    rb = [b - a for a, b in ranges]
    job = Job(N, cuda)
    ctxs = [mc.Context(cuda.index, block, b) for b in rb]
    cap = [mc.shard_bound(n, block)] + [mc.dist_gather_bound(b, block, nsub) for b in rb[1:]]
    outs = [torch.empty(c, dtype=torch.uint8, device=cuda) for c in cap]
    try:
        torch.cuda.synchronize(cuda)
        res, errs = run_ranks(N, lambda r: job.dists[r].compress_gather(
            ctxs[r], d_in.data_ptr() + ranges[r][0], rb[r], rb, nsub, outs[r].data_ptr(), cap[r],
            job.streams[r].cuda_stream))
        assert errs == [None] * N, errs
        h = hashlib.sha256(mc.write_header(n, n // block))
        h.update(memoryview(outs[0][:res[0]].cpu().numpy()))
        assert res[0] + 10 == want_bytes
        assert h.hexdigest() == want_sha
        # rank 0's final moves of the 7 peers' bytes behind its segment (timed on its stream)
        copy_ms = job.dists[0].gather_copy_ms()
        print(f"N=8 loopback: rank-0 share {share0 / 1e4:.1f} %, final copies {copy_ms:.3f} ms", flush=True)
        assert 0 <= copy_ms < 50, copy_ms
        assert all(job.dists[r].gather_copy_ms() < 0 for r in range(1, N))
    finally:
        for c in ctxs:
            c.close()
        job.close()


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_loop_concat_gather_and_allgather(nranks, cuda):
    """fcx_dist_concat at N > 1: sizes all-gather, then grouped receives at rank 0 (gather) or
    one broadcast per source rank (allgather), segments of uneven and zero length; a capacity
    failure on one rank fails every rank and the next call works"""
    import torch

    job = Job(nranks, cuda)
    g = torch.Generator().manual_seed(nranks)
    lens = [int(x) for x in torch.randint(0, 300000, (nranks,), generator=g)]
    lens[nranks // 2] = 0
    segs = [torch.randint(0, 256, (max(m, 1),), dtype=torch.uint8, generator=g).to(cuda) for m in lens]
    want = torch.cat([s[:m] for s, m in zip(segs, lens)])
    tot = sum(lens)
    outs = [torch.zeros(tot + 64, dtype=torch.uint8, device=cuda) for _ in range(nranks)]
    try:
        for mode in (mc.DIST_GATHER, mc.DIST_ALLGATHER):
            for o in outs:
                o.zero_()
            torch.cuda.synchronize(cuda)
            res, errs = run_ranks(nranks, lambda r: job.dists[r].concat(
                segs[r].data_ptr(), lens[r], outs[r].data_ptr(), outs[r].numel(), mode, job.streams[r].cuda_stream))
            assert errs == [None] * nranks, errs
            assert res == [tot] * nranks
            for r in range(nranks) if mode == mc.DIST_ALLGATHER else [0]:
                assert torch.equal(outs[r][:tot], want), (mode, r)
            # rank r > 0 with too little room (allgather) / rank 0 (gather): every rank fails
            bad = nranks - 1 if mode == mc.DIST_ALLGATHER else 0
            res, errs = run_ranks(nranks, lambda r: job.dists[r].concat(
                segs[r].data_ptr(), lens[r], outs[r].data_ptr(), 16 if r == bad else outs[r].numel(), mode,
                job.streams[r].cuda_stream))
            assert all(isinstance(e, mc.FcxError) for e in errs), errs
    finally:
        job.close()


def test_loop_local_compress_host(cuda):
    """fcx_dist_compress_host with three thread ranks in one handle (the CLI's -g N form):
    rounds smaller than the input, records in block order, equal to the reference's file"""
    d = mc.Dist.loop_local(3, cuda.index)
    try:
        assert d.size() == (3, 3) and d.transport() == "loopback"
        data = inputs.mosaic(77, 9 * 65536 + 1234)
        assert mc.write_header(len(data), 10) + d.compress_host(data, 65536, round_bytes=2 * 65536) == \
            oracle.compress_file(data, 65536)
        text = inputs.make({"type": "gen", "kind": "text", "seed": 8, "n": 2 << 20})
        assert mc.write_header(len(text), 32) + d.compress_host(text, 65536) == oracle.compress_file(text, 65536)
    finally:
        d.close()


def test_loop_unmatched_operation_times_out(cuda):
    """a rank whose peer never joins fails after the hub's timeout instead of hanging, and the
    aborted hub fails every later call"""
    import torch

    job = Job(2, cuda, timeout_ms=1500)
    seg = torch.arange(1000, dtype=torch.int64, device=cuda).to(torch.uint8)
    out = torch.zeros(4096, dtype=torch.uint8, device=cuda)
    try:
        res, errs = run_ranks(1, lambda r: job.dists[0].concat(seg.data_ptr(), 1000, out.data_ptr(), 4096,
                                                             mc.DIST_GATHER, job.streams[0].cuda_stream), timeout=30)
        assert isinstance(errs[0], mc.FcxError) and "waited" in str(errs[0])
        res, errs = run_ranks(2, lambda r: job.dists[r].concat(seg.data_ptr(), 1000, out.data_ptr(), 4096,
                                                             mc.DIST_GATHER, job.streams[r].cuda_stream), timeout=30)
        assert all(isinstance(e, mc.FcxError) for e in errs)
    finally:
        job.close()
