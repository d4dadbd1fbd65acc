"""Multi-rank sharding + concatenation (my_compress_amd.dist) on CPU with gloo,
world_size 2.  Each rank compresses its contiguous block range; the all-gather
concatenation must reproduce the single-process file byte for byte.  No GPU:
the per-rank block encoder here is the oracle (the kernels are covered by the
gpu tests); what is under test is the partition and the exchange."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import inputs
import oracle
from my_compress_amd import dist as fdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cases, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for idx, (spec, block) in enumerate(cases):
            data = inputs.make(spec)
            lo, hi = fdist.byte_range(len(data), block, rank, world)
            for codec, enc in (("lz77", oracle.compress_file), ("lz78", oracle.lz78_compress_file)):
                seg = enc(data[lo:hi], block)[10:] if hi > lo else b""
                t = torch.frombuffer(bytearray(seg), dtype=torch.uint8) if seg else torch.zeros(0, dtype=torch.uint8)
                for mode in ("allgather", "gather"):
                    whole = fdist.concat_segments(t, dist, mode=mode, dst=world - 1 if mode == "gather" else 0)
                    if whole is not None:
                        results[(idx, codec, mode, rank)] = fdist.assemble_file(len(data), block,
                                                                               whole.numpy().tobytes(), codec)
                # gather into the rank's own output buffer: rank 0's segment already sits at offset 0
                sizes, offs = fdist.exchange_sizes(t.numel(), dist, t.device)
                buf = torch.zeros(sum(sizes) + 16, dtype=torch.uint8)
                if rank == 0 and t.numel():
                    buf[:t.numel()] = t
                    t = buf[:t.numel()]
                n = fdist.gather_segments(t, buf, sizes, offs, dist, 0)
                if rank == 0:
                    results[(idx, codec, "inplace", 0)] = fdist.assemble_file(len(data), block,
                                                                             buf[:n].numpy().tobytes(), codec)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_concat_matches_single_process():
    cases = [
        ({"type": "gen", "kind": "text", "seed": 5, "n": 300000}, 65536),   # 5 blocks: uneven split 2/3
        ({"type": "mosaic", "seed": 7, "n": 200000}, 32768),
        ({"type": "gen", "kind": "rand", "seed": 1, "n": 5000}, 65536),     # 1 block: rank 1 is empty
    ]
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), cases, results), nprocs=2, join=True)
    for idx, (spec, block) in enumerate(cases):
        data = inputs.make(spec)
        want = {"lz77": oracle.compress_file(data, block), "lz78": oracle.lz78_compress_file(data, block)}
        for codec in ("lz77", "lz78"):
            for key in [(idx, codec, "allgather", 0), (idx, codec, "allgather", 1), (idx, codec, "gather", 1),
                        (idx, codec, "inplace", 0)]:
                assert results[key] == want[codec], key
            assert (idx, codec, "gather", 0) not in results   # gather lands on dst only


def test_block_ranges_partition():
    for nb in [0, 1, 2, 5, 8, 1024, 8192]:
        for world in [1, 2, 3, 4, 8]:
            rs = [fdist.block_range(nb, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == nb
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


def test_c_partition_matches_python():
    """fcx_dist_block_range (C, the CLI's -g N and fcx_dist_compress_host) and
    my_compress_amd.dist.block_range (the Python ranks) split identically"""
    import my_compress_amd as mc

    for nb in [0, 1, 2, 5, 8, 1023, 1024, 8192, 65535]:
        for world in [1, 2, 3, 4, 7, 8]:
            for r in range(world):
                assert mc.dist_block_range(nb, r, world) == fdist.block_range(nb, r, world)


def test_dist_needs_a_gpu_without_one():
    import torch

    import my_compress_amd as mc

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(mc.FcxError):
        mc.Dist.local([0])


# ---- gather-aware partition + pipelined gather (fcx_dist_compress_gather's protocol) ----------
def _gather_worker(rank, world, port, cases, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for idx, (spec, block, share, nsub, fail_rank) in enumerate(cases):
            data = inputs.make(spec)
            rb = [(lambda lo_hi: lo_hi[1] - lo_hi[0])(fdist.byte_range(len(data), block, r, world, share))
                  for r in range(world)]
            lo, hi = fdist.byte_range(len(data), block, rank, world, share)
            mine = data[lo:hi]

            def pieces():   # each sub-batch compressed only when the protocol asks for it
                for s, (a, b) in enumerate(fdist.piece_ranges(len(mine), block, nsub)):
                    if rank == fail_rank and s == nsub - 1:
                        raise RuntimeError("injected compress failure")
                    seg = oracle.compress_file(mine[a:b], block)[10:] if b > a else b""
                    yield torch.frombuffer(bytearray(seg), dtype=torch.uint8) if seg else torch.zeros(0, dtype=torch.uint8)

            try:
                if rank == 0:
                    own = oracle.compress_file(mine, block)[10:] if mine else b""
                    out = torch.zeros(2 * len(data) + 4096 * (len(data) // block + 2), dtype=torch.uint8)
                    own_t = torch.frombuffer(bytearray(own), dtype=torch.uint8) if own else torch.zeros(0, dtype=torch.uint8)
                    n = fdist.compress_gather(None, dist, rb, block, nsub, own=own_t, out=out)
                    results[(idx, rank)] = fdist.assemble_file(len(data), block, out[:n].numpy().tobytes())
                else:
                    results[(idx, rank)] = fdist.compress_gather(pieces(), dist, rb, block, nsub)
            except RuntimeError as e:
                results[(idx, rank)] = "error: " + str(e)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_pipelined_gather_uneven_partition(world):
    """rank 0 takes a larger block range (the gather-aware split), the peers send their ranges in
    sub-batches as they compress them; rank 0's assembled file equals the single-process oracle
    file byte for byte.  A peer whose compress fails publishes it: rank 0 raises, nobody hangs."""
    text = {"type": "gen", "kind": "text", "seed": 5, "n": 700000}
    cases = [
        (text, 65536, fdist.gather_share_ppm(world, "text"), 3, -1),
        (text, 65536, 600000, 4, -1),                                      # peers get 1-3 pieces of blocks
        ({"type": "mosaic", "seed": 9, "n": 333333}, 16384, 500000, 1, -1),
        ({"type": "mosaic", "seed": 9, "n": 333333}, 16384, 0, 5, -1),     # even split, 5 pieces
        ({"type": "gen", "kind": "rand", "seed": 1, "n": 70000}, 65536, 900000, 3, -1),   # peers (almost) empty
        (text, 65536, 500000, 2, world - 1),                               # injected failure
    ]
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_gather_worker, args=(world, _free_port(), cases, results), nprocs=world, join=True)
    for idx, (spec, block, share, nsub, fail_rank) in enumerate(cases):
        if fail_rank >= 0:   # every rank learns the job failed (rank 0's verdict), nobody hangs
            assert str(results[(idx, 0)]).startswith("error:") and "failed" in results[(idx, 0)], results[(idx, 0)]
            for r in range(world):
                assert str(results[(idx, r)]).startswith("error:"), (r, results[(idx, r)])
            continue
        data = inputs.make(spec)
        assert results[(idx, 0)] == oracle.compress_file(data, block), (idx, spec, share, nsub)


def test_weighted_partition():
    for nb in [0, 1, 2, 7, 1024, 8192]:
        for world in [1, 2, 3, 4, 8]:
            for ppm in [0, 1, 125000, 500000, 787000, 999999, 1000000]:
                rs = [fdist.block_range(nb, r, world, ppm) for r in range(world)]
                assert rs[0][0] == 0 and rs[-1][1] == nb
                assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
                if world > 1 and ppm:
                    assert rs[0][1] == nb * ppm // 1_000_000
                    peers = [b - a for a, b in rs[1:]]
                    assert max(peers) - min(peers) <= 1


def test_c_weighted_partition_matches_python():
    import my_compress_amd as mc

    for nb in [0, 1, 5, 1024, 8192, 65535]:
        for world in [1, 2, 3, 8]:
            for ppm in [0, 333333, 787000, 1000000]:
                for r in range(world):
                    assert mc.dist_block_range(nb, r, world, ppm) == fdist.block_range(nb, r, world, ppm)


def test_piece_ranges_cover_in_block_order():
    for n, block, nsub in [(0, 4096, 3), (1, 4096, 4), (10 * 4096 + 5, 4096, 4), (1 << 20, 65536, 64)]:
        pr = fdist.piece_ranges(n, block, nsub)
        assert len(pr) == nsub and pr[0][0] == 0 and pr[-1][1] == n
        assert all(pr[i][1] == pr[i + 1][0] for i in range(nsub - 1))
        assert all(a % block == 0 for a, _ in pr)


def test_gather_bound_holds_pieces():
    import my_compress_amd as mc

    for n, block, nsub in [(0, 1 << 20, 4), (5 << 20, 1 << 20, 4), (123456789, 1 << 16, 64), (1 << 30, 1 << 20, 8)]:
        want = sum((mc.shard_bound(hi - lo, block) + 15) // 16 * 16 for lo, hi in fdist.piece_ranges(n, block, nsub))
        assert mc.dist_gather_bound(n, block, nsub) >= max(want, mc.shard_bound(n, block))


def test_step_model_is_monotone_by_design():
    """the gather-aware split keeps the modelled strong-scaling step (1 GiB, gather to rank 0,
    64 GB/s per xGMI link, 4 pieces) below the one-GPU step at every N, for rand and text"""
    for kind in ("rand", "text"):
        c, r = fdist.COMPRESS_MS_PER_GIB[kind], fdist.RATIO[kind]
        t = [fdist.step_model_ms(fdist.gather_share_ppm(n, kind) / 1e6 if n > 1 else 1.0, n, c, r, 64.0, 4)
             for n in (1, 2, 4, 8)]
        assert t[0] > t[1] > t[2] > t[3], (kind, t)
        # the even split with one send at the end (round 3's step) is slower than one GPU at N = 2
        even = fdist.step_model_ms(0.5, 2, c, r, 64.0, 1)
        if kind == "rand":
            assert even > t[0]


# ---- calibration of the gather-aware split (bench.py --concat pipe at N > 1) -------------------
def _calib_worker(rank, world, port, results):
    import time

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # a deterministic probe: rank 0's time is the one used
        fixed = fdist.calibrate_share(dist, "rand", 4, 4.5 + rank, 100 << 20, (101 << 20) + rank * 1000,
                                      lambda: 0.004 if rank == 0 else 9.0)
        # the real pattern over gloo: every peer's segment to rank 0 at once
        seg = torch.full(((3 << 20) * rank,), 7, dtype=torch.uint8)

        def probe():
            sizes, offs = fdist.exchange_sizes(seg.numel(), dist, "cpu")
            buf = torch.empty(sum(sizes) + 1, dtype=torch.uint8)
            t0 = time.perf_counter()
            fdist.gather_segments(seg, buf, sizes, offs, dist, 0)
            return time.perf_counter() - t0

        real = fdist.calibrate_share(dist, "text", 4, 14.0, 64 << 20, seg.numel(), probe)
        results[rank] = (fixed, real)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_calibrated_share_gloo(world):
    """every rank derives the same share from the measured figures: the slowest rank's compress
    rate, the job's ratio and the gather link rate of rank 0's probe"""
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_calib_worker, args=(world, _free_port(), results), nprocs=world, join=True)
    fixed = [results[r][0] for r in range(world)]
    real = [results[r][1] for r in range(world)]
    assert all(f == fixed[0] for f in fixed) and all(x == real[0] for x in real)
    f = fixed[0]
    peer_bytes = (101 << 20) + (world - 1) * 1000
    assert f["c_ms_per_gib"] == 4.5 + world - 1 and f["probe_bytes"] == peer_bytes
    assert abs(f["link_gbps"] - peer_bytes / 0.004 / 1e9) < 1e-9
    ratio = sum((101 << 20) + r * 1000 for r in range(world)) / (world * (100 << 20))
    assert abs(f["ratio"] - ratio) < 1e-12
    assert f["share0_ppm"] == fdist.gather_share_ppm(world, "rand", f["link_gbps"], 4, c_ms=f["c_ms_per_gib"],
                                                     ratio=ratio)
    r = real[0]
    assert 0 < r["share0_ppm"] < 1_000_000 and r["link_gbps"] > 0 and r["probe_ms"] > 0
    assert r["probe_bytes"] == (3 << 20) * (world - 1)
