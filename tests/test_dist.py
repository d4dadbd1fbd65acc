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
