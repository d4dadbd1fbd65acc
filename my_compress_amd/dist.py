"""Multi-GPU sharding of the FCX7 compress path (and of FCX8, the -c lz78 codec,
whose records are framed the same way).

Blocks are independent (the window and the parse restart per block,
my_compress.cpp:1675-1703, and main() zeroes its buffers between blocks,
4118-4119), so N ranks take contiguous block ranges and compress them with no
data-path communication.  The one exchange is the final concatenation of the
per-rank segments ([u32 len][payload]... each) in rank order: an all-gather of
the segment sizes, then of the segments padded to the largest (RCCL over xGMI
on GPUs, gloo on CPU tensors in tests).  The 10-byte header is written by the
host from the global totals (main(), 4128-4129).
"""
import torch

from . import write_header


def block_range(nblocks: int, rank: int, world: int):
    """contiguous block range [b0, b1) of `rank`"""
    return nblocks * rank // world, nblocks * (rank + 1) // world


def byte_range(n: int, block_bytes: int, rank: int, world: int):
    nblocks = (n + block_bytes - 1) // block_bytes
    b0, b1 = block_range(nblocks, rank, world)
    return min(n, b0 * block_bytes), min(n, b1 * block_bytes)


def concat_segments(seg: torch.Tensor, dist, group=None) -> torch.Tensor:
    """all-gather the ranks' segments (1-D uint8 tensors of any length, on the
    backend's device) and return their concatenation in rank order, on every rank"""
    world = dist.get_world_size(group)
    dev = seg.device
    size = torch.tensor([seg.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, size, group=group)
    szs = [int(s.item()) for s in sizes]
    mx = max(max(szs), 1)
    send = torch.zeros(mx, dtype=torch.uint8, device=dev)
    send[:seg.numel()] = seg
    recv = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(recv, send, group=group)
    return torch.cat([recv[r][:szs[r]] for r in range(world)])


def assemble_file(total_in: int, block_bytes: int, body: bytes, codec: str = "lz77") -> bytes:
    """header + concatenated records; codec "lz78" writes the "FCX8" tag (-c lz78 files,
    same framing, main() 4079-4086)"""
    nblocks = (total_in + block_bytes - 1) // block_bytes
    hdr = write_header(total_in, nblocks)
    if codec == "lz78":
        hdr = b"FCX8" + hdr[4:]
    return hdr + body
