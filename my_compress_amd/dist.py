"""Multi-GPU sharding of the FCX7 compress path (and of FCX8, the -c lz78 codec,
whose records are framed the same way).

Blocks are independent (the window and the parse restart per block,
my_compress.cpp:1675-1703, and main() zeroes its buffers between blocks,
4118-4119), so N ranks take contiguous block ranges and compress them with no
data-path communication.  The one exchange is the final concatenation of the
per-rank segments ([u32 len][payload]... each) in rank order, which the
reference does by writing blocks to one file in order (4112-4114).  Two forms,
both writing straight into one contiguous output buffer (no padding, no second
copy), over RCCL/xGMI on GPUs and gloo on CPU tensors in tests:

  gather_segments     rank `dst` receives every segment at its offset (grouped
                      point-to-point receives, one per peer, all xGMI links at
                      once): 1/N of the all-gather's traffic; the file writer's form
  allgather_segments  every rank ends with the whole stream (one broadcast per
                      source rank, exact sizes, into the same offsets)

Both start with exchange_sizes (an all-gather of one int64 per rank).  The
10-byte header is written by the host from the global totals (main(),
4128-4129).
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


def exchange_sizes(seg_len: int, dist, device, group=None):
    """all-gather of the per-rank segment sizes; returns (sizes, offsets) in rank order"""
    world = dist.get_world_size(group)
    mine = torch.tensor([seg_len], dtype=torch.int64, device=device)
    allv = torch.empty(world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(allv, mine, group=group)
    sizes = [int(x) for x in allv.tolist()]
    offs = [0] * world
    for r in range(1, world):
        offs[r] = offs[r - 1] + sizes[r - 1]
    return sizes, offs


def _place_own(seg: torch.Tensor, out: torch.Tensor, off: int):
    """put this rank's segment at its offset of `out` unless it already lives there"""
    n = seg.numel()
    if n and seg.data_ptr() != out.data_ptr() + off:
        out[off:off + n].copy_(seg)


def gather_segments(seg: torch.Tensor, out, sizes, offs, dist, dst: int = 0, group=None) -> int:
    """rank `dst` receives every rank's segment into out[offs[r]:offs[r]+sizes[r]]
    (out: a 1-D uint8 tensor of >= sum(sizes) bytes on dst, ignored elsewhere).
    A segment that already is out[:n] on dst (the compress output buffer reused as
    the file buffer) is not copied.  Returns the total length."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    ops = []
    if rank == dst:
        _place_own(seg, out, offs[rank])
        for r in range(world):
            if r != dst and sizes[r]:
                ops.append(dist.P2POp(dist.irecv, out[offs[r]:offs[r] + sizes[r]], r, group))
    elif sizes[rank]:
        ops.append(dist.P2POp(dist.isend, seg[:sizes[rank]], dst, group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return sum(sizes)


def allgather_segments(seg: torch.Tensor, out: torch.Tensor, sizes, offs, dist, group=None) -> int:
    """every rank ends with the whole concatenation in out[:sum(sizes)]: one
    broadcast per source rank with its exact size (an all-gather-v without the
    padding of a plain all-gather).  Returns the total length."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    _place_own(seg, out, offs[rank])
    works = []
    for r in range(world):
        if sizes[r]:
            works.append(dist.broadcast(out[offs[r]:offs[r] + sizes[r]], src=r, group=group, async_op=True))
    for w in works:
        w.wait()
    return sum(sizes)


def concat_segments(seg: torch.Tensor, dist, group=None, mode: str = "allgather", dst: int = 0):
    """convenience: exchange sizes, then concatenate into a fresh buffer; returns the
    whole stream (on every rank for "allgather", on dst for "gather", else None)"""
    sizes, offs = exchange_sizes(seg.numel(), dist, seg.device, group)
    rank = dist.get_rank(group)
    out = None
    if mode == "allgather" or rank == dst:
        out = torch.empty(max(sum(sizes), 1), dtype=torch.uint8, device=seg.device)
    if mode == "allgather":
        n = allgather_segments(seg, out, sizes, offs, dist, group)
    elif mode == "gather":
        n = gather_segments(seg, out, sizes, offs, dist, dst, group)
    else:
        raise ValueError(mode)
    return out[:n] if out is not None else None


def assemble_file(total_in: int, block_bytes: int, body: bytes, codec: str = "lz77") -> bytes:
    """header + concatenated records; codec "lz78" writes the "FCX8" tag (-c lz78 files,
    same framing, main() 4079-4086)"""
    nblocks = (total_in + block_bytes - 1) // block_bytes
    hdr = write_header(total_in, nblocks)
    if codec == "lz78":
        hdr = b"FCX8" + hdr[4:]
    return hdr + body
