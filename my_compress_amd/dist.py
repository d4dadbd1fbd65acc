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


def block_range(nblocks: int, rank: int, world: int, share0_ppm: int = 0):
    """contiguous block range [b0, b1) of `rank`.  share0_ppm = 0: the even split (sizes differ
    by at most one block).  Otherwise the gather-aware split (fcx_dist_block_range_w): rank 0,
    the receiver of the concatenation, takes nblocks * share0_ppm // 10^6 blocks first, and
    ranks 1..N-1 split the rest evenly."""
    world = max(world, 1)
    if world == 1 or share0_ppm <= 0:
        return nblocks * rank // world, nblocks * (rank + 1) // world
    n0 = nblocks * min(share0_ppm, 1_000_000) // 1_000_000
    if rank == 0:
        return 0, n0
    p0, p1 = block_range(nblocks - n0, rank - 1, world - 1)
    return n0 + p0, n0 + p1


def byte_range(n: int, block_bytes: int, rank: int, world: int, share0_ppm: int = 0):
    nblocks = (n + block_bytes - 1) // block_bytes
    b0, b1 = block_range(nblocks, rank, world, share0_ppm)
    return min(n, b0 * block_bytes), min(n, b1 * block_bytes)


def piece_ranges(n: int, block_bytes: int, nsub: int):
    """the nsub sub-batches of a rank's n bytes (whole blocks, near-even), as fcx_dist's piece_range"""
    nb = (n + block_bytes - 1) // block_bytes
    out = []
    for s in range(nsub):
        b0, b1 = block_range(nb, s, nsub)
        out.append((min(n, b0 * block_bytes), min(n, b1 * block_bytes)))
    return out


# ---- the strong-scaling step model --------------------------------------------
# One GPU's compress time per GiB and output ratio for each synthetic kind at 1 MiB blocks
# (bench.py on one MI355X, profiles/r06_bench_n1.json), the defaults of gather_share_ppm.
COMPRESS_MS_PER_GIB = {"rand": 4.30, "text": 13.0, "zeros": 2.70, "runs": 11.9, "dna": 28.0, "mix": 14.0}
RATIO = {"rand": 1.0163, "text": 0.5805, "zeros": 0.0070, "runs": 0.0396, "dna": 0.3112, "mix": 0.487}


def step_model_ms(share0: float, world: int, c_ms: float, ratio: float, link_gbps: float, nsub: int,
                  gib: float = 1.0, copy_gbps: float = 2500.0):
    """modelled ms of one gather step of `gib` GiB: rank 0 compresses share0 of the input while
    each peer compresses (1 - share0) / (N - 1) of it in nsub pieces and sends each piece over its
    own link as soon as it is done (pipeline: first piece, then the slower of compress and send per
    piece, then the last send); rank 0 then moves the peers' bytes behind its segment (an HBM copy,
    read + write at copy_gbps).  c_ms: one GPU's compress ms per GiB."""
    if world <= 1:
        return gib * c_ms
    gp = (1.0 - share0) / (world - 1) * gib
    a = gp * c_ms / nsub                                   # one piece's compress
    b = gp * ratio * (1 << 30) / (link_gbps * 1e9) * 1e3 / nsub   # one piece's send
    peer = a + (nsub - 1) * max(a, b) + b
    copy = (1.0 - share0) * gib * ratio * (1 << 30) * 2 / (copy_gbps * 1e9) * 1e3
    return max(share0 * gib * c_ms, peer) + copy


def gather_share_ppm(world: int, kind: str = "rand", link_gbps: float = 64.0, nsub: int = 4,
                     c_ms: float = None, ratio: float = None) -> int:
    """rank 0's block share (ppm) that minimises step_model_ms; 0 (even split) for one rank"""
    if world <= 1:
        return 0
    c_ms = COMPRESS_MS_PER_GIB.get(kind, 14.1) if c_ms is None else c_ms
    ratio = RATIO.get(kind, 1.0) if ratio is None else ratio
    best = min(range(1000, 1_000_000, 1000), key=lambda p: step_model_ms(p / 1e6, world, c_ms, ratio, link_gbps, nsub))
    return best


def calibrate_share(dist, kind: str, nsub: int, c_ms_per_gib: float, in_bytes: int, out_bytes: int, probe,
                    device="cpu", group=None) -> dict:
    """the gather-aware share from one warmup step's measurements instead of assumed rates.
    Every rank passes its measured compress ms per GiB, its shard's input bytes and its compressed
    segment's bytes; probe() gathers every peer's segment to rank 0 over the job's transport (the
    real exchange pattern: all peers send at once, each over its own link) and returns its seconds
    (rank 0's value is used).  The link rate is the largest peer segment over that time; the compress
    rate is the slowest rank's; the ratio is the job's.  Returns, identically on every rank:
    share0_ppm (the step model's choice with the measured figures), link_gbps, c_ms_per_gib, ratio,
    probe_ms, probe_bytes (the largest peer segment) and the model's predicted step ms."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    mx = torch.tensor([float(c_ms_per_gib), float(out_bytes if rank else 0)], dtype=torch.float64, device=device)
    sm = torch.tensor([float(in_bytes), float(out_bytes)], dtype=torch.float64, device=device)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(sm, op=dist.ReduceOp.SUM, group=group)
    secs = torch.tensor([float(probe())], dtype=torch.float64, device=device)
    dist.broadcast(secs, 0, group=group)
    c_ms, peer_bytes = float(mx[0]), float(mx[1])
    ratio = float(sm[1]) / max(float(sm[0]), 1.0)
    t = max(float(secs[0]), 1e-6)
    link = peer_bytes / t / 1e9 if peer_bytes > 0 else float("inf")
    link_m = min(link, 1e4)   # (no peer bytes: the exchange costs nothing, the model wants a finite rate)
    share = gather_share_ppm(world, kind, link_m, nsub, c_ms=c_ms, ratio=ratio)
    gib = float(sm[0]) / (1 << 30)
    return {"share0_ppm": share, "link_gbps": link, "c_ms_per_gib": c_ms, "ratio": ratio, "probe_ms": t * 1e3,
            "probe_bytes": int(peer_bytes),
            "model_ms": step_model_ms(share / 1e6, world, c_ms, ratio, link_m, nsub, gib=gib)}


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


def compress_gather(pieces, dist, rank_bytes, block_bytes: int, nsub: int, own=None, out=None, group=None,
                    device=None, own_error=None):
    """fcx_dist_compress_gather's protocol over torch.distributed (the `--concat-impl torch` path
    and the gloo tests).  A peer passes `pieces`, an iterable of its nsub sub-batch segments in
    order (uint8 tensors, e.g. compressed one by one as they are consumed): each is sent as it is
    produced, an int64 pair (length, error) first, then its bytes.  Rank 0 passes its own
    segment `own` (already at out[:len], or copied there) and `out` (>= the whole
    concatenation); per round s it receives every peer's length pair, then every peer's bytes
    into a staging region per peer, and finally moves them behind its own segment in rank order.
    A peer that fails sends (-1, 1) for this and every later round.  Rank 0 then sends the job's
    verdict (0 or 1) to every peer, so every rank raises when any rank failed -- a peer's failure,
    a piece beyond its peer's staging bound (drained, not stored), rank 0's own failure
    (`own_error`, a message) or an `out` too small for the whole concatenation.  `device`: where a
    peer's control words live (its pieces' device; required under nccl, which cannot send CPU
    tensors).  Returns the concatenated length on rank 0, the bytes sent on a peer."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    dev = out.device if out is not None else torch.device(device if device is not None else "cpu")
    if rank != 0:
        sent, failed = 0, False
        it = iter(pieces)
        for s in range(nsub):
            seg = None
            if not failed:
                try:
                    seg = next(it)
                except Exception:   # a failed compress: publish it, keep the protocol
                    failed = True
            n = 0 if failed else int(seg.numel())
            words = torch.tensor([-1, 1] if failed else [n, 0], dtype=torch.int64, device=dev)
            dist.send(words, 0, group)
            if n:
                dist.send(seg.contiguous(), 0, group)
            sent += n
        verdict = torch.zeros(1, dtype=torch.int64, device=dev)
        dist.recv(verdict, 0, group)
        if failed:
            raise RuntimeError("compress_gather: this rank's compress failed")
        if int(verdict.item()):
            raise RuntimeError("compress_gather: rank 0 reports the job failed")
        return sent
    stage_cap = [0] + [sum(2 * (hi - lo) + 4096 * ((hi - lo + block_bytes - 1) // block_bytes) + 64
                           for lo, hi in piece_ranges(rank_bytes[r], block_bytes, nsub)) for r in range(1, world)]
    stage = [torch.empty(max(c, 1), dtype=torch.uint8, device=dev) for c in stage_cap]
    fill = [0] * world
    err = None
    for s in range(nsub):
        words = [torch.zeros(2, dtype=torch.int64, device=dev) for _ in range(world)]
        ops = [dist.P2POp(dist.irecv, words[r], r, group) for r in range(1, world)]
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        ops = []
        for r in range(1, world):
            n, e = int(words[r][0]), int(words[r][1])
            if e or n < 0:
                err = err or f"rank {r} failed in sub-batch {s}"
                continue
            if n and fill[r] + n > stage_cap[r]:   # beyond the peer's bound: drained, the job fails
                err = err or f"rank {r} sent a piece beyond its bound in sub-batch {s}"
                ops.append(dist.P2POp(dist.irecv, torch.empty(n, dtype=torch.uint8, device=dev), r, group))
            elif n:
                ops.append(dist.P2POp(dist.irecv, stage[r][fill[r]:fill[r] + n], r, group))
                fill[r] += n
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
    n_own = int(own.numel()) if own is not None else 0
    if not err and own_error:
        err = f"rank 0 failed: {own_error}"
    if not err and (out is None or n_own + sum(fill) > out.numel()):
        err = f"output capacity too small ({n_own + sum(fill)} B)"
    verdict = torch.tensor([1 if err else 0], dtype=torch.int64, device=dev)
    ops = [dist.P2POp(dist.isend, verdict, r, group) for r in range(1, world)]
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    if err:
        raise RuntimeError("compress_gather: " + err)
    _place_own(own if own is not None else torch.zeros(0, dtype=torch.uint8, device=dev), out, 0)
    off = n_own
    for r in range(1, world):
        out[off:off + fill[r]].copy_(stage[r][:fill[r]])
        off += fill[r]
    return off


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
