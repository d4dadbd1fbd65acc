#!/usr/bin/env python3
"""bench.py — compress throughput of the MI355X FCX7 LZ77 + Huffman path.

Metric (BASELINE.json): compress MB/s on 1 GB synthetic bytes at 1/2/4/8 MI355X;
% HBM roofline.  One process per GPU (torchrun for N > 1), RCCL over xGMI.

Headline (default, `scaling: strong`): ONE 1 GiB input (--global-mib) split into
contiguous block ranges over the N ranks.  A timed step is the
whole job: every rank compresses its device-resident shard into [u32 len][payload]
records in HBM and the segments end up concatenated in rank order in one contiguous
stream on rank 0.  --concat pipe (default): the gather-aware partition (rank 0, the
receiver, takes a larger block range, --share0, by default the share the step model
of my_compress_amd.dist picks) and fcx_dist_compress_gather: the peers compress in
--nsub pieces and send each piece over their xGMI link while the next compresses,
rank 0 compresses its range meanwhile.  --concat gather: even split, compress, then a
sizes all-gather and grouped point-to-point receives; `allgather`: every rank gets
the stream, one broadcast per source rank.  `value` = global input bytes x K / the
max-over-ranks time of K such steps.  At N=1 there is nothing to concatenate.
The compress-only rate (no exchange) is reported beside it.  The assembled stream
is checked against the reference's SHA-256 (HL-rand / HL-text / C3 / C5 digests,
SURVEY.md §8(c)) at every N.

Extra leg `weak` (N > 1; BASELINE config 4): rank r compresses bytes [r GiB,
(r+1) GiB) of the seed-4 rand stream, each rank's segment checked against the
reference's, the N segments gathered to rank 0.

    python bench.py                      # N=1, defaults
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        --master-port 29500 bench.py --gpus 8
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

METRIC = "compress MB/s on 1 GB synthetic bytes at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
GiB = 1 << 30
HL_DIGEST = {  # reference output digests of whole files: (kind, seed, bytes, block)
    ("rand", 4, GiB, 1 << 20): ("ee962534628bf6b2f79c51a44a65ac0845945e2fe9225e5be8f99f288912a69d", 1091294206),
    ("text", 3, GiB, 1 << 20): ("132a36b9d2592f8c37a82b51f545ddb67acec53fa1a31b7f1f6a04617a01a3d1", 624801500),
    ("text", 3, GiB, 1 << 18): ("20219e60c2e9aef6659801fbfc53c6873ec811686eedcb45c0896fc5547d63d0", 630008807),
    ("zeros", 0, GiB, 1 << 20): ("533fd45fbaa861a6060e9a5beac177cc0b64db691fc602a1e0e1e188afa5f912", 7521290),
    ("runs", 5, GiB, 1 << 20): ("4fced94fd4725ba3b1031dec67d63e1295b95ae08cc1cf0e34c84769f5313d26", 42548682),
    ("rand", 2, 64 << 20, 1 << 16): ("3b6853f2cf570b7a35c469efff62c15e0290b04ede45f6b47a97afc82c1878a5", 68819158),
    # the mix leg: the reference compiled in place, tests/golden/make_mix_digest.py
    ("mix", 0, GiB, 1 << 20): ("ce8bb8bc756a62fcd276d6a71b93456c18a7def3d77e555ea7eb8b92bfebffb5", 523200760),
}
SEEDS = {"rand": 4, "text": 3, "runs": 5, "zeros": 0, "dna": 6, "mix": 0}
# extra legs after the main one: name -> (kind, block bytes[, seed, MiB]); BASELINE configs 2
# (64 MiB of seed-2 random bytes at 64 KiB blocks), 3 and 5, plus "dna" (rand()%4 bytes: dense
# 3-byte buckets) and "mix" (1 MiB blocks cycling rand / text / runs / dna: every match unit in
# one call, tests/inputs.py mix_into)
LEGS = {"c2": ("rand", 1 << 16, 2, 64), "text": ("text", 1 << 20), "c3": ("text", 1 << 18),
        "zeros": ("zeros", 1 << 20), "runs": ("runs", 1 << 20), "dna": ("dna", 1 << 20), "mix": ("mix", 1 << 20)}
# legs whose first call on a fresh context is timed beside the steady state (cold_call)
COLD_LEGS = ("rand", "text", "mix")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_input(kind, seed, lo, hi, pinned=True):
    """bytes [lo, hi) of the synthetic stream `kind`/`seed` in a
    (pinned) host tensor.  rand jumps ahead in O(log lo); the other streams are
    generated from their start and sliced."""
    import torch

    import inputs

    n = hi - lo
    host = torch.empty(max(n, 1), dtype=torch.uint8)
    if pinned:
        host = host.pin_memory()
    if kind in ("rand", "dna"):
        inputs.rand_stream_into(seed, lo, host.data_ptr(), n, kind)
    elif kind == "mix" and lo:
        whole = torch.empty(hi, dtype=torch.uint8)
        inputs.mix_into(whole.data_ptr(), hi)
        host[:n].copy_(whole[lo:hi])
        del whole
    elif kind == "zeros" or lo == 0:
        inputs.generate_into(kind, seed, host.data_ptr(), n)
    else:
        whole = torch.empty(hi, dtype=torch.uint8)
        inputs.generate_into(kind, seed, whole.data_ptr(), hi)
        host[:n].copy_(whole[lo:hi])
        del whole
    return host


def max_over_ranks(dt, dist, dev):
    import torch

    if not dist:
        return dt
    tt = torch.tensor([dt], dtype=torch.float64)
    if dist.get_backend() != "gloo":
        tt = tt.to(dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


def timed(fn, steps, dist, dev):
    """barrier + synchronize on both sides of `steps` calls; max over ranks"""
    import torch

    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    return max_over_ranks(time.perf_counter() - t0, dist, dev)


def setup_leg(kind, seed, block, args, rank, world, dev, scaling, n_global, share0, concat, main_leg):
    """this rank's input (device-resident) and output buffers for one partition of the leg"""
    import torch

    import my_compress_amd as mc
    from my_compress_amd import dist as fdist

    if scaling == "strong":
        ranges = [fdist.byte_range(n_global, block, r, world, share0) for r in range(world)]
    else:
        per = n_global // world
        ranges = [(r * per, (r + 1) * per) for r in range(world)]
    lo, hi = ranges[rank]
    S = {"ranges": ranges, "rank_bytes": [b - a for a, b in ranges], "n": hi - lo, "share0": share0}
    n = S["n"]
    t = time.time()
    if scaling == "weak" and kind != "rand":
        host = make_input(kind, seed + rank, 0, n)   # independent per-rank streams
    else:
        host = make_input(kind, seed, lo, hi)
    S["gen_s"] = time.time() - t
    S["d_in"] = host.to(dev)
    S["host_path"] = None
    if world == 1 and args.host_path and main_leg:
        S["host_path"] = host_leg(host, n, block)
    del host
    # gather / pipe: rank 0's compress output buffer is also the file buffer (its segment sits at
    # offset 0); pipe: a peer's pieces sit at their bound offsets
    cap = mc.shard_bound(n_global if (concat in ("gather", "pipe") and rank == 0) else n, block)
    if concat == "pipe" and rank != 0:
        cap = mc.dist_gather_bound(n, block, args.nsub)
    S["cap"] = cap
    S["d_out"] = torch.empty(cap, dtype=torch.uint8, device=dev)
    S["whole"] = None
    if concat == "allgather":
        S["whole"] = torch.empty(mc.shard_bound(n_global, block), dtype=torch.uint8, device=dev)
    S["ctx"] = mc.Context(dev.index, block, max(n, block))
    return S


def calibrate_leg(S, kind, block, args, rank, world, dev, dist):
    """the pipe step's partition from measurements (one warmup step): this rank's compress ms per
    GiB (its whole shard, one timed call), its compressed bytes, and the link rate of the gather
    pattern itself (every peer's contiguous segment to rank 0 at once, over the same transport the
    step uses: fcx_dist_concat, or torch.distributed)"""
    import torch

    import my_compress_amd as mc
    from my_compress_amd import dist as fdist

    n, ctx, d_in, d_out, cap = S["n"], S["ctx"], S["d_in"], S["d_out"], S["cap"]
    sid = torch.cuda.current_stream(dev).cuda_stream
    seg = 0
    best = float("inf")
    for _ in range(2):   # (the first call also warms the context's scratch)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        seg = ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, sid) if n else 0
        best = min(best, time.perf_counter() - t0)
    c_ms = best * 1e3 / max(n / GiB, 1e-9) if n else 0.0
    gloo = dist.get_backend() == "gloo"

    def probe():
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if args.fcx_dist is not None:
            args.fcx_dist.concat(d_out.data_ptr(), seg, d_out.data_ptr(), cap, mc.DIST_GATHER, sid)
        else:
            sizes, offs = fdist.exchange_sizes(seg, dist, "cpu" if gloo else dev)
            if gloo:
                buf = torch.empty(sum(sizes) + 1, dtype=torch.uint8)
                fdist.gather_segments(d_out[:seg].cpu(), buf, sizes, offs, dist, 0)
            else:
                fdist.gather_segments(d_out[:seg], d_out, sizes, offs, dist, 0)
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0

    cal = fdist.calibrate_share(dist, kind, args.nsub, c_ms, n, seg, probe, device="cpu" if gloo else dev)
    cal["assumed_link_gbps"] = args.link_gbps
    cal["share0_ppm_assumed_link"] = S["share0"]
    return cal


def run_leg(kind, seed, block, args, rank, world, dev, dist, profile_stages, scaling="strong", main_leg=False,
            global_mib=None):
    """one leg.  strong: the global input of global_mib (default args.global_mib) MiB split over
    the ranks; weak: args.mib MiB per rank (rand: rank r = bytes [r*shard, (r+1)*shard) of one stream)."""
    import torch

    import my_compress_amd as mc
    from my_compress_amd import dist as fdist

    concat = args.concat if dist else "none"
    share0 = 0
    if scaling == "strong":
        n_global = (global_mib or args.global_mib) << 20
        if concat == "pipe" and world > 1:   # the gather-aware partition (the model at the assumed link rate)
            share0 = args.share0_ppm if args.share0_ppm >= 0 else fdist.gather_share_ppm(
                world, kind, args.link_gbps, args.nsub)
    else:
        n_global = (args.mib << 20) * world
    S = setup_leg(kind, seed, block, args, rank, world, dev, scaling, n_global, share0, concat, main_leg)
    calib = None
    if concat == "pipe" and scaling == "strong" and world > 1 and args.share0_ppm < 0 and args.calibrate:
        calib = calibrate_leg(S, kind, block, args, rank, world, dev, dist)
        if calib["share0_ppm"] != share0:   # re-partition with the measured figures
            nb = (n_global + block - 1) // block
            moved = fdist.block_range(nb, 0, world, calib["share0_ppm"]) != fdist.block_range(nb, 0, world, share0)
            share0 = calib["share0_ppm"]
            if moved:
                S["ctx"].close()
                S.clear()
                torch.cuda.empty_cache()
                S = setup_leg(kind, seed, block, args, rank, world, dev, scaling, n_global, share0, concat, main_leg)
    ranges, rank_bytes, n = S["ranges"], S["rank_bytes"], S["n"]
    d_in, d_out, cap, whole, ctx = S["d_in"], S["d_out"], S["cap"], S["whole"], S["ctx"]
    gen_s, host_path = S["gen_s"], S["host_path"]
    sid = torch.cuda.current_stream(dev).cuda_stream
    state = {}

    def compress():
        if n:
            ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, sid, sync=False)

    def pieces():   # torch pipe path, a peer: its sub-batches compressed one by one as they are sent
        o = 0
        for a, b in fdist.piece_ranges(n, block, args.nsub):
            pb = mc.shard_bound(b - a, block)
            got = ctx.compress_shard(d_in.data_ptr() + a, b - a, d_out.data_ptr() + o, pb, sid) if b > a else 0
            seg = d_out[o:o + got]
            yield seg.cpu() if dist.get_backend() == "gloo" else seg
            o += (pb + 15) // 16 * 16

    def step():   # the whole job: compress, sizes, concatenation in rank order
        if concat == "pipe":
            if args.fcx_dist is not None:   # C++ RCCL path: compress and gather overlapped
                state["total"] = args.fcx_dist.compress_gather(ctx, d_in.data_ptr(), n, rank_bytes, args.nsub,
                                                               d_out.data_ptr(), cap, sid)
                return
            gloo = dist.get_backend() == "gloo"
            if rank == 0:
                own = d_out[:ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, sid)] if n else d_out[:0]
                if gloo:   # rehearsal without RCCL: the pieces travel through host memory
                    hout = torch.empty(cap, dtype=torch.uint8)
                    tot = fdist.compress_gather(None, dist, rank_bytes, block, args.nsub, own=own.cpu(), out=hout)
                    d_out[:tot].copy_(hout[:tot])
                else:
                    tot = fdist.compress_gather(None, dist, rank_bytes, block, args.nsub, own=own, out=d_out)
                state["total"] = tot
            else:
                state["total"] = fdist.compress_gather(pieces(), dist, rank_bytes, block, args.nsub,
                                                       device=None if gloo else dev)
            return
        compress()
        seg_len = ctx.read_out_len() if n else 0
        if concat == "none":
            state["total"] = seg_len
            return
        if args.fcx_dist is not None:   # C++ RCCL path: sizes all-gather + gather / all-gather-v
            dst = d_out if concat == "gather" else whole
            mode = mc.DIST_GATHER if concat == "gather" else mc.DIST_ALLGATHER
            state["total"] = args.fcx_dist.concat(d_out.data_ptr(), seg_len, dst.data_ptr(), dst.numel(), mode, sid)
            state["seg"] = seg_len
            return
        sizes, offs = fdist.exchange_sizes(seg_len, dist, dev if dist.get_backend() != "gloo" else "cpu")
        seg = d_out[:seg_len]
        if dist.get_backend() == "gloo":   # rehearsal without RCCL: the segments travel through host memory
            hbuf = torch.empty(sum(sizes) + 1, dtype=torch.uint8)
            hseg = seg.cpu()
            if concat == "gather":
                fdist.gather_segments(hseg, hbuf, sizes, offs, dist, 0)
            else:
                fdist.allgather_segments(hseg, hbuf, sizes, offs, dist)
            if rank == 0:
                (d_out if concat == "gather" else whole)[:sum(sizes)].copy_(hbuf[:sum(sizes)])
        elif concat == "gather":
            fdist.gather_segments(seg, d_out, sizes, offs, dist, 0)
        else:
            fdist.allgather_segments(seg, whole, sizes, offs, dist)
        state["total"], state["seg"] = sum(sizes), seg_len

    step()   # validates the call, creates the communicators
    for _ in range(args.warmup):
        step()
    # compress only (device-resident, no exchange): K steps back to back, then the per-kernel hipEvent
    # times from K more steps outside the timed region (their per-step event reads synchronise)
    dt_c = timed(compress, args.steps, dist, dev)
    stage_sum = {}
    if profile_stages and n:
        ctx.set_profiling(True)
        for _ in range(args.steps):
            compress()
            for name, ms in ctx.stage_times():   # waits for this step's last event
                stage_sum[name] = stage_sum.get(name, 0.0) + ms
        ctx.set_profiling(False)
    seg_len = ctx.read_out_len() if n else 0
    # the whole job, K steps
    dt = timed(step, args.steps, dist, dev) if concat != "none" else dt_c
    total = state.get("total", seg_len)
    res = {
        "kind": kind, "block_bytes": block, "scaling": scaling, "global_bytes": n_global, "bytes_this_rank": n,
        "out_bytes": total, "ratio": total / max(n_global, 1), "concat": CONCAT_FORMS.get(concat, concat),
        "seconds": dt, "ms_per_step": dt / args.steps * 1e3, "value": n_global * args.steps / dt / 1e6,
        "compress_only": {"value": n_global * args.steps / dt_c / 1e6, "ms_per_step": dt_c / args.steps * 1e3,
                          "note": "device-resident compress of every rank's shard, no exchange (max over ranks)"},
        "gen_s": gen_s, "stages_ms": {k: v / args.steps for k, v in stage_sum.items()}, "host_path": host_path,
        "seg_bytes_rank0": seg_len,
    }
    if concat != "none":
        res["concat_ms_per_step"] = res["ms_per_step"] - res["compress_only"]["ms_per_step"]
        res["concat_impl"] = (f"fcx_dist (C++, {args.fcx_dist.transport()} transport)" if args.fcx_dist is not None
                              else f"torch.distributed ({dist.get_backend()})")
        res["partition"] = {"share0_ppm": share0, "rank_bytes": rank_bytes,
                            "nsub": args.nsub if concat == "pipe" else None}
        if concat == "pipe" and scaling == "strong":
            res["partition"]["model_ms_assumed_link"] = fdist.step_model_ms(
                (share0 / 1e6) if share0 else 1.0 / world, world, fdist.COMPRESS_MS_PER_GIB.get(kind, 14.1),
                fdist.RATIO.get(kind, 1.0), args.link_gbps, args.nsub, gib=n_global / GiB)
            res["partition"]["assumed_link_gbps"] = args.link_gbps
            if calib is not None:
                res["partition"]["calibration"] = calib
                res["partition"]["measured_link_gbps"] = calib["link_gbps"]
                res["partition"]["model_ms"] = calib["model_ms"]
                res["partition"]["source"] = "measured (one warmup step: compress rate, ratio, gather link rate)"
            else:
                res["partition"]["source"] = ("--share0" if args.share0_ppm >= 0 else
                                              f"step model at the assumed {args.link_gbps} GB/s link")
    res["match_kernel"] = ctx.match_kernel() if n else None   # (the timed steps' match stage)
    if n:   # tiles per match unit in the last call (fcx_route.hip)
        res["route"] = ctx.route_stats()
    if n and kind in COLD_LEGS and (main_leg or world == 1):
        res["cold_call"] = cold_call(d_in, n, cap, block, dev, res["compress_only"]["ms_per_step"])
    stats = ctx.stats() if n else {"tokens": 0, "matches": 0, "lazy_evals": 0, "lazy_tiles": 0}
    res["tokens"], res["matches"] = stats["tokens"], stats["matches"]
    res["lazy_evals"], res["lazy_tiles"] = stats["lazy_evals"], stats["lazy_tiles"]
    if not args.no_verify:
        res.update(verify(kind, seed, block, n_global, scaling, rank, world, dev, dist, d_out, whole, concat,
                          seg_len, total))
    if concat == "pipe" and n:   # (a peer's pieces sit at their bound offsets: its own records again)
        compress()
        seg_len = ctx.read_out_len()
    if not args.no_decode and (main_leg or world == 1):
        res["decode"] = decode_leg(d_out, seg_len, n, block, d_in, args, dev, dist, world)
    ctx.close()
    S.clear()
    del d_in, d_out, whole
    torch.cuda.empty_cache()
    return res


def verify(kind, seed, block, n_global, scaling, rank, world, dev, dist, d_out, whole, concat, seg_len, total):
    """digest of the assembled stream (rank 0) against the reference's; weak rand:
    every rank's segment against SURVEY.md B.3"""
    import torch

    import inputs
    import my_compress_amd as mc

    out = {}
    if scaling == "weak" and kind == "rand" and seed == 4 and n_global // world == GiB and concat == "pipe":
        # the segments arrive concatenated on rank 0: each rank's slice against SURVEY.md B.3
        oks = []
        if rank == 0:
            off = 0
            for r in range(world):
                want_bytes, want_prefix = inputs.C4_SEGMENTS[r] if r < len(inputs.C4_SEGMENTS) else (-1, "")
                h = hashlib.sha256(memoryview(d_out[off:off + want_bytes].cpu().numpy())).hexdigest()
                oks.append(int(want_bytes > 0 and off + want_bytes <= total and h[:16] == want_prefix))
                off += max(want_bytes, 0)
            oks[-1] &= int(off == total)
            out["rank_segments_bit_exact"] = oks
            out["bit_exact_vs_reference"] = all(oks)
        return out
    if scaling == "weak" and kind == "rand" and seed == 4 and n_global // world == GiB:
        ok = 0
        if rank < len(inputs.C4_SEGMENTS):
            want_bytes, want_prefix = inputs.C4_SEGMENTS[rank]
            h = hashlib.sha256(memoryview(d_out[:seg_len].cpu().numpy())).hexdigest()
            ok = int(seg_len == want_bytes and h[:16] == want_prefix)
        flags = torch.tensor([ok], dtype=torch.int64)
        if dist:
            if dist.get_backend() != "gloo":
                flags = flags.to(dev)
            allf = [torch.zeros_like(flags) for _ in range(world)]
            dist.all_gather(allf, flags)
            oks = [int(x.item()) for x in allf]
        else:
            oks = [ok]
        out["rank_segments_bit_exact"] = oks
        out["bit_exact_vs_reference"] = all(oks)
        return out
    key = (kind, seed, n_global, block)
    if key not in HL_DIGEST or rank != 0:
        return out
    stream = d_out if concat in ("none", "gather", "pipe") else whole
    h = hashlib.sha256(mc.write_header(n_global, (n_global + block - 1) // block))
    h.update(memoryview(stream[:total].cpu().numpy()))
    want_sha, want_bytes = HL_DIGEST[key]
    out["bit_exact_vs_reference"] = h.hexdigest() == want_sha and total + 10 == want_bytes
    out["checked"] = "sha256 of header + assembled stream on rank 0 vs the reference's file (SURVEY.md B.4)"
    return out


def cold_call(d_in, n, cap, block, dev, steady_ms):
    """the first compress call of a fresh context (it waits for its own route counts: no estimate
    yet) and its second call, each synchronous, against the steady state of back-to-back calls"""
    import torch

    import my_compress_amd as mc

    ctx = mc.Context(dev.index, block, n)
    sid = torch.cuda.current_stream(dev).cuda_stream
    # its own output buffer: d_out holds the step's assembled stream at N > 1 (rank 0's segment then
    # the peers'), and a compress may write a few bytes past its segment's end (whole words)
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    ms = []
    try:
        for _ in range(2):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, sid)
            ms.append((time.perf_counter() - t0) * 1e3)
        rs = ctx.route_stats()
    finally:
        ctx.close()
    return {"cold_ms": ms[0], "second_ms": ms[1], "steady_ms": steady_ms, "cold_vs_steady": ms[0] / steady_ms,
            "cold_value": n / ms[0] / 1e3, "rest_tiles_second_call": rs["rest"],
            "note": "one synchronous call of a fresh context (its first: the route counts are read back "
                    "before the units launch), then a second; steady = compress_only ms per step"}


def transition_leg(dev, block=1 << 20, shard_mib=256, calls=4):
    """one context, device-resident shards: `calls` rand shards, then `calls` text shards, each call
    synchronous.  The first text call runs with the estimate of the rand calls (its text tiles go to
    k_match_rest), so its time against the steady text call is the price of a change of kind; the
    stream path (fcx_compress_stream) sees the same on every shard whose kind changed"""
    import torch

    import my_compress_amd as mc

    n = shard_mib << 20
    ins = {k: make_input(k, SEEDS[k], 0, n).to(dev) for k in ("rand", "text")}
    cap = mc.shard_bound(n, block)
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    sid = torch.cuda.current_stream(dev).cuda_stream
    warm = make_input("mix", 0, 0, 64 << 20).to(dev)   # every match kernel's code loaded before timing
    w = mc.Context(dev.index, block, warm.numel())
    w.compress_shard(warm.data_ptr(), warm.numel(), d_out.data_ptr(), cap, sid)
    w.close()
    del warm
    ctx = mc.Context(dev.index, block, n)
    ms, rest = {"rand": [], "text": []}, []
    try:
        for k in ("rand", "text"):
            for _ in range(calls):
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                ctx.compress_shard(ins[k].data_ptr(), n, d_out.data_ptr(), cap, sid)
                ms[k].append((time.perf_counter() - t0) * 1e3)
                rest.append(ctx.route_stats()["rest"])
    finally:
        ctx.close()
    steady = min(ms["text"][1:])
    # the stream path (host memory in and out, fcx_compress_host in 64 MiB shards) over rand then
    # text on one context, against the two parts streamed apart on fresh contexts
    import ctypes

    hosts = {k: make_input(k, SEEDS[k], 0, n) for k in ("rand", "text")}
    both = torch.cat([hosts["rand"], hosts["text"]]).pin_memory()
    out = ctypes.create_string_buffer(mc.shard_bound(2 * n, block))
    got = ctypes.c_uint64(0)

    def stream(buf, nb):
        c = mc.Context(dev.index, block, 64 << 20)
        try:
            t0 = time.perf_counter()
            mc._check(mc.lib().fcx_compress_host(c._h, ctypes.cast(buf.data_ptr(), ctypes.POINTER(ctypes.c_uint8)), nb,
                                                 ctypes.cast(out, ctypes.POINTER(ctypes.c_uint8)), len(out),
                                                 ctypes.byref(got)), "fcx_compress_host")
            return (time.perf_counter() - t0) * 1e3
        finally:
            c.close()

    t_rand = min(stream(hosts["rand"], n) for _ in range(2))
    t_text = min(stream(hosts["text"], n) for _ in range(2))
    t_both = min(stream(both, 2 * n) for _ in range(2))
    return {"shard_mib": shard_mib, "rand_ms": ms["rand"], "text_ms": ms["text"], "rest_tiles": rest,
            "first_text_vs_steady": ms["text"][0] / steady,
            "stream_ms": {"rand": t_rand, "text": t_text, "rand_then_text": t_both},
            "stream_vs_parts": t_both / (t_rand + t_text),
            "note": "synchronous calls on one context: rand x %d then text x %d; stream: fcx_compress_host in "
                    "64 MiB shards (PCIe both ways), rand then text on one fresh context against each part "
                    "on its own" % (calls, calls)}


def host_leg(host, n, block, reps=3):
    """host-to-host rate (PCIe in both directions, pinned buffers, 256 MiB shards
    through the pipelined fcx_compress_stream path): reported beside `value`, never as it"""
    import ctypes

    import my_compress_amd as mc

    shard = (256 << 20) // block * block
    ctx = mc.Context(0, block, shard)
    cap = mc.shard_bound(n, block)
    out = ctypes.create_string_buffer(cap)
    got = ctypes.c_uint64(0)
    src = ctypes.cast(host.data_ptr(), ctypes.POINTER(ctypes.c_uint8))
    try:
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            mc._check(mc.lib().fcx_compress_host(ctx._h, src, n, ctypes.cast(out, ctypes.POINTER(ctypes.c_uint8)),
                                                 cap, ctypes.byref(got)), "fcx_compress_host")
            ts.append(time.perf_counter() - t0)
    finally:
        ctx.close()
    dt = min(ts)
    return {"value": n / dt / 1e6, "unit": "MB/s", "ms": dt * 1e3, "out_bytes": got.value,
            "note": "host memory in -> host memory out, 256 MiB shards, H2D/compute/D2H overlapped; "
                    "the output lands in pageable memory (one extra host copy)"}


def decode_leg(d_rec, rec_len, n, block, d_in, args, dev, dist, world):
    """GPU decoder on the leg's own records: K timed
    fcx_decompress_shard calls (device records -> device bytes), max over ranks,
    then a byte compare with the input"""
    import torch

    import my_compress_amd as mc

    nblocks = (n + block - 1) // block
    d_back = torch.empty(n, dtype=torch.uint8, device=dev)
    dctx = mc.DContext(dev.index)
    sid = torch.cuda.current_stream(dev).cuda_stream
    try:
        for _ in range(max(1, args.warmup)):
            dctx.decompress_shard(d_rec.data_ptr(), rec_len, nblocks, d_back.data_ptr(), n, sid)
        dctx.set_profiling(True)
        stage_sum = {}
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            dctx.decompress_shard(d_rec.data_ptr(), rec_len, nblocks, d_back.data_ptr(), n, sid)
            for name, ms in dctx.stage_times():
                stage_sum[name] = stage_sum.get(name, 0.0) + ms
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        dt = time.perf_counter() - t0
        if dist:
            tt = torch.tensor([dt], dtype=torch.float64)
            if dist.get_backend() != "gloo":
                tt = tt.to(dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt.item())
        ok = bool(torch.equal(d_back, d_in))
    finally:
        dctx.close()
    del d_back
    return {"value": world * n * args.steps / dt / 1e6, "unit": "MB/s (decoded bytes)",
            "ms_per_step": dt / args.steps * 1e3, "round_trip_exact": ok,
            "stages_ms": {k: v / args.steps for k, v in stage_sum.items()}}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpu_share():
    """threads the CPU baseline may use: the CPUs this process may run on
    (sched_getaffinity), capped by the cgroup CPU quota when one is set
    (/sys/fs/cgroup/cpu.max); returns (threads, how it was determined)"""
    aff = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) // int(period)))
            return min(aff, q), f"cgroup cpu.max quota {quota}/{period} = {q} CPUs (affinity {aff})"
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < aff:
        # the GPU box exports its per-GPU CPU share here (16) while affinity shows the whole host
        return int(omp), f"OMP_NUM_THREADS={omp}: the host's per-GPU CPU share (affinity shows {aff})"
    return aff, f"sched_getaffinity: {aff} CPUs (no cgroup quota)"


def cpu_baseline(kind, seed, block, threads=None, nblocks=None, nblocks_1t=8, mib_per_thread=8, mib_1t=8):
    """the reference's block encoder (oracle/_ref, compiled from /root/reference) on
    the first nblocks blocks of the same shard (default: mib_per_thread MiB per thread),
    one host thread per CPU of this process's share (host_cpu_share), plus the first
    nblocks_1t blocks (default: mib_1t MiB) on one thread (the reference is single-threaded)"""
    import oracle

    share, share_how = host_cpu_share()
    threads = threads or share
    per_thread = max(1, (mib_per_thread << 20) // block)
    nblocks = nblocks or min(256 * max(1, (1 << 20) // block), per_thread * threads)
    nblocks_1t = min(nblocks, max(nblocks_1t if block >= (1 << 20) else 0, (mib_1t << 20) // block, 1))

    R = oracle.ref()
    kind_used = "reference"
    if R is None:
        kind_used = "port"
    import inputs

    n = block * nblocks
    data = inputs.generate(kind, seed, n)
    blocks = [data[i:i + block] for i in range(0, n, block)]
    lock = threading.Lock()
    todo = list(range(len(blocks)))

    def worker():
        ob = ctypes.create_string_buffer(2 * block + 4096)
        while True:
            with lock:
                if not todo:
                    return
                i = todo.pop()
            if R is not None:
                R.ref_compress_block(blocks[i], len(blocks[i]), ob)
            else:
                oracle.orc().orc_compress_block(blocks[i], len(blocks[i]), ob, oracle.FINDER_SUNDAY)

    if R is not None:
        R.ref_set_quiet(1)
    t1 = time.perf_counter()
    ob1 = ctypes.create_string_buffer(2 * block + 4096)
    for i in range(min(nblocks_1t, len(blocks))):
        if R is not None:
            R.ref_compress_block(blocks[i], len(blocks[i]), ob1)
        else:
            oracle.orc().orc_compress_block(blocks[i], len(blocks[i]), ob1, oracle.FINDER_SUNDAY)
    one = min(nblocks_1t, len(blocks)) * block / (time.perf_counter() - t1) / 1e6
    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker) for _ in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    if R is not None:
        R.ref_set_quiet(0)
    return {"value": n / dt / 1e6, "unit": "MB/s", "cores": threads, "kind": kind_used,
            "sample": f"first {nblocks} x {block // 1024} KiB blocks of the {kind} shard, {threads} threads "
                      f"({'reference my_compress_file_lz77 compiled in place' if R is not None else 'oracle port'})",
            "seconds": dt, "one_thread_MBps": one, "one_thread_sample": f"first {nblocks_1t} blocks, 1 thread",
            "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(), "cores_source": share_how}


def lz78_leg(dev, mib=1024, block=1 << 20, reps=2, ref_blocks=2):
    """the -c lz78 codec (fcx_lz78.hip; my_compress_file_lz78 :3127) on a device-resident
    rand shard: compress rate, the first `ref_blocks` records checked against the
    reference compiled in place (the oracle when it is absent), and the reference timed
    on the same blocks on one core (it is single-threaded)"""
    import torch

    import inputs
    import my_compress_amd as mc
    import oracle

    n = mib << 20
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    inputs.generate_into("rand", 4, host.data_ptr(), n)
    d_in = host.to(dev)
    cap = mc.lz78_bound(n, block)
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    out_len = ctypes.c_uint64()
    st = torch.cuda.current_stream(dev).cuda_stream
    L = mc.lib()
    times = []
    for it in range(reps + 1):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        rc = L.fcx_lz78_compress_shard(d_in.data_ptr(), n, block, d_out.data_ptr(), cap, ctypes.byref(out_len), st)
        torch.cuda.synchronize(dev)
        if rc != 0:
            raise RuntimeError(L.fcx_last_error().decode())
        if it:
            times.append(time.perf_counter() - t0)
    dt = sum(times) / len(times)
    mc.lz78_release()
    head = d_out[:min(out_len.value, ref_blocks * (2 * block + 65536))].cpu().numpy().tobytes()
    R = oracle.ref()
    blocks = [bytes(host[i * block:(i + 1) * block].numpy()) for i in range(ref_blocks)]
    if R is not None:
        R.ref_set_quiet(1)
    t1 = time.perf_counter()
    want = [oracle.ref_lz78_compress_block(b) if R is not None else oracle.lz78_compress_block(b) for b in blocks]
    cpu_s = time.perf_counter() - t1
    if R is not None:
        R.ref_set_quiet(0)
    q, exact = 0, True
    for w in want:
        sz = int.from_bytes(head[q:q + 4], "little")
        exact &= head[q + 4:q + 4 + sz] == w
        q += 4 + sz
    return {"value": n / dt / 1e6, "unit": "MB/s", "ms_per_step": dt * 1e3, "ratio": out_len.value / n,
            "workload": f"rand {mib} MiB, {block // 1024} KiB blocks, device-resident",
            "bit_exact_first_blocks": exact, "checked_blocks": ref_blocks,
            "cpu_baseline": {"value": ref_blocks * block / cpu_s / 1e6, "unit": "MB/s", "cores": 1,
                             "kind": "reference" if R is not None else "port",
                             "sample": f"first {ref_blocks} x {block // 1024} KiB blocks, my_compress_file_lz78"}}


# the exchange each --concat form runs at N > 1 (named in the line's config)
CONCAT_FORMS = {
    "pipe": "pipe: each peer's segment sent to rank 0 in sub-batches as they finish (send/recv gather)",
    "gather": "gather: every peer's whole segment sent to rank 0 after the compress (send/recv)",
    "allgather": "allgather: every rank receives every segment (RCCL all-gather)",
    "none": "none",
}


def roofline(res, pmc_leg, pmc):
    """roofline of a leg's dominant kernel (largest hipEvent stage time over the K compress-only
    steps): achieved = the leg's algorithmic bytes on this rank (input + compressed
    output, 1 + r per input byte) / that kernel's average time; traffic = FETCH_SIZE x 2 + WRITE_SIZE
    per launch from the committed PMC summary for this leg (`pmc_leg`:stage), scaled to this shard"""
    stages = {k: v for k, v in res["stages_ms"].items() if k != "memset"}
    dom = max(stages, key=stages.get) if stages else None
    n = res["bytes_this_rank"]
    alg = n + res["seg_bytes_rank0"]
    achieved = alg / (stages[dom] * 1e-3) / 1e9 if dom else None
    traffic = None
    # the match stage runs one of k_match's units (fcx_ctx_match_kernel): the kernel name is that unit's
    kernel = (res.get("match_kernel") or "k_match") if dom == "match" else f"k_{dom}" if dom else None
    rt = res.get("route") or {}
    # (a unit counts when it searched at least 1 % of the tiles: a few misfiled samples handed on do not)
    units = [u for u in ("sparse", "runs", "key4", "nofilter", "uniform")
             if 100 * (rt.get(u, 0) - (rt.get("handed_on", 0) if u == "nofilter" else 0)) >= rt.get("tiles", 0) > 0]
    if dom == "match" and len(units) > 1:   # routed over several units: the stage is their launches together
        kernel = "k_match_{" + ",".join(dict(sparse="sparse", runs="runs", key4="k4", nofilter="nf",
                                              uniform="uniform")[u] for u in units) + "}"
    key = f"{pmc_leg}:{kernel[2:]}" if kernel else None
    if pmc_leg and key in pmc:   # PMC passes ran on a whole 1 GiB shard; scale to this rank's launch
        traffic = pmc[key].get("hbm_bytes_per_launch") * n / pmc[key].get("input_bytes", GiB)
    return {"bound": "hbm", "kernel": kernel, "achieved": achieved, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
            "alg_bytes_per_launch": alg, "kernel_ms": stages.get(dom),
            "note": "achieved = (this rank's input + its compressed segment) / the dominant kernel's average "
                    "hipEvent time over K profiled compress-only steps (outside the timed region); traffic = FETCH_SIZE x 2 + WRITE_SIZE per "
                    "launch from profiles/pmc_latest.json (rocprofv3 PMC passes), scaled to this shard",
            "path_achieved": alg / (res["compress_only"]["ms_per_step"] * 1e-3) / 1e9,
            "path_frac": alg / (res["compress_only"]["ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBS}


def load_pmc(path):
    if path and os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--kind", default="rand", choices=["rand", "text", "runs", "zeros", "dna", "mix"])
    ap.add_argument("--global-mib", type=int, default=1024, help="headline input size, split over the ranks")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="main leg: strong = --global-mib split N ways (default), weak = --mib per rank")
    ap.add_argument("--mib", type=int, default=1024, help="MiB per rank for weak scaling (the weak leg)")
    ap.add_argument("--block", type=int, default=1 << 20)
    ap.add_argument("--no-text", action="store_true", help="skip every extra leg")
    ap.add_argument("--legs", default="c2,text,c3,zeros,runs,dna,mix",
                    help="extra legs after the main one (comma list of " + ",".join(LEGS) + ")")
    ap.add_argument("--no-weak", action="store_true", help="skip the weak-scaling (config 4) leg at N > 1")
    ap.add_argument("--concat", default="pipe", choices=["pipe", "gather", "allgather", "none"],
                    help="pipe: gather-aware partition, compress and gather overlapped (fcx_dist_compress_gather); "
                         "gather: even split, compress, then gather to rank 0; allgather: the stream on every rank")
    ap.add_argument("--share0", dest="share0_ppm", type=int, default=-1,
                    help="pipe: rank 0's share of the blocks in ppm (-1 = the step model's choice)")
    ap.add_argument("--nsub", type=int, default=4, help="pipe: sub-batches per peer")
    ap.add_argument("--link-gbps", type=float, default=64.0,
                    help="pipe: xGMI GB/s per link and direction assumed by the partition model before calibration")
    ap.add_argument("--no-calibrate", dest="calibrate", action="store_false",
                    help="pipe, N > 1: keep the modelled share0 (default: re-partition from one measured warmup step)")
    ap.add_argument("--concat-impl", default="fcx", choices=["fcx", "torch"],
                    help="fcx: the C++ RCCL path (fcx_dist_concat); torch: torch.distributed P2P / broadcast")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--dist-rehearsal", action="store_true",
                    help="use the multi-rank code path (process group, concatenation) even at N=1 (under torchrun)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-decode", action="store_true", help="skip the GPU decoder timing")
    ap.add_argument("--no-host-path", dest="host_path", action="store_false",
                    help="skip the host-to-host (PCIe-inclusive) timing of the main leg")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-lz78", action="store_true", help="skip the -c lz78 codec leg")
    ap.add_argument("--no-transition", action="store_true", help="skip the rand -> text change-of-kind timing")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_latest.json"))
    args = ap.parse_args()

    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # FCX_BENCH_SAME_DEVICE=1: every rank on cuda:0 (rehearsing N>1 on a one-GPU box, with --dist-backend gloo)
    dev = torch.device("cuda:0" if os.environ.get("FCX_BENCH_SAME_DEVICE") == "1" else f"cuda:{local}")
    torch.cuda.set_device(dev)
    dist = None
    if world > 1 or args.dist_rehearsal:
        import torch.distributed as dist_

        if args.dist_backend == "nccl":
            dist_.init_process_group("nccl", device_id=dev)
        else:
            dist_.init_process_group("gloo")
        dist = dist_
    args.fcx_dist = None
    if dist and args.dist_backend == "nccl" and args.concat_impl == "fcx":
        # the C++ RCCL communicator of the concatenation (fcx_dist_init_rank); its unique id
        # travels over the torch process group
        import my_compress_amd as mc

        uid = torch.zeros(128, dtype=torch.uint8, device=dev)
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(mc.dist_unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, src=0)
        try:
            args.fcx_dist = mc.Dist.rank(world, rank, bytes(uid.cpu().numpy().tobytes()), dev.index)
            ok = 1
        except mc.FcxError as e:   # (the line then says concat_impl "torch.distributed (nccl)")
            print(f"rank {rank}: fcx_dist_init_rank failed ({e}); the torch.distributed path carries the exchange",
                  file=sys.stderr, flush=True)
            args.fcx_dist, ok = None, 0
        flag = torch.tensor([ok], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)   # every rank takes the same path
        if not int(flag.item()) and args.fcx_dist is not None:
            args.fcx_dist.close()
            args.fcx_dist = None
    main_res = run_leg(args.kind, SEEDS[args.kind], args.block, args, rank, world, dev, dist, True,
                       scaling=args.scaling, main_leg=True)
    legs = {}
    for name in ([] if args.no_text else [x for x in args.legs.split(",") if x]):
        kind, block = LEGS[name][:2]
        seed, mib = (LEGS[name][2], LEGS[name][3]) if len(LEGS[name]) > 2 else (SEEDS[kind], None)
        if kind == args.kind and block == args.block and seed == SEEDS[kind] and mib is None:
            continue
        legs[name] = run_leg(kind, seed, block, args, rank, world, dev, dist, True, global_mib=mib)
    weak = None
    if dist and not args.no_weak and args.scaling == "strong":
        weak = run_leg("rand", 4, 1 << 20, args, rank, world, dev, dist, False, scaling="weak")

    if rank == 0:
        pmc = load_pmc(args.pmc)
        n = main_res["bytes_this_rank"]
        roof = roofline(main_res, args.kind if args.block == 1 << 20 else None, pmc)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.kind, SEEDS[args.kind], args.block)
        part = main_res.get("partition") or {}
        shard_note = "the whole input" if world == 1 else (
            f"contiguous block ranges over {world} ranks" +
            (f", rank 0 (the receiver) {part['share0_ppm'] / 1e4:.1f} %" if part.get("share0_ppm") else ", even"))
        line = {
            "metric": METRIC, "value": main_res["value"], "unit": "MB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": main_res["ms_per_step"],
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: glibc rand()%256 seed 4 (SURVEY.md §8(d)); the 1 GiB input is SURVEY's HL-rand "
                    "(= the first GiB of BASELINE config 4); extra legs: text = enwik-style generator seed 3 at "
                    "1 MiB (HL-text) and 256 KiB blocks (C3), c2 = rand seed 2, 64 MiB at 64 KiB blocks (config 2), zeros "
                    "and runs seed 5 (config 5), dna = "
                    "'ACGT'[rand()%4] seed 6, mix = 1 MiB blocks cycling rand / text / runs / dna (every match "
                    "unit in one call)",
            "config": {"workload": f"{args.kind} {main_res['global_bytes'] >> 20} MiB, {args.block // 1024} KiB "
                                   f"blocks, {shard_note}; step = compress + concatenation of the segments "
                                   f"into one stream ({main_res['concat']})",
                       "kind": args.kind, "global_bytes": main_res["global_bytes"],
                       "bytes_per_gpu": n, "block_bytes": args.block,
                       "parallelism": (f"block-sharded x{world}, {main_res['concat']} over "
                                       f"{main_res.get('concat_impl')}" if world > 1 else "single GPU")},
            "roofline": roof,
            "cpu_baseline": cpu,
            "ratio": main_res["ratio"],
            "bit_exact_vs_reference": main_res.get("bit_exact_vs_reference"),
            "compress_only": main_res["compress_only"],
            "concat_ms_per_step": main_res.get("concat_ms_per_step"),
            "concat_impl": main_res.get("concat_impl"),
            "partition": main_res.get("partition"),
            "stages_ms": main_res["stages_ms"],
            "lazy_evals": main_res["lazy_evals"],
            "decode": main_res.get("decode"),
            "host_path": main_res.get("host_path"),
            "route": main_res.get("route"),
            "cold_call": main_res.get("cold_call"),
        }
        if world == 1 and not args.no_lz78 and not args.no_text:
            line["lz78"] = lz78_leg(dev)
        if world == 1 and not args.no_transition and not args.no_text:
            line["transition"] = transition_leg(dev)
        keep = ["value", "ms_per_step", "compress_only", "concat_ms_per_step", "ratio", "block_bytes", "stages_ms",
                "lazy_evals", "lazy_tiles", "decode", "bit_exact_vs_reference", "global_bytes", "partition",
                "concat_impl", "route", "cold_call"]
        for name, lr in legs.items():
            line[name] = {k: lr[k] for k in keep if k in lr}
            line[name]["roofline"] = roofline(lr, name, pmc)
            if world == 1 and not args.no_cpu_baseline:   # a smaller sample per extra leg: ~2 MiB per thread
                kind, block = LEGS[name][:2]
                seed = LEGS[name][2] if len(LEGS[name]) > 2 else SEEDS[kind]
                line[name]["cpu_baseline"] = cpu_baseline(kind, seed, block, mib_per_thread=2, mib_1t=2)
        if weak is not None:
            line["weak"] = {k: weak[k] for k in keep + ["rank_segments_bit_exact", "global_bytes"] if k in weak}
            line["weak"]["workload"] = (f"BASELINE config 4 sharding: rank r = bytes [r GiB, (r+1) GiB) of the "
                                        f"seed-4 rand stream, {world} GiB total, segments gathered to rank 0")
        # a compact per-leg summary as the LAST key, so a reader that keeps only the line's tail
        # (the driver keeps 8 KB) still sees every leg
        summ = {}

        def brief(name, v, lr=None):
            rf, cb = v.get("roofline") or {}, v.get("cpu_baseline") or {}
            summ[name] = {"value": round(v["value"], 1), "ms": round(v["ms_per_step"], 3),
                          "bit_exact": v.get("bit_exact_vs_reference"),
                          "frac": round(rf["frac"], 4) if rf.get("frac") else None,
                          "path_frac": round(rf["path_frac"], 4) if rf.get("path_frac") else None,
                          "cpu_MBps": round(cb["value"], 1) if cb.get("value") else None}
            if v.get("cold_call"):
                summ[name]["cold_vs_steady"] = round(v["cold_call"]["cold_vs_steady"], 3)

        brief(args.kind, line)
        for name in legs:
            brief(name, line[name])
        if "weak" in line:
            brief("weak", line["weak"])
        if "transition" in line:
            summ["transition"] = {"first_text_vs_steady": round(line["transition"]["first_text_vs_steady"], 3),
                                  "stream_vs_parts": round(line["transition"]["stream_vs_parts"], 3)}
        line["legs"] = summ
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        if args.fcx_dist is not None:
            args.fcx_dist.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
