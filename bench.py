#!/usr/bin/env python3
"""bench.py — compress throughput of the MI355X FCX7 LZ77 + Huffman path.

Metric (BASELINE.json): compress MB/s on 1 GB synthetic bytes at 1/2/4/8 MI355X;
% HBM roofline.  One process per GPU (torchrun for N > 1).  A "step" compresses
the rank's whole device-resident shard (1 GiB = 1024 x 1 MiB blocks by default)
into [u32 len][payload]... in HBM.  Shards are independent block ranges, so the
data path has no collective (scaling: weak); the RCCL all-gather that
concatenates the per-rank segments is timed after the timed region as its own
stage ("concat").

Default workload: rand = glibc rand()%256 seed 4, rank r = bytes [r GiB,
(r+1) GiB) of that one stream (BASELINE config 4 sharding; N=1 is SURVEY's
HL-rand, whose output digest is checked).  The text leg (seed 3 + rank; N=1 is
HL-text) is measured in the same run and reported under "text".

    python bench.py                      # N=1, defaults
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
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
HL_DIGEST = {  # reference output digests for the N=1 shards
    ("rand", 4, 1 << 30, 1 << 20): ("ee962534628bf6b2f79c51a44a65ac0845945e2fe9225e5be8f99f288912a69d", 1091294206),
    ("text", 3, 1 << 30, 1 << 20): ("132a36b9d2592f8c37a82b51f545ddb67acec53fa1a31b7f1f6a04617a01a3d1", 624801500),
    ("text", 3, 1 << 30, 1 << 18): ("20219e60c2e9aef6659801fbfc53c6873ec811686eedcb45c0896fc5547d63d0", 630008807),
    ("zeros", 0, 1 << 30, 1 << 20): ("533fd45fbaa861a6060e9a5beac177cc0b64db691fc602a1e0e1e188afa5f912", 7521290),
    ("runs", 5, 1 << 30, 1 << 20): ("4fced94fd4725ba3b1031dec67d63e1295b95ae08cc1cf0e34c84769f5313d26", 42548682),
}
# extra legs measured after the main one: name -> (kind, seed, block bytes); BASELINE configs 3 and 5
LEGS = {"text": ("text", 3, 1 << 20), "c3": ("text", 3, 1 << 18), "zeros": ("zeros", 0, 1 << 20),
        "runs": ("runs", 5, 1 << 20)}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_shard(kind, seed, rank, n):
    """pinned host tensor with rank's shard of the synthetic stream"""
    import torch

    import inputs

    G = inputs.gen_lib()
    G.fcxgen_skip.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    if kind == "rand":
        h = G.fcxgen_create(inputs.GEN_KIND["rand"], seed)
        G.fcxgen_skip(h, rank * n)   # one stream, rank r starts at byte r*n
        G.fcxgen_fill(h, host.data_ptr(), n)
        G.fcxgen_destroy(h)
    else:
        inputs.generate_into(kind, seed + rank, host.data_ptr(), n)
    return host


def run_leg(kind, seed, args, rank, world, dev, dist, profile_stages, block=None):
    import torch

    import my_compress_amd as mc

    n = args.mib << 20
    block = block or args.block
    t = time.time()
    host = make_shard(kind, seed, rank, n)
    gen_s = time.time() - t
    d_in = host.to(dev)
    host_path = None
    if world == 1 and args.host_path and kind == args.kind:
        host_path = host_leg(host, n, block)
    del host
    cap = mc.shard_bound(n, block)
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    ctx = mc.Context(dev.index, block, n)
    stream = torch.cuda.current_stream(dev)
    sid = stream.cuda_stream
    out_len = ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, sid)  # validates the call
    for _ in range(args.warmup):
        ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, sid, sync=False)
    ctx.set_profiling(profile_stages)
    stage_sum = {}
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, sid, sync=False)
        if profile_stages:
            for name, ms in ctx.stage_times():   # waits for this step's last event
                stage_sum[name] = stage_sum.get(name, 0.0) + ms
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    ctx.set_profiling(False)
    if dist:
        tt = torch.tensor([dt], dtype=torch.float64)
        if dist.get_backend() != "gloo":
            tt = tt.to(dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    out_len = ctx.read_out_len()   # segment size of the timed steps (device word)
    res = {
        "kind": kind, "block_bytes": block, "bytes_per_gpu": n, "out_bytes": out_len, "ratio": out_len / n,
        "seconds": dt, "ms_per_step": dt / args.steps * 1e3,
        "value": world * n * args.steps / dt / 1e6, "gen_s": gen_s,
        "stages_ms": {k: v / args.steps for k, v in stage_sum.items()},
        "host_path": host_path,
    }
    stats = ctx.stats()
    res["tokens"], res["matches"] = stats["tokens"], stats["matches"]
    res["lazy_evals"], res["lazy_tiles"] = stats["lazy_evals"], stats["lazy_tiles"]
    key = (kind, seed, n, block)
    if rank == 0 and world == 1 and key in HL_DIGEST and not args.no_verify:
        import my_compress_amd as mc2

        h = hashlib.sha256(mc2.write_header(n, (n + block - 1) // block))
        h.update(memoryview(d_out[:out_len].cpu().numpy()))
        want_sha, want_bytes = HL_DIGEST[key]
        res["bit_exact_vs_reference"] = h.hexdigest() == want_sha and out_len + 10 == want_bytes
    if not args.no_decode:
        res["decode"] = decode_leg(d_out, out_len, n, block, d_in, args, dev, dist, world)
    concat = None
    if dist and world > 1 and args.concat == "allgather":
        concat = allgather_concat(d_out, out_len, world, dev, dist)
    ctx.close()
    del d_in, d_out
    torch.cuda.empty_cache()
    return res, concat


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


def allgather_concat(d_out, seg_len, world, dev, dist):
    """RCCL all-gather of the per-rank segments (my_compress_amd.dist): sizes,
    then segments padded to the largest, assembled in rank order on every rank.
    With the gloo backend (rehearsal) the segments travel through host memory."""
    import torch

    from my_compress_amd import dist as fdist

    on_host = dist.get_backend() == "gloo"
    dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    seg = d_out[:seg_len]
    if on_host:
        seg = seg.cpu()
    whole = fdist.concat_segments(seg, dist)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    tt = torch.tensor([dt], dtype=torch.float64)
    if not on_host:
        tt = tt.to(dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    dt = float(tt.item())
    total = int(whole.numel())
    del whole
    return {"kind": "allgather" + ("(gloo,host)" if on_host else "(rccl)"), "ms": dt * 1e3, "bytes": total,
            "GBps_per_rank_recv": (total - seg_len) / dt / 1e9}


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


def cpu_baseline(kind, seed, block, threads=None, nblocks=None, nblocks_1t=8):
    """the reference's block encoder (oracle/_ref, compiled from /root/reference) on
    the first nblocks blocks of the same shard, one host thread per CPU of this
    process's share (host_cpu_share), plus the first nblocks_1t blocks on one thread
    (the reference is single-threaded)"""
    import oracle

    share, share_how = host_cpu_share()
    threads = threads or share
    nblocks = nblocks or min(256, 8 * threads)   # ~10-60 s of CPU work at 0.5-1 s per 1 MiB block

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
    ap.add_argument("--kind", default="rand", choices=["rand", "text", "runs", "zeros"])
    ap.add_argument("--mib", type=int, default=1024, help="MiB per GPU")
    ap.add_argument("--block", type=int, default=1 << 20)
    ap.add_argument("--no-text", action="store_true", help="skip every extra leg")
    ap.add_argument("--legs", default="text,c3,zeros,runs",
                    help="extra legs after the main one (comma list of " + ",".join(LEGS) + ")")
    ap.add_argument("--concat", default="allgather", choices=["allgather", "none"])
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-decode", action="store_true", help="skip the GPU decoder timing")
    ap.add_argument("--no-host-path", dest="host_path", action="store_false",
                    help="skip the host-to-host (PCIe-inclusive) timing of the main leg")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-lz78", action="store_true", help="skip the -c lz78 codec leg")
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
    if world > 1:
        import torch.distributed as dist_

        if args.dist_backend == "nccl":
            dist_.init_process_group("nccl", device_id=dev)
        else:
            dist_.init_process_group("gloo")
        dist = dist_
    seeds = {"rand": 4, "text": 3, "runs": 5, "zeros": 0}
    main_res, concat = run_leg(args.kind, seeds[args.kind], args, rank, world, dev, dist, True)
    legs = {}
    for name in ([] if args.no_text else [x for x in args.legs.split(",") if x]):
        kind, seed, block = LEGS[name]
        if kind == args.kind and block == args.block:
            continue
        legs[name], _ = run_leg(kind, seed, args, rank, world, dev, dist, True, block=block)

    if rank == 0:
        stages = {k: v for k, v in main_res["stages_ms"].items() if k != "memset"}
        dom = max(stages, key=stages.get) if stages else None
        n = main_res["bytes_per_gpu"]
        alg = n + main_res["out_bytes"]          # 1 + r bytes per input byte
        achieved = alg / (stages[dom] * 1e-3) / 1e9 if dom else None
        pmc = load_pmc(args.pmc)
        traffic = None
        key = f"{args.kind}:{dom}"
        if key in pmc:
            traffic = pmc[key].get("hbm_bytes_per_launch")
        roof = {"bound": "hbm", "kernel": f"k_{dom}" if dom else None, "achieved": achieved, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                "alg_bytes_per_launch": alg,
                "note": "algorithmic bytes = input + compressed output per launch (1 + r per input byte); "
                        "the path is compare/serial-bound, HBM fraction is small by construction",
                "path_achieved": alg / (main_res["ms_per_step"] * 1e-3) / 1e9}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.kind, seeds[args.kind], args.block)
        line = {
            "metric": METRIC, "value": main_res["value"], "unit": "MB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": main_res["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: glibc rand()%256 seed 4, rank r = bytes [r*shard, (r+1)*shard) of one stream "
                    "(SURVEY.md §8(d)); extra legs: text = enwik-style generator seed 3+rank at 1 MiB (HL-text) "
                    "and 256 KiB blocks (c3), zeros, runs seed 5+rank (BASELINE config 5)",
            "config": {"workload": f"{args.kind} {args.mib} MiB per GPU, {args.block // 1024} KiB blocks "
                                   f"(BASELINE config 4 sharding; N=1 = HL-{args.kind})",
                       "kind": args.kind, "bytes_per_gpu": n, "block_bytes": args.block,
                       "global_bytes": n * world, "parallelism": f"block-sharded x{world}"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "ratio": main_res["ratio"],
            "bit_exact_vs_reference": main_res.get("bit_exact_vs_reference"),
            "stages_ms": main_res["stages_ms"],
            "lazy_evals": main_res["lazy_evals"],
            "concat": concat,
            "decode": main_res.get("decode"),
            "host_path": main_res.get("host_path"),
        }
        if world == 1 and not args.no_lz78 and not args.no_text:
            line["lz78"] = lz78_leg(dev)
        for name, lr in legs.items():
            line[name] = {k: lr[k] for k in ["value", "ms_per_step", "ratio", "block_bytes", "stages_ms", "lazy_evals"]}
            if "decode" in lr:
                line[name]["decode"] = lr["decode"]
            line[name]["bit_exact_vs_reference"] = lr.get("bit_exact_vs_reference")
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
