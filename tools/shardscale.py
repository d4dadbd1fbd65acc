#!/usr/bin/env python3
"""Single-GPU predictor of the strong-scaling curve.

At N GPUs the headline job gives every rank a 1/N shard of the 1 GiB input, so the
per-rank compress time at N = 8/4/2/1 is the one-GPU time of a 128/256/512/1024 MiB
shard of the same stream.  This times each shard size back to back (device-resident
input, hipEvent stage times of one profiled pass) and writes one JSON object:

    python tools/shardscale.py --kind rand --out gpurun_out/shardscale_rand.json

The exchange (gather of the N-1 remote segments to rank 0 over xGMI) is not modelled
here; DESIGN §6 adds it from the link rate.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import inputs  # noqa: E402
import my_compress_amd as mc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="rand")
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--block", type=int, default=1 << 20)
    ap.add_argument("--sizes", default="128,256,512,1024", help="shard sizes in MiB")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    sizes = [int(s) for s in a.sizes.split(",")]
    n_max = max(sizes) << 20
    host = torch.empty(n_max, dtype=torch.uint8).pin_memory()
    inputs.generate_into(a.kind, a.seed, host.data_ptr(), n_max)
    dev = torch.device("cuda:0")
    d_in = host.to(dev)
    st = torch.cuda.current_stream().cuda_stream
    res = {"kind": a.kind, "seed": a.seed, "block": a.block, "device": torch.cuda.get_device_name(0),
           "note": "per-rank compress time of the 1 GiB headline job at N = 1024 / shard MiB (strong scaling), "
                   "one GPU, device-resident input; exchange not included", "shards": []}
    for mib in sizes:
        n = mib << 20
        cap = mc.shard_bound(n, a.block)
        d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
        ctx = mc.Context(0, a.block, n)
        ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, st)   # warm
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, st, sync=False)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        out_len = ctx.read_out_len()
        ctx.set_profiling(True)
        ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, st)
        stages = {name: round(t, 4) for name, t in ctx.stage_times()}
        ctx.set_profiling(False)
        ctx.close()
        del d_out
        row = {"shard_mib": mib, "predicts_n": 1024 // mib if 1024 % mib == 0 else None, "ms": round(ms, 4),
               "GBps": round(n / ms / 1e6, 2), "out_bytes": out_len, "stages_ms": stages}
        res["shards"].append(row)
        print(json.dumps(row), flush=True)
    base = next((r for r in res["shards"] if r["shard_mib"] == 1024), None)
    if base:
        for r in res["shards"]:
            r["speedup_vs_1GiB"] = round(base["ms"] / r["ms"], 3)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    t = time.time()
    main()
    print(f"done in {time.time() - t:.1f}s", flush=True)
