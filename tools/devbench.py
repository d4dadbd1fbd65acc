#!/usr/bin/env python3
"""Developer timing: compress a device-resident synthetic shard with per-stage
hipEvent timing and (optionally) check the output digest against the
reference's.

    python tools/devbench.py --kind text --gib 1 --block 1048576 --check hl_text_1GiB
"""
import argparse
import hashlib
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
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--block", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--check", default=None)
    ap.add_argument("--groups", default="0", help="comma list of fcx_ctx_set_groups values to time")
    ap.add_argument("--mode", type=int, default=0, help="fcx_ctx_set_match_mode (0: routed)")
    a = ap.parse_args()
    n = a.mib << 20
    t = time.time()
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    inputs.generate_into(a.kind, a.seed, host.data_ptr(), n)
    print(f"gen {a.kind} {a.mib} MiB: {time.time() - t:.1f}s", flush=True)
    dev = torch.device("cuda:0")
    d_in = host.to(dev)
    cap = mc.shard_bound(n, a.block)
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    ctx = mc.Context(0, a.block, n)
    ctx.set_match_mode(a.mode)
    st = torch.cuda.current_stream().cuda_stream
    got = ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, st)  # warm
    for G in [int(x) for x in a.groups.split(",")]:
        ctx.set_groups(G)
        ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, st)  # warm
        torch.cuda.synchronize()
        t = time.time()
        for r in range(a.reps):   # back to back, unprofiled
            ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, st, sync=False)
        torch.cuda.synchronize()
        dt = (time.time() - t) / a.reps
        got = ctx.read_out_len()
        print(f"groups {G}: {dt * 1e3:.3f} ms  {n / dt / 1e9:.2f} GB/s  out={got} ratio={got / n:.4f}"
              f"  {ctx.match_kernel()}", flush=True)
        ctx.set_profiling(True)
        ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, st)
        print("   " + "  ".join(f"{name} {ms:.3f}" for name, ms in ctx.stage_times()))
        ctx.set_profiling(False)
        if a.check:
            cfg = inputs.SURVEY_DIGESTS[a.check]
            h = hashlib.sha256(mc.write_header(n, (n + a.block - 1) // a.block))
            h.update(memoryview(d_out[:got].cpu().numpy()))
            print("   digest", "OK" if h.hexdigest() == cfg["out"] and got + 10 == cfg["bytes"] else "MISMATCH",
                  got + 10, cfg["bytes"], flush=True)
    print(ctx.stats())
    try:
        print("route", ctx.route_stats())
    except (mc.FcxError, AttributeError):
        pass
    ctx.close()


if __name__ == "__main__":
    main()
