#!/usr/bin/env python3
"""Decoder timing (development): GPU-compress a synthetic shard, then time the GPU
decoder on the device records and check the round trip."""
import argparse, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import inputs
import my_compress_amd as mc
ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="rand"); ap.add_argument("--seed", type=int, default=4)
ap.add_argument("--mib", type=int, default=256); ap.add_argument("--block", type=int, default=1 << 20)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
n = a.mib << 20
dev = torch.device("cuda:0")
host = torch.empty(n, dtype=torch.uint8).pin_memory()
inputs.generate_into(a.kind, a.seed, host.data_ptr(), n)
d_in = host.to(dev)
cap = mc.shard_bound(n, a.block)
d_rec = torch.empty(cap, dtype=torch.uint8, device=dev)
ctx = mc.Context(0, a.block, n)
sid = torch.cuda.current_stream().cuda_stream
m = ctx.compress_shard(d_in.data_ptr(), n, d_rec.data_ptr(), cap, sid)
ctx.close()
d_back = torch.empty(n, dtype=torch.uint8, device=dev)
dc = mc.DContext(0)
nb = (n + a.block - 1) // a.block
dc.set_profiling(True)
for r in range(a.reps):
    torch.cuda.synchronize(); t = time.perf_counter()
    got = dc.decompress_shard(d_rec.data_ptr(), m, nb, d_back.data_ptr(), n, sid)
    torch.cuda.synchronize(); dt = time.perf_counter() - t
    print(f"rep {r}: {dt*1e3:.2f} ms  {n/dt/1e9:.2f} GB/s", " ".join(f"{k}={v:.3f}" for k, v in dc.stage_times()))
print("round trip", "OK" if got == n and torch.equal(d_back, d_in) else "MISMATCH")
