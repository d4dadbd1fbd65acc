#!/usr/bin/env python3
"""k_match per-phase timing (development): the kernel alone through fcx_debug_match
with phase exits (16: staging + run count, 32: + sort, 64: + queries, 0: whole)."""
import argparse, ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import inputs
import my_compress_amd as mc
ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="rand"); ap.add_argument("--seed", type=int, default=4)
ap.add_argument("--mib", type=int, default=1024); ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--mode", type=int, default=0, help="fcx_ctx_set_match_mode (4: the 4-byte-key kernel)")
ap.add_argument("--phases", default="", help="comma-separated subset of the phase names")
a = ap.parse_args()
n = a.mib << 20
host = torch.empty(n, dtype=torch.uint8).pin_memory()
inputs.generate_into(a.kind, a.seed, host.data_ptr(), n)
d = host.to("cuda:0")
ctx = mc.Context(0, 1 << 20, n)
ctx.set_match_mode(a.mode)
L = mc.lib()
L.fcx_debug_match.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]
s = torch.cuda.current_stream()
res = {}
for name, bits in [("stage+count", 16), ("+filter", 4096), ("+sort", 32), ("+runtable", 8192 | 64), ("+eval-noloop", 16384 | 64), ("+eval-nofold", 32768 | 64), ("+queries", 64), ("+q-nocand", (1 << 22) | 64), ("+q-allA", (1 << 20) | 64), ("+q-allB", (1 << 21) | 64), ("+rmA1", 1 << 18), ("+rmA2", 1 << 19), ("+walks", 512), ("+jacobi", 256), ("+counts", 1024), ("+list", 2048), ("whole", 0), ("no-search", 1)]:
    if a.phases and name not in a.phases.split(","):
        continue
    ts = []
    for r in range(a.reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        mc._check(L.fcx_debug_match(ctx._h, ctypes.c_void_p(d.data_ptr()), n, bits, ctypes.c_void_p(s.cuda_stream)), "dbg")
        e1.record(s)
        torch.cuda.synchronize()
        if r: ts.append(e0.elapsed_time(e1))
    res[name] = min(ts)
    print(f"{a.kind} {name:12s} {res[name]:.3f} ms")
