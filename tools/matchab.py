#!/usr/bin/env python3
"""k_match A/B timing (development): the kernel alone through fcx_debug_match for each dbg value
given (experiment bits of k_match<true>), min over reps.  python tools/matchab.py --kind text 0x100000 0"""
import argparse, ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import inputs
import my_compress_amd as mc
ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="text"); ap.add_argument("--seed", type=int, default=None)
ap.add_argument("--mib", type=int, default=256); ap.add_argument("--reps", type=int, default=5)
ap.add_argument("bits", nargs="+")
a = ap.parse_args()
seed = a.seed if a.seed is not None else {"rand": 4, "text": 3, "runs": 5, "zeros": 0, "dna": 5}[a.kind]
n = a.mib << 20
host = torch.empty(n, dtype=torch.uint8).pin_memory()
inputs.generate_into(a.kind, seed, host.data_ptr(), n)
d = host.to("cuda:0")
ctx = mc.Context(0, 1 << 20, n)
L = mc.lib()
L.fcx_debug_match.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]
s = torch.cuda.current_stream()
for b in a.bits:
    bits = int(b, 0)
    ts = []
    for r in range(a.reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        mc._check(L.fcx_debug_match(ctx._h, ctypes.c_void_p(d.data_ptr()), n, bits, ctypes.c_void_p(s.cuda_stream)), "dbg")
        e1.record(s)
        torch.cuda.synchronize()
        if r: ts.append(e0.elapsed_time(e1))
    print(f"{a.kind} dbg={b:>10s} {min(ts):.3f} ms  ({min(ts) * 1024 / a.mib:.2f} ms/GiB)", flush=True)
