#!/usr/bin/env python3
"""k_emit / k_tree path timing (development): compress a device-resident shard with fcx_debug_emit_bits
set to each value given and print the emit stage's hipEvent time (the output is invalid while a
bit is set).  python tools/emitab.py --kind rand 0 1 2 4 8"""
import argparse, ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import inputs
import my_compress_amd as mc
ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="rand"); ap.add_argument("--mib", type=int, default=1024)
ap.add_argument("--block", type=int, default=1 << 20); ap.add_argument("--seed", type=int, default=None)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--stage", default="emit", help="stage to report (emit; tree with bits >= 0x10000)")
ap.add_argument("bits", nargs="+")
a = ap.parse_args()
seed = a.seed if a.seed is not None else {"rand": 4, "text": 3, "runs": 5, "zeros": 0, "dna": 5}[a.kind]
n = a.mib << 20
host = torch.empty(n, dtype=torch.uint8).pin_memory()
inputs.generate_into(a.kind, seed, host.data_ptr(), n)
d_in = host.to("cuda:0")
cap = mc.shard_bound(n, a.block)
d_out = torch.empty(cap, dtype=torch.uint8, device="cuda:0")
ctx = mc.Context(0, a.block, n)
L = mc.lib()
L.fcx_debug_emit_bits.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
st = torch.cuda.current_stream().cuda_stream
for b in a.bits:
    mc._check(L.fcx_debug_emit_bits(ctx._h, int(b, 0)), "bits")
    best = None
    for r in range(a.reps):
        ctx.set_profiling(True)
        try:
            ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, st)
        except Exception:
            pass   # invalid output while bits are set
        torch.cuda.synchronize()
        t = dict(ctx.stage_times())
        best = t[a.stage] if best is None else min(best, t[a.stage])
    print(f"{a.kind} {a.stage} bits={b:>8s} {best:.3f} ms", flush=True)
mc._check(L.fcx_debug_emit_bits(ctx._h, 0), "bits")
