"""Throughput of the -c lz78 codec on one GPU (device-resident input, 1 MiB blocks).
LZ78 is a serial-dictionary parse per block; this measures where it stands, it is
not the headline metric.  Usage: python tools/lz78bench.py [MiB]"""
import ctypes
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

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
n, block = mib << 20, 1 << 20
res = {}
for kind in ("rand", "text"):
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    inputs.generate_into(kind, 4, host.data_ptr(), n)
    d_in = host.to("cuda:0")
    cap = mc.lz78_bound(n, block)
    d_out = torch.empty(cap, dtype=torch.uint8, device="cuda:0")
    out_len = ctypes.c_uint64()
    st = torch.cuda.current_stream().cuda_stream
    L = mc.lib()
    for it in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = L.fcx_lz78_compress_shard(d_in.data_ptr(), n, block, d_out.data_ptr(), cap, ctypes.byref(out_len), st)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        assert rc == 0, L.fcx_last_error()
    comp = bytes(d_out[:out_len.value].cpu().numpy())
    hdr = b"FCX8" + n.to_bytes(4, "little") + (n // block).to_bytes(2, "little")
    t1 = time.perf_counter()
    dec = mc.decompress_lz78(hdr + comp)
    dt_dec = time.perf_counter() - t1
    # the reference decoder drops a block's trailing 0x00 unless the block's last token
    # was a whole-remainder (index, '\0') token (my_compress.cpp:1858-1863, 3701-3703)
    src = bytes(host.numpy())
    q, ok = 0, True
    for o in range(0, n, block):
        blk = src[o:o + block]
        if dec[q:q + len(blk)] == blk:
            q += len(blk)
        elif blk[-1] == 0 and dec[q:q + len(blk) - 1] == blk[:-1]:
            q += len(blk) - 1
        else:
            ok = False
            break
    ok = ok and q == len(dec)
    res[kind] = {"compress_MBps": n / dt / 1e6, "ms": dt * 1e3, "ratio": out_len.value / n,
                 "decode_host_to_host_MBps": n / dt_dec / 1e6,
                 "round_trip_modulo_tail_zero_rule": ok}
    print(kind, json.dumps(res[kind]), flush=True)
print(json.dumps({"lz78": res, "mib": mib, "block_bytes": block}))
