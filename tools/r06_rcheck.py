"""Development: routed compress of rand / text shards of several sizes (k_classify's rounds per workgroup
R = 1..4) against the forced unrouted units; prints mismatches."""
import ctypes, sys, torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import inputs
import my_compress_amd as mc

dev = torch.device("cuda:0")
B = 1 << 20
for kind, mode in (("rand", 7), ("text", 5)):
    for mib in (1020, 768, 512, 300, 1024):
        n = mib << 20
        h = torch.empty(n, dtype=torch.uint8).pin_memory()
        inputs.generate_into(kind, 1, h.data_ptr(), n)
        d_in = h.to(dev)
        cap = mc.shard_bound(n, B)
        outs = []
        for m in (0, mode):
            ctx = mc.Context(0, B, n)
            ctx.set_match_mode(m)
            d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
            k = ctx.compress_shard(d_in.data_ptr(), n, d_out.data_ptr(), cap, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            outs.append((k, d_out[:k].clone()))
            rs = ctx.route_stats() if m == 0 else None
            ctx.close()
        same = outs[0][0] == outs[1][0] and torch.equal(outs[0][1], outs[1][1])
        print(kind, mib, "MiB", "routed == forced:", same, outs[0][0], outs[1][0], rs, flush=True)
        del d_in, h
