import sys, json, hashlib
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import torch, inputs, my_compress_amd as mc
g = json.load(open('/root/repo/tests/golden/golden.json'))
for case in g['cases']:
    if case['name'] not in ('kat30', 'tiny_262'): continue
    data = inputs.make(case)
    got = mc.compress(data, case['block'])
    want = bytes.fromhex(case['out_hex'])
    print(case['name'], len(got), len(want))
    print(' got ', got.hex())
    print(' want', want.hex())
    diff = [i for i in range(min(len(got), len(want))) if got[i] != want[i]]
    print(' diff at', diff[:40])
