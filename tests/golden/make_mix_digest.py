#!/usr/bin/env python3
"""Reference digest of the bench's `mix` leg: 1 GiB whose 1 MiB blocks cycle through rand / text /
runs / dna (tests/inputs.py mix_into), compressed by the reference's own block encoder
(oracle/_ref/libref.so: /root/reference/my_compress.cpp compiled in place, my_compress_file_lz77
:2115) and framed as main() writes the file (:4073-4136).  Blocks are independent, so they are
encoded on several host threads and written in block order.  Prints the JSON entry committed in
tests/inputs.py (SURVEY_DIGESTS["mix_1GiB"]) and bench.py (HL_DIGEST).

    python tests/golden/make_mix_digest.py [--mib 1024] [--threads 8]
"""
import argparse
import ctypes
import hashlib
import json
import os
import struct
import sys
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import inputs  # noqa: E402
import oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    n, block = a.mib << 20, inputs.MIX_BLOCK
    R = oracle.ref()
    if R is None:
        sys.exit("oracle/_ref/libref.so not built (make -C oracle ref)")
    R.ref_set_quiet(1)
    data = inputs.generate("mix", 0, n)
    nb = (n + block - 1) // block
    recs = [None] * nb
    lock = threading.Lock()
    todo = list(range(nb))

    def worker():
        ob = ctypes.create_string_buffer(2 * block + 4096)
        while True:
            with lock:
                if not todo:
                    return
                i = todo.pop()
            blk = data[i * block:(i + 1) * block]
            k = R.ref_compress_block(blk, len(blk), ob)
            recs[i] = struct.pack("<I", k) + ob.raw[:k]

    ths = [threading.Thread(target=worker) for _ in range(a.threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    R.ref_set_quiet(0)
    h = hashlib.sha256(b"FCX7" + struct.pack("<IH", n & 0xFFFFFFFF, nb & 0xFFFF))
    size = 10
    for r in recs:
        h.update(r)
        size += len(r)
    print(json.dumps({"kind": "mix", "n": n, "block": block, "in": hashlib.sha256(data).hexdigest(),
                      "out": h.hexdigest(), "bytes": size}))


if __name__ == "__main__":
    main()
