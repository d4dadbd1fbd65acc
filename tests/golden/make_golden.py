#!/usr/bin/env python3
"""Generate tests/golden/golden.json from the REFERENCE compiled in place.

Container-only (needs oracle/_ref/libref.so, built by `make -C oracle ref` from
/root/reference/my_compress.cpp).  The committed JSON holds only data: input
specs (re-creatable by tests/inputs.py on any machine), SHA-256 digests and
sizes of the reference's .fcx output, full hex for the small ones, and the
reference's own known-answer results for the primitives on the path.

    python tests/golden/make_golden.py            # writes tests/golden/golden.json
"""
import ctypes
import hashlib
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import inputs  # noqa: E402

REF = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref.so"))
REF.ref_compress_block.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p]
REF.ref_compress_block.restype = ctypes.c_uint32
REF.ref_lz77_tokens.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
REF.ref_lz77_tokens.restype = ctypes.c_uint32
REF.ref_sunday.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_char_p, ctypes.c_int32]
REF.ref_sunday.restype = ctypes.c_int32
REF.ref_golomb_encode.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
REF.ref_golomb_encode.restype = ctypes.c_uint32
REF.ref_combine_bits.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint8, ctypes.c_void_p]
REF.ref_huffman_tree.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
REF.ref_huffman_tree.restype = ctypes.c_uint32
REF.ref_decompress_block.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
REF.ref_decompress_block.restype = ctypes.c_int64
REF.ref_set_quiet(1)


def ref_file(data: bytes, block: int) -> bytes:
    """main()'s compress loop (my_compress.cpp:4073-4136) around the reference block encoder."""
    nblk = (len(data) + block - 1) // block
    out = bytearray(b"FCX7" + struct.pack("<IH", len(data) & 0xFFFFFFFF, nblk & 0xFFFF))
    ob = ctypes.create_string_buffer(2 * block + 4096)
    for off in range(0, len(data), block):
        blk = data[off:off + block]
        n = REF.ref_compress_block(blk, len(blk), ob)
        out += struct.pack("<I", n) + ob.raw[:n]
    return bytes(out)


def ref_decode_file(blob: bytes) -> bytes:
    """main()'s decompress loop (my_compress.cpp:4160-4204) around the reference
    block decoder my_decompress_file_lz77 (2255-2393): the decoded bytes of every
    record, concatenated, quirks included (single-symbol sub-streams decode as
    zeros 930-984; a match token past pCnt stops the block, 2336-2339)."""
    nblk = struct.unpack_from("<H", blob, 8)[0]
    off, out = 10, bytearray()
    ob = ctypes.create_string_buffer((1 << 20) + 4096)
    for _ in range(nblk):
        (n,) = struct.unpack_from("<I", blob, off)
        got = REF.ref_decompress_block(blob[off + 4:off + 4 + n], n, ob, len(ob))
        out += ob.raw[:got]
        off += 4 + n
    return bytes(out)


def ref_tokens(data: bytes):
    n = len(data)
    p = (ctypes.c_uint32 * (n + 1))()
    l = (ctypes.c_uint32 * (n + 1))()
    c = (ctypes.c_uint8 * (n + 1))()
    N = REF.ref_lz77_tokens(data, n, p, l, c)
    return [[p[i], l[i], c[i]] for i in range(N)]


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def main():
    cases = []
    for spec in inputs.golden_specs():
        data = inputs.make(spec)
        out = ref_file(data, spec["block"])
        rec = dict(spec)
        rec.update(in_sha256=sha(data), in_bytes=len(data), out_bytes=len(out), out_sha256=sha(out))
        dec = ref_decode_file(out)
        rec.update(dec_bytes=len(dec), dec_sha256=sha(dec), dec_is_input=dec == data)
        if len(out) <= 4096:
            rec["out_hex"] = out.hex()
        cases.append(rec)
        print(f"{spec['name']:40s} in={len(data):9d} out={len(out):9d} {rec['out_sha256'][:12]}", file=sys.stderr)

    token_cases = []
    for spec in inputs.token_specs():
        data = inputs.make(spec)
        token_cases.append(dict(spec, in_sha256=sha(data), tokens=ref_tokens(data)))

    # the reference's own self-test KATs (my_compress.cpp:3749-3759 active prints;
    # 3779-3867 disabled tests), evaluated by the reference itself
    kat = {}
    s1 = b"bbc abcdab abcdabcdabde"
    s2 = b"bbc abcdab abcdabcdabcd"
    s3 = b"bbc abcdab abcdabcdaacd"
    kat["sunday"] = [
        [s1.hex(), 23, b"abcdabd".hex(), 7, REF.ref_sunday(s1 + b"\0", 23, b"abcdabd", 7)],
        [s2.hex(), 23, s2[15:23].hex(), 8, REF.ref_sunday(s2 + b"\0", 23, s2[15:], 8)],
        [s3.hex(), 23, s3[15:23].hex(), 8, REF.ref_sunday(s3 + b"\0", 23, s3[15:], 8)],
        [s3.hex(), 22, s3[15:23].hex(), 8, REF.ref_sunday(s3 + b"\0", 22, s3[15:], 8)],
        [s3.hex(), 23, s3[15:19].hex(), 4, REF.ref_sunday(s3 + b"\0", 23, s3[15:], 4)],
    ]
    vals = (ctypes.c_uint32 * 10)(*[i * 17 for i in range(10)])
    words = (ctypes.c_uint32 * 64)()
    nw = REF.ref_golomb_encode(vals, 10, words)
    kat["golomb"] = {"in": [i * 17 for i in range(10)], "words": [words[i] for i in range(nw)]}
    # lengths 3..257 as they occur in the parse
    vals2 = list(range(3, 258))
    v2 = (ctypes.c_uint32 * len(vals2))(*vals2)
    words2 = (ctypes.c_uint32 * 4096)()
    nw2 = REF.ref_golomb_encode(v2, len(vals2), words2)
    kat["golomb_3_257"] = {"in": vals2, "words": [words2[i] for i in range(nw2)]}
    cb = (ctypes.c_uint32 * 4)(0x123, 0x345, 0x567, 0x789)
    cbo = (ctypes.c_uint8 * 7)()
    REF.ref_combine_bits(cb, 4, 12, cbo)
    kat["combine_bits"] = {"in": [0x123, 0x345, 0x567, 0x789], "bits": 12, "out": list(cbo)}
    pv = [1, 2047, 1024, 5, 300, 2046, 7]
    cb2 = (ctypes.c_uint32 * len(pv))(*pv)
    cbo2 = (ctypes.c_uint8 * ((11 * len(pv)) // 8 + 1))()
    REF.ref_combine_bits(cb2, len(pv), 11, cbo2)
    kat["combine_bits_11"] = {"in": pv, "bits": 11, "out": list(cbo2)}
    # my_compress_file_lz77 (2115-2253) on totalBytes = 0: a valid call with a 17-byte payload
    eb = ctypes.create_string_buffer(4096)
    en = REF.ref_compress_block(b"", 0, eb)
    kat["empty_block"] = {"in_bytes": 0, "out_hex": eb.raw[:en].hex()}
    wts = [0, 5, 29, 7, 0, 8, 14, 23, 3, 11, 0]
    w = (ctypes.c_uint32 * 11)(*wts)
    nodes = (ctypes.c_uint32 * (4 * 21))()
    real = REF.ref_huffman_tree(w, 11, nodes)
    kat["huffman_tree"] = {"weights": wts, "real": real, "nodes": [list(nodes[4 * i:4 * i + 4]) for i in range(21)]}
    # ties everywhere: equal weights exercise the strict '<' re-insertion rule (588)
    wts2 = [4, 4, 4, 4, 8, 8, 2, 2, 16, 1, 1, 0, 3, 3]
    w2 = (ctypes.c_uint32 * len(wts2))(*wts2)
    nodes2 = (ctypes.c_uint32 * (4 * (2 * len(wts2) - 1)))()
    real2 = REF.ref_huffman_tree(w2, len(wts2), nodes2)
    kat["huffman_tree_ties"] = {"weights": wts2, "real": real2,
                                "nodes": [list(nodes2[4 * i:4 * i + 4]) for i in range(2 * len(wts2) - 1)]}

    doc = {
        "about": "Reference outputs for my_compress.cpp -c lz77 (YuBinRen/my_compress), generated by "
                 "tests/golden/make_golden.py from oracle/_ref (the reference compiled in place). "
                 "Inputs are re-created from their spec by tests/inputs.py.",
        "cases": cases,
        "tokens": token_cases,
        "kat": kat,
        "survey_digests": inputs.SURVEY_DIGESTS,
    }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(doc, f, indent=1)
    print("wrote golden.json", file=sys.stderr)


if __name__ == "__main__":
    main()
