"""Deterministic test inputs, shared by the tests, the
golden-vector script and smoke().

Every input is described by a small JSON-able spec and re-created by `make(spec)`
from tools/libfcxgen.so (glibc TYPE_3 rand embedded), so the committed fixtures
carry data specs + expected outputs, never bulk bytes.
"""
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN_KIND = {"rand": 0, "zeros": 1, "runs": 2, "text": 3, "dna": 4}
MiB = 1 << 20

_gen = None


def gen_lib():
    global _gen
    if _gen is None:
        _gen = ctypes.CDLL(os.path.join(ROOT, "tools", "libfcxgen.so"))
        _gen.fcxgen_generate.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
        _gen.fcxgen_create.argtypes = [ctypes.c_int, ctypes.c_uint32]
        _gen.fcxgen_create.restype = ctypes.c_void_p
        _gen.fcxgen_fill.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        _gen.fcxgen_destroy.argtypes = [ctypes.c_void_p]
        _gen.fcxgen_rand_values.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
    return _gen


# the `mix` input (bench leg `mix`): 1 MiB blocks cycling through four kinds -- block i is block
# i // 4 of the stream MIX_STREAMS[i % 4] (the same streams and seeds as the per-kind bench legs)
MIX_STREAMS = (("rand", 4), ("text", 3), ("runs", 5), ("dna", 6))
MIX_BLOCK = MiB


def mix_into(ptr: int, n: int) -> None:
    nb = (n + MIX_BLOCK - 1) // MIX_BLOCK
    for k, (kind, seed) in enumerate(MIX_STREAMS):
        mine = range(k, nb, len(MIX_STREAMS))
        if not len(mine):
            continue
        tmp = ctypes.create_string_buffer(len(mine) * MIX_BLOCK)
        gen_lib().fcxgen_generate(GEN_KIND[kind], seed, tmp, len(mine) * MIX_BLOCK)
        for j, i in enumerate(mine):
            ln = min(MIX_BLOCK, n - i * MIX_BLOCK)
            ctypes.memmove(ptr + i * MIX_BLOCK, ctypes.addressof(tmp) + j * MIX_BLOCK, ln)


def generate(kind: str, seed: int, n: int) -> bytes:
    buf = ctypes.create_string_buffer(max(n, 1))
    generate_into(kind, seed, ctypes.addressof(buf), n)
    return buf.raw[:n]


def generate_into(kind: str, seed: int, ptr: int, n: int) -> None:
    """fill host memory at `ptr` (e.g. a pinned torch tensor) with n bytes (kind "mix": mix_into,
    the seed is unused)"""
    if kind == "mix":
        mix_into(ptr, n)
    else:
        gen_lib().fcxgen_generate(GEN_KIND[kind], seed, ctypes.c_void_p(ptr), n)


def _lcg(seed):
    x = seed & 0xFFFFFFFF
    while True:
        x = (1103515245 * x + 12345) & 0x7FFFFFFF
        yield x


def mosaic(seed: int, n: int) -> bytes:
    """concatenation of pieces of every kind and many lengths: sparse/dense
    transitions inside blocks and tiles (long zero runs inside text, periodic
    stretches, random bursts)."""
    r = _lcg(seed)
    out = bytearray()
    kinds = ["text", "rand", "runs", "zeros", "period", "text", "runs"]
    while len(out) < n:
        k = kinds[next(r) % len(kinds)]
        ln = 1 + next(r) % 9000
        if k == "period":
            per = 1 + next(r) % 9
            pat = generate("rand", next(r), per)
            piece = (pat * (ln // per + 1))[:ln]
        else:
            piece = generate(k, next(r) % 1000 + 1, ln)
        out += piece
    return bytes(out[:n])


def make(spec) -> bytes:
    t = spec["type"]
    if t == "tiny":          # bytes (7i+3) mod 256
        return bytes((7 * i + 3) % 256 for i in range(spec["n"]))
    if t == "seq":
        return bytes(range(spec["n"]))
    if t == "repeat":
        return bytes.fromhex(spec["hex"]) * spec["count"]
    if t == "gen":
        return generate(spec["kind"], spec["seed"], spec["n"])
    if t == "mosaic":
        return mosaic(spec["seed"], spec["n"])
    if t == "concat":
        return b"".join(make(s) for s in spec["parts"])
    raise ValueError(t)


def _g(kind, seed, n, block, name=None):
    return {"name": name or f"{kind}_s{seed}_{n}_b{block}", "type": "gen", "kind": kind,
            "seed": seed, "n": n, "block": block}


def golden_specs():
    S = []
    for n in [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 16, 17, 31, 64, 258, 259, 262, 1000]:
        S.append({"name": f"tiny_{n}", "type": "tiny", "n": n, "block": MiB})
    S.append({"name": "seq16", "type": "seq", "n": 16, "block": MiB})
    S.append({"name": "seq256x40", "type": "repeat", "hex": bytes(range(256)).hex(), "count": 40, "block": MiB})
    S.append({"name": "abcabd_x1000", "type": "repeat", "hex": b"abcabcabcabd".hex(), "count": 1000, "block": MiB})
    S.append({"name": "A_x100000", "type": "repeat", "hex": b"A".hex(), "count": 100000, "block": MiB})
    S.append({"name": "kat30", "type": "repeat", "hex": b"aacaacabcabaaacbaaacccaacabcad".hex(), "count": 1, "block": MiB})
    for per in [1, 2, 3, 5, 8, 13]:
        S.append({"name": f"period{per}", "type": "repeat", "hex": bytes((37 * i + 11) % 251 for i in range(per)).hex(),
                  "count": 70000 // per, "block": 65536})
    for kind, seed in [("rand", 1), ("text", 1), ("runs", 1), ("zeros", 0)]:
        for block in [MiB, 65536, 262144]:
            S.append(_g(kind, seed, MiB, block))
    S.append(_g("text", 7, 300000, 4096))
    S.append(_g("rand", 8, 100000, 1000))
    S.append(_g("runs", 9, 200000, 10000))
    S.append(_g("text", 11, 77777, 65536))
    S.append(_g("zeros", 0, 5000, 1000))
    for seed in [1, 2, 3]:
        for block in [65536, MiB]:
            S.append({"name": f"mosaic_s{seed}_b{block}", "type": "mosaic", "seed": seed, "n": 600000, "block": block})
    S.append({"name": "text_zeros_text", "type": "concat", "block": MiB, "parts": [
        {"type": "gen", "kind": "text", "seed": 21, "n": 100000},
        {"type": "gen", "kind": "zeros", "seed": 0, "n": 50000},
        {"type": "gen", "kind": "text", "seed": 22, "n": 100000}]})
    # a chars stream whose random stretch has Huffman codes far above 8 bits (text sets
    # the frequencies): chunks there take several encode staging windows
    S.append({"name": "text_rand_text_longcodes", "type": "concat", "block": MiB, "parts": [
        {"type": "gen", "kind": "text", "seed": 23, "n": 600000},
        {"type": "gen", "kind": "rand", "seed": 24, "n": 40000},
        {"type": "gen", "kind": "text", "seed": 25, "n": 300000}]})
    S.append({"name": "text_plus_partial", "type": "concat", "block": 262144, "parts": [
        {"type": "gen", "kind": "text", "seed": 5, "n": MiB + 12345}]})
    # decoder quirks (my_compress.cpp:2255-2393): an all-literal block whose flag bytes
    # are all 0xFF has a one-symbol flags stream, which the reference decodes as zeros,
    # so its first "match" token finds pCnt exhausted and the block stops empty
    # (2336-2339); 4100 bytes leave a partial last flag byte (two symbols, decodes fine)
    S.append(_g("rand", 31, 4096, 4096, name="quirk_rand4k_empty"))
    S.append(_g("rand", 32, 4 * 4096, 4096, name="quirk_rand4k_x4"))
    S.append(_g("rand", 33, 4100, 8192, name="quirk_rand4100"))
    S.append({"name": "quirk_text_rand_text", "type": "concat", "block": 4096, "parts": [
        {"type": "gen", "kind": "text", "seed": 34, "n": 6000},
        {"type": "gen", "kind": "rand", "seed": 35, "n": 8192},
        {"type": "gen", "kind": "text", "seed": 36, "n": 6000}]})
    S.append({"name": "quirk_two_symbols", "type": "repeat", "hex": b"AB".hex(), "count": 3000, "block": 1000})
    return S


def token_specs():
    return [
        {"name": "kat30", "type": "repeat", "hex": b"aacaacabcabaaacbaaacccaacabcad".hex(), "count": 1},
        {"name": "abc300", "type": "repeat", "hex": b"abc".hex(), "count": 100},
        {"name": "text5000", "type": "gen", "kind": "text", "seed": 3, "n": 5000},
        {"name": "runs3000", "type": "gen", "kind": "runs", "seed": 4, "n": 3000},
        {"name": "mosaic20000", "type": "mosaic", "seed": 9, "n": 20000},
    ]


# Digests of the reference's output on the full-size configs (SURVEY.md §8(c),
# Appendix B.4): produced by the survey with the same in-place reference build
# (8 processes over block ranges, byte-identical to the CLI).
SURVEY_DIGESTS = {
    "cfg2_rand_64MiB": {"kind": "rand", "seed": 2, "n": 64 * MiB, "block": 65536,
                        "in": "d0ea0741abb3435057409137cdc79331b78c64ab0c5cbe8678e6fae40d3179cf",
                        "bytes": 68819158, "out": "3b6853f2cf570b7a35c469efff62c15e0290b04ede45f6b47a97afc82c1878a5"},
    "cfg3_text_1GiB": {"kind": "text", "seed": 3, "n": 1024 * MiB, "block": 262144,
                       "in": "713e4aa36f5d3604cc756c4abf995bc0355d1c7387379c60bcd24b8556c3bdea",
                       "bytes": 630008807, "out": "20219e60c2e9aef6659801fbfc53c6873ec811686eedcb45c0896fc5547d63d0"},
    "cfg5a_zeros_1GiB": {"kind": "zeros", "seed": 0, "n": 1024 * MiB, "block": MiB,
                         "in": "49bc20df15e412a64472421e13fe86ff1c5165e18b2afccf160d4dc19fe68a14",
                         "bytes": 7521290, "out": "533fd45fbaa861a6060e9a5beac177cc0b64db691fc602a1e0e1e188afa5f912"},
    "cfg5b_runs_1GiB": {"kind": "runs", "seed": 5, "n": 1024 * MiB, "block": MiB,
                        "in": "18cddd87a89e44af896056a31ae955c56deea5bf47ab1de5ab491796d5115ef3",
                        "bytes": 42548682, "out": "4fced94fd4725ba3b1031dec67d63e1295b95ae08cc1cf0e34c84769f5313d26"},
    # not a SURVEY digest: the bench's `mix` leg, made here by the reference compiled in place
    # (tests/golden/make_mix_digest.py)
    "mix_1GiB": {"kind": "mix", "seed": 0, "n": 1024 * MiB, "block": MiB,
                 "in": "02afe5c4c67cbf572024632afed721e1d90bb58f44b40259422cb3fd23db3ae2",
                 "bytes": 523200760, "out": "ce8bb8bc756a62fcd276d6a71b93456c18a7def3d77e555ea7eb8b92bfebffb5"},
    "hl_text_1GiB": {"kind": "text", "seed": 3, "n": 1024 * MiB, "block": MiB,
                     "in": "713e4aa36f5d3604cc756c4abf995bc0355d1c7387379c60bcd24b8556c3bdea",
                     "bytes": 624801500, "out": "132a36b9d2592f8c37a82b51f545ddb67acec53fa1a31b7f1f6a04617a01a3d1"},
    "hl_rand_1GiB": {"kind": "rand", "seed": 4, "n": 1024 * MiB, "block": MiB,
                     "in": "2a96181ea4cf7c0c9cfff49677640efe0a5a0b12ee5d0379f2bdf06d9c41f29d",
                     "bytes": 1091294206, "out": "ee962534628bf6b2f79c51a44a65ac0845945e2fe9225e5be8f99f288912a69d"},
}

# BASELINE config 4 (8 GiB rand seed 4, 1 MiB blocks) split over 8 ranks: rank r
# compresses bytes [r GiB, (r+1) GiB) of the one stream into its segment of
# [u32 len][payload] records (no header).  Sizes and sha256 prefixes of the
# reference's segments; the whole file is
# 10 + sum(bytes) = 8,730,352,595 B with sha256 8f1cae2f... (header total wraps to 0).
C4_SEGMENTS = [
    (1091294196, "6e3350797c82335d"),
    (1091294015, "baccd8ba445a9881"),
    (1091294276, "9b42660291458d16"),
    (1091294478, "df0203068ca7daa3"),
    (1091294029, "7330de83672cbb7d"),
    (1091293907, "d31a6f66f351bab0"),
    (1091293647, "3663bdd18b38bc7f"),
    (1091294037, "018665b30a10d61d"),
]
C4_FILE = {"bytes": 8730352595, "out": "8f1cae2fa6fbc3b597bd90b83fd0998ffeb7d827e199a9f6aa3c25fea587656c"}


def rand_stream_into(seed: int, offset: int, ptr: int, n: int, kind: str = "rand") -> None:
    """bytes [offset, offset + n) of the rand (or dna) stream of `seed` (one glibc
    rand() per byte), via the generator's O(log offset) jump-ahead: rank shards of
    one global input"""
    G = gen_lib()
    G.fcxgen_skip.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    h = G.fcxgen_create(GEN_KIND[kind], seed)
    try:
        G.fcxgen_skip(h, offset)
        G.fcxgen_fill(h, ctypes.c_void_p(ptr), n)
    finally:
        G.fcxgen_destroy(h)

