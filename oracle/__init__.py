"""oracle — CPU checkers for the FCX7 / LZ77 compress path.

TEST INFRASTRUCTURE ONLY.  Imported solely by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg, and only as the checker / the timed CPU
baseline — never as the thing measured or shipped.  The product
(my_compress_amd/) never imports or links anything here.

  liboracle.so   clean-room C restatement (fcx_oracle.c) of my_compress.cpp's
                 -c lz77 path; pinned by tests/test_oracle.py against the
                 reference's own KATs and against _ref/libref.so.
  _ref/libref.so the reference itself, compiled in place from
                 /root/reference/my_compress.cpp (oracle/Makefile, container
                 only; travels to the GPU box prebuilt, may be absent).
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
FINDER_SUNDAY, FINDER_EXHAUSTIVE = 0, 1
_orc = None
_ref = None


def orc():
    global _orc
    if _orc is None:
        L = ctypes.CDLL(os.path.join(HERE, "liboracle.so"))
        L.orc_compress_file.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                        ctypes.c_uint64, ctypes.c_int]
        L.orc_compress_file.restype = ctypes.c_uint64
        L.orc_decompress_file.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
        L.orc_decompress_file.restype = ctypes.c_int64
        L.orc_compress_block.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
        L.orc_compress_block.restype = ctypes.c_uint32
        L.orc_decompress_block.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
        L.orc_decompress_block.restype = ctypes.c_int64
        L.orc_lz77_parse.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p]
        L.orc_lz77_parse.restype = ctypes.c_uint32
        L.orc_sunday_search.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_char_p, ctypes.c_int32]
        L.orc_sunday_search.restype = ctypes.c_int32
        L.orc_golomb_encode.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        L.orc_golomb_encode.restype = ctypes.c_uint32
        L.orc_combine_bits.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
        L.orc_huffman_tree.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        L.orc_huffman_tree.restype = ctypes.c_uint32
        L.orc_huffman_stream.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p]
        L.orc_huffman_stream.restype = ctypes.c_uint32
        _orc = L
    return _orc


def ref():
    """the reference compiled in place, or None when oracle/_ref was not built/shipped"""
    global _ref
    if _ref is None:
        path = os.path.join(HERE, "_ref", "libref.so")
        if not os.path.exists(path):
            return None
        L = ctypes.CDLL(path)
        L.ref_compress_block.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p]
        L.ref_compress_block.restype = ctypes.c_uint32
        L.ref_set_quiet.argtypes = [ctypes.c_int]
        L.ref_set_quiet(1)   # the reference printf()s per block (my_compress.cpp:2249)
        _ref = L
    return _ref


def compress_file(data: bytes, block: int, finder: int = FINDER_EXHAUSTIVE) -> bytes:
    nb = (len(data) + block - 1) // block
    cap = 2 * len(data) + 4096 * (nb + 2)
    out = ctypes.create_string_buffer(cap)
    n = orc().orc_compress_file(data, len(data), block, out, cap, finder)
    if n == 0:
        raise RuntimeError("oracle compress failed")
    return out.raw[:n]


def decompress_file(blob: bytes, cap: int) -> bytes:
    out = ctypes.create_string_buffer(max(cap, 1))
    n = orc().orc_decompress_file(blob, len(blob), out, cap)
    if n < 0:
        raise RuntimeError("oracle decompress failed")
    return out.raw[:n]


def compress_block(block: bytes, finder: int = FINDER_EXHAUSTIVE) -> bytes:
    out = ctypes.create_string_buffer(2 * len(block) + 4096)
    n = orc().orc_compress_block(block, len(block), out, finder)
    return out.raw[:n]


def parse(data: bytes, finder: int = FINDER_EXHAUSTIVE):
    n = len(data)
    p = (ctypes.c_uint32 * (n + 1))()
    l = (ctypes.c_uint32 * (n + 1))()
    c = (ctypes.c_uint8 * (n + 1))()
    N = orc().orc_lz77_parse(data, n, finder, p, l, c)
    return [[p[i], l[i], c[i]] for i in range(N)]


def ref_compress_file(data: bytes, block: int) -> bytes:
    """the reference block encoder framed like main(); requires oracle/_ref"""
    import struct
    R = ref()
    if R is None:
        raise RuntimeError("oracle/_ref/libref.so not built")
    nb = (len(data) + block - 1) // block
    out = bytearray(b"FCX7" + struct.pack("<IH", len(data) & 0xFFFFFFFF, nb & 0xFFFF))
    ob = ctypes.create_string_buffer(2 * block + 4096)
    for off in range(0, len(data), block):
        blk = data[off:off + block]
        n = R.ref_compress_block(blk, len(blk), ob)
        out += struct.pack("<I", n) + ob.raw[:n]
    return bytes(out)


# ---- -c lz78 (lz78_oracle.c; reference my_compress.cpp:1832-1934, 3127-3710) ----
def _lz78_bind(L):
    if getattr(L, "_lz78", False):
        return L
    L.orc_lz78_parse.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    L.orc_lz78_parse.restype = ctypes.c_uint32
    L.orc_lz78_compress_block.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p]
    L.orc_lz78_compress_block.restype = ctypes.c_uint32
    L.orc_lz78_decompress_block.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
    L.orc_lz78_decompress_block.restype = ctypes.c_int64
    L.orc_lz78_compress_file.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                         ctypes.c_uint64]
    L.orc_lz78_compress_file.restype = ctypes.c_uint64
    L.orc_lz78_decompress_file.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
    L.orc_lz78_decompress_file.restype = ctypes.c_int64
    L._lz78 = True
    return L


def lz78_bound(n: int, block: int) -> int:
    """output capacity for an FCX8 file: ≤ 4 B per input byte + 64 KiB per block"""
    nb = max(1, (n + block - 1) // block)
    return 10 + 4 * n + (65536 + 4) * nb


def lz78_parse(data: bytes):
    n = len(data)
    idx = (ctypes.c_uint32 * (n + 1))()
    c = (ctypes.c_uint8 * (n + 1))()
    N = _lz78_bind(orc()).orc_lz78_parse(data, n, idx, c)
    return [(idx[i], c[i]) for i in range(N)]


def lz78_compress_block(block: bytes) -> bytes:
    out = ctypes.create_string_buffer(4 * len(block) + 65536)
    n = _lz78_bind(orc()).orc_lz78_compress_block(block, len(block), out)
    return out.raw[:n]


def lz78_decompress_block(payload: bytes, cap: int) -> bytes:
    out = ctypes.create_string_buffer(max(cap, 1))
    n = _lz78_bind(orc()).orc_lz78_decompress_block(payload, len(payload), out, cap)
    if n < 0:
        raise RuntimeError("oracle lz78 decompress failed")
    return out.raw[:n]


def lz78_compress_file(data: bytes, block: int) -> bytes:
    cap = lz78_bound(len(data), block)
    out = ctypes.create_string_buffer(cap)
    n = _lz78_bind(orc()).orc_lz78_compress_file(data, len(data), block, out, cap)
    if n == 0:
        raise RuntimeError("oracle lz78 compress failed")
    return out.raw[:n]


def lz78_decompress_file(blob: bytes, cap: int) -> bytes:
    out = ctypes.create_string_buffer(max(cap, 1))
    n = _lz78_bind(orc()).orc_lz78_decompress_file(blob, len(blob), out, cap)
    if n < 0:
        raise RuntimeError("oracle lz78 decompress failed")
    return out.raw[:n]


def _ref_lz78_bind(R):
    if getattr(R, "_lz78", False):
        return R
    R.ref_lz78_compress_block.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p]
    R.ref_lz78_compress_block.restype = ctypes.c_uint32
    R.ref_lz78_tokens.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    R.ref_lz78_tokens.restype = ctypes.c_uint32
    R.ref_lz78_decompress_block.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
    R.ref_lz78_decompress_block.restype = ctypes.c_int64
    R._lz78 = True
    return R


def ref_lz78_tokens(data: bytes):
    R = ref()
    if R is None:
        raise RuntimeError("oracle/_ref/libref.so not built")
    n = len(data)
    idx = (ctypes.c_uint32 * (n + 1))()
    c = (ctypes.c_uint8 * (n + 1))()
    N = _ref_lz78_bind(R).ref_lz78_tokens(data, n, idx, c)
    return [(idx[i], c[i]) for i in range(N)]


def ref_lz78_compress_block(block: bytes) -> bytes:
    R = ref()
    if R is None:
        raise RuntimeError("oracle/_ref/libref.so not built")
    out = ctypes.create_string_buffer(4 * len(block) + 65536)
    n = _ref_lz78_bind(R).ref_lz78_compress_block(block, len(block), out)
    return out.raw[:n]


def ref_lz78_decompress_block(payload: bytes, cap: int) -> bytes:
    R = ref()
    if R is None:
        raise RuntimeError("oracle/_ref/libref.so not built")
    out = ctypes.create_string_buffer(max(cap, 1))
    n = _ref_lz78_bind(R).ref_lz78_decompress_block(payload, len(payload), out, cap)
    return out.raw[:min(n, cap)]


def ref_lz78_compress_file(data: bytes, block: int) -> bytes:
    """the reference lz78 block encoder framed like main() with -c lz78 ("FCX8")"""
    import struct
    nb = (len(data) + block - 1) // block
    out = bytearray(b"FCX8" + struct.pack("<IH", len(data) & 0xFFFFFFFF, nb & 0xFFFF))
    for off in range(0, len(data), block):
        p = ref_lz78_compress_block(data[off:off + block])
        out += struct.pack("<I", len(p)) + p
    return bytes(out)
