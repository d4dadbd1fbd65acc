"""my_compress_amd — MI355X-native LZ77 + Huffman compressor (FCX7 byte stream).

Python mirror of the reference's compress interface over the C ABI in
include/fcx.h (lib/libfcx.so, hand-written HIP kernels for gfx950):

    my_compress_file_lz77(block) -> payload      # my_compress.cpp:2115
    my_decompress_file_lz77(payload) -> block    # my_compress.cpp:2255
    compress(data, block_bytes) -> FCX7 file     # main() compress loop, :4073-4136
    decompress(blob) -> data                     # main() decompress loop, :4137-4204
    Context(...).compress_shard(d_in, n, d_out, cap, stream)   # device-resident batch

The compress path runs only on the GPU: a missing extension or device raises
(FcxError / ImportError); there is no CPU fallback.
"""
import ctypes
import os
import struct

__all__ = [
    "FcxError", "lib", "lib_path", "Context", "my_compress_file_lz77", "my_decompress_file_lz77",
    "compress", "decompress", "shard_bound", "write_header", "BLOCK_BYTES", "HEADER_BYTES",
]

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
BLOCK_BYTES = 1 << 20   # BLOCK_BYTES, my_compress.cpp:113
HEADER_BYTES = 10       # stCmpFileHead, my_compress.cpp:101-109

_lib = None


class FcxError(RuntimeError):
    pass


def lib_path() -> str:
    # FCX_LIB: alternative in-tree build for A/B experiments (tools/); default lib/libfcx.so
    return os.environ.get("FCX_LIB") or os.path.join(PKG_DIR, "lib", "libfcx.so")


def lib():
    """Load lib/libfcx.so (built by __graft_entry__.build()); raises if missing."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(path)
    c_u8p = ctypes.c_void_p
    L.fcx_compress_block.argtypes = [ctypes.c_void_p, ctypes.c_uint32, c_u8p]
    L.fcx_compress_block.restype = ctypes.c_uint32
    L.fcx_decompress_block.argtypes = [c_u8p, ctypes.c_uint32, c_u8p, ctypes.c_uint64]
    L.fcx_decompress_block.restype = ctypes.c_int64
    L.fcx_write_header.argtypes = [c_u8p, ctypes.c_uint64, ctypes.c_uint64]
    L.fcx_parse_header.argtypes = [c_u8p, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint16),
                                   ctypes.c_char_p]
    L.fcx_shard_bound.argtypes = [ctypes.c_uint64, ctypes.c_uint32]
    L.fcx_shard_bound.restype = ctypes.c_uint64
    L.fcx_ctx_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64]
    L.fcx_ctx_destroy.argtypes = [ctypes.c_void_p]
    L.fcx_ctx_destroy.restype = None
    L.fcx_compress_shard.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                     ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p]
    L.fcx_ctx_device_out_len.argtypes = [ctypes.c_void_p]
    L.fcx_ctx_device_out_len.restype = ctypes.c_void_p
    L.fcx_ctx_read_out_len.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    L.fcx_compress_host.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_uint64, c_u8p, ctypes.c_uint64,
                                    ctypes.POINTER(ctypes.c_uint64)]
    L.fcx_ctx_set_profiling.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.fcx_ctx_set_match_mode.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.fcx_ctx_set_groups.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.fcx_ctx_stage_count.argtypes = [ctypes.c_void_p]
    L.fcx_ctx_stage.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                ctypes.POINTER(ctypes.c_float)]
    L.fcx_ctx_stats.argtypes = [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_uint64)] * 5
    L.fcx_ctx_match_kernel.argtypes = [ctypes.c_void_p]
    L.fcx_ctx_match_kernel.restype = ctypes.c_int
    if hasattr(L, "fcx_ctx_route_stats"):   # (absent from an older FCX_LIB build used for A/B timing)
        L.fcx_ctx_route_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    L.fcx_compress_stream.argtypes = [ctypes.c_void_p, READ_FN, WRITE_FN, ctypes.c_void_p, ctypes.c_uint64,
                                      ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_uint64)]
    L.fcx_decompress_stream.argtypes = [ctypes.c_void_p, READ_FN, WRITE_FN, ctypes.c_void_p, ctypes.c_uint64,
                                        ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64),
                                        ctypes.POINTER(ctypes.c_uint64)]
    L.fcx_dctx_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int]
    L.fcx_dctx_destroy.argtypes = [ctypes.c_void_p]
    L.fcx_dctx_destroy.restype = None
    L.fcx_decompress_shard.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                       ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.c_void_p]
    L.fcx_decompress_host.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_uint64, c_u8p, ctypes.c_uint64,
                                      ctypes.POINTER(ctypes.c_uint64)]
    L.fcx_dctx_set_profiling.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.fcx_dctx_stage_count.argtypes = [ctypes.c_void_p]
    L.fcx_dctx_stage.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                 ctypes.POINTER(ctypes.c_float)]
    L.fcx_lz78_compress_shard.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p]
    L.fcx_lz78_compress_host.argtypes = [c_u8p, ctypes.c_uint64, ctypes.c_uint32, c_u8p, ctypes.c_uint64,
                                         ctypes.POINTER(ctypes.c_uint64)]
    L.fcx_lz78_compress_block.argtypes = [ctypes.c_void_p, ctypes.c_uint32, c_u8p]
    L.fcx_lz78_compress_block.restype = ctypes.c_uint32
    L.fcx_lz78_release.argtypes = []
    L.fcx_lz78_decompress_block.argtypes = [c_u8p, ctypes.c_uint32, c_u8p, ctypes.c_uint64]
    L.fcx_lz78_decompress_block.restype = ctypes.c_int64
    L.fcx_lz78_decompress_host.argtypes = [c_u8p, ctypes.c_uint64, c_u8p, ctypes.c_uint64,
                                           ctypes.POINTER(ctypes.c_uint64)]
    P64 = ctypes.POINTER(ctypes.c_uint64)
    L.fcx_dist_block_range.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, P64, P64]
    L.fcx_dist_block_range.restype = None
    L.fcx_dist_block_range_w.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, P64, P64]
    L.fcx_dist_block_range_w.restype = None
    L.fcx_dist_gather_bound.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
    L.fcx_dist_gather_bound.restype = ctypes.c_uint64
    L.fcx_dist_compress_gather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, P64,
                                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, P64, ctypes.c_void_p]
    L.fcx_dist_unique_id.argtypes = [c_u8p]
    L.fcx_dist_init_rank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int, c_u8p, ctypes.c_int]
    L.fcx_dist_init_local.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    L.fcx_dist_destroy.argtypes = [ctypes.c_void_p]
    L.fcx_dist_destroy.restype = None
    L.fcx_dist_size.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    L.fcx_dist_concat.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                  ctypes.c_uint64, P64, ctypes.c_int, ctypes.c_void_p]
    L.fcx_dist_compress_host.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                         c_u8p, ctypes.c_uint64, P64]
    L.fcx_dist_transport.argtypes = [ctypes.c_void_p]
    L.fcx_dist_transport.restype = ctypes.c_char_p
    L.fcx_loop_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int, ctypes.c_uint32]
    L.fcx_loop_destroy.argtypes = [ctypes.c_void_p]
    L.fcx_loop_destroy.restype = None
    L.fcx_dist_init_loop.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_int]
    L.fcx_dist_init_loop_local.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int,
                                           ctypes.c_uint32]
    L.fcx_dist_debug_fail.argtypes = [ctypes.c_void_p, ctypes.c_int]
    if hasattr(L, "fcx_dist_gather_copy_ms"):
        L.fcx_dist_gather_copy_ms.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
    L.fcx_last_error.restype = ctypes.c_char_p
    L.fcx_version.restype = ctypes.c_char_p
    _lib = L
    return L


# fcx_read_fn / fcx_write_fn (include/fcx.h)
READ_FN = ctypes.CFUNCTYPE(ctypes.c_int64, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint64)
WRITE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint64)


def _stream_fns(src, sink):
    """ctypes callbacks over a binary reader (.readinto) and writer (.write)"""
    def rd(_u, buf, cap):
        mv = (ctypes.c_uint8 * cap).from_address(ctypes.addressof(buf.contents))
        return src.readinto(memoryview(mv).cast("B"))

    def wr(_u, buf, n):
        sink.write(ctypes.string_at(buf, n))
        return 0

    return READ_FN(rd), WRITE_FN(wr)


def _check(rc, what):
    if rc != 0:
        raise FcxError(f"{what} failed ({rc}): {lib().fcx_last_error().decode(errors='replace')}")


def shard_bound(n: int, block_bytes: int = BLOCK_BYTES) -> int:
    return int(lib().fcx_shard_bound(n, block_bytes))


def write_header(total_in: int, nblocks: int) -> bytes:
    buf = ctypes.create_string_buffer(HEADER_BYTES)
    _check(lib().fcx_write_header(buf, total_in, nblocks), "fcx_write_header")
    return buf.raw


class Context:
    """fcx_ctx: device, block size, scratch in HBM for shards up to max_shard_bytes."""

    def __init__(self, device: int = 0, block_bytes: int = BLOCK_BYTES, max_shard_bytes: int = BLOCK_BYTES):
        self._h = ctypes.c_void_p()
        self.block_bytes = block_bytes
        _check(lib().fcx_ctx_create(ctypes.byref(self._h), device, block_bytes, max_shard_bytes), "fcx_ctx_create")

    def close(self):
        if self._h:
            lib().fcx_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def compress_shard(self, d_in: int, n: int, d_out: int, cap: int, stream: int = 0, sync: bool = True):
        """device pointers in, [u32 len][payload]... at d_out; returns bytes (sync) or None"""
        out = ctypes.c_uint64(0)
        _check(lib().fcx_compress_shard(self._h, ctypes.c_void_p(d_in), n, ctypes.c_void_p(d_out), cap,
                                        ctypes.byref(out) if sync else None, ctypes.c_void_p(stream)),
               "fcx_compress_shard")
        return out.value if sync else None

    def device_out_len_ptr(self) -> int:
        return int(lib().fcx_ctx_device_out_len(self._h))

    def read_out_len(self) -> int:
        """waits for the device; output bytes of the last compress_shard"""
        out = ctypes.c_uint64(0)
        _check(lib().fcx_ctx_read_out_len(self._h, ctypes.byref(out)), "fcx_ctx_read_out_len")
        return out.value

    def compress_host(self, data: bytes) -> bytes:
        cap = shard_bound(len(data), self.block_bytes)
        out = ctypes.create_string_buffer(cap)
        got = ctypes.c_uint64(0)
        _check(lib().fcx_compress_host(self._h, data, len(data), out, cap, ctypes.byref(got)), "fcx_compress_host")
        return out.raw[:got.value]

    def compress_stream(self, src, sink, shard_bytes: int):
        """pipelined stream path: records of src (binary reader) to sink (binary writer);
        returns (total_in, total_out, nblocks)"""
        rd, wr = _stream_fns(src, sink)
        vals = [ctypes.c_uint64() for _ in range(3)]
        _check(lib().fcx_compress_stream(self._h, rd, wr, None, shard_bytes, *[ctypes.byref(v) for v in vals]),
               "fcx_compress_stream")
        return tuple(v.value for v in vals)

    def set_profiling(self, on: bool = True):
        _check(lib().fcx_ctx_set_profiling(self._h, 1 if on else 0), "fcx_ctx_set_profiling")

    def set_match_mode(self, mode: int):
        """testing: 0 auto, 1 bucket search, 2 run table for whole tiles, 3 the general
        kernel, 4 the 4-byte-key kernel, 5 the no-filter kernel, 6 the runs kernel, 7 the sparse
        kernel (same output; fcx.h)"""
        _check(lib().fcx_ctx_set_match_mode(self._h, mode), "fcx_ctx_set_match_mode")

    def set_groups(self, groups: int):
        """pipelined launch: block groups over two streams (0 = automatic); same output"""
        _check(lib().fcx_ctx_set_groups(self._h, groups), "fcx_ctx_set_groups")

    def stage_times(self):
        """[(stage name, device ms)] of the last profiled compress_shard"""
        res = []
        for i in range(lib().fcx_ctx_stage_count(self._h)):
            name = ctypes.c_char_p()
            ms = ctypes.c_float()
            _check(lib().fcx_ctx_stage(self._h, i, ctypes.byref(name), ctypes.byref(ms)), "fcx_ctx_stage")
            res.append((name.value.decode(), ms.value))
        return res

    def stats(self):
        vals = [ctypes.c_uint64() for _ in range(5)]
        _check(lib().fcx_ctx_stats(self._h, *[ctypes.byref(v) for v in vals]), "fcx_ctx_stats")
        return dict(zip(["tokens", "matches", "lazy_evals", "lazy_tiles", "tiles"], [v.value for v in vals]))

    MATCH_KERNELS = ("k_match", "k_match_k4", "k_match_nf", "k_match_runs", "k_match_sparse", "k_match_uniform")

    def match_kernel(self) -> str:
        """the kernel the last compress_shard call's match stage ran (fcx_ctx_match_kernel; routed:
        the unit given the most tiles)"""
        return self.MATCH_KERNELS[lib().fcx_ctx_match_kernel(self._h)]

    ROUTE_STATS = ("sparse", "runs", "key4", "nofilter", "handed_on", "tiles", "rest", "cold", "uniform")

    def route_stats(self) -> dict:
        """how the last (routed) call's tiles were searched (fcx_ctx_route_stats): tiles per unit
        list, tiles handed on (to the no-filter and runs lists), tiles with bytes, tiles left to the
        units' remainder kernels, whether the call waited for its own counts (a context's first
        call), and the uniform unit's tiles"""
        n = len(self.ROUTE_STATS)
        vals = (ctypes.c_uint64 * n)()
        _check(lib().fcx_ctx_route_stats(self._h, vals, n), "fcx_ctx_route_stats")
        return dict(zip(self.ROUTE_STATS, [int(v) for v in vals]))


class DContext:
    """fcx_dctx: the GPU decoder (my_decompress_file_lz77 :2255 for whole runs of block records)."""

    def __init__(self, device: int = 0):
        self._h = ctypes.c_void_p()
        _check(lib().fcx_dctx_create(ctypes.byref(self._h), device), "fcx_dctx_create")

    def close(self):
        if self._h:
            lib().fcx_dctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def decompress_shard(self, d_in: int, in_len: int, nblocks: int, d_out: int, cap: int, stream: int = 0) -> int:
        """device records in, decoded bytes at d_out; returns the decoded byte count"""
        out = ctypes.c_uint64(0)
        _check(lib().fcx_decompress_shard(self._h, ctypes.c_void_p(d_in), in_len, nblocks, ctypes.c_void_p(d_out),
                                          cap, ctypes.byref(out), ctypes.c_void_p(stream)), "fcx_decompress_shard")
        return out.value

    def decompress_host(self, blob: bytes, cap: int = None) -> bytes:
        """a whole FCX7 file -> the decoded bytes, on the GPU"""
        if cap is None:
            cap = max(16, struct.unpack_from("<I", blob, 4)[0] if len(blob) >= HEADER_BYTES else 0)
        out = ctypes.create_string_buffer(cap)
        got = ctypes.c_uint64(0)
        _check(lib().fcx_decompress_host(self._h, blob, len(blob), out, cap, ctypes.byref(got)),
               "fcx_decompress_host")
        return out.raw[:got.value]

    def decompress_stream(self, src, sink):
        """FCX7 file from src (binary reader) to sink through the GPU decoder;
        returns (header total, decoded bytes, records)"""
        rd, wr = _stream_fns(src, sink)
        t = ctypes.c_uint32()
        o, n = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().fcx_decompress_stream(self._h, rd, wr, None, 0, ctypes.byref(t), ctypes.byref(o), ctypes.byref(n)),
               "fcx_decompress_stream")
        return t.value, o.value, n.value

    def set_profiling(self, on: bool = True):
        _check(lib().fcx_dctx_set_profiling(self._h, 1 if on else 0), "fcx_dctx_set_profiling")

    def stage_times(self):
        res = []
        for i in range(lib().fcx_dctx_stage_count(self._h)):
            name = ctypes.c_char_p()
            ms = ctypes.c_float()
            _check(lib().fcx_dctx_stage(self._h, i, ctypes.byref(name), ctypes.byref(ms)), "fcx_dctx_stage")
            res.append((name.value.decode(), ms.value))
        return res


def decompress_gpu(blob: bytes, cap: int = None, device: int = 0, ctx: "DContext" = None) -> bytes:
    """whole FCX7 file -> bytes with the GPU decoder (cap defaults to the header's total,
    which wraps mod 2^32: pass cap for larger files)"""
    own = ctx is None
    if own:
        ctx = DContext(device)
    try:
        return ctx.decompress_host(blob, cap)
    finally:
        if own:
            ctx.close()


def my_compress_file_lz77(block: bytes) -> bytes:
    """one block (<= 1 MiB) -> payload, same bytes as my_compress_file_lz77 (:2115)"""
    n = len(block)
    out = ctypes.create_string_buffer(2 * n + 4096)
    got = lib().fcx_compress_block(block, n, out)
    if got == 0:
        raise FcxError(f"fcx_compress_block failed: {lib().fcx_last_error().decode(errors='replace')}")
    return out.raw[:got]


def my_decompress_file_lz77(payload: bytes, cap: int = BLOCK_BYTES + 8) -> bytes:
    """payload -> block bytes (reference decoder semantics, :2255)"""
    out = ctypes.create_string_buffer(cap)
    got = lib().fcx_decompress_block(payload, len(payload), out, cap)
    if got < 0:
        raise FcxError(f"fcx_decompress_block failed ({got})")
    return out.raw[:got]


def compress(data: bytes, block_bytes: int = BLOCK_BYTES, device: int = 0, ctx: "Context" = None) -> bytes:
    """whole FCX7 file for `data` (header + [u32 len][payload] per block)"""
    nblocks = (len(data) + block_bytes - 1) // block_bytes
    if not data:
        return write_header(0, 0)
    own = ctx is None
    if own:
        ctx = Context(device, block_bytes, min(len(data), 256 << 20))
    try:
        body = ctx.compress_host(data)
    finally:
        if own:
            ctx.close()
    return write_header(len(data), nblocks) + body


def decompress(blob: bytes) -> bytes:
    if len(blob) < HEADER_BYTES or blob[:3] != b"FCX" or blob[3:4] != b"7":
        raise FcxError("not an FCX7 (LZ77) stream")
    total, nblocks = struct.unpack_from("<IH", blob, 4)
    off, out = HEADER_BYTES, []
    for _ in range(nblocks):
        (sz,) = struct.unpack_from("<I", blob, off)
        off += 4
        out.append(my_decompress_file_lz77(blob[off:off + sz]))
        off += sz
    return b"".join(out)


# ---- -c lz78 (FCX8): my_compress_file_lz78 (my_compress.cpp:3127-3476) on the GPU ----
def lz78_bound(n: int, block_bytes: int = BLOCK_BYTES) -> int:
    """output capacity for compress_lz78: records are <= ~9.1 B per input byte + ~600 B"""
    nb = (n + block_bytes - 1) // block_bytes
    return HEADER_BYTES + 10 * n + 4096 * max(nb, 1)


def my_compress_file_lz78(block: bytes) -> bytes:
    """one block (<= 1 MiB) -> payload, same bytes as my_compress_file_lz78 (:3127)"""
    n = len(block)
    if n == 0:
        return b""
    out = ctypes.create_string_buffer(10 * n + 4096)
    got = lib().fcx_lz78_compress_block(block, n, out)
    if got == 0:
        raise FcxError(f"fcx_lz78_compress_block failed: {lib().fcx_last_error().decode(errors='replace')}")
    return out.raw[:got]


def compress_lz78(data: bytes, block_bytes: int = BLOCK_BYTES) -> bytes:
    """whole FCX8 file for `data` (main() with -c lz78, :4073-4136)"""
    cap = lz78_bound(len(data), block_bytes)
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_uint64()
    try:
        _check(lib().fcx_lz78_compress_host(data, len(data), block_bytes, out, cap, ctypes.byref(n)),
               "fcx_lz78_compress_host")
    finally:
        lib().fcx_lz78_release()   # the codec caches ~40 B of device scratch per input byte
    return out.raw[:n.value]


def my_decompress_file_lz78(payload: bytes, cap: int = BLOCK_BYTES + 8) -> bytes:
    """one payload -> block bytes on the GPU (reference decoder semantics, :3478)"""
    out = ctypes.create_string_buffer(max(cap, 1))
    got = lib().fcx_lz78_decompress_block(payload, len(payload), out, cap)
    if got < 0:
        raise FcxError(f"fcx_lz78_decompress_block failed ({got}): {lib().fcx_last_error().decode(errors='replace')}")
    return out.raw[:got]


def decompress_lz78(blob: bytes, cap: int = None) -> bytes:
    """whole FCX8 file -> bytes on the GPU (main() decompress mode, :4137-4204)"""
    caps = [cap]
    if cap is None:   # the header's total (+ slack), then the per-block bound if the total wrapped
        total, nb = struct.unpack_from("<IH", blob, 4) if len(blob) >= HEADER_BYTES else (0, 0)
        caps = [total + 64 * nb + 64, nb * (BLOCK_BYTES + 8) + 1]
    for i, c in enumerate(caps):
        out = ctypes.create_string_buffer(max(c, 1))
        n = ctypes.c_uint64()
        rc = lib().fcx_lz78_decompress_host(blob, len(blob), out, c, ctypes.byref(n))
        if rc == -2 and i + 1 < len(caps):   # FCX_ERR_CAPACITY
            continue
        _check(rc, "fcx_lz78_decompress_host")
        return out.raw[:n.value]


def lz78_release() -> None:
    """frees the LZ78 compress scratch cached on the current HIP device"""
    _check(lib().fcx_lz78_release(), "fcx_lz78_release")


# ---- multi-GPU (fcx_dist_*: block ranges per GPU, RCCL concatenation) ----------------
DIST_GATHER, DIST_ALLGATHER = 0, 1


def dist_block_range(nblocks: int, rank: int, nranks: int, share0_ppm: int = 0):
    """the C partition (fcx_dist_block_range, or fcx_dist_block_range_w with a rank-0 share);
    equals my_compress_amd.dist.block_range"""
    b0, b1 = ctypes.c_uint64(), ctypes.c_uint64()
    if share0_ppm:
        lib().fcx_dist_block_range_w(nblocks, rank, nranks, share0_ppm, ctypes.byref(b0), ctypes.byref(b1))
    else:
        lib().fcx_dist_block_range(nblocks, rank, nranks, ctypes.byref(b0), ctypes.byref(b1))
    return b0.value, b1.value


def dist_gather_bound(n: int, block_bytes: int, nsub: int) -> int:
    """a peer's d_out capacity for Dist.compress_gather (pieces at their bound offsets)"""
    return int(lib().fcx_dist_gather_bound(n, block_bytes, nsub))


def dist_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    _check(lib().fcx_dist_unique_id(buf), "fcx_dist_unique_id")
    return buf.raw


class Loop:
    """fcx_loop: the in-process loopback transport's hub (include/fcx.h).  Thread ranks on one
    device run the multi-rank protocols over it: Dist.loop(hub, r) per thread rank."""

    def __init__(self, nranks: int, device: int = 0, timeout_ms: int = 60000):
        self._h = ctypes.c_void_p()
        _check(lib().fcx_loop_create(ctypes.byref(self._h), nranks, device, timeout_ms), "fcx_loop_create")
        self.nranks = nranks

    def close(self):
        if self._h:
            lib().fcx_loop_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Dist:
    """fcx_dist: communicator(s) of the multi-GPU compress path.
    Dist.local([0, 1, ...]) drives several devices from this process (the CLI's -g N);
    Dist.rank(n, r, uid, device) is one rank of a process-per-GPU job (RCCL);
    Dist.loop(hub, r) / Dist.loop_local(n, device) are the same forms over the loopback
    transport (thread ranks of one process on one device)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def local(cls, devices):
        h = ctypes.c_void_p()
        arr = (ctypes.c_int * len(devices))(*devices)
        _check(lib().fcx_dist_init_local(ctypes.byref(h), len(devices), arr), "fcx_dist_init_local")
        return cls(h)

    @classmethod
    def rank(cls, nranks: int, rank: int, uid: bytes, device: int = 0):
        h = ctypes.c_void_p()
        _check(lib().fcx_dist_init_rank(ctypes.byref(h), nranks, rank, uid, device), "fcx_dist_init_rank")
        return cls(h)

    @classmethod
    def loop(cls, hub: "Loop", rank: int):
        h = ctypes.c_void_p()
        _check(lib().fcx_dist_init_loop(ctypes.byref(h), hub._h, rank), "fcx_dist_init_loop")
        return cls(h)

    @classmethod
    def loop_local(cls, nranks: int, device: int = 0, timeout_ms: int = 60000):
        h = ctypes.c_void_p()
        _check(lib().fcx_dist_init_loop_local(ctypes.byref(h), nranks, device, timeout_ms), "fcx_dist_init_loop_local")
        return cls(h)

    def transport(self) -> str:
        return lib().fcx_dist_transport(self._h).decode()

    def debug_fail(self, piece: int):
        """testing: as a peer of compress_gather, treat sub-batch `piece` as failed (-1 = off)"""
        _check(lib().fcx_dist_debug_fail(self._h, piece), "fcx_dist_debug_fail")

    def gather_copy_ms(self) -> float:
        """rank 0 of the last compress_gather: device ms of its final moves of the peers' bytes
        behind its own segment (-1 on a peer)"""
        v = ctypes.c_float(-1.0)
        _check(lib().fcx_dist_gather_copy_ms(self._h, ctypes.byref(v)), "fcx_dist_gather_copy_ms")
        return float(v.value)

    def close(self):
        if self._h:
            lib().fcx_dist_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def size(self):
        n, loc = ctypes.c_int(), ctypes.c_int()
        _check(lib().fcx_dist_size(self._h, ctypes.byref(n), ctypes.byref(loc)), "fcx_dist_size")
        return n.value, loc.value

    def concat(self, d_seg: int, seg_len: int, d_out: int, cap: int, mode: int = DIST_GATHER, stream: int = 0) -> int:
        """this rank's device segment -> the concatenation in rank order at d_out; returns its length"""
        tot = ctypes.c_uint64()
        _check(lib().fcx_dist_concat(self._h, 0, ctypes.c_void_p(d_seg), seg_len, ctypes.c_void_p(d_out), cap,
                                     ctypes.byref(tot), mode, ctypes.c_void_p(stream)), "fcx_dist_concat")
        return tot.value

    def compress_gather(self, ctx: "Context", d_in: int, n: int, rank_bytes, nsub: int, d_out: int, cap: int,
                        stream: int = 0) -> int:
        """the strong-scaling step (fcx_dist_compress_gather): this rank compresses its n device
        bytes (peers: in nsub pieces, each sent to rank 0 when done) and rank 0 ends with every
        rank's records in block order at d_out; returns that length on rank 0, bytes sent elsewhere"""
        rb = (ctypes.c_uint64 * len(rank_bytes))(*rank_bytes)
        tot = ctypes.c_uint64()
        _check(lib().fcx_dist_compress_gather(self._h, ctx._h, ctypes.c_void_p(d_in), n, rb, nsub,
                                              ctypes.c_void_p(d_out), cap, ctypes.byref(tot),
                                              ctypes.c_void_p(stream)), "fcx_dist_compress_gather")
        return tot.value

    def compress_host(self, data: bytes, block_bytes: int = BLOCK_BYTES, round_bytes: int = 0) -> bytes:
        """records ([u32 len][payload]...) of data, block ranges over this process's devices"""
        cap = shard_bound(len(data), block_bytes)
        out = ctypes.create_string_buffer(max(cap, 1))
        got = ctypes.c_uint64()
        _check(lib().fcx_dist_compress_host(self._h, data, len(data), block_bytes, round_bytes, out, cap,
                                            ctypes.byref(got)), "fcx_dist_compress_host")
        return out.raw[:got.value]

