// fcx_stream.hip — pipelined host I/O around the device paths.
//
// The reference's main() (my_compress.cpp:4073-4136 compress, 4137-4204
// decompress) reads a block, codes it and writes it, strictly in turn.  Here a
// file streams through two pipeline slots, each a pinned host buffer and its
// device twin: while the GPU compresses shard k, the host reads shard k+1 into
// the other slot's pinned buffer and writes shard k-1's records, and the copies
// run on their own streams (H2D, D2H) so PCIe overlaps compute as well.  Files
// larger than host memory or HBM stream through in shard-sized pieces.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "fcx.h"

namespace fcx {
void set_last_error(const std::string &m);
}

namespace {

int sfail(int code, const std::string &m) {
    fcx::set_last_error(m);
    return code;
}

#define SHIP(expr)                                                                                    \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess) return sfail(FCX_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct Slot {
    uint8_t *hin = nullptr, *hout = nullptr, *din = nullptr, *dout = nullptr;
    uint64_t *hlen = nullptr;   // pinned copy of the device length / error words
    uint64_t n = 0;             // input bytes in this slot
    hipEvent_t h2d = nullptr, comp = nullptr, d2h = nullptr;
};

struct Pipeline {
    Slot s[2];
    hipStream_t sin = nullptr, scomp = nullptr, sout = nullptr;
    int device = -1;
    uint64_t in_bytes = 0, out_bytes = 0;
    ~Pipeline() {
        for (auto &x : s) {
            if (x.hin) (void)hipHostFree(x.hin);
            if (x.hout) (void)hipHostFree(x.hout);
            if (x.hlen) (void)hipHostFree(x.hlen);
            if (x.din) (void)hipFree(x.din);
            if (x.dout) (void)hipFree(x.dout);
            for (hipEvent_t e : {x.h2d, x.comp, x.d2h})
                if (e) (void)hipEventDestroy(e);
        }
        for (hipStream_t q : {sin, scomp, sout})
            if (q) (void)hipStreamDestroy(q);
    }
    int init(int dev, uint64_t in_b, uint64_t out_b) {
        device = dev;
        in_bytes = in_b;
        out_bytes = out_b;
        SHIP(hipStreamCreateWithFlags(&sin, hipStreamNonBlocking));
        SHIP(hipStreamCreateWithFlags(&scomp, hipStreamNonBlocking));
        SHIP(hipStreamCreateWithFlags(&sout, hipStreamNonBlocking));
        for (auto &x : s) {
            SHIP(hipHostMalloc((void **)&x.hin, in_bytes ? in_bytes : 16, hipHostMallocDefault));
            SHIP(hipHostMalloc((void **)&x.hout, out_bytes ? out_bytes : 16, hipHostMallocDefault));
            SHIP(hipHostMalloc((void **)&x.hlen, 16, hipHostMallocDefault));
            SHIP(hipMalloc((void **)&x.din, in_bytes ? in_bytes : 16));
            SHIP(hipMalloc((void **)&x.dout, out_bytes ? out_bytes : 16));
            SHIP(hipEventCreateWithFlags(&x.h2d, hipEventDisableTiming));
            SHIP(hipEventCreateWithFlags(&x.comp, hipEventDisableTiming));
            SHIP(hipEventCreateWithFlags(&x.d2h, hipEventDisableTiming));
            SHIP(hipEventRecord(x.comp, scomp));   // slots start free
            SHIP(hipEventRecord(x.d2h, sout));
            SHIP(hipEventRecord(x.h2d, sin));
        }
        return FCX_OK;
    }
};

// pinned/device slots are kept per host thread (one set for each direction) and
// reused while they are large enough: per-block calls do not re-pin memory
thread_local Pipeline *g_pipe[2] = {nullptr, nullptr};
struct PipeFree {
    ~PipeFree() { for (auto &p : g_pipe) { delete p; p = nullptr; } }
};
thread_local PipeFree g_pipe_free;

int get_pipe(int which, int dev, uint64_t in_b, uint64_t out_b, Pipeline **out) {
    (void)&g_pipe_free;
    Pipeline *&p = g_pipe[which];
    if (p && (p->device != dev || p->in_bytes < in_b || p->out_bytes < out_b)) {
        (void)hipDeviceSynchronize();
        delete p;
        p = nullptr;
    }
    if (!p) {
        p = new Pipeline();
        const int r = p->init(dev, in_b, out_b);
        if (r) { delete p; p = nullptr; return r; }
    }
    for (auto &x : p->s) x.n = 0;
    *out = p;
    return FCX_OK;
}

// fills buf with up to cap bytes (short only at end of input); <0 on error
int64_t read_full(fcx_read_fn rd, void *user, uint8_t *buf, uint64_t cap) {
    uint64_t got = 0;
    while (got < cap) {
        const int64_t r = rd(user, buf + got, cap - got);
        if (r < 0) return r;
        if (r == 0) break;
        got += (uint64_t)r;
    }
    return (int64_t)got;
}

// host-to-host copies of the memory paths (a shard into / out of the pinned staging): one thread moves
// ~10 GB/s, so a 256 MiB shard's copy in and out took longer than its H2D, compress and D2H together;
// large copies are split over up to kCopyThreads threads (64-B aligned pieces of >= 8 MiB)
constexpr uint64_t kCopyPiece = 8ull << 20;
constexpr unsigned kCopyThreads = 8;
void par_memcpy(uint8_t *dst, const uint8_t *src, uint64_t n) {
    const uint64_t t = n / kCopyPiece < kCopyThreads ? n / kCopyPiece : kCopyThreads;
    if (t <= 1) { memcpy(dst, src, n); return; }
    const uint64_t per = (n / t + 63) & ~63ull;
    std::vector<std::thread> th;
    th.reserve(t - 1);
    for (uint64_t i = 1; i < t; i++) {
        const uint64_t a = i * per, b = i + 1 == t ? n : (i + 1) * per;
        if (a < b) th.emplace_back([=] { memcpy(dst + a, src + a, b - a); });
    }
    memcpy(dst, src, per < n ? per : n);
    for (auto &x : th) x.join();
}

struct MemIO {   // fcx_compress_host / fcx_decompress_* over memory
    const uint8_t *in;
    uint64_t in_len, in_pos;
    uint8_t *out;
    uint64_t cap, out_pos;
};
int64_t mem_read(void *u, uint8_t *buf, uint64_t cap) {
    MemIO *m = (MemIO *)u;
    const uint64_t n = m->in_len - m->in_pos < cap ? m->in_len - m->in_pos : cap;
    par_memcpy(buf, m->in + m->in_pos, n);
    m->in_pos += n;
    return (int64_t)n;
}
int mem_write(void *u, const uint8_t *buf, uint64_t n) {
    MemIO *m = (MemIO *)u;
    if (n > m->cap - m->out_pos) return FCX_ERR_CAPACITY;
    par_memcpy(m->out + m->out_pos, buf, n);
    m->out_pos += n;
    return 0;
}

}  // namespace

extern "C" {

int fcx_compress_stream(fcx_ctx *ctx, fcx_read_fn rd, fcx_write_fn wr, void *user, uint64_t shard_bytes,
                        uint64_t *total_in, uint64_t *total_out, uint64_t *nblocks) {
    if (!ctx || !rd || !wr) return sfail(FCX_ERR_ARG, "fcx_compress_stream: NULL argument");
    uint32_t B = 0;
    int dev = 0;
    if (fcx_ctx_info(ctx, &dev, &B, nullptr)) return FCX_ERR_ARG;
    SHIP(hipSetDevice(dev));
    const uint64_t shard = shard_bytes >= B ? shard_bytes / B * B : B;
    const uint64_t cap = fcx_shard_bound(shard, B);
    Pipeline *PP = nullptr;
    int r = get_pipe(0, dev, shard, cap, &PP);
    if (r) return r;
    Pipeline &P = *PP;
    const uint64_t *dlen = fcx_ctx_device_out_len(ctx);
    uint64_t tin = 0, tout = 0, tblocks = 0;
    // finish shard in slot x in two halves: length back and the records' D2H issued (start), then,
    // after the host has read the next shard into the slot's input buffer meanwhile, the D2H
    // waited for and the records written (finish)
    uint64_t olen_pending = 0;
    auto drain_start = [&](Slot &x) -> int {
        SHIP(hipEventSynchronize(x.comp));
        const uint32_t e = (uint32_t)x.hlen[1];
        if (e & 4u) return sfail(FCX_ERR_CAPACITY, "shard output capacity");
        if (e) return sfail(FCX_ERR_INTERNAL, "device invariant violated (error bits " + std::to_string(e) + ")");
        olen_pending = x.hlen[0];
        SHIP(hipMemcpyAsync(x.hout, x.dout, olen_pending, hipMemcpyDeviceToHost, P.sout));
        SHIP(hipEventRecord(x.d2h, P.sout));
        return FCX_OK;
    };
    auto drain_finish = [&](Slot &x) -> int {
        SHIP(hipEventSynchronize(x.d2h));
        const int w = wr(user, x.hout, olen_pending);
        if (w) return sfail(w < 0 ? w : FCX_ERR_ARG, "write callback failed");
        tout += olen_pending;
        x.n = 0;
        return FCX_OK;
    };
    auto drain = [&](Slot &x) -> int {
        const int rr = drain_start(x);
        return rr ? rr : drain_finish(x);
    };
    int64_t got = read_full(rd, user, P.s[0].hin, shard);
    if (got < 0) return sfail(FCX_ERR_ARG, "read callback failed");
    for (uint32_t k = 0; got > 0; k++) {
        Slot &x = P.s[k & 1], &y = P.s[(k + 1) & 1];
        x.n = (uint64_t)got;
        tin += x.n;
        tblocks += (x.n + B - 1) / B;
        SHIP(hipStreamWaitEvent(P.sin, x.comp, 0));     // x.din free again (shard k-2 compressed)
        SHIP(hipMemcpyAsync(x.din, x.hin, x.n, hipMemcpyHostToDevice, P.sin));
        SHIP(hipEventRecord(x.h2d, P.sin));
        SHIP(hipStreamWaitEvent(P.scomp, x.h2d, 0));
        SHIP(hipStreamWaitEvent(P.scomp, x.d2h, 0));   // x.dout free again
        if ((r = fcx_compress_shard(ctx, x.din, x.n, x.dout, cap, nullptr, P.scomp))) return r;
        SHIP(hipMemcpyAsync(x.hlen, dlen, 16, hipMemcpyDeviceToHost, P.scomp));
        SHIP(hipEventRecord(x.comp, P.scomp));
        // while the GPU works on slot x: read the next shard into y (its H2D is long done)
        // and write y's finished records
        const bool last = x.n < shard;
        got = 0;
        const bool ydrain = y.n != 0;
        if (ydrain) { if ((r = drain_start(y))) return r; }
        if (!last) {   // (y.hin: its H2D is long done; y's records go out through y.hout meanwhile)
            SHIP(hipEventSynchronize(y.h2d));
            got = read_full(rd, user, y.hin, shard);
            if (got < 0) return sfail(FCX_ERR_ARG, "read callback failed");
        }
        if (ydrain) { if ((r = drain_finish(y))) return r; }
    }
    for (auto &x : P.s)
        if (x.n) { if ((r = drain(x))) return r; }
    if (total_in) *total_in = tin;
    if (total_out) *total_out = tout;
    if (nblocks) *nblocks = tblocks;
    return FCX_OK;
}

int fcx_compress_host(fcx_ctx *ctx, const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    if (!ctx || (!in && n) || !out) return sfail(FCX_ERR_ARG, "fcx_compress_host: NULL argument");
    uint64_t shard = 0;
    if (fcx_ctx_info(ctx, nullptr, nullptr, &shard)) return FCX_ERR_ARG;
    MemIO m{in, n, 0, out, cap, 0};
    const int r = fcx_compress_stream(ctx, mem_read, mem_write, &m, shard, nullptr, nullptr, nullptr);
    if (r) return r;
    if (out_len) *out_len = m.out_pos;
    return FCX_OK;
}

int fcx_decompress_stream(fcx_dctx *dctx, fcx_read_fn rd, fcx_write_fn wr, void *user, uint64_t max_in,
                          uint32_t *hdr_total, uint64_t *total_out, uint64_t *nblocks) {
    if (!dctx || !rd || !wr) return sfail(FCX_ERR_ARG, "fcx_decompress_stream: NULL argument");
    uint8_t hdr[FCX_HEADER_BYTES];
    if (read_full(rd, user, hdr, sizeof(hdr)) != (int64_t)sizeof(hdr)) return sfail(FCX_ERR_FORMAT, "short header");
    uint32_t total = 0;
    char kind = 0;
    int r = fcx_parse_header(hdr, &total, nullptr, &kind);
    if (r) return r;
    if (kind != '7') return sfail(FCX_ERR_FORMAT, "LZ78 streams are outside this build's scope");
    int dev = 0;
    if (fcx_dctx_device(dctx, &dev)) return FCX_ERR_ARG;
    SHIP(hipSetDevice(dev));
    // groups of whole records: up to kGroup blocks (<= 1 MiB decoded each) per device call
    // (max_in, when known, bounds the staging: small inputs do not pin a whole group)
    constexpr uint32_t kGroup = 256;
    const uint64_t rec_max = 2ull * FCX_MAX_BLOCK_BYTES + 4096 + 4;
    uint64_t in_cap = (uint64_t)kGroup * rec_max;
    uint64_t out_cap = (uint64_t)kGroup * FCX_MAX_BLOCK_BYTES;
    if (max_in && max_in < in_cap) {
        in_cap = max_in;
        // each record of >= 4 + 3 bytes decodes to <= 1 MiB
        out_cap = (uint64_t)FCX_MAX_BLOCK_BYTES * ((max_in + 6) / 7 < kGroup ? (max_in + 6) / 7 : kGroup);
    }
    Pipeline *PP = nullptr;
    if ((r = get_pipe(1, dev, in_cap, out_cap, &PP))) return r;
    Pipeline &P = *PP;
    Slot &x = P.s[0];
    uint64_t tout = 0, tblocks = 0;
    bool eof = false;
    while (!eof) {
        uint64_t used = 0;
        uint32_t nb = 0;
        while (nb < kGroup) {
            uint32_t len;
            const int64_t g = read_full(rd, user, (uint8_t *)&len, 4);
            if (g == 0) { eof = true; break; }
            if (g != 4) return sfail(FCX_ERR_FORMAT, "truncated block record");
            if (len > 2 * FCX_MAX_BLOCK_BYTES + 4096) return sfail(FCX_ERR_FORMAT, "block record too long");
            if (used + 4 + (uint64_t)len > in_cap) return sfail(FCX_ERR_FORMAT, "truncated block record");
            memcpy(x.hin + used, &len, 4);
            if (read_full(rd, user, x.hin + used + 4, len) != (int64_t)len)
                return sfail(FCX_ERR_FORMAT, "truncated block record");
            used += 4 + (uint64_t)len;
            nb++;
        }
        if (nb == 0) break;
        SHIP(hipMemcpyAsync(x.din, x.hin, used, hipMemcpyHostToDevice, P.scomp));
        uint64_t got = 0;
        if ((r = fcx_decompress_shard(dctx, x.din, used, nb, x.dout, out_cap, &got, P.scomp))) return r;
        SHIP(hipMemcpyAsync(x.hout, x.dout, got, hipMemcpyDeviceToHost, P.scomp));
        SHIP(hipStreamSynchronize(P.scomp));
        const int w = wr(user, x.hout, got);
        if (w) return sfail(w < 0 ? w : FCX_ERR_ARG, "write callback failed");
        tout += got;
        tblocks += nb;
    }
    if (hdr_total) *hdr_total = total;
    if (total_out) *total_out = tout;
    if (nblocks) *nblocks = tblocks;
    return FCX_OK;
}

int fcx_decompress_host(fcx_dctx *dctx, const uint8_t *in, uint64_t in_len, uint8_t *out, uint64_t cap,
                        uint64_t *out_len) {
    if (!dctx || !in || (cap && !out)) return sfail(FCX_ERR_ARG, "fcx_decompress_host: NULL argument");
    if (in_len < FCX_HEADER_BYTES || memcmp(in, "FCX7", 4) != 0) return sfail(FCX_ERR_FORMAT, "not an FCX7 stream");
    MemIO m{in, in_len, 0, out, cap, 0};
    const int r = fcx_decompress_stream(dctx, mem_read, mem_write, &m, in_len - FCX_HEADER_BYTES, nullptr, nullptr,
                                        nullptr);
    if (r) return r;
    if (out_len) *out_len = m.out_pos;
    return FCX_OK;
}

}  // extern "C"
