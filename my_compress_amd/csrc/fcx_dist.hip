// fcx_dist.hip — multi-GPU compress: contiguous block ranges per GPU, segments
// concatenated in block order over RCCL (xGMI).  See include/fcx.h (fcx_dist_*).
//
// The reference compresses its 1 MiB blocks one after the other and writes each
// [u32 len][payload] record to one file in order (my_compress.cpp:4090-4122,
// 4112-4114).  Blocks are independent (:1675-1703), so N ranks take contiguous block
// ranges; the only exchange is the concatenation: an all-gather of the u64 segment
// sizes, then the segments land at their offsets of one contiguous buffer — a gather
// to rank 0 (grouped ncclSend/ncclRecv: every peer's link carries its own segment at
// once, 1/N of an all-gather's traffic) or an all-gather-v (one ncclBroadcast per
// source rank with its exact size; no padding, no second copy).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "fcx.h"

namespace fcx {
void set_last_error(const std::string &m);
}

namespace {

int dfail(int code, const std::string &msg) {
    fcx::set_last_error(msg);
    return code;
}

#define DHIP(expr)                                                                              \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess) return dfail(FCX_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define DNCCL(expr)                                                                             \
    do {                                                                                        \
        ncclResult_t r_ = (expr);                                                               \
        if (r_ != ncclSuccess) return dfail(FCX_ERR_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

}  // namespace

struct fcx_dist {
    int nranks = 0;                  // ranks of the job
    int base_rank = 0;               // rank of local index 0
    std::vector<int> devices;        // per local rank
    std::vector<ncclComm_t> comms;   // per local rank
    std::vector<uint64_t *> d_sizes; // per local rank: 2 x nranks u64 (size + capacity all-gather)
    // fcx_dist_compress_host's per-device resources, kept across calls
    uint32_t block = 0;
    std::vector<fcx_ctx *> ctx;
    std::vector<uint8_t *> din, dout;
    std::vector<hipStream_t> st;
    std::vector<uint64_t> dincap, dcap;
    // fcx_dist_compress_gather's resources (process-per-GPU form), made on first use and kept
    hipStream_t cst = nullptr;       // the exchange's stream (beside the caller's compress stream)
    uint64_t *d_words = nullptr;     // 2 u64 per (sub-batch, rank): piece length, error bits
    uint64_t *h_words = nullptr;     // pinned mirror
    std::vector<hipEvent_t> ev;      // per sub-batch: compressed and its length copied
    uint8_t *d_stage = nullptr;      // rank 0: the peers' pieces as they arrive
    uint64_t stage_cap = 0;
};

namespace {

constexpr uint64_t kFailed = ~0ull;   // size-exchange word of a rank whose compress failed

// sizes all-gather + segment placement for local rank li (one host thread per local rank).
// Every rank always enters both phases, whatever happened before: `status` != FCX_OK (this
// rank's compress failed) travels as a sentinel size, and each rank also publishes the
// capacity it receives into, so the exchange hands every rank the same facts and every
// rank reaches the same verdict (skip the data phase and fail, or run it) -- no rank is
// left waiting in a send or receive that its peer never posts.
int concat_local(fcx_dist *d, int li, const uint8_t *d_seg, uint64_t seg_len, uint8_t *d_out, uint64_t cap,
                 uint64_t *total, int mode, hipStream_t st, int status = FCX_OK) {
    const int n = d->nranks, rank = d->base_rank + li;
    ncclComm_t comm = d->comms[li];
    DHIP(hipSetDevice(d->devices[li]));
    uint64_t *ds = d->d_sizes[li];
    const bool receives = mode == FCX_DIST_ALLGATHER || rank == 0;
    const uint64_t mine[2] = {status ? kFailed : seg_len, receives ? cap : kFailed};
    DHIP(hipMemcpyAsync(ds + 2 * rank, mine, sizeof(mine), hipMemcpyHostToDevice, st));
    DNCCL(ncclAllGather(ds + 2 * rank, ds, 2, ncclUint64, comm, st));
    std::vector<uint64_t> words(2 * (size_t)n), sizes(n), offs(n, 0);
    DHIP(hipMemcpyAsync(words.data(), ds, words.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    DHIP(hipStreamSynchronize(st));
    if (status) return status;   // (this rank's own message is already set)
    for (int r = 0; r < n; r++) {
        if (words[2 * r] == kFailed)
            return dfail(FCX_ERR_RCCL, "fcx_dist_concat: rank " + std::to_string(r) + " failed; no segment exchanged");
        sizes[r] = words[2 * r];
    }
    for (int r = 1; r < n; r++) offs[r] = offs[r - 1] + sizes[r - 1];
    const uint64_t tot = offs[n - 1] + sizes[n - 1];
    *total = tot;
    for (int r = 0; r < n; r++)   // every receiving rank's capacity, judged identically everywhere
        if (words[2 * r + 1] != kFailed && tot > words[2 * r + 1])
            return dfail(FCX_ERR_CAPACITY, "fcx_dist_concat: output capacity of rank " + std::to_string(r) +
                                               " too small (" + std::to_string(tot) + " B)");
    // own segment to its offset (skipped when it already lives there); the exchanged size
    // is what every peer expects, so it is the one sent and received
    const uint64_t own = sizes[rank];
    if (receives && own && d_seg != d_out + offs[rank])
        DHIP(hipMemcpyAsync(d_out + offs[rank], d_seg, own, hipMemcpyDeviceToDevice, st));
    DNCCL(ncclGroupStart());
    if (mode == FCX_DIST_GATHER) {
        if (rank == 0) {
            for (int r = 1; r < n; r++)
                if (sizes[r]) DNCCL(ncclRecv(d_out + offs[r], sizes[r], ncclUint8, r, comm, st));
        } else if (own) {
            DNCCL(ncclSend(d_seg, own, ncclUint8, 0, comm, st));
        }
    } else {
        for (int r = 0; r < n; r++)
            if (sizes[r]) DNCCL(ncclBroadcast(d_out + offs[r], d_out + offs[r], sizes[r], ncclUint8, r, comm, st));
    }
    DNCCL(ncclGroupEnd());
    DHIP(hipStreamSynchronize(st));
    if (own != seg_len) return dfail(FCX_ERR_INTERNAL, "fcx_dist_concat: size exchange mismatch");
    return FCX_OK;
}

// fcx_dist_compress_gather's stream, length words and events (sized for FCX_DIST_MAX_SUB
// sub-batches of every rank), and rank 0's staging buffer of at least `stage` bytes
int ensure_gather(fcx_dist *d, uint64_t stage) {
    DHIP(hipSetDevice(d->devices[0]));
    const size_t words = 2ull * FCX_DIST_MAX_SUB * (size_t)d->nranks;
    if (!d->cst) {
        DHIP(hipStreamCreateWithFlags(&d->cst, hipStreamNonBlocking));
        DHIP(hipMalloc((void **)&d->d_words, words * sizeof(uint64_t)));
        DHIP(hipHostMalloc((void **)&d->h_words, words * sizeof(uint64_t), hipHostMallocDefault));
        d->ev.assign(FCX_DIST_MAX_SUB, nullptr);
        for (auto &e : d->ev) DHIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    if (stage > d->stage_cap) {
        if (d->d_stage) DHIP(hipFree(d->d_stage));
        d->d_stage = nullptr;
        d->stage_cap = 0;
        if (hipMalloc((void **)&d->d_stage, stage) != hipSuccess)
            return dfail(FCX_ERR_NOMEM, "fcx_dist_compress_gather: staging buffer of " + std::to_string(stage) + " B");
        d->stage_cap = stage;
    }
    return FCX_OK;
}

void release_gather(fcx_dist *d) {
    if (d->devices.empty()) return;
    (void)hipSetDevice(d->devices[0]);
    if (d->cst) (void)hipStreamSynchronize(d->cst);
    for (auto e : d->ev)
        if (e) (void)hipEventDestroy(e);
    d->ev.clear();
    if (d->cst) (void)hipStreamDestroy(d->cst);
    if (d->d_words) (void)hipFree(d->d_words);
    if (d->h_words) (void)hipHostFree(d->h_words);
    if (d->d_stage) (void)hipFree(d->d_stage);
    d->cst = nullptr; d->d_words = nullptr; d->h_words = nullptr; d->d_stage = nullptr; d->stage_cap = 0;
}

inline uint64_t round16(uint64_t x) { return (x + 15) & ~15ull; }

// sub-batch s of nsub of a rank's n bytes: whole blocks, the near-even split of block_range
void piece_range(uint64_t n, uint32_t block, uint32_t s, uint32_t nsub, uint64_t *lo, uint64_t *hi) {
    const uint64_t nb = (n + block - 1) / block;
    uint64_t b0, b1;
    fcx_dist_block_range(nb, (int)s, (int)nsub, &b0, &b1);
    *lo = b0 * block < n ? b0 * block : n;
    *hi = b1 * block < n ? b1 * block : n;
}

// bytes a rank's pieces take at their bound offsets (a peer's d_out; rank 0's staging region)
uint64_t pieces_bound(uint64_t n, uint32_t block, uint32_t nsub) {
    uint64_t t = 0;
    for (uint32_t s = 0; s < nsub; s++) {
        uint64_t lo, hi;
        piece_range(n, block, s, nsub, &lo, &hi);
        t += round16(fcx_shard_bound(hi - lo, block));
    }
    return t;
}

void release_local(fcx_dist *d) {
    for (size_t i = 0; i < d->ctx.size(); i++) {
        (void)hipSetDevice(d->devices[i]);
        if (d->st[i]) (void)hipStreamDestroy(d->st[i]);
        if (d->din[i]) (void)hipFree(d->din[i]);
        if (d->dout[i]) (void)hipFree(d->dout[i]);
        fcx_ctx_destroy(d->ctx[i]);
    }
    d->ctx.clear(); d->din.clear(); d->dout.clear(); d->st.clear(); d->dincap.clear(); d->dcap.clear();
    d->block = 0;
}

// (re)allocates fcx_dist_compress_host's resources when the block size changes or a call
// needs more than the cached ones hold: `per` input bytes per device, and output for the
// whole round (`round` input bytes) on device 0, one device's range elsewhere
int ensure_local(fcx_dist *d, uint32_t block, uint64_t per, uint64_t round) {
    const size_t nd = d->devices.size();
    bool ok = d->block == block && d->ctx.size() == nd;
    for (size_t i = 0; ok && i < nd; i++)
        ok = d->dincap[i] >= per && d->dcap[i] >= fcx_shard_bound(i == 0 ? round : per, block);
    if (ok) return FCX_OK;
    release_local(d);
    d->ctx.assign(nd, nullptr); d->din.assign(nd, nullptr); d->dout.assign(nd, nullptr);
    d->st.assign(nd, nullptr); d->dincap.assign(nd, 0); d->dcap.assign(nd, 0);
    d->block = block;
    for (size_t i = 0; i < nd; i++) {   // one device at a time
        int r = FCX_OK;
        if (hipSetDevice(d->devices[i]) != hipSuccess || hipStreamCreate(&d->st[i]) != hipSuccess)
            r = dfail(FCX_ERR_HIP, "fcx_dist_compress_host: stream");
        if (!r) r = fcx_ctx_create(&d->ctx[i], d->devices[i], block, per);
        d->dincap[i] = per;
        d->dcap[i] = fcx_shard_bound(i == 0 ? round : per, block);
        if (!r && (hipMalloc((void **)&d->din[i], per) != hipSuccess ||
                   hipMalloc((void **)&d->dout[i], d->dcap[i]) != hipSuccess))
            r = dfail(FCX_ERR_NOMEM, "fcx_dist_compress_host: device buffers");
        if (r) { release_local(d); return r; }
    }
    return FCX_OK;
}

int make_dist(fcx_dist **out, fcx_dist *d) {
    d->d_sizes.resize(d->devices.size(), nullptr);
    for (size_t i = 0; i < d->devices.size(); i++) {
        DHIP(hipSetDevice(d->devices[i]));
        DHIP(hipMalloc((void **)&d->d_sizes[i], 2 * sizeof(uint64_t) * (size_t)d->nranks));
    }
    *out = d;
    return FCX_OK;
}

}  // namespace

extern "C" {

void fcx_dist_block_range(uint64_t nblocks, int rank, int nranks, uint64_t *b0, uint64_t *b1) {
    // same arithmetic as my_compress_amd.dist.block_range: sizes differ by at most one
    if (nranks <= 0) nranks = 1;
    if (b0) *b0 = nblocks * (uint64_t)rank / (uint64_t)nranks;
    if (b1) *b1 = nblocks * (uint64_t)(rank + 1) / (uint64_t)nranks;
}

void fcx_dist_block_range_w(uint64_t nblocks, int rank, int nranks, uint32_t share0_ppm, uint64_t *b0,
                            uint64_t *b1) {
    // same arithmetic as my_compress_amd.dist.block_range(..., share0_ppm): rank 0 (the gather's
    // receiver) takes floor(nblocks * ppm / 10^6) blocks, ranks 1..N-1 split the rest near-evenly
    if (nranks <= 1 || share0_ppm == 0) { fcx_dist_block_range(nblocks, rank, nranks, b0, b1); return; }
    const uint64_t ppm = share0_ppm > 1000000u ? 1000000u : share0_ppm;
    const uint64_t n0 = (uint64_t)((unsigned __int128)nblocks * ppm / 1000000u);
    uint64_t lo = 0, hi = n0;
    if (rank > 0) {
        uint64_t p0, p1;
        fcx_dist_block_range(nblocks - n0, rank - 1, nranks - 1, &p0, &p1);
        lo = n0 + p0;
        hi = n0 + p1;
    }
    if (b0) *b0 = lo;
    if (b1) *b1 = hi;
}

uint64_t fcx_dist_gather_bound(uint64_t n, uint32_t block_bytes, uint32_t nsub) {
    if (block_bytes == 0) return 0;
    if (nsub < 1) nsub = 1;
    const uint64_t p = pieces_bound(n, block_bytes, nsub > FCX_DIST_MAX_SUB ? FCX_DIST_MAX_SUB : nsub);
    const uint64_t w = fcx_shard_bound(n, block_bytes);
    return p > w ? p : w;
}

int fcx_dist_compress_gather(fcx_dist *d, fcx_ctx *c, const uint8_t *d_in, uint64_t n, const uint64_t *rank_bytes,
                             uint32_t nsub, uint8_t *d_out, uint64_t cap, uint64_t *total, void *stream) {
    if (!d || !c || !rank_bytes || !total || !d_out || (n && !d_in) || nsub < 1 || nsub > FCX_DIST_MAX_SUB)
        return dfail(FCX_ERR_ARG, "fcx_dist_compress_gather: bad argument");
    if (d->comms.size() != 1)
        return dfail(FCX_ERR_ARG, "fcx_dist_compress_gather: one rank per process (fcx_dist_init_rank)");
    const int N = d->nranks, rank = d->base_rank;
    if (rank_bytes[rank] != n) return dfail(FCX_ERR_ARG, "fcx_dist_compress_gather: rank_bytes[rank] != n");
    int dev = 0;
    uint32_t B = 0;
    int rc = fcx_ctx_info(c, &dev, &B, nullptr);
    if (rc) return rc;
    if (dev != d->devices[0]) return dfail(FCX_ERR_ARG, "fcx_dist_compress_gather: context on another device");
    hipStream_t st = (hipStream_t)stream;
    ncclComm_t comm = d->comms[0];
    *total = 0;
    uint64_t stage = 0;
    std::vector<uint64_t> soff(N, 0);   // rank 0: each peer's staging region
    if (rank == 0)
        for (int r = 1; r < N; r++) {
            soff[r] = stage;
            stage += pieces_bound(rank_bytes[r], B, nsub);
        }
    if ((rc = ensure_gather(d, stage))) return rc;
    uint64_t *dw = d->d_words, *hw = d->h_words;
    if (rank == 0) {
        // own range straight into d_out at offset 0 (a failure is reported after the peers' pieces
        // are drained, so no peer is left in a send), the peers' pieces into the staging regions
        // on the exchange stream meanwhile: per round s, every peer's length words, then its bytes
        int own_rc = fcx_compress_shard(c, d_in, n, d_out, cap, nullptr, st);
        std::vector<uint64_t> fill(N, 0);
        std::string peer_err;
        for (uint32_t s = 0; s < nsub && N > 1; s++) {
            uint64_t *ws = dw + 2ull * s * N, *hs = hw + 2ull * s * N;
            DNCCL(ncclGroupStart());
            for (int r = 1; r < N; r++) DNCCL(ncclRecv(ws + 2 * r, 2, ncclUint64, r, comm, d->cst));
            DNCCL(ncclGroupEnd());
            DHIP(hipMemcpyAsync(hs, ws, 2ull * N * sizeof(uint64_t), hipMemcpyDeviceToHost, d->cst));
            DHIP(hipStreamSynchronize(d->cst));
            DNCCL(ncclGroupStart());
            for (int r = 1; r < N; r++) {
                const uint64_t len = hs[2 * r], err = hs[2 * r + 1];
                if (err || len == kFailed) {
                    if (peer_err.empty()) peer_err = "rank " + std::to_string(r) + " failed in sub-batch " + std::to_string(s);
                    continue;
                }
                if (len == 0) continue;
                if (fill[r] + len > pieces_bound(rank_bytes[r], B, nsub))   // (bounded by construction)
                    return dfail(FCX_ERR_INTERNAL, "fcx_dist_compress_gather: piece beyond its bound");
                DNCCL(ncclRecv(d->d_stage + soff[r] + fill[r], len, ncclUint8, r, comm, d->cst));
                fill[r] += len;
            }
            DNCCL(ncclGroupEnd());
        }
        DHIP(hipStreamSynchronize(d->cst));
        uint64_t own = 0;
        if (!own_rc) own_rc = fcx_ctx_read_out_len(c, &own);
        if (own_rc) return own_rc;
        if (!peer_err.empty()) return dfail(FCX_ERR_RCCL, "fcx_dist_compress_gather: " + peer_err);
        uint64_t off = own;
        for (int r = 1; r < N; r++) off += fill[r];
        if (off > cap) return dfail(FCX_ERR_CAPACITY, "fcx_dist_compress_gather: output capacity too small (" +
                                                          std::to_string(off) + " B)");
        off = own;
        for (int r = 1; r < N; r++) {   // the peers' bytes behind the own segment, in rank order
            if (fill[r]) DHIP(hipMemcpyAsync(d_out + off, d->d_stage + soff[r], fill[r], hipMemcpyDeviceToDevice, st));
            off += fill[r];
        }
        DHIP(hipStreamSynchronize(st));
        *total = off;
        return FCX_OK;
    }
    // a peer: every piece's compress is enqueued at once at its bound offset of d_out; each piece's
    // length words follow it on the compress stream, and the exchange stream sends them and then
    // the piece's bytes as soon as the piece is done, while the next piece compresses
    std::vector<uint64_t> ro(nsub, 0), lens(nsub, 0);
    int status = FCX_OK;
    std::string msg;
    uint64_t o = 0;
    for (uint32_t s = 0; s < nsub; s++) {
        uint64_t lo, hi;
        piece_range(n, B, s, nsub, &lo, &hi);
        ro[s] = o;
        const uint64_t pb = round16(fcx_shard_bound(hi - lo, B));
        if (status == FCX_OK && o + pb > cap) {
            status = dfail(FCX_ERR_CAPACITY, "fcx_dist_compress_gather: peer output capacity too small (see fcx_dist_gather_bound)");
            msg = fcx_last_error();
        }
        if (status == FCX_OK) {
            status = fcx_compress_shard(c, d_in + lo, hi - lo, d_out + o, pb, nullptr, st);
            if (status) msg = fcx_last_error();
        }
        if (status == FCX_OK) {
            DHIP(hipMemcpyAsync(dw + 2 * s, fcx_ctx_device_out_len(c), 2 * sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
            DHIP(hipMemcpyAsync(hw + 2 * s, dw + 2 * s, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
            DHIP(hipEventRecord(d->ev[s], st));
        }
        o += pb;
    }
    uint64_t sent = 0;
    for (uint32_t s = 0; s < nsub; s++) {
        bool ok = status == FCX_OK && hipEventSynchronize(d->ev[s]) == hipSuccess;
        if (ok && hw[2 * s + 1]) {
            status = dfail(hw[2 * s + 1] & 4u ? FCX_ERR_CAPACITY : FCX_ERR_INTERNAL,
                           "fcx_dist_compress_gather: device error bits " + std::to_string(hw[2 * s + 1]));
            msg = fcx_last_error();
            ok = false;
        }
        if (!ok) {   // publish the failure in this and every later round (rank 0 keeps the protocol)
            if (status == FCX_OK) { status = dfail(FCX_ERR_HIP, "fcx_dist_compress_gather: compress failed"); msg = fcx_last_error(); }
            hw[2 * s] = kFailed;
            hw[2 * s + 1] = 1;
            DHIP(hipMemcpyAsync(dw + 2 * s, hw + 2 * s, 2 * sizeof(uint64_t), hipMemcpyHostToDevice, d->cst));
        } else {
            lens[s] = hw[2 * s];
            DHIP(hipStreamWaitEvent(d->cst, d->ev[s], 0));
        }
        DNCCL(ncclSend(dw + 2 * s, 2, ncclUint64, 0, comm, d->cst));
        if (ok && lens[s]) DNCCL(ncclSend(d_out + ro[s], lens[s], ncclUint8, 0, comm, d->cst));
        sent += lens[s];
    }
    DHIP(hipStreamSynchronize(d->cst));
    DHIP(hipStreamSynchronize(st));
    if (status) return dfail(status, msg);
    *total = sent;
    return FCX_OK;
}

int fcx_dist_unique_id(uint8_t *id) {
    if (!id) return dfail(FCX_ERR_ARG, "fcx_dist_unique_id: NULL");
    ncclUniqueId u;
    DNCCL(ncclGetUniqueId(&u));
    memcpy(id, u.internal, FCX_DIST_ID_BYTES);
    return FCX_OK;
}

int fcx_dist_init_rank(fcx_dist **out, int nranks, int rank, const uint8_t *id, int device) {
    if (!out || !id || nranks <= 0 || rank < 0 || rank >= nranks) return dfail(FCX_ERR_ARG, "fcx_dist_init_rank: bad argument");
    *out = nullptr;
    DHIP(hipSetDevice(device));
    ncclUniqueId u;
    memcpy(u.internal, id, FCX_DIST_ID_BYTES);
    ncclComm_t comm;
    DNCCL(ncclCommInitRank(&comm, nranks, u, rank));
    fcx_dist *d = new fcx_dist();
    d->nranks = nranks;
    d->base_rank = rank;
    d->devices = {device};
    d->comms = {comm};
    const int r = make_dist(out, d);
    if (r) fcx_dist_destroy(d);
    return r;
}

int fcx_dist_init_local(fcx_dist **out, int ndev, const int *devices) {
    if (!out || ndev <= 0 || !devices) return dfail(FCX_ERR_ARG, "fcx_dist_init_local: bad argument");
    *out = nullptr;
    int have = 0;
    if (hipGetDeviceCount(&have) != hipSuccess || have == 0) return dfail(FCX_ERR_HIP, "no HIP device: the compress path is GPU-only");
    for (int i = 0; i < ndev; i++)
        if (devices[i] < 0 || devices[i] >= have) return dfail(FCX_ERR_ARG, "fcx_dist_init_local: bad device index");
    std::vector<ncclComm_t> comms(ndev);
    DNCCL(ncclCommInitAll(comms.data(), ndev, devices));
    fcx_dist *d = new fcx_dist();
    d->nranks = ndev;
    d->base_rank = 0;
    d->devices.assign(devices, devices + ndev);
    d->comms = comms;
    const int r = make_dist(out, d);
    if (r) fcx_dist_destroy(d);
    return r;
}

void fcx_dist_destroy(fcx_dist *d) {
    if (!d) return;
    release_local(d);
    release_gather(d);
    for (size_t i = 0; i < d->comms.size(); i++) {
        (void)hipSetDevice(d->devices[i]);
        (void)hipDeviceSynchronize();
        if (i < d->d_sizes.size() && d->d_sizes[i]) (void)hipFree(d->d_sizes[i]);
        (void)ncclCommDestroy(d->comms[i]);
    }
    delete d;
}

int fcx_dist_size(fcx_dist *d, int *nranks, int *nlocal) {
    if (!d) return dfail(FCX_ERR_ARG, "NULL dist");
    if (nranks) *nranks = d->nranks;
    if (nlocal) *nlocal = (int)d->comms.size();
    return FCX_OK;
}

int fcx_dist_concat(fcx_dist *d, int local, const uint8_t *d_seg, uint64_t seg_len, uint8_t *d_out, uint64_t cap,
                    uint64_t *total, int mode, void *stream) {
    if (!d || !total || local < 0 || local >= (int)d->comms.size() || (seg_len && !d_seg) ||
        (mode != FCX_DIST_GATHER && mode != FCX_DIST_ALLGATHER))
        return dfail(FCX_ERR_ARG, "fcx_dist_concat: bad argument");
    if (d->comms.size() > 1) return dfail(FCX_ERR_ARG, "fcx_dist_concat: a multi-device process uses fcx_dist_compress_host");
    return concat_local(d, local, d_seg, seg_len, d_out, cap, total, mode, (hipStream_t)stream);
}

int fcx_dist_compress_host(fcx_dist *d, const uint8_t *in, uint64_t n, uint32_t block_bytes, uint64_t round_bytes,
                           uint8_t *out, uint64_t cap, uint64_t *out_len) {
    if (!d || (n && !in) || !out || !out_len || block_bytes == 0 || block_bytes > FCX_MAX_BLOCK_BYTES)
        return dfail(FCX_ERR_ARG, "fcx_dist_compress_host: bad argument");
    if (d->base_rank != 0 || (int)d->comms.size() != d->nranks)
        return dfail(FCX_ERR_ARG, "fcx_dist_compress_host: needs every rank in this process (fcx_dist_init_local)");
    *out_len = 0;
    if (n == 0) return FCX_OK;
    const int nd = d->nranks;
    const uint64_t per = ((round_bytes ? round_bytes : (1ull << 30)) + block_bytes - 1) / block_bytes * block_bytes;
    const uint64_t round_max = per * (uint64_t)nd;
    const uint64_t rn0 = n < round_max ? n : round_max;
    // per device: context, input and output buffers (device 0's output receives the round),
    // kept in the fcx_dist between calls (the CLI's -g N calls once per round of input)
    int r0 = ensure_local(d, block_bytes, per < rn0 ? per : rn0, rn0);
    if (r0) return r0;
    std::vector<fcx_ctx *> &ctx = d->ctx;
    std::vector<uint8_t *> &din = d->din, &dout = d->dout;
    std::vector<hipStream_t> &st = d->st;
    std::vector<uint64_t> &dcap = d->dcap;
    std::vector<int> rc(nd, FCX_OK);
    std::vector<std::string> err(nd);
    uint64_t done_in = 0, done_out = 0;
    while (done_in < n) {
        const uint64_t rn = n - done_in < round_max ? n - done_in : round_max;
        const uint64_t nb = (rn + block_bytes - 1) / block_bytes;
        uint64_t total = 0;
        auto work = [&](int i) {
            uint64_t b0, b1;
            fcx_dist_block_range(nb, i, nd, &b0, &b1);
            const uint64_t lo = b0 * block_bytes < rn ? b0 * block_bytes : rn;
            const uint64_t hi = b1 * block_bytes < rn ? b1 * block_bytes : rn;
            int r = FCX_OK;
            uint64_t seg = 0, tot = 0;
            if (hipSetDevice(d->devices[i]) != hipSuccess) r = dfail(FCX_ERR_HIP, "hipSetDevice");
            if (!r && hi > lo && hipMemcpyAsync(din[i], in + done_in + lo, hi - lo, hipMemcpyHostToDevice, st[i]) != hipSuccess)
                r = dfail(FCX_ERR_HIP, "fcx_dist_compress_host: H2D");
            if (!r && hi > lo) r = fcx_compress_shard(ctx[i], din[i], hi - lo, dout[i], dcap[i], &seg, st[i]);
            // every rank enters the exchange, failed or not (a failure is published there)
            r = concat_local(d, i, dout[i], seg, dout[0], dcap[0], &tot, FCX_DIST_GATHER, st[i], r);
            if (i == 0) total = tot;
            rc[i] = r;
            if (r) err[i] = fcx_last_error();
        };
        std::vector<std::thread> th;
        for (int i = 1; i < nd; i++) th.emplace_back(work, i);
        work(0);
        for (auto &t : th) t.join();
        for (int i = 0; i < nd; i++)
            if (rc[i]) {
                return dfail(rc[i], "device " + std::to_string(d->devices[i]) + ": " + err[i]);
            }
        if (done_out + total > cap) return dfail(FCX_ERR_CAPACITY, "fcx_dist_compress_host: output capacity too small");
        (void)hipSetDevice(d->devices[0]);
        if (hipMemcpy(out + done_out, dout[0], total, hipMemcpyDeviceToHost) != hipSuccess)
            return dfail(FCX_ERR_HIP, "fcx_dist_compress_host: D2H");
        done_out += total;
        done_in += rn;
    }
    *out_len = done_out;
    return FCX_OK;
}

}  // extern "C"
