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
    std::vector<uint64_t *> d_sizes; // per local rank: nranks u64 (size all-gather)
};

namespace {

// sizes all-gather + segment placement for local rank li (one host thread per local rank)
int concat_local(fcx_dist *d, int li, const uint8_t *d_seg, uint64_t seg_len, uint8_t *d_out, uint64_t cap,
                 uint64_t *total, int mode, hipStream_t st) {
    const int n = d->nranks, rank = d->base_rank + li;
    ncclComm_t comm = d->comms[li];
    DHIP(hipSetDevice(d->devices[li]));
    uint64_t *ds = d->d_sizes[li];
    DHIP(hipMemcpyAsync(ds + rank, &seg_len, sizeof(uint64_t), hipMemcpyHostToDevice, st));
    DNCCL(ncclAllGather(ds + rank, ds, 1, ncclUint64, comm, st));
    std::vector<uint64_t> sizes(n), offs(n, 0);
    DHIP(hipMemcpyAsync(sizes.data(), ds, n * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    DHIP(hipStreamSynchronize(st));
    for (int r = 1; r < n; r++) offs[r] = offs[r - 1] + sizes[r - 1];
    const uint64_t tot = offs[n - 1] + sizes[n - 1];
    *total = tot;
    if (sizes[rank] != seg_len) return dfail(FCX_ERR_INTERNAL, "fcx_dist_concat: size exchange mismatch");
    const bool receives = mode == FCX_DIST_ALLGATHER || rank == 0;
    if (receives && tot > cap) return dfail(FCX_ERR_CAPACITY, "fcx_dist_concat: output capacity too small");
    // own segment to its offset (skipped when it already lives there)
    if (receives && seg_len && d_seg != d_out + offs[rank])
        DHIP(hipMemcpyAsync(d_out + offs[rank], d_seg, seg_len, hipMemcpyDeviceToDevice, st));
    DNCCL(ncclGroupStart());
    if (mode == FCX_DIST_GATHER) {
        if (rank == 0) {
            for (int r = 1; r < n; r++)
                if (sizes[r]) DNCCL(ncclRecv(d_out + offs[r], sizes[r], ncclUint8, r, comm, st));
        } else if (seg_len) {
            DNCCL(ncclSend(d_seg, seg_len, ncclUint8, 0, comm, st));
        }
    } else {
        for (int r = 0; r < n; r++)
            if (sizes[r]) DNCCL(ncclBroadcast(d_out + offs[r], d_out + offs[r], sizes[r], ncclUint8, r, comm, st));
    }
    DNCCL(ncclGroupEnd());
    DHIP(hipStreamSynchronize(st));
    return FCX_OK;
}

int make_dist(fcx_dist **out, fcx_dist *d) {
    d->d_sizes.resize(d->devices.size(), nullptr);
    for (size_t i = 0; i < d->devices.size(); i++) {
        DHIP(hipSetDevice(d->devices[i]));
        DHIP(hipMalloc((void **)&d->d_sizes[i], sizeof(uint64_t) * (size_t)d->nranks));
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
    // per device: context, input and output buffers (device 0's output receives the round)
    std::vector<fcx_ctx *> ctx(nd, nullptr);
    std::vector<uint8_t *> din(nd, nullptr), dout(nd, nullptr);
    std::vector<hipStream_t> st(nd, nullptr);
    std::vector<uint64_t> dcap(nd, 0);
    std::vector<int> rc(nd, FCX_OK);
    std::vector<std::string> err(nd);
    uint64_t done_in = 0, done_out = 0;
    auto release = [&]() {
        for (int i = 0; i < nd; i++) {
            (void)hipSetDevice(d->devices[i]);
            if (st[i]) (void)hipStreamDestroy(st[i]);
            if (din[i]) (void)hipFree(din[i]);
            if (dout[i]) (void)hipFree(dout[i]);
            fcx_ctx_destroy(ctx[i]);
        }
    };
    {   // allocation, one device at a time
        const uint64_t rn = n < round_max ? n : round_max;
        for (int i = 0; i < nd; i++) {
            int r = FCX_OK;
            if (hipSetDevice(d->devices[i]) != hipSuccess || hipStreamCreate(&st[i]) != hipSuccess)
                r = dfail(FCX_ERR_HIP, "fcx_dist_compress_host: stream");
            if (!r) r = fcx_ctx_create(&ctx[i], d->devices[i], block_bytes, per);
            dcap[i] = fcx_shard_bound(i == 0 ? rn : per, block_bytes);
            if (!r && (hipMalloc((void **)&din[i], per) != hipSuccess || hipMalloc((void **)&dout[i], dcap[i]) != hipSuccess))
                r = dfail(FCX_ERR_NOMEM, "fcx_dist_compress_host: device buffers");
            if (r) { release(); return r; }
        }
    }
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
            if (!r) r = concat_local(d, i, dout[i], seg, dout[0], dcap[0], &tot, FCX_DIST_GATHER, st[i]);
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
                const int r = dfail(rc[i], "device " + std::to_string(d->devices[i]) + ": " + err[i]);
                release();
                return r;
            }
        if (done_out + total > cap) { release(); return dfail(FCX_ERR_CAPACITY, "fcx_dist_compress_host: output capacity too small"); }
        (void)hipSetDevice(d->devices[0]);
        if (hipMemcpy(out + done_out, dout[0], total, hipMemcpyDeviceToHost) != hipSuccess) {
            release();
            return dfail(FCX_ERR_HIP, "fcx_dist_compress_host: D2H");
        }
        done_out += total;
        done_in += rn;
    }
    release();
    *out_len = done_out;
    return FCX_OK;
}

}  // extern "C"
