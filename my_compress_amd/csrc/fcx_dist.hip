// fcx_dist.hip — multi-GPU compress: contiguous block ranges per GPU, segments
// concatenated in block order over RCCL (xGMI).  See include/fcx.h (fcx_dist_*).
//
// The reference compresses its 1 MiB blocks one after the other and writes each
// [u32 len][payload] record to one file in order (my_compress.cpp:4090-4122,
// 4112-4114).  Blocks are independent (:1675-1703), so N ranks take contiguous block
// ranges; the only exchange is the concatenation: an all-gather of the u64 segment
// sizes, then the segments land at their offsets of one contiguous buffer — a gather
// to rank 0 (grouped send/recv: every peer's link carries its own segment at once,
// 1/N of an all-gather's traffic) or an all-gather-v (one broadcast per source rank
// with its exact size; no padding, no second copy).
//
// The protocols talk to a Transport (group start/end, send/recv of device bytes, a
// small all-gather, a broadcast).  The product transport is RCCL.  The loopback
// transport runs the same protocol code between host threads of one process on one
// GPU ("thread ranks", each with its own fcx_ctx and streams): a matched send/recv
// pair becomes one device-to-device copy on the hub's stream, ordered after both
// sides' stream positions by events, and both sides' streams wait for the copy.
// It exists so that the N > 1 exchange runs on a one-GPU box (tests/test_gpu_dist.py).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
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
#define DTRY(expr)                                                                              \
    do {                                                                                        \
        int rc_ = (expr);                                                                       \
        if (rc_) return rc_;                                                                    \
    } while (0)

// ---- transport seam ------------------------------------------------------------------------
// Semantics are NCCL's: ops between group_start/group_end are issued together at group_end;
// an op outside a group is a group of one; every op is ordered on its stream.
struct Transport {
    virtual ~Transport() = default;
    virtual const char *name() const = 0;
    virtual int group_start() = 0;
    virtual int group_end() = 0;
    virtual int send(const void *buf, uint64_t bytes, int peer, hipStream_t st) = 0;
    virtual int recv(void *buf, uint64_t bytes, int peer, hipStream_t st) = 0;
    // every rank's `bytes` at sbuf land at rbuf + rank * bytes on every rank
    virtual int allgather(const void *sbuf, void *rbuf, uint64_t bytes, hipStream_t st) = 0;
    // root's `bytes` at sbuf land at rbuf on every rank
    virtual int broadcast(const void *sbuf, void *rbuf, uint64_t bytes, int root, hipStream_t st) = 0;
    // the communicator is unusable afterwards (peers blocked on it are released with an error)
    virtual void abort() = 0;
};

struct RcclTransport final : Transport {
    ncclComm_t comm = nullptr;
    bool aborted = false;
    explicit RcclTransport(ncclComm_t c) : comm(c) {}
    ~RcclTransport() override {
        if (comm && !aborted) (void)ncclCommDestroy(comm);
    }
    const char *name() const override { return "rccl"; }
    int group_start() override { DNCCL(ncclGroupStart()); return FCX_OK; }
    int group_end() override { DNCCL(ncclGroupEnd()); return FCX_OK; }
    int send(const void *buf, uint64_t bytes, int peer, hipStream_t st) override {
        DNCCL(ncclSend(buf, bytes, ncclUint8, peer, comm, st));
        return FCX_OK;
    }
    int recv(void *buf, uint64_t bytes, int peer, hipStream_t st) override {
        DNCCL(ncclRecv(buf, bytes, ncclUint8, peer, comm, st));
        return FCX_OK;
    }
    int allgather(const void *sbuf, void *rbuf, uint64_t bytes, hipStream_t st) override {
        DNCCL(ncclAllGather(sbuf, rbuf, bytes, ncclUint8, comm, st));
        return FCX_OK;
    }
    int broadcast(const void *sbuf, void *rbuf, uint64_t bytes, int root, hipStream_t st) override {
        DNCCL(ncclBroadcast(sbuf, rbuf, bytes, ncclUint8, root, comm, st));
        return FCX_OK;
    }
    void abort() override {
        if (comm && !aborted) (void)ncclCommAbort(comm);
        aborted = true;
    }
};

// ---- loopback: thread ranks of one process on one device -------------------------------------
enum OpKind { kSend, kRecv, kAllGather, kBcast };

struct LoopDone {          // the hub's "copy done" event, waited for by every op it completes
    hipEvent_t ev = nullptr;
    int refs = 0;
};

struct LoopOp {
    OpKind kind = kSend;
    int rank = 0, peer = 0;            // p2p: own rank and the other side; broadcast: peer = root
    const void *sbuf = nullptr;
    void *rbuf = nullptr;
    uint64_t bytes = 0;
    hipStream_t st = nullptr;
    hipEvent_t posted = nullptr;       // the op's position on its stream
    LoopDone *done = nullptr;
    bool matched = false;
    int err = FCX_OK;
    std::string msg;
};

}  // namespace

struct fcx_loop {
    int nranks = 0;
    int device = -1;
    uint32_t timeout_ms = 60000;
    std::mutex mu;
    std::condition_variable cv;
    hipStream_t st = nullptr;                      // copies of matched ops, in match order
    std::vector<std::deque<LoopOp *>> sendq, recvq;   // per (src * n + dst), FIFO like NCCL
    std::map<uint64_t, std::vector<LoopOp *>> coll;   // k-th collective of every rank
    std::vector<uint64_t> coll_seq;                // per rank: collectives posted
    std::vector<hipEvent_t> free_ev, retired_ev;
    int attached = 0;
    bool creator_gone = false;
    bool aborted = false;
    std::string abort_msg;

    // (all below with mu held)
    hipEvent_t event() {
        if (free_ev.empty())
            for (size_t i = 0; i < retired_ev.size();) {
                if (hipEventQuery(retired_ev[i]) == hipSuccess) {
                    free_ev.push_back(retired_ev[i]);
                    retired_ev[i] = retired_ev.back();
                    retired_ev.pop_back();
                } else {
                    i++;
                }
            }
        if (!free_ev.empty()) {
            hipEvent_t e = free_ev.back();
            free_ev.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
        return e;
    }
    void retire(hipEvent_t e) {
        if (e) retired_ev.push_back(e);
    }
    // the hub stream waits for every op's stream position, runs `copies`, records the done event
    // every op's stream will wait for
    void complete(const std::vector<LoopOp *> &ops, const std::vector<std::pair<LoopOp *, LoopOp *>> &copies,
                  int err, const std::string &msg) {
        LoopDone *dn = new LoopDone();
        dn->refs = (int)ops.size();
        for (LoopOp *o : ops) (void)hipStreamWaitEvent(st, o->posted, 0);
        if (!err)
            for (auto &c : copies)   // (dst op, src op): src's sbuf -> dst's rbuf (+ offset for allgather)
                if (c.first->bytes) {
                    uint8_t *dst = (uint8_t *)c.first->rbuf;
                    if (c.first->kind == kAllGather) dst += (uint64_t)c.second->rank * c.second->bytes;
                    if (dst != c.second->sbuf &&
                        hipMemcpyAsync(dst, c.second->sbuf, c.first->bytes, hipMemcpyDeviceToDevice, st) != hipSuccess)
                        err = FCX_ERR_HIP;
                }
        dn->ev = event();
        if (!dn->ev || hipEventRecord(dn->ev, st) != hipSuccess) err = FCX_ERR_HIP;
        for (LoopOp *o : ops) {
            retire(o->posted);
            o->posted = nullptr;
            o->done = dn;
            o->matched = true;
            if (err) {
                o->err = err;
                o->msg = msg.empty() ? "loopback transport: device copy failed" : msg;
            }
        }
    }
    void post(LoopOp *o) {
        const int n = nranks;
        if (o->kind == kSend || o->kind == kRecv) {
            const int src = o->kind == kSend ? o->rank : o->peer, dst = o->kind == kSend ? o->peer : o->rank;
            auto &mine = (o->kind == kSend ? sendq : recvq)[(size_t)src * n + dst];
            auto &other = (o->kind == kSend ? recvq : sendq)[(size_t)src * n + dst];
            if (other.empty()) {
                mine.push_back(o);
                return;
            }
            LoopOp *p = other.front();
            other.pop_front();
            LoopOp *s = o->kind == kSend ? o : p, *r = o->kind == kSend ? p : o;
            const bool ok = s->bytes == r->bytes;
            complete({s, r}, {{r, s}}, ok ? FCX_OK : FCX_ERR_RCCL,
                     ok ? std::string() : "loopback transport: rank " + std::to_string(src) + " sends " +
                                              std::to_string(s->bytes) + " B, rank " + std::to_string(dst) +
                                              " receives " + std::to_string(r->bytes) + " B");
            return;
        }
        auto &v = coll[coll_seq[o->rank]++];
        v.push_back(o);
        if ((int)v.size() < n) return;
        std::vector<LoopOp *> ops(v.begin(), v.end());
        coll.erase(coll_seq[o->rank] - 1);
        std::vector<LoopOp *> by_rank(n, nullptr);
        bool ok = true;
        for (LoopOp *x : ops) {
            ok &= x->kind == ops[0]->kind && x->bytes == ops[0]->bytes && x->peer == ops[0]->peer;
            if (x->rank >= 0 && x->rank < n) by_rank[x->rank] = x;
        }
        std::vector<std::pair<LoopOp *, LoopOp *>> copies;
        if (ok) {
            for (int r = 0; r < n; r++) ok &= by_rank[r] != nullptr;
        }
        if (ok && ops[0]->kind == kAllGather) {
            for (int r = 0; r < n; r++)
                for (int q = 0; q < n; q++) copies.push_back({by_rank[r], by_rank[q]});
        } else if (ok) {
            const int root = ops[0]->peer;
            ok = root >= 0 && root < n;
            if (ok)
                for (int r = 0; r < n; r++) copies.push_back({by_rank[r], by_rank[root]});
        }
        complete(ops, copies, ok ? FCX_OK : FCX_ERR_RCCL,
                 ok ? std::string() : "loopback transport: ranks disagree on a collective (kind, size or root)");
    }
    void abort_all(const std::string &why) {
        if (!aborted) {
            aborted = true;
            abort_msg = why;
        }
        for (auto &q : sendq) q.clear();
        for (auto &q : recvq) q.clear();
        coll.clear();
        cv.notify_all();
    }
    // (mu NOT held) drops the creator's or one attached rank's reference; the hub is freed by the
    // call that drops the last one (the transition and the check share one critical section)
    void drop(bool creator) {
        bool last;
        {
            std::lock_guard<std::mutex> lk(mu);
            if (creator)
                creator_gone = true;
            else
                attached--;
            last = creator_gone && attached == 0;
        }
        if (!last) return;
        if (st) {
            (void)hipSetDevice(device);
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
        for (auto e : free_ev) (void)hipEventDestroy(e);
        for (auto e : retired_ev) (void)hipEventDestroy(e);
        delete this;
    }
};

namespace {

struct LoopTransport final : Transport {
    fcx_loop *hub;
    int rank;
    int depth = 0;
    std::vector<std::unique_ptr<LoopOp>> pending;
    LoopTransport(fcx_loop *h, int r) : hub(h), rank(r) {}
    ~LoopTransport() override { hub->drop(false); }
    const char *name() const override { return "loopback"; }
    int group_start() override {
        depth++;
        return FCX_OK;
    }
    int group_end() override {
        if (depth <= 0) return dfail(FCX_ERR_ARG, "loopback transport: group_end without group_start");
        if (--depth) return FCX_OK;
        return flush();
    }
    int add(std::unique_ptr<LoopOp> o) {
        o->rank = rank;
        pending.push_back(std::move(o));
        return depth ? FCX_OK : flush();
    }
    int send(const void *buf, uint64_t bytes, int peer, hipStream_t st) override {
        if (peer < 0 || peer >= hub->nranks || peer == rank) return dfail(FCX_ERR_ARG, "loopback transport: bad peer");
        auto o = std::make_unique<LoopOp>();
        o->kind = kSend; o->peer = peer; o->sbuf = buf; o->bytes = bytes; o->st = st;
        return add(std::move(o));
    }
    int recv(void *buf, uint64_t bytes, int peer, hipStream_t st) override {
        if (peer < 0 || peer >= hub->nranks || peer == rank) return dfail(FCX_ERR_ARG, "loopback transport: bad peer");
        auto o = std::make_unique<LoopOp>();
        o->kind = kRecv; o->peer = peer; o->rbuf = buf; o->bytes = bytes; o->st = st;
        return add(std::move(o));
    }
    int allgather(const void *sbuf, void *rbuf, uint64_t bytes, hipStream_t st) override {
        auto o = std::make_unique<LoopOp>();
        o->kind = kAllGather; o->peer = -1; o->sbuf = sbuf; o->rbuf = rbuf; o->bytes = bytes; o->st = st;
        return add(std::move(o));
    }
    int broadcast(const void *sbuf, void *rbuf, uint64_t bytes, int root, hipStream_t st) override {
        auto o = std::make_unique<LoopOp>();
        o->kind = kBcast; o->peer = root; o->sbuf = sbuf; o->rbuf = rbuf; o->bytes = bytes; o->st = st;
        return add(std::move(o));
    }
    void abort() override {
        std::lock_guard<std::mutex> lk(hub->mu);
        hub->abort_all("loopback transport: rank " + std::to_string(rank) + " aborted the communicator");
    }
    // issues the pending group: records each op's stream position, posts it to the hub (the side
    // that completes a pair enqueues the copy), waits until every op is matched, then orders each
    // op's stream after its copy.  An op never matched within the hub's timeout aborts the hub, so
    // a protocol error fails every rank instead of hanging one.
    int flush() {
        std::vector<std::unique_ptr<LoopOp>> ops;
        ops.swap(pending);
        if (ops.empty()) return FCX_OK;
        DHIP(hipSetDevice(hub->device));
        std::unique_lock<std::mutex> lk(hub->mu);
        if (hub->aborted) return dfail(FCX_ERR_RCCL, hub->abort_msg);
        for (size_t i = 0; i < ops.size(); i++) {
            ops[i]->posted = hub->event();
            if (!ops[i]->posted || hipEventRecord(ops[i]->posted, ops[i]->st) != hipSuccess) {
                for (size_t j = 0; j <= i; j++)   // nothing was posted: every event taken goes back
                    if (ops[j]->posted) hub->retire(ops[j]->posted);
                return dfail(FCX_ERR_HIP, "loopback transport: event record");
            }
        }
        for (auto &o : ops) hub->post(o.get());
        hub->cv.notify_all();
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(hub->timeout_ms);
        auto all_matched = [&] {
            for (auto &o : ops)
                if (!o->matched) return false;
            return true;
        };
        while (!all_matched() && !hub->aborted)
            if (hub->cv.wait_until(lk, deadline) == std::cv_status::timeout && !all_matched()) {
                hub->abort_all("loopback transport: rank " + std::to_string(rank) + " waited " +
                               std::to_string(hub->timeout_ms) + " ms for a matching operation");
                break;
            }
        if (!all_matched()) {   // aborted: the unmatched ops were dropped from the hub's queues
            for (auto &o : ops) {
                if (!o->matched) hub->retire(o->posted);
                if (o->matched && o->done && --o->done->refs == 0) {
                    hub->retire(o->done->ev);
                    delete o->done;
                }
            }
            return dfail(FCX_ERR_RCCL, hub->abort_msg);
        }
        int rc = FCX_OK;
        std::string msg;
        for (auto &o : ops) {
            if (hipStreamWaitEvent(o->st, o->done->ev, 0) != hipSuccess && !rc) {
                rc = FCX_ERR_HIP;
                msg = "loopback transport: stream wait";
            }
            if (o->err && !rc) {
                rc = o->err;
                msg = o->msg;
            }
            if (--o->done->refs == 0) {
                hub->retire(o->done->ev);
                delete o->done;
            }
        }
        return rc ? dfail(rc, msg) : FCX_OK;
    }
};

}  // namespace

struct fcx_dist {
    int nranks = 0;                  // ranks of the job
    int base_rank = 0;               // rank of local index 0
    std::vector<int> devices;        // per local rank
    std::vector<std::unique_ptr<Transport>> tr;   // per local rank
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
    uint64_t *d_ctl = nullptr;       // [0, 1] the failure words (never written by a compress stream); [2] verdict
    uint64_t *h_ctl = nullptr;       // pinned mirror of the verdict
    std::vector<hipEvent_t> ev;      // per sub-batch: compressed and its length copied
    uint8_t *d_stage = nullptr;      // rank 0: the peers' pieces as they arrive
    uint64_t stage_cap = 0;
    uint8_t *d_drain = nullptr;      // rank 0: a piece beyond its peer's bound, received and dropped
    uint64_t drain_cap = 0;
    hipEvent_t copy_ev[2] = {nullptr, nullptr};   // rank 0: around the final moves of the peers' bytes
    float copy_ms = -1.f;            // their duration in the last gather (-1: none timed)
    int fail_piece = -1;             // testing: a peer treats this piece as failed (fcx_dist_debug_fail)
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
    Transport &t = *d->tr[li];
    DHIP(hipSetDevice(d->devices[li]));
    uint64_t *ds = d->d_sizes[li];
    const bool receives = mode == FCX_DIST_ALLGATHER || rank == 0;
    const uint64_t mine[2] = {status ? kFailed : seg_len, receives ? cap : kFailed};
    DHIP(hipMemcpyAsync(ds + 2 * rank, mine, sizeof(mine), hipMemcpyHostToDevice, st));
    DTRY(t.allgather(ds + 2 * rank, ds, sizeof(mine), st));
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
    DTRY(t.group_start());
    int rc = FCX_OK;
    if (mode == FCX_DIST_GATHER) {
        if (rank == 0) {
            for (int r = 1; r < n && !rc; r++)
                if (sizes[r]) rc = t.recv(d_out + offs[r], sizes[r], r, st);
        } else if (own) {
            rc = t.send(d_seg, own, 0, st);
        }
    } else {
        for (int r = 0; r < n && !rc; r++)
            if (sizes[r]) rc = t.broadcast(d_out + offs[r], d_out + offs[r], sizes[r], r, st);
    }
    const int rc2 = t.group_end();
    if (rc) return rc;
    if (rc2) return rc2;
    DHIP(hipStreamSynchronize(st));
    if (own != seg_len) return dfail(FCX_ERR_INTERNAL, "fcx_dist_concat: size exchange mismatch");
    return FCX_OK;
}

// fcx_dist_compress_gather's stream, length words, control words and events (sized for
// FCX_DIST_MAX_SUB sub-batches of every rank), and rank 0's staging buffer of >= `stage` bytes
int ensure_gather(fcx_dist *d, uint64_t stage) {
    DHIP(hipSetDevice(d->devices[0]));
    const size_t words = 2ull * FCX_DIST_MAX_SUB * (size_t)d->nranks;
    if (!d->cst) {
        DHIP(hipStreamCreateWithFlags(&d->cst, hipStreamNonBlocking));
        DHIP(hipMalloc((void **)&d->d_words, words * sizeof(uint64_t)));
        DHIP(hipHostMalloc((void **)&d->h_words, words * sizeof(uint64_t), hipHostMallocDefault));
        DHIP(hipMalloc((void **)&d->d_ctl, 4 * sizeof(uint64_t)));
        DHIP(hipHostMalloc((void **)&d->h_ctl, 4 * sizeof(uint64_t), hipHostMallocDefault));
        const uint64_t ctl[4] = {kFailed, 1, 0, 0};
        DHIP(hipMemcpy(d->d_ctl, ctl, sizeof(ctl), hipMemcpyHostToDevice));
        d->ev.assign(FCX_DIST_MAX_SUB, nullptr);
        for (auto &e : d->ev) DHIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        for (auto &e : d->copy_ev) DHIP(hipEventCreate(&e));
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
    for (auto &e : d->copy_ev) {
        if (e) (void)hipEventDestroy(e);
        e = nullptr;
    }
    if (d->cst) (void)hipStreamDestroy(d->cst);
    if (d->d_words) (void)hipFree(d->d_words);
    if (d->h_words) (void)hipHostFree(d->h_words);
    if (d->d_ctl) (void)hipFree(d->d_ctl);
    if (d->h_ctl) (void)hipHostFree(d->h_ctl);
    if (d->d_stage) (void)hipFree(d->d_stage);
    if (d->d_drain) (void)hipFree(d->d_drain);
    d->cst = nullptr; d->d_words = nullptr; d->h_words = nullptr; d->d_ctl = nullptr; d->h_ctl = nullptr;
    d->d_stage = nullptr; d->stage_cap = 0;
    d->d_drain = nullptr; d->drain_cap = 0;
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

int need_device(int device) {
    int have = 0;
    if (hipGetDeviceCount(&have) != hipSuccess || have == 0)
        return dfail(FCX_ERR_HIP, "no HIP device: the compress path is GPU-only");
    if (device < 0 || device >= have) return dfail(FCX_ERR_ARG, "bad device index");
    return FCX_OK;
}

// rank 0's side of fcx_dist_compress_gather
int gather_root(fcx_dist *d, fcx_ctx *c, const uint8_t *d_in, uint64_t n, const uint64_t *rank_bytes,
                uint32_t nsub, uint32_t B, uint8_t *d_out, uint64_t cap, uint64_t *total, hipStream_t st) {
    const int N = d->nranks;
    Transport &t = *d->tr[0];
    std::vector<uint64_t> soff(N, 0), bound(N, 0);   // each peer's staging region
    uint64_t stage = 0;
    for (int r = 1; r < N; r++) {
        soff[r] = stage;
        bound[r] = pieces_bound(rank_bytes[r], B, nsub);
        stage += bound[r];
    }
    DTRY(ensure_gather(d, stage));
    uint64_t *dw = d->d_words, *hw = d->h_words;
    // own range straight into d_out at offset 0 (a failure is reported after the peers' pieces
    // are drained, so no peer is left in a send), the peers' pieces into the staging regions on
    // the exchange stream meanwhile: per round s, every peer's length words, then its bytes
    int own_rc = fcx_compress_shard(c, d_in, n, d_out, cap, nullptr, st);
    std::string own_msg = own_rc ? fcx_last_error() : "";
    std::vector<uint64_t> fill(N, 0);
    std::string peer_err;
    for (uint32_t s = 0; s < nsub && N > 1; s++) {
        uint64_t *ws = dw + 2ull * s * N, *hs = hw + 2ull * s * N;
        DTRY(t.group_start());
        int rc = FCX_OK;
        for (int r = 1; r < N && !rc; r++) rc = t.recv(ws + 2 * r, 2 * sizeof(uint64_t), r, d->cst);
        const int rc2 = t.group_end();
        DTRY(rc);
        DTRY(rc2);
        DHIP(hipMemcpyAsync(hs, ws, 2ull * N * sizeof(uint64_t), hipMemcpyDeviceToHost, d->cst));
        DHIP(hipStreamSynchronize(d->cst));
        // a piece beyond its peer's staging bound (the ranks disagree on rank_bytes; a peer checks
        // its pieces against the same bound otherwise) is still received -- into the drain buffer,
        // so the peer's send completes and the protocol runs on to the failing verdict
        uint64_t drain = 0;
        for (int r = 1; r < N; r++) {
            const uint64_t len = hs[2 * r], err = hs[2 * r + 1];
            if (!err && len != kFailed && len && fill[r] + len > bound[r]) drain = std::max(drain, len);
        }
        if (drain > d->drain_cap) {
            if (d->d_drain) DHIP(hipFree(d->d_drain));
            d->d_drain = nullptr;
            d->drain_cap = 0;
            if (hipMalloc((void **)&d->d_drain, drain) != hipSuccess)
                return dfail(FCX_ERR_NOMEM, "fcx_dist_compress_gather: drain buffer of " + std::to_string(drain) + " B");
            d->drain_cap = drain;
        }
        DTRY(t.group_start());
        for (int r = 1; r < N && !rc; r++) {
            const uint64_t len = hs[2 * r], err = hs[2 * r + 1];
            if (err || len == kFailed) {
                if (peer_err.empty()) peer_err = "rank " + std::to_string(r) + " failed in sub-batch " + std::to_string(s);
                continue;
            }
            if (len == 0) continue;
            if (fill[r] + len > bound[r]) {
                if (peer_err.empty()) peer_err = "rank " + std::to_string(r) + " sent a piece beyond its bound";
                rc = t.recv(d->d_drain, len, r, d->cst);   // (concurrent drains of one round share it: dropped)
                continue;
            }
            rc = t.recv(d->d_stage + soff[r] + fill[r], len, r, d->cst);
            fill[r] += len;
        }
        const int rc3 = t.group_end();
        DTRY(rc);
        DTRY(rc3);
    }
    DHIP(hipStreamSynchronize(d->cst));
    uint64_t own = 0;
    if (!own_rc) {
        own_rc = fcx_ctx_read_out_len(c, &own);
        if (own_rc) own_msg = fcx_last_error();
    }
    uint64_t off = own;
    for (int r = 1; r < N; r++) off += fill[r];
    int verdict = own_rc;
    std::string msg = own_msg;
    if (!verdict && !peer_err.empty()) {
        verdict = FCX_ERR_RCCL;
        msg = "fcx_dist_compress_gather: " + peer_err;
    }
    if (!verdict && off > cap) {
        verdict = FCX_ERR_CAPACITY;
        msg = "fcx_dist_compress_gather: output capacity too small (" + std::to_string(off) + " B)";
    }
    if (N > 1) {   // the job's verdict to every peer, so every rank returns the same outcome
        d->h_ctl[2] = (uint64_t)(int64_t)verdict;
        DHIP(hipMemcpyAsync(d->d_ctl + 2, d->h_ctl + 2, sizeof(uint64_t), hipMemcpyHostToDevice, d->cst));
        DTRY(t.group_start());
        int rc = FCX_OK;
        for (int r = 1; r < N && !rc; r++) rc = t.send(d->d_ctl + 2, sizeof(uint64_t), r, d->cst);
        const int rc2 = t.group_end();
        DTRY(rc);
        DTRY(rc2);
    }
    if (verdict) {
        DHIP(hipStreamSynchronize(d->cst));
        DHIP(hipStreamSynchronize(st));
        return dfail(verdict, msg);
    }
    off = own;
    DHIP(hipEventRecord(d->copy_ev[0], st));
    for (int r = 1; r < N; r++) {   // the peers' bytes behind the own segment, in rank order
        if (fill[r]) DHIP(hipMemcpyAsync(d_out + off, d->d_stage + soff[r], fill[r], hipMemcpyDeviceToDevice, st));
        off += fill[r];
    }
    DHIP(hipEventRecord(d->copy_ev[1], st));
    DHIP(hipStreamSynchronize(d->cst));
    DHIP(hipStreamSynchronize(st));
    if (hipEventElapsedTime(&d->copy_ms, d->copy_ev[0], d->copy_ev[1]) != hipSuccess) d->copy_ms = -1.f;
    *total = off;
    return FCX_OK;
}

// a peer's side: every piece's compress is enqueued at once at its bound offset of d_out; each
// piece's length words follow it on the compress stream, and the exchange stream sends them and
// then the piece's bytes as soon as the piece is done, while the next piece compresses.  A failed
// piece (and every later one) is announced with the constant failure words d_ctl[0..1], which no
// compress-stream copy ever writes, so a pending copy cannot turn the announcement into a length.
int gather_peer(fcx_dist *d, fcx_ctx *c, const uint8_t *d_in, uint64_t n, uint32_t nsub, uint32_t B,
                uint8_t *d_out, uint64_t cap, uint64_t *total, hipStream_t st) {
    Transport &t = *d->tr[0];
    DTRY(ensure_gather(d, 0));
    uint64_t *dw = d->d_words, *hw = d->h_words;
    std::vector<uint64_t> ro(nsub, 0), pb(nsub, 0), lens(nsub, 0);
    int status = FCX_OK;
    std::string msg;
    uint32_t enq = 0;   // pieces enqueued before a host-side failure
    uint64_t o = 0;
    for (uint32_t s = 0; s < nsub; s++) {
        uint64_t lo, hi;
        piece_range(n, B, s, nsub, &lo, &hi);
        ro[s] = o;
        pb[s] = round16(fcx_shard_bound(hi - lo, B));
        if (status == FCX_OK && o + pb[s] > cap) {
            status = dfail(FCX_ERR_CAPACITY, "fcx_dist_compress_gather: peer output capacity too small (see fcx_dist_gather_bound)");
            msg = fcx_last_error();
        }
        if (status == FCX_OK) {
            status = fcx_compress_shard(c, d_in + lo, hi - lo, d_out + o, pb[s], nullptr, st);
            if (status) msg = fcx_last_error();
        }
        if (status == FCX_OK) {
            DHIP(hipMemcpyAsync(dw + 2 * s, fcx_ctx_device_out_len(c), 2 * sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
            DHIP(hipMemcpyAsync(hw + 2 * s, dw + 2 * s, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
            DHIP(hipEventRecord(d->ev[s], st));
            enq = s + 1;
        }
        o += pb[s];
    }
    uint64_t sent = 0;
    bool failed = false;
    for (uint32_t s = 0; s < nsub; s++) {
        if (!failed) {
            if (s >= enq) {
                failed = true;
            } else if (hipEventSynchronize(d->ev[s]) != hipSuccess) {
                failed = true;
                if (status == FCX_OK) { status = dfail(FCX_ERR_HIP, "fcx_dist_compress_gather: compress failed"); msg = fcx_last_error(); }
            } else if (hw[2 * s + 1]) {
                failed = true;
                status = dfail(hw[2 * s + 1] & 4u ? FCX_ERR_CAPACITY : FCX_ERR_INTERNAL,
                               "fcx_dist_compress_gather: device error bits " + std::to_string(hw[2 * s + 1]));
                msg = fcx_last_error();
            } else if (hw[2 * s] > pb[s]) {
                failed = true;
                status = dfail(FCX_ERR_INTERNAL, "fcx_dist_compress_gather: piece longer than its bound");
                msg = fcx_last_error();
            } else if ((int)s == d->fail_piece) {
                failed = true;
                status = dfail(FCX_ERR_INTERNAL, "fcx_dist_compress_gather: injected failure (fcx_dist_debug_fail)");
                msg = fcx_last_error();
            }
        }
        if (failed) {   // this and every later round: the constant failure words
            DTRY(t.send(d->d_ctl, 2 * sizeof(uint64_t), 0, d->cst));
            continue;
        }
        lens[s] = hw[2 * s];
        DHIP(hipStreamWaitEvent(d->cst, d->ev[s], 0));
        DTRY(t.send(dw + 2 * s, 2 * sizeof(uint64_t), 0, d->cst));
        if (lens[s]) DTRY(t.send(d_out + ro[s], lens[s], 0, d->cst));
        sent += lens[s];
    }
    // the job's verdict from rank 0
    DTRY(t.recv(d->d_ctl + 2, sizeof(uint64_t), 0, d->cst));
    DHIP(hipMemcpyAsync(d->h_ctl + 2, d->d_ctl + 2, sizeof(uint64_t), hipMemcpyDeviceToHost, d->cst));
    DHIP(hipStreamSynchronize(d->cst));
    DHIP(hipStreamSynchronize(st));
    if (status) return dfail(status, msg);
    const int64_t verdict = (int64_t)d->h_ctl[2];
    if (verdict)
        return dfail(verdict < 0 && verdict >= FCX_ERR_RCCL ? (int)verdict : FCX_ERR_RCCL,
                     "fcx_dist_compress_gather: rank 0 reports the job failed (code " + std::to_string(verdict) + ")");
    *total = sent;
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
    if (d->tr.size() != 1)
        return dfail(FCX_ERR_ARG, "fcx_dist_compress_gather: one rank per handle (fcx_dist_init_rank / fcx_dist_init_loop)");
    const int rank = d->base_rank;
    if (rank_bytes[rank] != n) return dfail(FCX_ERR_ARG, "fcx_dist_compress_gather: rank_bytes[rank] != n");
    int dev = 0;
    uint32_t B = 0;
    DTRY(fcx_ctx_info(c, &dev, &B, nullptr));
    if (dev != d->devices[0]) return dfail(FCX_ERR_ARG, "fcx_dist_compress_gather: context on another device");
    *total = 0;
    DHIP(hipSetDevice(dev));
    if (rank == 0) return gather_root(d, c, d_in, n, rank_bytes, nsub, B, d_out, cap, total, (hipStream_t)stream);
    return gather_peer(d, c, d_in, n, nsub, B, d_out, cap, total, (hipStream_t)stream);
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
    d->tr.emplace_back(new RcclTransport(comm));
    const int r = make_dist(out, d);
    if (r) fcx_dist_destroy(d);
    return r;
}

int fcx_dist_init_local(fcx_dist **out, int ndev, const int *devices) {
    if (!out || ndev <= 0 || !devices) return dfail(FCX_ERR_ARG, "fcx_dist_init_local: bad argument");
    *out = nullptr;
    for (int i = 0; i < ndev; i++) DTRY(need_device(devices[i]));
    std::vector<ncclComm_t> comms(ndev);
    DNCCL(ncclCommInitAll(comms.data(), ndev, devices));
    fcx_dist *d = new fcx_dist();
    d->nranks = ndev;
    d->base_rank = 0;
    d->devices.assign(devices, devices + ndev);
    for (auto cm : comms) d->tr.emplace_back(new RcclTransport(cm));
    const int r = make_dist(out, d);
    if (r) fcx_dist_destroy(d);
    return r;
}

int fcx_loop_create(fcx_loop **out, int nranks, int device, uint32_t timeout_ms) {
    if (!out || nranks <= 0) return dfail(FCX_ERR_ARG, "fcx_loop_create: bad argument");
    *out = nullptr;
    DTRY(need_device(device));
    DHIP(hipSetDevice(device));
    fcx_loop *h = new fcx_loop();
    h->nranks = nranks;
    h->device = device;
    h->timeout_ms = timeout_ms ? timeout_ms : 60000;
    h->sendq.resize((size_t)nranks * nranks);
    h->recvq.resize((size_t)nranks * nranks);
    h->coll_seq.assign(nranks, 0);
    if (hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return dfail(FCX_ERR_HIP, "fcx_loop_create: stream");
    }
    *out = h;
    return FCX_OK;
}

void fcx_loop_destroy(fcx_loop *h) {
    if (h) h->drop(true);
}

int fcx_dist_init_loop(fcx_dist **out, fcx_loop *h, int rank) {
    if (!out || !h || rank < 0 || rank >= h->nranks) return dfail(FCX_ERR_ARG, "fcx_dist_init_loop: bad argument");
    *out = nullptr;
    {
        std::lock_guard<std::mutex> lk(h->mu);
        h->attached++;
    }
    fcx_dist *d = new fcx_dist();
    d->nranks = h->nranks;
    d->base_rank = rank;
    d->devices = {h->device};
    d->tr.emplace_back(new LoopTransport(h, rank));
    const int r = make_dist(out, d);
    if (r) fcx_dist_destroy(d);
    return r;
}

int fcx_dist_init_loop_local(fcx_dist **out, int nranks, int device, uint32_t timeout_ms) {
    if (!out || nranks <= 0) return dfail(FCX_ERR_ARG, "fcx_dist_init_loop_local: bad argument");
    *out = nullptr;
    fcx_loop *h = nullptr;
    DTRY(fcx_loop_create(&h, nranks, device, timeout_ms));
    fcx_dist *d = new fcx_dist();
    d->nranks = nranks;
    d->base_rank = 0;
    d->devices.assign(nranks, device);
    {
        std::lock_guard<std::mutex> lk(h->mu);
        h->attached += nranks;
    }
    for (int r = 0; r < nranks; r++) d->tr.emplace_back(new LoopTransport(h, r));
    fcx_loop_destroy(h);   // (the transports keep the hub)
    const int r = make_dist(out, d);
    if (r) fcx_dist_destroy(d);
    return r;
}

const char *fcx_dist_transport(fcx_dist *d) { return d && !d->tr.empty() ? d->tr[0]->name() : ""; }

int fcx_dist_gather_copy_ms(fcx_dist *d, float *ms) {
    if (!d || !ms) return dfail(FCX_ERR_ARG, "fcx_dist_gather_copy_ms: NULL argument");
    *ms = d->copy_ms;
    return FCX_OK;
}

int fcx_dist_debug_fail(fcx_dist *d, int piece) {
    if (!d) return dfail(FCX_ERR_ARG, "NULL dist");
    d->fail_piece = piece;
    return FCX_OK;
}

void fcx_dist_destroy(fcx_dist *d) {
    if (!d) return;
    release_local(d);
    release_gather(d);
    for (size_t i = 0; i < d->devices.size(); i++) {
        (void)hipSetDevice(d->devices[i]);
        if (i < d->d_sizes.size() && d->d_sizes[i]) {
            (void)hipDeviceSynchronize();
            (void)hipFree(d->d_sizes[i]);
        }
    }
    d->tr.clear();
    delete d;
}

int fcx_dist_size(fcx_dist *d, int *nranks, int *nlocal) {
    if (!d) return dfail(FCX_ERR_ARG, "NULL dist");
    if (nranks) *nranks = d->nranks;
    if (nlocal) *nlocal = (int)d->tr.size();
    return FCX_OK;
}

int fcx_dist_concat(fcx_dist *d, int local, const uint8_t *d_seg, uint64_t seg_len, uint8_t *d_out, uint64_t cap,
                    uint64_t *total, int mode, void *stream) {
    if (!d || !total || local < 0 || local >= (int)d->tr.size() || (seg_len && !d_seg) ||
        (mode != FCX_DIST_GATHER && mode != FCX_DIST_ALLGATHER))
        return dfail(FCX_ERR_ARG, "fcx_dist_concat: bad argument");
    if (d->tr.size() > 1) return dfail(FCX_ERR_ARG, "fcx_dist_concat: a multi-device process uses fcx_dist_compress_host");
    return concat_local(d, local, d_seg, seg_len, d_out, cap, total, mode, (hipStream_t)stream);
}

int fcx_dist_compress_host(fcx_dist *d, const uint8_t *in, uint64_t n, uint32_t block_bytes, uint64_t round_bytes,
                           uint8_t *out, uint64_t cap, uint64_t *out_len) {
    if (!d || (n && !in) || !out || !out_len || block_bytes == 0 || block_bytes > FCX_MAX_BLOCK_BYTES)
        return dfail(FCX_ERR_ARG, "fcx_dist_compress_host: bad argument");
    if (d->base_rank != 0 || (int)d->tr.size() != d->nranks)
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
