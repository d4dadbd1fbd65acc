// fcx_entropy.hip — Huffman sub-streams and block-record assembly (gfx950).
//
// Each block payload carries four Huffman sub-streams (my_huffman_encode_char,
// my_compress.cpp:987-1104): the literal-flag bitmap (only when > 1 byte,
// 2095-2108), the chars of every token, the 11-bit packed distances and the
// golomb words.  The reference tree is NOT canonical:
//   leaves = symbols with weight > 0, stably sorted by (weight, symbol) (458-498);
//   each step merges list[0] (left) and list[1] (right) and re-inserts the sum
//   after every entry of weight <= sum (strict '<' at 588).
// Because merged weights never decrease, that list is exactly the stable merge
// of two FIFO queues — sorted leaves and internal nodes in creation order —
// taking the leaf on a weight tie.  k_tree runs that two-queue form in one wave
// per (block, stream), then serialises the tree (1013-1066) and the code table:
// code = root->leaf path, left = 0, root decision in bit 0 (LSB-first, 869-924).
//
//   (histograms)   the chars: a u16 row of counts per tile, built by k_emit (fcx_parse.hip)
//   k_tree         sums the chars rows, or counts the bytes of a finished flag / distance /
//                  golomb stream; builds the tree (closed form for balanced weights, a fixed
//                  point for other long merges, else the serial two-queue merge), header
//                  bytes, code table and W, and clears the stream's chunk status words
//   k_block_layout record layout and size per block
//   k_scan_blocks  record offsets across the shard (+ capacity check)
//   k_encode       a chunk of 8192 symbols per workgroup (a chars lane whose 64 symbols are a run
//                  of input bytes, per k_emit's segment descriptor, reads them from the input):
//                  its bit count, then its starting bit
//                  by decoupled look-back over the stream's earlier chunks (8-byte status
//                  words: aggregate or inclusive prefix, and the chunk's last 32 code bits);
//                  each lane packs its 64 codes into whole words in LDS; the words are stored
//                  plainly at the record's (unaligned) byte offset, the first one merged with
//                  the previous chunk's last bits (the word the two chunks share is this
//                  chunk's to write; a stream's last chunk also writes its partial last word)
//   k_headers      lengths, counts and tree headers of every record
#include "fcx_device.h"

namespace fcx {

constexpr uint32_t kErrCodeLen = 1u, kErrCapacity = 4u;

__device__ inline bool stream_active(const BlockInfo &bi, uint32_t s) {
    if (s == 0) return bi.slen[0] > 1;   // flags are Huffman-coded only when > 1 byte
    if (s == 3) return bi.gbits > 0;     // no golomb words -> nothing written (989-990)
    return true;
}

__device__ inline void chunk_of(const Layout &L, uint32_t r, uint32_t &s, uint32_t &c) {
    s = 0;
    while (s < kStreams - 1 && r >= L.cpb[s]) { r -= L.cpb[s]; s++; }
    c = r;
}

// ---------------------------------------------------------------------------
// a chunk's workgroup: kEncT lanes of kSymL consecutive symbols (64 B per lane in flight:
// two waves per 8 KiB chunk, so a CU holds 16 chunks' loads at once)
constexpr uint32_t kEncT = 128;
constexpr uint32_t kSymL = kChunk / kEncT;   // 64
constexpr uint32_t kSymW = kSymL / 4;        // 16 words
static_assert(kSymL % 16 == 0, "whole 16-B loads");
static_assert(kSymL == kCharSeg, "one chars segment descriptor per lane");

__device__ inline uint32_t chunk_symbols(const uint32_t *w4, uint32_t i0, uint32_t i1, uint32_t *out32 /*kSymW words*/) {
    // loads the (up to) kSymL symbols [i0, i1) as 16-B loads, all in flight together (i0 is
    // a multiple of kSymL and stream strides are multiples of 16; a read past a block's
    // stream lands in the next block's stride or the 64 B of slack at the buffer end),
    // bytes past i1 zeroed
    const uint32_t n = i1 > i0 ? i1 - i0 : 0;
    if (n == 0) {
#pragma unroll
        for (uint32_t q = 0; q < kSymW; q++) out32[q] = 0;
        return 0;
    }
    const uint4 *p = (const uint4 *)(w4 + (i0 >> 2));
    uint4 v[kSymW / 4];
#pragma unroll
    for (uint32_t q = 0; q < kSymW / 4; q++) v[q] = p[q];
#pragma unroll
    for (uint32_t q = 0; q < kSymW / 4; q++) {
        out32[4 * q] = v[q].x; out32[4 * q + 1] = v[q].y; out32[4 * q + 2] = v[q].z; out32[4 * q + 3] = v[q].w;
    }
    if (n < kSymL)
#pragma unroll
        for (uint32_t q = 0; q < kSymW; q++) {
            const uint32_t lo = 4 * q;
            out32[q] = lo >= n ? 0u : (n - lo >= 4 ? out32[q] : out32[q] & ((1u << (8 * (n - lo))) - 1u));
        }
    return n;
}

// the same symbols where the lane's chars segment is a run of input bytes (k_emit's descriptor):
// bytes p[i0, i1) at any alignment.  A whole segment is four unaligned 16-B loads (gfx950 global
// loads take any byte address; the compiler emits the same for a byte-aligned copy); a short one
// (the stream's last) reads its bytes one by one, so nothing past p[i1 - 1] is touched
__device__ inline uint32_t input_symbols(const uint8_t *p, uint32_t i0, uint32_t i1, uint32_t *out32 /*kSymW words*/) {
    const uint32_t n = i1 > i0 ? i1 - i0 : 0;
    if (n == kSymL) {
#pragma unroll
        for (uint32_t q = 0; q < kSymW / 4; q++) {
            uint4 v;
            __builtin_memcpy(&v, p + i0 + 16 * q, 16);
            out32[4 * q] = v.x; out32[4 * q + 1] = v.y; out32[4 * q + 2] = v.z; out32[4 * q + 3] = v.w;
        }
        return n;
    }
#pragma unroll
    for (uint32_t q = 0; q < kSymW; q++) out32[q] = 0;
    for (uint32_t j = 0; j < n; j++) out32[j >> 2] |= (uint32_t)p[i0 + j] << (8 * (j & 3));
    return n;
}

__device__ inline const uint8_t *stream_base(const Layout &L, uint32_t s, uint32_t b, const uint8_t *s0,
                                             const uint8_t *s1, const uint8_t *s2, const uint8_t *s3) {
    return (s == 0 ? s0 : s == 1 ? s1 : s == 2 ? s2 : s3) + (uint64_t)b * L.sstride[s];
}

// ---------------------------------------------------------------------------
constexpr uint32_t kTreeT = 256;   // k_tree workgroup: four waves (the chars rows are summed by all of them; the merge is serial)
constexpr uint32_t kTreeW = kTreeT / 64;
constexpr uint32_t kJacobiMin = 64, kJacobiMax = 40;   // k_tree: merges solved as a fixed point
static_assert(kTreeW * 256 >= 2 * 512, "the fixed point's P arrays in the weights scratch");

// kDev = true carries development timing exits (fcx_debug_emit_bits bits 16..19; the compress stops
// after this kernel while they are set); the product launches k_tree<false>
template <bool kDev>
__global__ __launch_bounds__(kTreeT) void k_tree(Layout L, const uint16_t *__restrict__ thist, const uint8_t *__restrict__ s0,
                                                 const uint8_t *__restrict__ s2, const uint8_t *__restrict__ s3,
                                                 BlockInfo *__restrict__ binfo, uint32_t *__restrict__ ctab,
                                                 uint8_t *__restrict__ ltab, uint8_t *__restrict__ hhdr,
                                                 uint64_t *__restrict__ cstat, uint32_t *__restrict__ err,
                                                 uint32_t dbg_in) {
    const uint32_t dbg = kDev ? dbg_in : 0u;
    __shared__ __attribute__((aligned(16))) uint32_t w[256];
    // one region, two lives: the stream byte counts (u16 x 16 lane slots per byte value) while the
    // flag / distance / golomb bytes are counted, then the leaf queue, merge and code arrays
    __shared__ __attribute__((aligned(16))) uint32_t big[256 * 16];
    uint32_t *sw = big, *ss = big + 260, *ln = big + 520, *iw = big + 776, *il = big + 1032, *ir = big + 1288;
    uint32_t *par = big + 1544, *sk = big + 2056;   // (sk 16-B aligned: 2056 = 4 x 514)
    uint32_t (*part)[256] = (uint32_t (*)[256])(big + 2312);   // chars rows (the chars stream only)
    __shared__ uint32_t s_red[kTreeW];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t b = blockIdx.x / kStreams, s = blockIdx.x % kStreams;
    BlockInfo &bi = binfo[b];
    // (the record's fields this prologue tests, read together before its first branch)
    const uint32_t lazy_tiles = bi.lazy_tiles, slen0 = bi.slen[0], gbits = bi.gbits;
    asm volatile("" ::"s"(lazy_tiles), "s"(slen0), "s"(gbits));
    // the call's lazy tiles (k_stitch walked them serially), for the routing of later calls
    // (fcx_capi.hip: a unit that left tiles lazy is launched over its list, where hand-ons work)
    if (s == 0 && tid == 0 && lazy_tiles) atomicAdd(err + 2, lazy_tiles);
    if (s == 0 ? slen0 <= 1 : s == 3 ? gbits == 0 : false) {   // (stream_active)
        if (tid == 0) { bi.hdrlen[s] = 0; bi.nwords[s] = 0; }
        return;
    }
    const uint32_t hb = (b * kStreams + s) * 256;
    uint32_t r0 = 0;
    for (uint32_t q = 0; q < s; q++) r0 += L.cpb[q];
    for (uint32_t c = tid; c < 2 * L.cpb[s]; c += kTreeT) cstat[2 * ((uint64_t)b * L.cpb_total + r0) + c] = 0;   // k_encode's look-back
    const uint32_t ntl = (bi.len + kTile - 1) / kTile;
    if (s == 1) {   // chars: wave wv sums the tile rows t = wv mod kTreeW (lane: symbols 4 lane .. 4 lane + 3)
        const uint2 *rows = (const uint2 *)(thist + (uint64_t)b * L.tpb * 256);
        uint32_t acc[4] = {0, 0, 0, 0};
#pragma unroll 16
        for (uint32_t t = wv; t < ntl; t += kTreeW) {
            const uint2 v = rows[(uint64_t)t * 64 + lane];
            acc[0] += v.x & 0xFFFFu; acc[1] += v.x >> 16; acc[2] += v.y & 0xFFFFu; acc[3] += v.y >> 16;
        }
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) part[wv][4 * lane + q] = acc[q];
        __syncthreads();
#pragma unroll
        for (uint32_t u = 0; u < 256 / kTreeT; u++) {
            const uint32_t sym = tid + kTreeT * u;
            uint32_t t = 0;
#pragma unroll
            for (uint32_t q = 0; q < kTreeW; q++) t += part[q][sym];
            w[sym] = t;
        }
    } else {
        // flags / distances / golomb words: the stream's slen bytes, counted straight from the
        // finished stream (the bits past the stream's last one are zero: k_stitch cleared the words
        // k_emit ORs into, so the (11 pCnt)/8 + 1-th byte (2192) and the golomb words' tails count
        // as the zeros the reference counts).  Zero and 0xFF bytes (runs of flags and unary golomb
        // codes) are counted in registers, the rest by LDS atomics
        const uint8_t *sb = (s == 0 ? s0 : s == 2 ? s2 : s3) + (uint64_t)b * L.sstride[s];
        const uint32_t nby = bi.slen[s], nq = nby / 16;
        // byte value by counts into word 16 by + (lane & 15), half (lane >> 4) & 1: the 32 lanes of a
        // bank group add to 32 different banks (random bytes no longer pile onto a few banks); 8 lanes
        // share a u16 counter, at most slen / 32 < 2^16 bytes (slen < 2 MiB)
        for (uint32_t x = tid; x < 256 * 16 / 4; x += kTreeT) ((uint4 *)big)[x] = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
        uint32_t c00 = 0, cff = 0;
        const uint32_t slot = lane & 15u, inc = 1u << (16 * ((lane >> 4) & 1u));
        auto count4 = [&](uint32_t v, uint32_t nb) {
#pragma unroll
            for (uint32_t q = 0; q < 4; q++) {
                const uint32_t by = (v >> (8 * q)) & 0xFFu;
                if (q >= nb) break;
                if (by == 0) c00++;
                else if (by == 0xFFu) cff++;
                else atomicAdd(&big[16 * by + slot], inc);
            }
        };
        const uint4 *s4 = (const uint4 *)sb;   // (stream strides are multiples of 16)
        constexpr uint32_t kDeep = 8;          // 16-B loads in flight per lane (text distances: ~200 KB a block)
        for (uint32_t q0 = 0; q0 < nq; q0 += kDeep * kTreeT) {
            uint4 v[kDeep];
#pragma unroll
            for (uint32_t u = 0; u < kDeep; u++) {
                const uint32_t q = q0 + tid + kTreeT * u;
                v[u] = q < nq ? s4[q] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (uint32_t u = 0; u < kDeep; u++) {
                const uint32_t nb = q0 + tid + kTreeT * u < nq ? 4u : 0u;
                count4(v[u].x, nb); count4(v[u].y, nb); count4(v[u].z, nb); count4(v[u].w, nb);
            }
        }
        if (tid < nby - 16 * nq) count4(sb[16 * nq + tid], 1);
        c00 = wave_sum_u32(c00);
        cff = wave_sum_u32(cff);
        __syncthreads();
        {   // byte tid's count: its 16 words, both halves
            const uint4 *r4 = (const uint4 *)(big + 16 * tid);
            uint32_t t = 0;
#pragma unroll
            for (uint32_t q = 0; q < 4; q++) {
                const uint4 v4 = r4[q];
                t += (v4.x & 0xFFFFu) + (v4.x >> 16) + (v4.y & 0xFFFFu) + (v4.y >> 16) + (v4.z & 0xFFFFu) + (v4.z >> 16) +
                     (v4.w & 0xFFFFu) + (v4.w >> 16);
            }
            w[tid] = t;
        }
        __syncthreads();
        if (lane == 0) { atomicAdd(&w[0], c00); atomicAdd(&w[0xFF], cff); }
        __syncthreads();
    }
    if (dbg & 1u) { if (w[tid] == 0x12345u) err[1] = 1; return; }   // (timing: weights only)
    uint32_t nz = 0;
#pragma unroll
    for (uint32_t u = 0; u < 256 / kTreeT; u++) nz += w[tid + kTreeT * u] != 0 ? 1u : 0u;
    const uint32_t real = (uint32_t)__syncthreads_count(nz >= 1) + (uint32_t)__syncthreads_count(nz >= 2);
    // stable sort of the leaves by (weight, symbol): rank = number of smaller keys.  A weight is at
    // most the block size (<= 2^20 symbols), so weight << 8 | symbol fits 32 bits
#pragma unroll
    for (uint32_t u = 0; u < 256 / kTreeT; u++) {
        const uint32_t sym = tid + kTreeT * u, wt = w[sym];
        sk[sym] = wt ? (wt << 8) | sym : 0xFFFFFFFFu;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < 256 / kTreeT; u++) {
        const uint32_t sym = tid + kTreeT * u, key = sk[sym];
        if (key != 0xFFFFFFFFu) {
            uint32_t rank = 0;
#pragma unroll 4
            for (uint32_t j = 0; j < 256; j += 4) {
                const uint4 k4 = *(const uint4 *)&sk[j];
                rank += (k4.x < key ? 1u : 0u) + (k4.y < key ? 1u : 0u) + (k4.z < key ? 1u : 0u) + (k4.w < key ? 1u : 0u);
            }
            sw[rank] = key >> 8;
            ss[rank] = sym;
        }
    }
    __syncthreads();
    if (dbg & 2u) { if (sw[tid] == 0x12345u) err[1] = 1; return; }   // (timing: + rank sort)
    const uint32_t nint = real >= 2 ? real - 1 : 0;
    // When the two lightest leaves outweigh the heaviest (w0 + w1 > w_max: the chars of random data),
    // every internal node outweighs every leaf, so the leaves are consumed first, in pairs, and the
    // sequence S = sorted leaves, then internal nodes in creation order, is nondecreasing (node k =
    // S[2k] + S[2k+1] >= S[2k-2] + S[2k-1] = node k-1): the merge takes S[2k] (left) and S[2k+1]
    // (right) at step k, a closed form every thread evaluates for its own nodes
    const bool fifo = nint && sw[0] + sw[1] > sw[real - 1];
    if (fifo) {
        for (uint32_t kk = tid; kk < nint; kk += kTreeT) {
            const uint32_t a = 2 * kk, c = 2 * kk + 1;
            const uint32_t id0 = a < real ? ss[a] : 256 + (a - real), id1 = c < real ? ss[c] : 256 + (c - real);
            il[kk] = id0;
            ir[kk] = id1;
            par[id0] = 256 + kk;
            par[id1] = 256 + kk;
        }
    }
    // Otherwise a long merge (>= kJacobiMin internal nodes) is solved as a fixed point, all threads
    // at once: the picks P are the sorted merge of the leaves L and the internal weights I (a leaf
    // first on a tie) and I[k] = P[2k] + P[2k+1].  From I = infinity, each round ranks every leaf and
    // internal node into P by binary search and recomputes I; I only decreases towards the merge's
    // (I[0] is right after one round, and I[k] is right one round after every node P[0..2k+1] uses),
    // and the measured histograms settle in 8-15 rounds.  Past kJacobiMax rounds, or for short
    // merges, one thread runs the two-queue merge below.
    bool merged = fifo;
    if (!fifo && nint >= kJacobiMin) {
        constexpr uint32_t kInf = 0xFFFFFFFFu;
        uint32_t *pw = &part[0][0], *pid = &part[2][0];   // P's weights and ids (the weights phase is over)
        for (uint32_t kk = tid; kk < nint; kk += kTreeT) iw[kk] = kInf;
        __syncthreads();
        for (uint32_t it = 0; it < kJacobiMax && !merged; it++) {
            for (uint32_t t = tid; t < real; t += kTreeT) {   // leaf t: after the internal nodes lighter than it
                const uint32_t wl = sw[t];
                uint32_t lo = 0, hi = nint;
                while (lo < hi) { const uint32_t md = (lo + hi) >> 1; if (iw[md] < wl) lo = md + 1; else hi = md; }
                pw[t + lo] = wl;
                pid[t + lo] = ss[t];
            }
            for (uint32_t j = tid; j < nint; j += kTreeT) {   // internal j: after the leaves no heavier than it
                const uint32_t wi = iw[j];
                uint32_t lo = 0, hi = real;
                while (lo < hi) { const uint32_t md = (lo + hi) >> 1; if (sw[md] <= wi) lo = md + 1; else hi = md; }
                pw[j + lo] = wi;
                pid[j + lo] = 256 + j;
            }
            __syncthreads();
            bool ch = false;
            for (uint32_t kk = tid; kk < nint; kk += kTreeT) {
                const uint32_t a = pw[2 * kk], c = pw[2 * kk + 1];
                const uint32_t nv = (a == kInf || c == kInf) ? kInf : a + c;
                ch = ch || nv != iw[kk];
                iw[kk] = nv;   // (read by the other threads only after the barrier below)
            }
            merged = __syncthreads_or(ch ? 1 : 0) == 0;
        }
        if (merged)
            for (uint32_t kk = tid; kk < nint; kk += kTreeT) {
                const uint32_t id0 = pid[2 * kk], id1 = pid[2 * kk + 1];
                il[kk] = id0;
                ir[kk] = id1;
                par[id0] = 256 + kk;
                par[id1] = 256 + kk;
            }
    }
    if (!merged && tid == 0 && nint) {
        // two-queue merge == the reference's sorted-list re-insertion (570-611).  Each step
        // reads both queue heads two deep at once (one LDS round trip per step)
        uint32_t lq = 0, iq = 0;
        for (uint32_t kk = 0; kk < nint; kk++) {
            const uint32_t L0 = sw[lq], L1 = sw[lq + 1], S0 = ss[lq], S1 = ss[lq + 1];
            const uint32_t I0 = iw[iq], I1 = iw[iq + 1];
            uint32_t id0, w0, id1, w1;
            if (lq < real && (iq >= kk || L0 <= I0)) {   // first: leaf
                id0 = S0; w0 = L0;
                if (lq + 1 < real && (iq >= kk || L1 <= I0)) { id1 = S1; w1 = L1; lq += 2; }
                else { id1 = 256 + iq; w1 = I0; lq += 1; iq += 1; }
            } else {                                      // first: internal node
                id0 = 256 + iq; w0 = I0;
                if (lq < real && (iq + 1 >= kk || L0 <= I1)) { id1 = S0; w1 = L0; lq += 1; iq += 1; }
                else { id1 = 256 + iq + 1; w1 = I1; iq += 2; }
            }
            iw[kk] = w0 + w1;
            il[kk] = id0;
            ir[kk] = id1;
            par[id0] = 256 + kk;
            par[id1] = 256 + kk;
        }
    }
    __syncthreads();
    if (dbg & 4u) { if (iw[tid] == 0x12345u) err[1] = 1; return; }   // (timing: + merge)
    const uint32_t root = 256 + nint - 1;
    uint32_t bits = 0;   // this thread's symbols' share of the stream's code bits
#pragma unroll
    for (uint32_t u = 0; u < 256 / kTreeT; u++) {   // code of a symbol: root -> leaf path, root decision in bit 0
        const uint32_t sym = tid + kTreeT * u;
        uint32_t code = 0, len = 0;
        if (nint && w[sym]) {
            uint32_t cur = sym;
            while (cur != root && len <= 32) {
                const uint32_t p = par[cur];
                code = (code << 1) | (ir[p - 256] == cur ? 1u : 0u);
                len++;
                cur = p;
            }
            if (len > 32) atomicOr(err, kErrCodeLen);
        }
        ctab[hb + sym] = code;
        ltab[hb + sym] = (uint8_t)len;
        ln[sym] = len;
        bits += w[sym] * len;
    }
    if (dbg & 8u) { if (bits == 0x12345u) err[1] = 1; return; }   // (timing: + codes)
    const uint32_t wsum = wave_sum_u32(bits);
    if (lane == 0) s_red[wv] = wsum;
    __syncthreads();
    uint64_t carry = 0;
    for (uint32_t q = 0; q < kTreeW; q++) carry += s_red[q];
    // header: [u8 ts][ceil(2ts/8) B internal-child bitmap][ts x (u8 l, u8 r)]
    const uint32_t ts = nint, nbm = (2 * ts + 7) / 8;
    uint8_t *hdr = hhdr + (uint64_t)(b * kStreams + s) * kHuffHdrStride;
    if (tid == 0) hdr[0] = (uint8_t)ts;
    if (tid < nbm) {
        uint32_t byte = 0;
        for (uint32_t q = 0; q < 8; q++) {
            const uint32_t node = (8 * tid + q) >> 1;
            if (node < ts) {
                const uint32_t ch = (q & 1) ? ir[node] : il[node];
                if (ch >= 256) byte |= 1u << q;
            }
        }
        hdr[1 + tid] = (uint8_t)byte;
    }
    for (uint32_t kk = tid; kk < ts; kk += kTreeT) {
        const uint32_t l = il[kk], r = ir[kk];
        hdr[1 + nbm + 2 * kk] = (uint8_t)(l >= 256 ? (256 - real) + (l - 256) : l);
        hdr[1 + nbm + 2 * kk + 1] = (uint8_t)(r >= 256 ? (256 - real) + (r - 256) : r);
    }
    if (tid == 0) {
        bi.hdrlen[s] = 1 + nbm + 2 * ts;
        bi.nwords[s] = (uint32_t)((carry + 31) / 32);
    }
}

// ---------------------------------------------------------------------------
// record layout of one block: offsets relative to the record start
struct RecLayout {
    uint32_t hdr_rel[kStreams];    // tree header (or raw flag bytes for s=0 when not Huffman-coded)
    uint32_t words_rel[kStreams];  // first code word
    uint32_t n_rel, pcnt_rel, g_rel, rec_bytes;
};

__device__ inline RecLayout record_layout(const BlockInfo &bi) {
    RecLayout R;
    uint32_t o = 4;          // u32 payload length (written by main(), 4112)
    R.n_rel = o; o += 4;     // u32 N (2137-2139)
    for (uint32_t s = 0; s < kStreams; s++) {
        if (s == 2) { R.pcnt_rel = o; o += 4; }  // u32 pCnt (2187-2189)
        if (s == 3) { R.g_rel = o; o += 4; }     // u32 golombLen (2226-2228)
        R.hdr_rel[s] = o;
        if (s == 0 && bi.slen[0] <= 1) {          // raw flag byte(s) (2103-2107)
            R.words_rel[0] = o;
            o += bi.slen[0];
        } else if (s == 3 && bi.gbits == 0) {
            R.words_rel[3] = o;
        } else {
            o += bi.hdrlen[s];
            o += 4;          // u32 W
            R.words_rel[s] = o;
            o += 4 * bi.nwords[s];
        }
    }
    R.rec_bytes = o;
    return R;
}

__global__ __launch_bounds__(64) void k_block_layout(uint32_t nblocks, BlockInfo *__restrict__ binfo) {
    const uint32_t b = blockIdx.x * 64 + threadIdx.x;
    if (b >= nblocks) return;
    BlockInfo &bi = binfo[b];
    const RecLayout R = record_layout(bi);
    for (uint32_t s = 0; s < kStreams; s++) bi.words_rel[s] = R.words_rel[s];
    bi.rec_bytes = R.rec_bytes;
}

__global__ __launch_bounds__(1024) void k_scan_blocks(uint32_t nblocks, const BlockInfo *__restrict__ binfo,
                                                      uint64_t *__restrict__ blk_off, uint64_t *__restrict__ total,
                                                      uint64_t cap, uint32_t *__restrict__ err) {
    __shared__ uint64_t wsum[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // offsets continue after the records of the shard's earlier block groups (fcx_compress_shard's
    // pipelined launch: their scans ran before this one); 0 for the first group
    uint64_t carry = *total;
    for (uint32_t b0 = 0; b0 < nblocks; b0 += 1024) {
        const uint32_t b = b0 + tid;
        const uint64_t v = b < nblocks ? binfo[b].rec_bytes : 0;
        uint64_t inc = v;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t lo = __shfl_up((uint32_t)inc, o, 64), hi = __shfl_up((uint32_t)(inc >> 32), o, 64);
            if (lane >= (uint32_t)o) inc += ((uint64_t)hi << 32) | lo;
        }
        if (lane == 63) wsum[wv] = inc;
        __syncthreads();
        uint64_t pre = carry, all = carry;
        for (uint32_t q = 0; q < 16; q++) {
            if (q < wv) pre += wsum[q];
            all += wsum[q];
        }
        if (b < nblocks) blk_off[b] = pre + inc - v;
        carry = all;
        __syncthreads();
    }
    if (tid == 0) {
        *total = carry;
        if (carry > cap) atomicOr(err, kErrCapacity);
    }
}

// staging words: the whole chunk at <= 8 bits per symbol (one pass; random data's chars
// are exactly 8); longer codes (<= 32 bits) go through several windows of this size
constexpr uint32_t kEncWords = kChunk / 4 + 2;

// k_encode's decoupled look-back: two words per chunk, cleared by k_tree.  [0] status: flag
// (bit 62: aggregate = this chunk's bit count, bit 63: inclusive prefix = the stream's bits
// through this chunk) | count; [1] the chunk's last 32 code bits | bit 63 once published (the
// next chunk merges them into the word the two share)
constexpr uint64_t kStAgg = 1ull << 62, kStInc = 2ull << 62, kStTail = 1ull << 63;
__device__ inline uint64_t st_word(uint64_t flag, uint32_t v) { return flag | (v & 0x3FFFFFFFu); }

// the chunk's last 32 code bits (staged bits [e - 32, e), e >= 32) for the next chunk
__device__ inline void publish_tail(uint64_t *st, const uint32_t *ws, uint32_t e) {
    const uint32_t lo = ws[(e - 32) >> 5], hi = ws[(e - 1) >> 5];
    const uint32_t tail = (uint32_t)((((uint64_t)hi << 32) | lo) >> ((e - 32) & 31));
    __hip_atomic_store(st + 1, kStTail | tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the first output word: the previous chunk's last sh0 bits below this chunk's first bits
// (waits for the previous chunk's tail; it publishes right after staging its words)
__device__ inline void merge_head(uint64_t *st, uint32_t *o32, uint32_t w0v, uint32_t sh0) {
    uint64_t t;
    do t = __hip_atomic_load(st - 2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (!(t & kStTail));
    o32[0] = w0v | ((uint32_t)t >> (32 - sh0));
}

__global__ __launch_bounds__(kEncT) __attribute__((amdgpu_waves_per_eu(8))) void k_encode(Layout L, const BlockInfo *__restrict__ binfo,
                                                 const uint8_t *__restrict__ s0, const uint8_t *__restrict__ s1,
                                                 const uint8_t *__restrict__ s2, const uint8_t *__restrict__ s3,
                                                 const uint32_t *__restrict__ ctab, const uint8_t *__restrict__ ltab,
                                                 uint64_t *__restrict__ cstat,
                                                 const uint64_t *__restrict__ blk_off, uint8_t *__restrict__ out,
                                                 const uint32_t *__restrict__ err, const uint8_t *__restrict__ in,
                                                 const uint32_t *__restrict__ sdesc) {
    constexpr uint32_t kW = kEncT / 64;
    __shared__ uint32_t ct[256], lt[256];
    __shared__ uint32_t ws[kEncWords];
    __shared__ uint32_t red[kW];
    __shared__ uint32_t s_pre;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t b = blockIdx.x / L.cpb_total, r = blockIdx.x % L.cpb_total;
    uint32_t s, c;
    chunk_of(L, r, s, c);
    // loads in two rounds: error word + block info, then everything else at once
    const uint32_t errv = *err;
    const BlockInfo &bi = binfo[b];
    // chars: is this lane's segment a run of input bytes (k_emit's descriptor)?
    // (the last chunk of a block whose size is not a multiple of kChunk has lanes past the block's
    // descriptors: they hold no symbols and read none)
    const uint32_t nseg = (L.B + kCharSeg - 1) / kCharSeg, seg = c * (kChunk / kCharSeg) + tid;
    const uint32_t cd = s == 1 && seg < nseg ? sdesc[(uint64_t)b * nseg + seg] : kCdMixed;
    const uint32_t len = bi.slen[s], c0 = c * kChunk;
    if (errv || !stream_active(bi, s) || c0 >= len) return;
    const uint32_t c1 = min(len, c0 + kChunk);
    const bool lastc = c1 == len;   // the stream's last chunk
    const uint32_t hb = (b * kStreams + s) * 256;
    uint32_t ctv[256 / kEncT], ltv[256 / kEncT];
#pragma unroll
    for (uint32_t u = 0; u < 256 / kEncT; u++) { ctv[u] = ctab[hb + tid + kEncT * u]; ltv[u] = ltab[hb + tid + kEncT * u]; }
    const uint8_t *base = (s == 0 ? s0 : s == 1 ? s1 : s == 2 ? s2 : s3) + (uint64_t)b * L.sstride[s];
    const uint32_t i0 = c0 + kSymL * tid, i1 = min(c1, i0 + kSymL);
    uint32_t sym[kSymW];
    const uint32_t n = cd != kCdMixed ? input_symbols(in + (uint64_t)b * L.B + cd, i0, i1, sym)
                                      : chunk_symbols((const uint32_t *)base, i0, i1, sym);
    const uint32_t n_chunk = c1 - c0;
    const uint64_t obyte = blk_off[b] + bi.words_rel[s];
    uint64_t *st = cstat + 2 * ((uint64_t)b * L.cpb_total + r);   // this chunk's words; st[-2k]: k chunks back
    bool all8 = true;
#pragma unroll
    for (uint32_t u = 0; u < 256 / kEncT; u++) {
        ct[tid + kEncT * u] = ctv[u];
        lt[tid + kEncT * u] = ltv[u];
        all8 = all8 && ltv[u] == 8;
    }
    // all 256 symbols with 8-bit codes (the chars of random data): the code stream is a
    // byte substitution
    const bool byte8 = __syncthreads_and(all8) != 0;
    if (byte8) {
        // every symbol of the stream is 8 bits: the chunk starts 8 c0 bits into the stream (no
        // look-back), and its bytes are a substitution.  Whole words inside the chunk are plain
        // stores; a word shared with the previous or next chunk gets this chunk's bytes only
        // (byte stores), so no chunk waits for a neighbour.  The stream's last chunk writes
        // whole words through the stream's W code words (zeros past the codes, 849-928; the
        // bytes after them belong to headers that k_headers writes later).
        const uint32_t T = 8 * n_chunk;
        const uint64_t g0 = 8 * obyte + 8ull * c0;
        const uint32_t sh0 = (uint32_t)(g0 & 31);
        const uint32_t nw = (sh0 + T + 31) >> 5;
        uint32_t *o32 = (uint32_t *)out + (g0 >> 5);
        for (uint32_t x = tid; x < nw; x += kEncT) ws[x] = 0u;
        uint32_t v[kSymW + 1];
#pragma unroll
        for (uint32_t q = 0; q < kSymW; q++) {
            const uint32_t w = sym[q];
            v[q] = ct[w & 0xFF] | (ct[(w >> 8) & 0xFF] << 8) | (ct[(w >> 16) & 0xFF] << 16) | (ct[w >> 24] << 24);
            if (4 * q >= n) v[q] = 0;
            else if (n - 4 * q < 4) v[q] &= (1u << (8 * (n - 4 * q))) - 1u;
        }
        // this lane's bytes start at staging byte sh0/8 + kSymL tid: shift into kSymW + 1
        // words, the first and last two shared with the neighbouring lanes
        const uint32_t bo = (sh0 >> 3) + kSymL * tid, sb = 8 * (bo & 3), w0 = bo >> 2;
        v[kSymW] = 0;
        __syncthreads();
        if (n) {
            uint32_t prev = 0;
#pragma unroll
            for (uint32_t q = 0; q <= kSymW; q++) {
                const uint32_t cur = v[q];
                const uint32_t o = sb ? (cur << sb) | (prev >> (32 - sb)) : cur;
                prev = cur;
                if (q == 0 || q >= kSymW - 1) { if (o) atomicOr(&ws[w0 + q], o); }
                else ws[w0 + q] = o;
            }
        }
        __syncthreads();
        const uint32_t e = sh0 + T;   // end bit in the staging
        const uint32_t nst = lastc ? (uint32_t)(((8 * obyte + 32ull * bi.nwords[s] - 1) >> 5) - (g0 >> 5) + 1) : nw;
        const uint32_t xa = sh0 ? 1u : 0u;                                     // first whole word
        const uint32_t xz = lastc ? nst : ((e & 31) ? nw - 1 : nw);           // end of whole words
        for (uint32_t x = xa + tid; x < xz; x += kEncT) o32[x] = x < nw ? ws[x] : 0u;
        // edge words: bytes [sh0/8, 4) of word 0, bytes [0, (e & 31)/8) of word nw - 1
        uint8_t *o8 = (uint8_t *)o32;
        if (tid < 4) {
            const uint32_t q = tid;
            // word 0 shared with the previous chunk (or the record's header bytes): bytes from sh0/8
            // (a one-word chunk that is not the stream's last: only up to its end)
            if (sh0 && q >= (sh0 >> 3) && (lastc || nw > 1 || 8 * q < e)) o8[q] = (uint8_t)(ws[0] >> (8 * q));
            // the last word shared with the next chunk: bytes below the end bit
            if (!lastc && (e & 31) && !(nw == 1 && sh0) && 8 * q < (e & 31))
                o8[4 * (nw - 1) + q] = (uint8_t)(ws[nw - 1] >> (8 * q));
        }
        return;
    }
    // ---- this chunk's bit count and this lane's bit offset in it
    uint32_t nb = 0;
    for (uint32_t q = 0; q < n; q++) nb += lt[(sym[q >> 2] >> (8 * (q & 3))) & 0xFF];
    const uint32_t inc = wave_incl_scan(nb);
    if (lane == 63) red[wv] = inc;
    __syncthreads();
    uint32_t tb = inc - nb, T = 0;
    for (uint32_t q = 0; q < kW; q++) {
        if (q < wv) tb += red[q];
        T += red[q];
    }
    if (T == 0) return;   // one symbol in the stream: no code bits (W = 0)
    // ---- decoupled look-back (wave 0): the stream's bits before this chunk
    if (wv == 0) {
        uint32_t excl = 0;
        if (c == 0) {
            if (lane == 0) __hip_atomic_store(st, st_word(kStInc, T), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0) __hip_atomic_store(st, st_word(kStAgg, T), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            uint32_t back = 1;   // lane i reads the chunk back + i places back
            for (;;) {
                const bool have = back + lane <= c;
                const uint64_t v = have ? __hip_atomic_load(st - 2 * (back + lane), __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT)
                                        : kStInc;   // before the stream: an inclusive 0
                const uint64_t rdy = __ballot((v >> 62) != 0), incm = __ballot((v >> 62) == 2);
                const uint32_t fnr = ~rdy ? (uint32_t)__builtin_ctzll(~rdy) : 64u;   // first lane not ready
                const uint32_t fin = incm ? (uint32_t)__builtin_ctzll(incm) : 64u;   // first inclusive prefix
                const uint32_t upto = fin < fnr ? fin + 1 : fnr;   // lanes whose counts are summed now
                excl += wave_sum_u32(lane < upto ? (uint32_t)v & 0x3FFFFFFFu : 0u);
                if (fin < fnr) break;
                back += fnr;   // (fnr == 0: the previous chunk has not published yet; poll again)
            }
            if (lane == 0) __hip_atomic_store(st, st_word(kStInc, excl + T), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) s_pre = excl;
    }
    __syncthreads();
    const uint64_t g0 = 8 * obyte + s_pre;   // first bit of this chunk in the output
    const uint32_t sh0 = (uint32_t)(g0 & 31);
    // the word the previous chunk ends in is this chunk's to write: its low sh0 bits are the
    // previous chunk's last ones, merged in last (the record's header bytes, written later, for
    // a stream's first chunk)
    const bool merge = c > 0 && sh0 != 0;
    const uint32_t nw = (sh0 + T + 31) >> 5;
    // the last word: this chunk's to write only when it ends on a word boundary (else the next
    // chunk writes it, merged); the stream's last chunk writes through the end of the stream's
    // W code words (zero bits past its codes, 849-928: W = ceil(bits / 32))
    const uint32_t nst = lastc ? (uint32_t)(((8 * obyte + 32ull * bi.nwords[s] - 1) >> 5) - (g0 >> 5) + 1)
                               : (((sh0 + T) & 31) == 0 ? nw : nw - 1);
    uint32_t *o32 = (uint32_t *)out + (g0 >> 5);
    uint32_t w0v = 0;   // (thread 0) the first staged word, kept for the merge
    // this lane's codes cover bits [p0, p1) of the staging words; whole words inside
    // that range are this lane's alone (plain LDS stores), the two end words are shared.
    // Windows of kEncWords words: a lane writes the words of its range inside the window.
    const uint32_t p0 = sh0 + tb, p1 = p0 + nb;
    uint32_t prevlast = 0;   // the previous window's last word (a tail may straddle two windows)
    for (uint32_t wb = 0; wb < nw; wb += kEncWords) {
        const uint32_t we = min(nw, wb + kEncWords);
        if (wb) prevlast = ws[kEncWords - 1];
        __syncthreads();
        for (uint32_t x = tid; x < we - wb; x += kEncT) ws[x] = 0u;
        __syncthreads();
        if (nb && (p0 >> 5) < we && ((p1 - 1) >> 5) >= wb) {
            uint32_t wi = p0 >> 5, ap = p0 & 31;
            uint64_t acc = 0;
            for (uint32_t q = 0; q < n; q++) {
                const uint32_t sy = (sym[q >> 2] >> (8 * (q & 3))) & 0xFF;
                acc |= (uint64_t)ct[sy] << ap;
                ap += lt[sy];
                if (ap >= 32) {
                    if (wi >= wb && wi < we) {
                        if (32 * wi >= p0 && 32 * wi + 32 <= p1) ws[wi - wb] = (uint32_t)acc;
                        else atomicOr(&ws[wi - wb], (uint32_t)acc);
                    }
                    acc >>= 32;
                    ap -= 32;
                    wi++;
                    if (wi >= we) break;
                }
            }
            if (ap && wi >= wb && wi < we) atomicOr(&ws[wi - wb], (uint32_t)acc);
        }
        __syncthreads();
        if (tid == 0 && wb == 0) w0v = ws[0];
        if (!lastc && tid == 0 && we == nw) {   // the window holding the chunk's end: publish its last bits
            const uint32_t e = sh0 + T - 32 * wb;   // end bit inside this window
            if (e >= 32) publish_tail(st, ws, e);
            else __hip_atomic_store(st + 1, kStTail | (((uint64_t)ws[0] << 32 | prevlast) >> e), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
        }
        for (uint32_t x = wb + (wb == 0 && merge ? 1 : 0) + tid; x < min(we, nst); x += kEncT) o32[x] = ws[x - wb];
        __syncthreads();
    }
    for (uint32_t x = nw + tid; x < nst; x += kEncT) o32[x] = 0u;   // (the last chunk's zero tail)
    if (merge && tid == 0) merge_head(st, o32, w0v, sh0);
}

__device__ inline void put_bytes(uint8_t *dst, const uint8_t *src, uint32_t n, uint32_t lane) {
    for (uint32_t i = lane; i < n; i += 64) dst[i] = src[i];
}
__device__ inline void put_u32(uint8_t *dst, uint32_t v, uint32_t lane) {
    if (lane < 4) dst[lane] = (uint8_t)(v >> (8 * lane));
}

__global__ __launch_bounds__(64) void k_headers(const BlockInfo *__restrict__ binfo, const uint8_t *__restrict__ s0,
                                                uint32_t s0_stride, const uint8_t *__restrict__ hhdr,
                                                const uint64_t *__restrict__ blk_off, uint8_t *__restrict__ out,
                                                const uint32_t *__restrict__ err) {
    if (*err) return;
    const uint32_t lane = threadIdx.x, b = blockIdx.x;
    const BlockInfo &bi = binfo[b];
    const RecLayout R = record_layout(bi);
    uint8_t *rec = out + blk_off[b];
    put_u32(rec, R.rec_bytes - 4, lane);
    put_u32(rec + R.n_rel, bi.ntok, lane);
    put_u32(rec + R.pcnt_rel, bi.nmatch, lane);
    put_u32(rec + R.g_rel, (bi.gbits + 31) / 32, lane);
    for (uint32_t s = 0; s < kStreams; s++) {
        if (s == 0 && bi.slen[0] <= 1) {
            put_bytes(rec + R.hdr_rel[0], s0 + (uint64_t)b * s0_stride, bi.slen[0], lane);
            continue;
        }
        if (s == 3 && bi.gbits == 0) continue;
        const uint8_t *h = hhdr + (uint64_t)(b * kStreams + s) * kHuffHdrStride;
        put_bytes(rec + R.hdr_rel[s], h, bi.hdrlen[s], lane);
        put_u32(rec + R.hdr_rel[s] + bi.hdrlen[s], bi.nwords[s], lane);
    }
}

// ---------------------------------------------------------------------------
void launch_entropy(const Layout &L, BlockInfo *binfo, uint8_t *s0, uint8_t *s1, uint8_t *s2, uint8_t *s3,
                    const uint16_t *thist, uint32_t *ctab,
                    uint8_t *ltab, uint8_t *hhdr, uint64_t *cstat, uint64_t *blk_off, uint64_t *total, uint8_t *out,
                    uint64_t cap, uint32_t *err, const uint8_t *in, const uint32_t *sdesc, hipStream_t st, hipEvent_t *ev,
                    hipEvent_t wait_scan, hipEvent_t rec_scan, uint32_t tree_dbg) {
    const uint32_t nchunks = L.nblocks * L.cpb_total;
    if (ev) (void)hipEventRecord(ev[0], st);   // (the histograms are k_emit's: no stage of their own)
    if (tree_dbg) {   // (development: k_tree's timing exits; nothing after it runs)
        hipLaunchKernelGGL(k_tree<true>, dim3(L.nblocks * kStreams), dim3(kTreeT), 0, st, L, thist, s0, s2, s3, binfo,
                           ctab, ltab, hhdr, cstat, err, tree_dbg);
        if (ev)
            for (int q = 1; q <= 6; q++) (void)hipEventRecord(ev[q], st);
        return;
    }
    hipLaunchKernelGGL(k_tree<false>, dim3(L.nblocks * kStreams), dim3(kTreeT), 0, st, L, thist, s0, s2, s3, binfo, ctab,
                       ltab, hhdr, cstat, err, 0u);
    if (ev) (void)hipEventRecord(ev[1], st);
    hipLaunchKernelGGL(k_block_layout, dim3((L.nblocks + 63) / 64), dim3(64), 0, st, L.nblocks, binfo);
    if (ev) (void)hipEventRecord(ev[2], st);
    if (wait_scan) (void)hipStreamWaitEvent(st, wait_scan, 0);   // the previous group's record offsets
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, st, L.nblocks, binfo, blk_off, total, cap, err);
    if (rec_scan) (void)hipEventRecord(rec_scan, st);
    if (ev) (void)hipEventRecord(ev[3], st);
    if (ev) (void)hipEventRecord(ev[4], st);   // (no edge zeroing: k_encode stores every word whole)
    hipLaunchKernelGGL(k_encode, dim3(nchunks), dim3(kEncT), 0, st, L, binfo, s0, s1, s2, s3, ctab, ltab, cstat,
                       blk_off, out, err, in, sdesc);
    if (ev) (void)hipEventRecord(ev[5], st);
    hipLaunchKernelGGL(k_headers, dim3(L.nblocks), dim3(64), 0, st, binfo, s0, L.sstride[0], hhdr, blk_off, out, err);
    if (ev) (void)hipEventRecord(ev[6], st);
}

}  // namespace fcx
