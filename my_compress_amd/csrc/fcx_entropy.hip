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
//   k_hist         256-bin histogram of every 8192-symbol chunk (per-wave LDS
//                  bins, runs of equal bytes counted in registers first)
//   k_tree         sums a stream's chunk histograms, builds the tree, header
//                  bytes, code table, W, and every chunk's starting bit offset
//                  (chunk histogram . code lengths) - no second pass over the data
//   k_block_layout record layout and size per block
//   k_scan_blocks  record offsets across the shard (+ capacity check)
//   k_zero_edges   zero the words the encoder ORs into (the two edge words of every
//                  chunk; every other output byte is stored whole by k_encode or k_headers)
//   k_encode       each lane packs its 64 codes into whole words (LDS atomics only
//                  for the two words it shares with neighbours); the chunk's words
//                  are stored at the record's (unaligned) byte offset: interior
//                  words plain, chunk-edge words atomicOr
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

__device__ inline const uint8_t *stream_base(const Layout &L, uint32_t s, uint32_t b, const uint8_t *s0,
                                             const uint8_t *s1, const uint8_t *s2, const uint8_t *s3) {
    return (s == 0 ? s0 : s == 1 ? s1 : s == 2 ? s2 : s3) + (uint64_t)b * L.sstride[s];
}

__global__ __launch_bounds__(kEncT) void k_hist(Layout L, const BlockInfo *__restrict__ binfo,
                                                const uint8_t *__restrict__ s0, const uint8_t *__restrict__ s1,
                                                const uint8_t *__restrict__ s2, const uint8_t *__restrict__ s3,
                                                uint32_t *__restrict__ hist) {
    constexpr uint32_t kW = kEncT / 64;
    constexpr uint32_t kCopies = 4;   // sub-histograms per wave (lane & 3): fewer same-address atomics
    __shared__ uint32_t h[kW][kCopies][256];
    const uint32_t tid = threadIdx.x, wv = tid >> 6, cp = tid & (kCopies - 1);
    const uint32_t b = blockIdx.x / L.cpb_total;
    uint32_t s, c;
    chunk_of(L, blockIdx.x % L.cpb_total, s, c);
    const BlockInfo &bi = binfo[b];
    if (!stream_active(bi, s)) return;
    const uint32_t len = bi.slen[s], c0 = c * kChunk;
    if (c0 >= len) return;
    const uint32_t c1 = min(len, c0 + kChunk);
    // each lane counts a strip of kSymL consecutive symbols, runs of one byte value first
    const uint32_t i0 = c0 + kSymL * tid, i1 = min(c1, i0 + kSymL);
    uint32_t sym[kSymW];
    const uint32_t n = chunk_symbols((const uint32_t *)stream_base(L, s, b, s0, s1, s2, s3), i0, i1, sym);
    for (uint32_t x = tid; x < kW * kCopies * 256; x += kEncT) (&h[0][0][0])[x] = 0;
    __syncthreads();
    uint32_t cur = sym[0] & 0xFF, run = 0;
    for (uint32_t q = 0; q < n; q++) {
        const uint32_t v = (sym[q >> 2] >> (8 * (q & 3))) & 0xFF;
        if (v != cur) {
            atomicAdd(&h[wv][cp][cur], run);
            cur = v;
            run = 0;
        }
        run++;
    }
    if (run) atomicAdd(&h[wv][cp][cur], run);
    __syncthreads();
    for (uint32_t x = tid; x < 256; x += kEncT) {
        uint32_t t = 0;
#pragma unroll
        for (uint32_t w = 0; w < kW; w++)
#pragma unroll
            for (uint32_t c = 0; c < kCopies; c++) t += h[w][c][x];
        hist[(uint64_t)blockIdx.x * 256 + x] = t;
    }
}

// ---------------------------------------------------------------------------
constexpr uint32_t kTreeT = 128;   // k_tree workgroup: two waves (more trees per CU: the merge is serial)
constexpr uint32_t kTreeW = kTreeT / 64;

__global__ __launch_bounds__(kTreeT) void k_tree(Layout L, const uint32_t *__restrict__ hist,
                                                 BlockInfo *__restrict__ binfo, uint32_t *__restrict__ ctab,
                                                 uint8_t *__restrict__ ltab, uint8_t *__restrict__ hhdr,
                                                 uint32_t *__restrict__ chunk_off, uint32_t *__restrict__ err) {
    __shared__ __attribute__((aligned(16))) uint32_t w[256];
    __shared__ uint32_t sw[257], ss[257], ln[256];   // (the merge reads the leaf queue two deep)
    __shared__ uint32_t iw[256], il[256], ir[256], par[512];
    __shared__ uint32_t part[kTreeW][256];
    __shared__ uint32_t s_red[kTreeW];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t b = blockIdx.x / kStreams, s = blockIdx.x % kStreams;
    BlockInfo &bi = binfo[b];
    if (!stream_active(bi, s)) {
        if (tid == 0) { bi.hdrlen[s] = 0; bi.nwords[s] = 0; }
        return;
    }
    const uint32_t hb = (b * kStreams + s) * 256;
    uint32_t r0 = 0;
    for (uint32_t q = 0; q < s; q++) r0 += L.cpb[q];
    const uint32_t nch = (bi.slen[s] + kChunk - 1) / kChunk;
    const uint32_t *hc = hist + ((uint64_t)b * L.cpb_total + r0) * 256;   // this stream's chunk histograms
    {   // symbol weights: wave wv sums the chunks c = wv mod kTreeW (lane: symbols lane + 64 q)
        uint32_t acc[4] = {0, 0, 0, 0};
#pragma unroll 8
        for (uint32_t c = wv; c < nch; c += kTreeW)
#pragma unroll
            for (uint32_t q = 0; q < 4; q++) acc[q] += hc[c * 256 + lane + 64 * q];
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) part[wv][lane + 64 * q] = acc[q];
    }
    __syncthreads();
    uint32_t nz = 0;
#pragma unroll
    for (uint32_t u = 0; u < 256 / kTreeT; u++) {
        const uint32_t sym = tid + kTreeT * u;
        uint32_t t = 0;
#pragma unroll
        for (uint32_t q = 0; q < kTreeW; q++) t += part[q][sym];
        w[sym] = t;
        nz += t != 0 ? 1u : 0u;
    }
    const uint32_t real = (uint32_t)__syncthreads_count(nz >= 1) + (uint32_t)__syncthreads_count(nz >= 2);
    // stable sort of the leaves by (weight, symbol): rank = number of smaller keys
#pragma unroll
    for (uint32_t u = 0; u < 256 / kTreeT; u++) {
        const uint32_t sym = tid + kTreeT * u, wt = w[sym];
        if (wt) {
            const uint64_t key = ((uint64_t)wt << 8) | sym;
            uint32_t rank = 0;
            for (uint32_t j = 0; j < 256; j += 4) {
                const uint4 w4 = *(const uint4 *)&w[j];
                const uint32_t wj[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
                for (uint32_t v = 0; v < 4; v++)
                    rank += (wj[v] != 0 && (((uint64_t)wj[v] << 8) | (j + v)) < key) ? 1u : 0u;
            }
            sw[rank] = wt;
            ss[rank] = sym;
        }
    }
    __syncthreads();
    const uint32_t nint = real >= 2 ? real - 1 : 0;
    if (tid == 0 && nint) {
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
    const uint32_t root = 256 + nint - 1;
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
    }
    __syncthreads();
    // starting bit of every chunk: chunk histogram . code lengths (thread c: chunk c, its
    // 256 counts in 64 independent 16-B loads), exclusive scan in chunk order
    uint64_t carry = 0;
    for (uint32_t c0 = 0; c0 < nch; c0 += kTreeT) {
        const uint32_t c = c0 + tid;
        uint32_t bitsc = 0;
        if (c < nch) {
            const uint4 *h4 = (const uint4 *)(hc + (uint64_t)c * 256);
#pragma unroll 16
            for (uint32_t q = 0; q < 64; q++) {
                const uint4 v = h4[q];
                bitsc += v.x * ln[4 * q] + v.y * ln[4 * q + 1] + v.z * ln[4 * q + 2] + v.w * ln[4 * q + 3];
            }
        }
        const uint32_t inc = wave_incl_scan(bitsc);
        if (lane == 63) s_red[wv] = inc;
        __syncthreads();
        uint32_t pre = 0, all = 0;
        for (uint32_t q = 0; q < kTreeW; q++) {
            if (q < wv) pre += s_red[q];
            all += s_red[q];
        }
        if (c < nch) chunk_off[(uint64_t)b * L.cpb_total + r0 + c] = (uint32_t)(carry + pre + inc - bitsc);
        carry += all;
        __syncthreads();
    }
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

__global__ __launch_bounds__(256) void k_zero_edges(Layout L, const BlockInfo *__restrict__ binfo,
                                                    const uint32_t *__restrict__ chunk_off,
                                                    const uint64_t *__restrict__ blk_off, uint8_t *__restrict__ out,
                                                    const uint32_t *__restrict__ err) {
    if (*err & kErrCapacity) return;
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= (uint64_t)L.nblocks * L.cpb_total) return;
    const uint32_t b = (uint32_t)(q / L.cpb_total), r = (uint32_t)(q % L.cpb_total);
    uint32_t s, c;
    chunk_of(L, r, s, c);
    const BlockInfo &bi = binfo[b];
    const uint32_t len = bi.slen[s], c0 = c * kChunk;
    if (!stream_active(bi, s) || c0 >= len) return;
    const uint64_t base = 8 * (blk_off[b] + bi.words_rel[s]);
    const uint64_t g0 = base + chunk_off[q];
    uint32_t *o32 = (uint32_t *)out;
    if (c0 + kChunk < len) {   // the chunk ends where the next one starts
        const uint64_t g1 = base + chunk_off[q + 1];
        o32[g0 >> 5] = 0;
        if (g1 > g0) o32[(g1 - 1) >> 5] = 0;
    } else {                   // last chunk: every word through the end of the stream's words
        const uint64_t g1 = base + 32ull * bi.nwords[s];
        for (uint64_t w = g0 >> 5; w <= (g1 > g0 ? (g1 - 1) >> 5 : g0 >> 5); w++) o32[w] = 0;
    }
}

// staging words: the whole chunk at <= 8 bits per symbol (one pass; random data's chars
// are exactly 8); longer codes (<= 32 bits) go through several windows of this size
constexpr uint32_t kEncWords = kChunk / 4 + 2;

__global__ __launch_bounds__(kEncT) void k_encode(Layout L, const BlockInfo *__restrict__ binfo,
                                                 const uint8_t *__restrict__ s0, const uint8_t *__restrict__ s1,
                                                 const uint8_t *__restrict__ s2, const uint8_t *__restrict__ s3,
                                                 const uint32_t *__restrict__ ctab, const uint8_t *__restrict__ ltab,
                                                 const uint32_t *__restrict__ chunk_off,
                                                 const uint64_t *__restrict__ blk_off, uint8_t *__restrict__ out,
                                                 const uint32_t *__restrict__ err) {
    constexpr uint32_t kW = kEncT / 64;
    __shared__ uint32_t ct[256], lt[256];
    __shared__ uint32_t ws[kEncWords];
    __shared__ uint32_t red[kW];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t b = blockIdx.x / L.cpb_total, r = blockIdx.x % L.cpb_total;
    uint32_t s, c;
    chunk_of(L, r, s, c);
    // loads in two rounds: error word + block info, then everything else at once
    const uint32_t errv = *err;
    const BlockInfo &bi = binfo[b];
    const uint32_t len = bi.slen[s], c0 = c * kChunk;
    if (errv || !stream_active(bi, s) || c0 >= len) return;
    const uint32_t c1 = min(len, c0 + kChunk);
    const uint32_t hb = (b * kStreams + s) * 256;
    uint32_t ctv[256 / kEncT], ltv[256 / kEncT];
#pragma unroll
    for (uint32_t u = 0; u < 256 / kEncT; u++) { ctv[u] = ctab[hb + tid + kEncT * u]; ltv[u] = ltab[hb + tid + kEncT * u]; }
    const uint8_t *base = (s == 0 ? s0 : s == 1 ? s1 : s == 2 ? s2 : s3) + (uint64_t)b * L.sstride[s];
    const uint32_t i0 = c0 + kSymL * tid, i1 = min(c1, i0 + kSymL);
    uint32_t sym[kSymW];
    const uint32_t n = chunk_symbols((const uint32_t *)base, i0, i1, sym);
    const uint64_t obyte = blk_off[b] + bi.words_rel[s];
    const uint32_t coff = chunk_off[(uint64_t)b * L.cpb_total + r];
    bool all8 = true;
#pragma unroll
    for (uint32_t u = 0; u < 256 / kEncT; u++) {
        ct[tid + kEncT * u] = ctv[u];
        lt[tid + kEncT * u] = ltv[u];
        all8 = all8 && ltv[u] == 8;
    }
    // all 256 symbols with 8-bit codes (the chars of random data): the code stream is a
    // byte substitution at a byte-aligned offset
    const bool byte8 = __syncthreads_and(all8) != 0;
    if (byte8) {
        const uint64_t g0 = 8 * obyte + coff;
        const uint32_t sh0 = (uint32_t)(g0 & 31), nw = (sh0 + 8 * (c1 - c0) + 31) >> 5;
        for (uint32_t x = tid; x < nw; x += kEncT) ws[x] = 0;
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
        uint32_t *o32 = (uint32_t *)out + (g0 >> 5);
        for (uint32_t x = tid; x < nw; x += kEncT) {
            const uint32_t val = ws[x];
            if (x == 0 || x == nw - 1) { if (val) atomicOr(&o32[x], val); }
            else o32[x] = val;
        }
        return;
    }
    uint32_t nb = 0;
    for (uint32_t q = 0; q < n; q++) nb += lt[(sym[q >> 2] >> (8 * (q & 3))) & 0xFF];
    // block exclusive scan of nb
    const uint32_t inc = wave_incl_scan(nb);
    if (lane == 63) red[wv] = inc;
    __syncthreads();
    uint32_t pre = 0, ctot = 0;
    for (uint32_t q = 0; q < kW; q++) {
        if (q < wv) pre += red[q];
        ctot += red[q];
    }
    const uint32_t tb = pre + inc - nb;
    const uint64_t g0 = 8 * obyte + coff;
    const uint64_t gw = g0 >> 5;
    const uint32_t sh0 = (uint32_t)(g0 & 31);
    const uint32_t nw = (sh0 + ctot + 31) >> 5;
    // this lane's codes cover bits [p0, p1) of the staging words; whole words inside
    // that range are this lane's alone (plain LDS stores), the two end words are shared.
    // Windows of kEncWords words: a lane writes the words of its range inside the window.
    const uint32_t p0 = sh0 + tb, p1 = p0 + nb;
    uint32_t *o32 = (uint32_t *)out + gw;
    for (uint32_t wb = 0; wb < nw; wb += kEncWords) {
        const uint32_t we = min(nw, wb + kEncWords);
        for (uint32_t x = tid; x < we - wb; x += kEncT) ws[x] = 0;
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
        for (uint32_t x = wb + tid; x < we; x += kEncT) {
            const uint32_t v = ws[x - wb];
            if (x == 0 || x == nw - 1) { if (v) atomicOr(&o32[x], v); }
            else o32[x] = v;
        }
        __syncthreads();
    }
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
                    uint32_t *hist, uint32_t *ctab, uint8_t *ltab, uint8_t *hhdr, uint32_t *chunk_off,
                    uint64_t *blk_off, uint64_t *total, uint8_t *out, uint64_t cap, uint32_t *err, hipStream_t st,
                    hipEvent_t *ev, hipEvent_t wait_scan, hipEvent_t rec_scan) {
    const uint32_t nchunks = L.nblocks * L.cpb_total;
    hipLaunchKernelGGL(k_hist, dim3(nchunks), dim3(kEncT), 0, st, L, binfo, s0, s1, s2, s3, hist);
    if (ev) (void)hipEventRecord(ev[0], st);
    hipLaunchKernelGGL(k_tree, dim3(L.nblocks * kStreams), dim3(kTreeT), 0, st, L, hist, binfo, ctab, ltab, hhdr,
                       chunk_off, err);
    if (ev) (void)hipEventRecord(ev[1], st);
    hipLaunchKernelGGL(k_block_layout, dim3((L.nblocks + 63) / 64), dim3(64), 0, st, L.nblocks, binfo);
    if (ev) (void)hipEventRecord(ev[2], st);
    if (wait_scan) (void)hipStreamWaitEvent(st, wait_scan, 0);   // the previous group's record offsets
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, st, L.nblocks, binfo, blk_off, total, cap, err);
    if (rec_scan) (void)hipEventRecord(rec_scan, st);
    if (ev) (void)hipEventRecord(ev[3], st);
    hipLaunchKernelGGL(k_zero_edges, dim3((nchunks + 255) / 256), dim3(256), 0, st, L, binfo, chunk_off, blk_off, out,
                       err);
    if (ev) (void)hipEventRecord(ev[4], st);
    hipLaunchKernelGGL(k_encode, dim3(nchunks), dim3(kEncT), 0, st, L, binfo, s0, s1, s2, s3, ctab, ltab, chunk_off,
                       blk_off, out, err);
    if (ev) (void)hipEventRecord(ev[5], st);
    hipLaunchKernelGGL(k_headers, dim3(L.nblocks), dim3(64), 0, st, binfo, s0, L.sstride[0], hhdr, blk_off, out, err);
    if (ev) (void)hipEventRecord(ev[6], st);
}

}  // namespace fcx
