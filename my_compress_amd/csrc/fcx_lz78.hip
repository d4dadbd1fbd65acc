// fcx_lz78.hip — the `-c lz78` block codec (FCX8) on gfx950.
//
// Reference: my_compress_file_lz78 (my_compress.cpp:3127-3476) over
// my_LZ78_compress (1832-1899).  Blocks are independent (each call restarts the
// dictionary), so the device work is block-parallel; inside a block the LZ78
// parse is a serial trie walk (each phrase's start depends on the previous
// phrase), so it runs one lane per block over an open-addressed trie in HBM.
// Everything after the parse is position-parallel:
//
//   k78_parse     wave per block (lane 0 walks): trie walk -> tokens (idx[t], c[t]),
//                 N, max idx; root children in LDS, depth-1 children dense, deeper hashed
//   k78_mark      token-parallel: bitmap of used indices (3180-3206), char histogram
//   k78_rank      workgroup per block: popcount prefix of the bitmap -> rank base per
//                 word, wcnt (mapIdx 3216-3219)
//   k78_group     token-parallel: rank -> (group = r/256, in-group position r%256),
//                 group counts (3224-3254)
//   k78_tree      workgroup per block: the group tree (create_huffman_tree 535-617 on
//                 G leaves, 3258-3307) and the char tree (987-1066), both as a bitonic
//                 sort of (weight, symbol) in LDS + the two-queue merge that equals the
//                 reference's insertion order; code tables; the record layout
//   k78_scan      record offsets across the shard
//   k78_tilesum / k78_tilescan / k78_pack
//                 bit offsets of every 8192-token tile, then each lane packs its 32
//                 group codes and 32 char codes LSB-first into word staging
//                 (huffman_encode_idxGroup 2927-3006, huffman_encode_char 849-928)
//   k78_write     byte-parallel assembly of [u32 len][payload] records
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <mutex>
#include <vector>
#include <algorithm>

#include "fcx.h"

namespace fcx78 {

constexpr uint32_t kTileTok = 8192;   // tokens per pack tile (256 lanes x 32)
constexpr uint32_t kSortCap = 8192;   // bitonic sort capacity (>= the max group count 4097 of a 1 MiB block)
constexpr uint32_t kGroupLds = 4112;  // LDS group counters: >= groups of a 1 MiB block, ceil((2^20 + 1) / 256)
static_assert(kGroupLds >= FCX_MAX_BLOCK_BYTES / 256 + 1 && kSortCap >= FCX_MAX_BLOCK_BYTES / 256 + 1, "group capacity");

struct Rec78 {
    uint32_t N, maxi, wcnt, G;
    uint32_t Wg, Wc, ts, hlen;   // group words, char words, char tree size, char header bytes
    uint32_t nbm;                // index bitmap bytes
    uint32_t o_G, o_tree, o_N, o_gw, o_gpos, o_chdr, o_Wc, o_cw;   // offsets inside the record
    uint32_t rec;                // 4 + payload
    uint32_t err;
};

struct Scratch {
    uint32_t B, nb, cap_log2, Gmax, tiles;
    uint64_t *slot;      // nb << cap_log2
    uint32_t *d1;        // nb << 16 (depth-1 children, dense; null when dense1 == 0)
    uint32_t dense1;     // blocks >= kDense1Min: dense depth-1 table, else depth 1 is hashed too
    uint32_t *idx;       // nb * B
    uint8_t *c;          // nb * B
    uint32_t *bm;        // nb * bmw
    uint32_t *rbase;     // nb * bmw
    uint32_t bmw;
    uint16_t *grp;       // nb * B
    uint8_t *gpos;       // nb * B
    uint32_t *gcnt;      // nb * Gmax
    uint32_t *chist;     // nb * 256
    uint32_t *gcode;     // nb * Gmax
    uint8_t *glen;       // nb * Gmax
    uint32_t *ccode;     // nb * 256
    uint8_t *clen;       // nb * 256
    uint32_t *tree;      // nb * 2 * Gmax (group tree children, u32 pairs)
    uint32_t *par;       // nb * 2 * Gmax (parent scratch)
    uint32_t *iw;        // nb * Gmax (internal-node weights scratch)
    uint8_t *chdr;       // nb * 576
    uint32_t *tbits;     // nb * tiles * 2
    uint32_t *gstage;    // nb * (B + 2)
    uint32_t *cstage;    // nb * (B + 2)
    Rec78 *rec;          // nb
    uint64_t *off;       // nb (record offsets in the output)
    uint64_t *total;     // 1 (running output bytes across batches)
};

__device__ inline uint64_t trie_hash(uint64_t key) { return (key * 0x9E3779B97F4A7C15ull) >> 17; }

// block size from which the depth-1 children get the dense 256 KiB table: a small block has
// few 2-byte phrases (<= B/2), so they share the hash table (then <= B/2 entries in B + 2
// slots), and a batch of tiny blocks no longer allocates and zeroes 256 KiB per block
constexpr uint32_t kDense1Min = 65536;

// ---------------------------------------------------------------------------
// my_LZ78_compress (1832-1899): phrase = longest dictionary prefix + 1 byte; token
// (prefix index or 0, byte); the phrase enters the dictionary at the next index.  A
// block whose remainder is a dictionary string ends with (its index, 0) (1858-1863).
// The dictionary is a set of strings with ids, so it can be held as three tables
// with the same contents as one trie: the root's children in LDS (256 ids), the
// depth-1 children as a dense 256x256 table per block (256 KiB, L2/MALL-resident),
// deeper children in the open-addressed hash table (blocks < kDense1Min: depth 1 too).
// One wave per block, lane 0 walks.
template <bool DENSE1>
__global__ __launch_bounds__(64) void k78_parse(const uint8_t *__restrict__ in, uint64_t n, Scratch S, uint64_t base_blk) {
    __shared__ uint32_t root[256];
    const uint32_t b = blockIdx.x;
    for (uint32_t i = threadIdx.x; i < 256; i += 64) root[i] = 0;
    __syncthreads();
    if (threadIdx.x != 0) return;
    const uint64_t off = (base_blk + b) * (uint64_t)S.B;
    Rec78 &R = S.rec[b];
    if (off >= n) {
        R.N = 0;
        return;
    }
    const uint32_t len = (uint32_t)min((uint64_t)S.B, n - off);
    const uint8_t *src = in + off;
    uint64_t *slot = S.slot + ((uint64_t)b << S.cap_log2);
    uint32_t *d1 = DENSE1 ? S.d1 + ((uint64_t)b << 16) : nullptr;
    const uint64_t mask = (1ull << S.cap_log2) - 1;
    uint32_t *idx = S.idx + (uint64_t)b * S.B;
    uint8_t *cc = S.c + (uint64_t)b * S.B;
    uint32_t N = 0, next = 1, pos = 0, maxi = 0;
    auto emit = [&](uint32_t node, uint32_t ch) {
        idx[N] = node;
        cc[N] = (uint8_t)ch;
        N++;
        maxi = max(maxi, node);
    };
    while (pos < len) {
        // a phrase's first two bytes are known when it starts: their loads and the
        // depth-1 lookup issue together, so the dependent chain per phrase is one input
        // load, one depth-1 load, then the hashed levels
        const uint32_t b0 = src[pos], b1 = pos + 1 < len ? src[pos + 1] : 0u;
        const uint32_t b2 = pos + 2 < len ? src[pos + 2] : 0u, b3 = pos + 3 < len ? src[pos + 3] : 0u;
        const uint32_t c0 = root[b0], c1 = DENSE1 ? d1[(b0 << 8) | b1] : 0u;
        if (!c0) {   // new 1-byte phrase
            root[b0] = next++;
            emit(0, b0);
            pos += 1;
            continue;
        }
        if (pos + 1 == len) {   // whole remainder is a dictionary string (1858-1863)
            emit(c0, 0);
            break;
        }
        uint32_t node, ahead, nahead;   // bytes already loaded past the node's phrase
        if (DENSE1) {
            if (!c1) {   // new 2-byte phrase
                d1[(b0 << 8) | b1] = next++;
                emit(c0, b1);
                pos += 2;
                continue;
            }
            node = c1;
            pos += 2;
            ahead = b2 | (b3 << 8);
            nahead = 2;
        } else {     // hashed depth 1: the walk below starts at the root child
            node = c0;
            pos += 1;
            ahead = b1 | (b2 << 8) | (b3 << 16);
            nahead = 3;
        }
        bool put = false;
        uint64_t h = 0, key = 0;
        while (pos < len) {
            const uint32_t byte = nahead ? (ahead & 0xFF) : src[pos];
            ahead >>= 8;
            nahead -= nahead ? 1 : 0;
            key = (((uint64_t)node << 8) | byte) + 1;
            uint32_t child = 0;
            for (h = trie_hash(key) & mask;; h = (h + 1) & mask) {
                const uint64_t s = slot[h];
                if (s == 0) break;
                if ((s >> 24) == key) {
                    child = (uint32_t)(s & 0xFFFFFFu);
                    break;
                }
            }
            if (!child) {
                put = true;   // h is the empty slot that ended the probe
                break;
            }
            node = child;
            pos++;
        }
        if (!put) {   // whole remainder found
            emit(node, 0);
            break;
        }
        slot[h] = (key << 24) | next++;
        emit(node, (uint32_t)((key - 1) & 0xFF));
        pos++;
    }
    R.N = N;
    R.maxi = maxi;
    R.err = 0;
}

// token-parallel: used-index bitmap + char histogram
__global__ __launch_bounds__(256) void k78_mark(Scratch S) {
    __shared__ uint32_t h[256];
    const uint32_t b = blockIdx.y, tid = threadIdx.x;
    const uint32_t N = S.rec[b].N;
    const uint32_t t0 = blockIdx.x * kTileTok;
    if (t0 >= N) return;
    h[tid] = 0;
    __syncthreads();
    const uint32_t *idx = S.idx + (uint64_t)b * S.B;
    const uint8_t *cc = S.c + (uint64_t)b * S.B;
    uint32_t *bm = S.bm + (uint64_t)b * S.bmw;
    const uint32_t t1 = min(N, t0 + kTileTok);
    for (uint32_t t = t0 + tid; t < t1; t += 256) {
        const uint32_t v = idx[t];
        atomicOr(&bm[v >> 5], 1u << (v & 31));
        atomicAdd(&h[cc[t]], 1u);
    }
    __syncthreads();
    if (h[tid]) atomicAdd(&S.chist[(uint64_t)b * 256 + tid], h[tid]);
}

// workgroup per block: exclusive popcount prefix over the bitmap words
__global__ __launch_bounds__(1024) void k78_rank(Scratch S) {
    __shared__ uint32_t part[1024];
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    Rec78 &R = S.rec[b];
    if (R.N == 0) return;
    const uint32_t nw = R.maxi / 32 + 1;
    const uint32_t per = (nw + 1023) / 1024;
    const uint32_t w0 = min(nw, tid * per), w1 = min(nw, w0 + per);
    const uint32_t *bm = S.bm + (uint64_t)b * S.bmw;
    uint32_t *rb = S.rbase + (uint64_t)b * S.bmw;
    uint32_t sum = 0;
    for (uint32_t w = w0; w < w1; w++) sum += __popc(bm[w]);
    part[tid] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {   // Hillis-Steele inclusive scan
        const uint32_t v = tid >= d ? part[tid - d] : 0u;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    uint32_t run = part[tid] - sum;
    for (uint32_t w = w0; w < w1; w++) {
        rb[w] = run;
        run += __popc(bm[w]);
    }
    if (tid == 1023) {
        R.wcnt = part[1023];
        R.G = (part[1023] + 255) / 256;
        R.nbm = R.maxi / 8 + 1;
    }
}

// token-parallel: rank -> group / in-group position, group counts
__global__ __launch_bounds__(256) void k78_group(Scratch S) {
    // group counts of the tile in LDS (G <= kGroupLds for blocks <= 1 MiB), flushed once
    __shared__ uint32_t lc[kGroupLds];
    const uint32_t b = blockIdx.y, tid = threadIdx.x;
    const Rec78 &R = S.rec[b];
    const uint32_t N = R.N;
    const uint32_t t0 = blockIdx.x * kTileTok;
    if (t0 >= N) return;
    const uint32_t G = R.G;
    const bool lds = G <= kGroupLds;
    if (lds)
        for (uint32_t g = tid; g < G; g += 256) lc[g] = 0;
    __syncthreads();
    const uint32_t *idx = S.idx + (uint64_t)b * S.B;
    const uint32_t *bm = S.bm + (uint64_t)b * S.bmw;
    const uint32_t *rb = S.rbase + (uint64_t)b * S.bmw;
    uint16_t *grp = S.grp + (uint64_t)b * S.B;
    uint8_t *gp = S.gpos + (uint64_t)b * S.B;
    uint32_t *gc = S.gcnt + (uint64_t)b * S.Gmax;
    const uint32_t t1 = min(N, t0 + kTileTok);
    for (uint32_t t = t0 + tid; t < t1; t += 256) {
        const uint32_t v = idx[t];
        const uint32_t r = rb[v >> 5] + __popc(bm[v >> 5] & ((1u << (v & 31)) - 1u));
        grp[t] = (uint16_t)(r >> 8);
        gp[t] = (uint8_t)(r & 255);
        if (lds) atomicAdd(&lc[r >> 8], 1u);
        else atomicAdd(&gc[r >> 8], 1u);
    }
    __syncthreads();
    if (lds)
        for (uint32_t g = tid; g < G; g += 256)
            if (lc[g]) atomicAdd(&gc[g], lc[g]);
}

// ---------------------------------------------------------------------------
// create_huffman_tree (535-617) on n leaves of weight w[] (zero = absent): leaves
// stably sorted by weight (sort key (w, symbol)), each merge takes the two list
// heads (left, right) and re-inserts after every weight <= sum, which is the
// two-queue merge taking the leaf on a tie.  Internal node k is n + (n - real) + k.
// lc/rc[k] hold its children (raw node numbers); parent[] is indexed by node.
// Codes: leaf -> root walk, root edge in bit 0 (869-924, 2947-2992).  Returns real;
// sets *bad on a code longer than 32 bits.
__device__ uint32_t wg_tree(uint32_t n, const uint32_t *w, uint64_t *keys /*LDS kSortCap*/, uint32_t *lc,
                            uint32_t *rc, uint32_t *par, uint32_t *iw, uint32_t *code, uint8_t *clen,
                            uint32_t *s_real, uint32_t *bad) {
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    uint32_t P = 1;
    while (P < n) P <<= 1;
    if (tid == 0) *s_real = 0;
    __syncthreads();
    for (uint32_t i = tid; i < P; i += nt) {
        const uint32_t wi = i < n ? w[i] : 0u;
        keys[i] = wi ? ((uint64_t)wi << 32) | i : ~0ull;
        if (wi) atomicAdd(s_real, 1u);
    }
    for (uint32_t i = tid; i < 2 * n; i += nt) par[i] = 0;
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = tid; i < P; i += nt) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const uint64_t a = keys[i], c = keys[l];
                    const bool up = (i & k) == 0;
                    if ((a > c) == up) {
                        keys[i] = c;
                        keys[l] = a;
                    }
                }
            }
            __syncthreads();
        }
    const uint32_t real = *s_real;
    const uint32_t nbase = n + (n - real);
    if (tid == 0 && real > 1) {
        uint32_t lh = 0, ih = 0, it = 0;
        for (uint32_t k = 0; k + 1 < real; k++) {
            uint32_t pick[2], pw[2];
            for (int q = 0; q < 2; q++) {
                const bool leaf = lh < real && (ih == it || (uint32_t)(keys[lh] >> 32) <= iw[ih]);
                if (leaf) {
                    pw[q] = (uint32_t)(keys[lh] >> 32);
                    pick[q] = (uint32_t)keys[lh];
                    lh++;
                } else {
                    pw[q] = iw[ih];
                    pick[q] = nbase + ih;
                    ih++;
                }
            }
            const uint32_t node = nbase + k;
            lc[k] = pick[0];
            rc[k] = pick[1];
            par[pick[0]] = node;
            par[pick[1]] = node;
            iw[it++] = pw[0] + pw[1];
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < n; i += nt) {
        uint32_t bits = 0, depth = 0, cur = i, p = par[i];
        if (w[i] && real > 1)
            while (p != 0 && p < 2 * n - 1) {
                if (depth == 32) {
                    *bad = 1;
                    break;
                }
                bits = (bits << 1) | (lc[p - nbase] == cur ? 0u : 1u);
                depth++;
                cur = p;
                p = par[p];
            }
        code[i] = bits;
        clen[i] = (uint8_t)depth;
    }
    __syncthreads();
    return real;
}

__global__ __launch_bounds__(256) void k78_tree(Scratch S) {
    __shared__ uint64_t keys[kSortCap];
    __shared__ uint32_t s_real, s_bad;
    __shared__ uint64_t s_bits[2];
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    Rec78 &R = S.rec[b];
    if (R.N == 0) return;
    if (tid == 0) {
        s_bad = 0;
        s_bits[0] = s_bits[1] = 0;
    }
    __syncthreads();
    const uint32_t G = R.G, Gm = S.Gmax;
    uint32_t *lc = S.tree + (uint64_t)b * 2 * Gm, *rc = lc + Gm;
    uint32_t *par = S.par + (uint64_t)b * 2 * Gm, *iw = S.iw + (uint64_t)b * Gm;
    const uint32_t *gc = S.gcnt + (uint64_t)b * Gm;
    uint32_t *gcode = S.gcode + (uint64_t)b * Gm;
    uint8_t *glen = S.glen + (uint64_t)b * Gm;
    if (G > 1) {
        wg_tree(G, gc, keys, lc, rc, par, iw, gcode, glen, &s_real, &s_bad);
        uint64_t part = 0;
        for (uint32_t g = tid; g < G; g += 256) part += (uint64_t)gc[g] * glen[g];
        atomicAdd((unsigned long long *)&s_bits[0], (unsigned long long)part);
    }
    // char tree (987-1066): the same builder on 256 symbols.  The group tree's parents
    // and internal weights are spent (its codes and children are stored), so the char
    // tree borrows that scratch: children in iw[0..511], weights iw[512..767], par[0..511].
    __syncthreads();
    const uint32_t *ch = S.chist + (uint64_t)b * 256;
    uint32_t *ccode = S.ccode + (uint64_t)b * 256;
    uint8_t *cl = S.clen + (uint64_t)b * 256;
    uint32_t *xlc = iw, *xrc = iw + 256;
    const uint32_t real = wg_tree(256, ch, keys, xlc, xrc, par, iw + 512, ccode, cl, &s_real, &s_bad);
    atomicAdd((unsigned long long *)&s_bits[1], (unsigned long long)ch[tid] * cl[tid]);
    const uint32_t ts = real > 1 ? real - 1 : 0, hb = (2 * ts + 7) / 8;
    uint8_t *hdr = S.chdr + (uint64_t)b * 576;
    // [u8 ts][hb bytes: bit k set = child k of the pairs is internal][ts x (u8 l, u8 r)]
    for (uint32_t q = tid; q < hb; q += 256) {
        uint32_t v = 0;
        for (uint32_t k = 8 * q; k < min(8 * q + 8, 2 * ts); k++)
            if (((k & 1) ? xrc[k >> 1] : xlc[k >> 1]) >= 256) v |= 1u << (k & 7);
        hdr[1 + q] = (uint8_t)v;
    }
    for (uint32_t j = tid; j < ts; j += 256) {
        const uint32_t l = xlc[j], r = xrc[j];
        hdr[1 + hb + 2 * j] = (uint8_t)(l >= 256 ? l - 256 : l);
        hdr[1 + hb + 2 * j + 1] = (uint8_t)(r >= 256 ? r - 256 : r);
    }
    if (tid == 0) hdr[0] = (uint8_t)ts;
    __syncthreads();
    if (tid == 0) {
        const uint32_t N = R.N;
        R.Wg = G > 1 ? (uint32_t)((s_bits[0] + 31) / 32) : 0u;
        R.Wc = (uint32_t)((s_bits[1] + 31) / 32);
        R.ts = ts;
        R.hlen = 1 + hb + 2 * ts;
        uint32_t o = 4 + 4 + R.nbm;   // [u32 len][u32 wcnt][bitmap]
        R.o_G = o;
        o += 4;
        R.o_tree = o;
        if (G > 1) {
            o += 8 * (G - 1);
            R.o_N = o;
            o += 8;   // N, Wg
            R.o_gw = o;
            o += 4 * R.Wg;
        } else {
            R.o_N = o;
            o += 4;
            R.o_gw = o;
        }
        R.o_gpos = o;
        o += N;
        R.o_chdr = o;
        o += R.hlen;
        R.o_Wc = o;
        o += 4;
        R.o_cw = o;
        o += 4 * R.Wc;
        R.rec = o;
        R.err = s_bad;
    }
}

// record offsets across the shard (one workgroup; serial chunks + LDS scan)
__global__ __launch_bounds__(1024) void k78_scan(Scratch S, uint64_t cap, uint32_t *err) {
    __shared__ uint64_t part[1024];
    const uint32_t tid = threadIdx.x, nb = S.nb;
    const uint32_t per = (nb + 1023) / 1024, b0 = min(nb, tid * per), b1 = min(nb, b0 + per);
    uint64_t sum = 0;
    for (uint32_t b = b0; b < b1; b++) {
        const Rec78 &R = S.rec[b];
        if (R.N) sum += R.rec;
        if (R.N && R.err) atomicOr(err, 1u);
    }
    part[tid] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint64_t v = tid >= d ? part[tid - d] : 0ull;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    const uint64_t base = *S.total;
    uint64_t run = base + part[tid] - sum;
    for (uint32_t b = b0; b < b1; b++) {
        S.off[b] = run;
        if (S.rec[b].N) run += S.rec[b].rec;
    }
    __syncthreads();
    if (tid == 1023) {
        *S.total = base + part[1023];
        if (base + part[1023] > cap) atomicOr(err, 2u);
    }
}

__device__ inline void tok_codes(const Scratch &S, uint32_t b, uint32_t t, uint32_t G, uint32_t &gcw, uint32_t &glw,
                                 uint32_t &ccw, uint32_t &clw) {
    const uint8_t sym = S.c[(uint64_t)b * S.B + t];
    ccw = S.ccode[(uint64_t)b * 256 + sym];
    clw = S.clen[(uint64_t)b * 256 + sym];
    if (G > 1) {
        const uint32_t g = S.grp[(uint64_t)b * S.B + t];
        gcw = S.gcode[(uint64_t)b * S.Gmax + g];
        glw = S.glen[(uint64_t)b * S.Gmax + g];
    } else {
        gcw = glw = 0;
    }
}

// bits of each tile (both streams)
__global__ __launch_bounds__(256) void k78_tilesum(Scratch S) {
    __shared__ uint32_t sg, sc;
    const uint32_t b = blockIdx.y, tid = threadIdx.x;
    const Rec78 &R = S.rec[b];
    const uint32_t t0 = blockIdx.x * kTileTok;
    if (t0 >= R.N) return;
    if (tid == 0) sg = sc = 0;
    __syncthreads();
    uint32_t a = 0, c = 0;
    for (uint32_t t = t0 + tid * 32; t < min(R.N, t0 + tid * 32 + 32); t++) {
        uint32_t gcw, glw, ccw, clw;
        tok_codes(S, b, t, R.G, gcw, glw, ccw, clw);
        a += glw;
        c += clw;
    }
    atomicAdd(&sg, a);
    atomicAdd(&sc, c);
    __syncthreads();
    if (tid == 0) {
        S.tbits[((uint64_t)b * S.tiles + blockIdx.x) * 2] = sg;
        S.tbits[((uint64_t)b * S.tiles + blockIdx.x) * 2 + 1] = sc;
    }
}

__global__ __launch_bounds__(64) void k78_tilescan(Scratch S) {
    const uint32_t b = blockIdx.x * 64 + threadIdx.x;
    if (b >= S.nb || S.rec[b].N == 0) return;
    const uint32_t nt = (S.rec[b].N + kTileTok - 1) / kTileTok;
    uint32_t a = 0, c = 0;
    uint32_t *tb = S.tbits + (uint64_t)b * S.tiles * 2;
    for (uint32_t i = 0; i < nt; i++) {
        const uint32_t x = tb[2 * i], y = tb[2 * i + 1];
        tb[2 * i] = a;
        tb[2 * i + 1] = c;
        a += x;
        c += y;
    }
}

__device__ inline void put_bits(uint32_t *w, uint32_t off, uint32_t code, uint32_t len) {
    if (!len) return;
    const uint64_t v = (uint64_t)code << (off & 31);
    atomicOr(&w[off >> 5], (uint32_t)v);
    if ((off & 31) + len > 32) atomicOr(&w[(off >> 5) + 1], (uint32_t)(v >> 32));
}

__global__ __launch_bounds__(256) void k78_pack(Scratch S) {
    __shared__ uint32_t pg[256], pc[256];
    const uint32_t b = blockIdx.y, tid = threadIdx.x;
    const Rec78 &R = S.rec[b];
    const uint32_t t0 = blockIdx.x * kTileTok;
    if (t0 >= R.N) return;
    const uint32_t i0 = t0 + tid * 32, i1 = min(R.N, i0 + 32);
    uint32_t a = 0, c = 0;
    for (uint32_t t = i0; t < i1; t++) {
        uint32_t gcw, glw, ccw, clw;
        tok_codes(S, b, t, R.G, gcw, glw, ccw, clw);
        a += glw;
        c += clw;
    }
    pg[tid] = a;
    pc[tid] = c;
    __syncthreads();
    for (uint32_t d = 1; d < 256; d <<= 1) {
        const uint32_t x = tid >= d ? pg[tid - d] : 0u, y = tid >= d ? pc[tid - d] : 0u;
        __syncthreads();
        pg[tid] += x;
        pc[tid] += y;
        __syncthreads();
    }
    const uint32_t *tb = S.tbits + ((uint64_t)b * S.tiles + blockIdx.x) * 2;
    uint32_t og = tb[0] + pg[tid] - a, oc = tb[1] + pc[tid] - c;
    uint32_t *gw = S.gstage + (uint64_t)b * (S.B + 2), *cw = S.cstage + (uint64_t)b * (S.B + 2);
    for (uint32_t t = i0; t < i1; t++) {
        uint32_t gcw, glw, ccw, clw;
        tok_codes(S, b, t, R.G, gcw, glw, ccw, clw);
        put_bits(gw, og, gcw, glw);
        put_bits(cw, oc, ccw, clw);
        og += glw;
        oc += clw;
    }
}

__device__ inline uint8_t u32_byte(uint32_t v, uint32_t k) { return (uint8_t)(v >> (8 * k)); }

// byte-parallel record assembly (layout: my_compress_file_lz78 3127-3476)
__global__ __launch_bounds__(256) void k78_write(Scratch S, uint8_t *__restrict__ out, const uint32_t *err) {
    const uint32_t b = blockIdx.y;
    const Rec78 &R = S.rec[b];
    if (R.N == 0 || *err) return;
    uint8_t *o = out + S.off[b];
    const uint32_t rec = R.rec;
    const uint8_t *bmb = (const uint8_t *)(S.bm + (uint64_t)b * S.bmw);
    const uint32_t *lc = S.tree + (uint64_t)b * 2 * S.Gmax, *rc = lc + S.Gmax;
    const uint8_t *gw = (const uint8_t *)(S.gstage + (uint64_t)b * (S.B + 2));
    const uint8_t *cw = (const uint8_t *)(S.cstage + (uint64_t)b * (S.B + 2));
    const uint8_t *gp = S.gpos + (uint64_t)b * S.B;
    const uint8_t *hdr = S.chdr + (uint64_t)b * 576;
    for (uint32_t p = blockIdx.x * 256 + threadIdx.x; p < rec; p += gridDim.x * 256) {
        uint8_t v;
        if (p < 4) v = u32_byte(rec - 4, p);
        else if (p < 8) v = u32_byte(R.wcnt, p - 4);
        else if (p < R.o_G) v = bmb[p - 8];
        else if (p < R.o_tree) v = u32_byte(R.G, p - R.o_G);
        else if (p < R.o_N) {
            const uint32_t q = p - R.o_tree, j = q / 8, k = q % 8;
            v = u32_byte(k < 4 ? lc[j] : rc[j], k & 3);
        } else if (R.G > 1 && p < R.o_N + 4) v = u32_byte(R.N, p - R.o_N);
        else if (R.G > 1 && p < R.o_gw) v = u32_byte(R.Wg, p - R.o_N - 4);
        else if (R.G <= 1 && p < R.o_gw) v = u32_byte(R.N, p - R.o_N);
        else if (p < R.o_gpos) v = gw[p - R.o_gw];
        else if (p < R.o_chdr) v = gp[p - R.o_gpos];
        else if (p < R.o_Wc) v = hdr[p - R.o_chdr];
        else if (p < R.o_cw) v = u32_byte(R.Wc, p - R.o_Wc);
        else v = cw[p - R.o_cw];
        o[p] = v;
    }
}

}  // namespace fcx78

using namespace fcx78;

namespace fcx {
void set_last_error(const std::string &m);   // fcx_capi.hip (fcx_last_error)
}
namespace {
int fail78(int code, const std::string &m) {
    fcx::set_last_error(m);
    return code;
}
#define H78(expr)                                                                               \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess) return fail78(FCX_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct Alloc78 {
    Scratch S{};
    void *mem = nullptr;
};

// Compress scratch is kept per device between calls (grow-only; ~40 GB for a 1 GiB
// batch), so repeated shards do not pay hipMalloc/hipFree; fcx_lz78_release frees it.
// Calls on one device are serialised on its slot.
struct Cache78 {
    std::mutex mu;
    void *mem = nullptr;
    uint64_t bytes = 0;
};
Cache78 g_cache[64];

Cache78 *cache_for_current_device() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    return &g_cache[dev];
}

int setup(Alloc78 &A, Cache78 &C, uint32_t B, uint32_t nb) {
    Scratch &S = A.S;
    S.B = B;
    S.nb = nb;
    S.cap_log2 = 10;
    // only phrases of >= 3 bytes reach the hash table, so it holds <= B/3 entries:
    // B + 2 slots keep the load <= 1/3 and always leave an empty slot
    while ((1ull << S.cap_log2) < (uint64_t)B + 2) S.cap_log2++;
    S.Gmax = B / 256 + 2;
    if (S.Gmax < 1024) S.Gmax = 1024;   // the char tree borrows iw[0..511]; parents need 2*256
    S.tiles = (B + 1 + kTileTok - 1) / kTileTok;
    S.bmw = B / 32 + 2;
    S.dense1 = B >= kDense1Min ? 1u : 0u;
    const uint64_t nbl = nb;
    uint64_t sz[] = {
        (nbl << S.cap_log2) * 8, nbl * B * 4, nbl * B, nbl * S.bmw * 4, nbl * S.bmw * 4, nbl * B * 2, nbl * B,
        nbl * S.Gmax * 4, nbl * 256 * 4, nbl * S.Gmax * 4, nbl * S.Gmax, nbl * 256 * 4, nbl * 256,
        nbl * 2 * S.Gmax * 4, nbl * 2 * S.Gmax * 4, nbl * S.Gmax * 4, nbl * 576, nbl * S.tiles * 8,
        nbl * (B + 2) * 4, nbl * (B + 2) * 4, nbl * sizeof(Rec78), nbl * 8, 8, S.dense1 ? (nbl << 16) * 4 : 0};
    constexpr int K = sizeof(sz) / sizeof(sz[0]);
    uint64_t offs[K], tot = 0;
    for (int i = 0; i < K; i++) {
        offs[i] = tot;
        tot += (sz[i] + 255) & ~255ull;
    }
    if (C.bytes < tot) {
        if (C.mem) (void)hipFree(C.mem);
        C.mem = nullptr;
        C.bytes = 0;
        H78(hipMalloc(&C.mem, tot));
        C.bytes = tot;
    }
    A.mem = C.mem;
    char *m = (char *)A.mem;
    S.slot = (uint64_t *)(m + offs[0]);
    S.idx = (uint32_t *)(m + offs[1]);
    S.c = (uint8_t *)(m + offs[2]);
    S.bm = (uint32_t *)(m + offs[3]);
    S.rbase = (uint32_t *)(m + offs[4]);
    S.grp = (uint16_t *)(m + offs[5]);
    S.gpos = (uint8_t *)(m + offs[6]);
    S.gcnt = (uint32_t *)(m + offs[7]);
    S.chist = (uint32_t *)(m + offs[8]);
    S.gcode = (uint32_t *)(m + offs[9]);
    S.glen = (uint8_t *)(m + offs[10]);
    S.ccode = (uint32_t *)(m + offs[11]);
    S.clen = (uint8_t *)(m + offs[12]);
    S.tree = (uint32_t *)(m + offs[13]);
    S.par = (uint32_t *)(m + offs[14]);
    S.iw = (uint32_t *)(m + offs[15]);
    S.chdr = (uint8_t *)(m + offs[16]);
    S.tbits = (uint32_t *)(m + offs[17]);
    S.gstage = (uint32_t *)(m + offs[18]);
    S.cstage = (uint32_t *)(m + offs[19]);
    S.rec = (Rec78 *)(m + offs[20]);
    S.off = (uint64_t *)(m + offs[21]);
    S.total = (uint64_t *)(m + offs[22]);
    S.d1 = S.dense1 ? (uint32_t *)(m + offs[23]) : nullptr;
    return FCX_OK;
}

// scratch is ~40 B per input byte of a batch (the trie 16 B): 1 GiB batches (~40 GB of
// HBM) because the parse has one walker per block and rate grows with walkers in flight
// (256 MiB: 539 MB/s, 1 GiB: 1386 MB/s on rand)
constexpr uint64_t kBatchBytes = 1024ull << 20;
constexpr uint64_t kScratchBudget = 64ull << 30;
}  // namespace

extern "C" {

int fcx_lz78_compress_shard(const uint8_t *d_in, uint64_t n, uint32_t block_bytes, uint8_t *d_out, uint64_t cap,
                            uint64_t *out_len, void *stream) {
    if (!d_out || !out_len || (n && !d_in)) return fail78(FCX_ERR_ARG, "fcx_lz78_compress_shard: NULL argument");
    if (block_bytes == 0 || block_bytes > FCX_MAX_BLOCK_BYTES)
        return fail78(FCX_ERR_ARG, "fcx_lz78_compress_shard: block_bytes must be in [1, 1 MiB]");
    *out_len = 0;
    if (n == 0) return FCX_OK;
    hipStream_t st = (hipStream_t)stream;
    const uint64_t nblk = (n + block_bytes - 1) / block_bytes;
    // blocks per batch: <= 1 GiB of input, and per-block scratch (trie, dense depth-1
    // table, group tables: large for tiny blocks) within a 64 GiB budget
    uint32_t cl2 = 10;
    while ((1ull << cl2) < (uint64_t)block_bytes + 2) cl2++;
    const uint64_t per_block = (8ull << cl2) + (block_bytes >= kDense1Min ? 1ull << 18 : 0) +
                               64ull * std::max<uint32_t>(1024, block_bytes / 256 + 2) +
                               24ull * block_bytes + 4096;
    const uint64_t by_budget = std::max<uint64_t>(1, kScratchBudget / per_block);
    const uint32_t batch = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>(std::min<uint64_t>(nblk, kBatchBytes / block_bytes), by_budget));
    Cache78 *C = cache_for_current_device();
    if (!C) return fail78(FCX_ERR_HIP, "fcx_lz78_compress_shard: no current HIP device");
    std::lock_guard<std::mutex> lock(C->mu);
    Alloc78 A;
    if (int rc = setup(A, *C, block_bytes, batch)) return rc;
    Scratch S = A.S;
    uint32_t *d_err = nullptr;
    H78(hipMalloc(&d_err, 4));
    struct ErrFree {
        uint32_t *p;
        ~ErrFree() { (void)hipFree(p); }
    } ef{d_err};
    H78(hipMemsetAsync(d_err, 0, 4, st));
    H78(hipMemsetAsync(S.total, 0, 8, st));
    for (uint64_t b0 = 0; b0 < nblk; b0 += batch) {
        S.nb = (uint32_t)std::min<uint64_t>(batch, nblk - b0);
        const uint32_t nb = S.nb;
        H78(hipMemsetAsync(S.slot, 0, ((uint64_t)nb << S.cap_log2) * 8, st));
        if (S.dense1) H78(hipMemsetAsync(S.d1, 0, ((uint64_t)nb << 16) * 4, st));
        H78(hipMemsetAsync(S.bm, 0, (uint64_t)nb * S.bmw * 4, st));
        H78(hipMemsetAsync(S.gcnt, 0, (uint64_t)nb * S.Gmax * 4, st));
        H78(hipMemsetAsync(S.chist, 0, (uint64_t)nb * 256 * 4, st));
        H78(hipMemsetAsync(S.gstage, 0, (uint64_t)nb * (S.B + 2) * 4, st));
        H78(hipMemsetAsync(S.cstage, 0, (uint64_t)nb * (S.B + 2) * 4, st));
        const dim3 tok_grid(S.tiles, nb);
        if (S.dense1) k78_parse<true><<<nb, 64, 0, st>>>(d_in, n, S, b0);
        else k78_parse<false><<<nb, 64, 0, st>>>(d_in, n, S, b0);
        k78_mark<<<tok_grid, 256, 0, st>>>(S);
        k78_rank<<<nb, 1024, 0, st>>>(S);
        k78_group<<<tok_grid, 256, 0, st>>>(S);
        k78_tree<<<nb, 256, 0, st>>>(S);
        k78_scan<<<1, 1024, 0, st>>>(S, cap, d_err);
        k78_tilesum<<<tok_grid, 256, 0, st>>>(S);
        k78_tilescan<<<(nb + 63) / 64, 64, 0, st>>>(S);
        k78_pack<<<tok_grid, 256, 0, st>>>(S);
        k78_write<<<dim3(64, nb), 256, 0, st>>>(S, d_out, d_err);
        H78(hipGetLastError());
    }
    uint32_t herr = 0;
    uint64_t total = 0;
    H78(hipMemcpyAsync(&herr, d_err, 4, hipMemcpyDeviceToHost, st));
    H78(hipMemcpyAsync(&total, S.total, 8, hipMemcpyDeviceToHost, st));
    H78(hipStreamSynchronize(st));
    if (herr & 2) return fail78(FCX_ERR_CAPACITY, "fcx_lz78_compress_shard: output capacity exceeded");
    if (herr & 1) return fail78(FCX_ERR_INTERNAL, "fcx_lz78_compress_shard: Huffman code longer than 32 bits");
    *out_len = total;
    return FCX_OK;
}

int fcx_lz78_release(void) {
    Cache78 *C = cache_for_current_device();
    if (!C) return fail78(FCX_ERR_HIP, "fcx_lz78_release: no current HIP device");
    std::lock_guard<std::mutex> lock(C->mu);
    if (C->mem) H78(hipFree(C->mem));
    C->mem = nullptr;
    C->bytes = 0;
    return FCX_OK;
}

int fcx_lz78_compress_host(const uint8_t *in, uint64_t n, uint32_t block_bytes, uint8_t *out, uint64_t cap,
                           uint64_t *out_len) {
    if (!in || !out || !out_len) return fail78(FCX_ERR_ARG, "fcx_lz78_compress_host: NULL argument");
    if (cap < FCX_HEADER_BYTES) return fail78(FCX_ERR_CAPACITY, "fcx_lz78_compress_host: capacity below the header");
    if (block_bytes == 0 || block_bytes > FCX_MAX_BLOCK_BYTES)
        return fail78(FCX_ERR_ARG, "fcx_lz78_compress_host: block_bytes must be in [1, 1 MiB]");
    const uint64_t nblk = (n + block_bytes - 1) / block_bytes;
    memcpy(out, "FCX8", 4);   // stCmpFileHead (101-109) with the lz78 tag (4079-4086)
    const uint32_t tot32 = (uint32_t)n;
    const uint16_t nb16 = (uint16_t)nblk;
    memcpy(out + 4, &tot32, 4);
    memcpy(out + 8, &nb16, 2);
    *out_len = FCX_HEADER_BYTES;
    if (n == 0) return FCX_OK;
    uint8_t *d_in = nullptr, *d_out = nullptr;
    H78(hipMalloc(&d_in, n));
    struct F {
        uint8_t **a, **b;
        ~F() {
            if (*a) (void)hipFree(*a);
            if (*b) (void)hipFree(*b);
        }
    } f{&d_in, &d_out};
    const uint64_t dcap = cap - FCX_HEADER_BYTES;
    H78(hipMalloc(&d_out, dcap ? dcap : 16));
    H78(hipMemcpy(d_in, in, n, hipMemcpyHostToDevice));
    uint64_t len = 0;
    if (int rc = fcx_lz78_compress_shard(d_in, n, block_bytes, d_out, dcap, &len, nullptr)) return rc;
    H78(hipMemcpy(out + FCX_HEADER_BYTES, d_out, len, hipMemcpyDeviceToHost));
    *out_len = FCX_HEADER_BYTES + len;
    return FCX_OK;
}

uint32_t fcx_lz78_compress_block(const void *in, uint32_t len, uint8_t *out) {
    if (!in || !out || len == 0 || len > FCX_MAX_BLOCK_BYTES) return 0;
    uint8_t *d_in = nullptr, *d_out = nullptr;
    const uint64_t cap = 10ull * len + 4096;
    if (hipMalloc(&d_in, len) != hipSuccess) return 0;
    if (hipMalloc(&d_out, cap) != hipSuccess) {
        (void)hipFree(d_in);
        return 0;
    }
    uint64_t got = 0;
    uint32_t ret = 0;
    if (hipMemcpy(d_in, in, len, hipMemcpyHostToDevice) == hipSuccess &&
        fcx_lz78_compress_shard(d_in, len, len, d_out, cap, &got, nullptr) == FCX_OK && got >= 4 &&
        hipMemcpy(out, d_out + 4, got - 4, hipMemcpyDeviceToHost) == hipSuccess)
        ret = (uint32_t)(got - 4);
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return ret;
}

}  // extern "C"

// ===========================================================================
// Decoder: my_decompress_file_lz78 (my_compress.cpp:3478-3710).  Every phrase copies
// an earlier phrase of the same block, so a block decodes serially; records are
// independent, so one lane decodes one record (group codes, char codes, in-group
// positions and phrase copies in a single pass), and a byte-parallel kernel packs
// the decoded blocks densely.
namespace fcx78 {

struct Dec78 {
    uint32_t B;             // per-record output capacity (FCX_MAX_BLOCK_BYTES + 8)
    uint32_t nb;
    const uint8_t *in;      // the records' payloads
    const uint64_t *roff;   // payload offset per record
    const uint32_t *rlen;   // payload bytes per record
    uint8_t *out;           // nb * B decoded bytes
    uint32_t *pindex;       // nb * (B + 2)
    uint32_t *pstart;       // nb * B
    uint32_t *plen;         // nb * B
    uint32_t *lc;           // nb * 2 * Gmax
    uint32_t Gmax;
    uint64_t *dlen;         // decoded bytes per record, or ~0 = malformed
};

__device__ inline uint32_t rd32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

struct BitRd {   // LSB-first u32 words, W of them
    const uint8_t *w;
    uint32_t W, i, cur, left;
    __device__ int next() {   // -1 when exhausted
        if (left == 0) {
            if (i >= W) return -1;
            cur = rd32(w + 4ull * i++);
            left = 32;
        }
        const int b = cur & 1;
        cur >>= 1;
        left--;
        return b;
    }
};

__device__ int64_t dec_block(const uint8_t *in, uint32_t len, uint8_t *out, uint64_t cap, uint32_t *pindex,
                             uint32_t *pstart, uint32_t *plen, uint32_t *glc, uint32_t Gmax, uint8_t *tpairs,
                             uint8_t *tbm) {
    const uint8_t *q = in, *end = in + len;
    if (len < 4) return -1;
    const uint32_t wcnt = rd32(q);
    q += 4;
    if (wcnt == 0 || wcnt > cap + 2) return -1;   // the reference reads pIndex[-1] (3502)
    {   // 3494-3500: indices of the set bits, ascending
        uint32_t i = 0;   // byte at a time, set bits by find-first-set
        for (uint64_t v8 = 0; i < wcnt; v8++) {
            if ((uint64_t)(end - q) <= v8) return -1;
            for (uint32_t x = q[v8]; x && i < wcnt; x &= x - 1) pindex[i++] = (uint32_t)(8 * v8 + __ffs(x) - 1);
        }
    }
    q += pindex[wcnt - 1] / 8 + 1;
    if (end - q < 4) return -1;
    const uint32_t G = rd32(q);
    q += 4;
    uint32_t N;
    BitRd gr{nullptr, 0, 0, 0, 0};
    uint32_t *grc = glc + Gmax;
    if (G > 1) {
        if (G > Gmax || (uint64_t)(end - q) < 8ull * (G - 1) + 8) return -1;
        for (uint32_t j = 0; j + 1 < G; j++) {
            glc[j] = rd32(q);
            grc[j] = rd32(q + 4);
            q += 8;
        }
        N = rd32(q);
        const uint32_t W = rd32(q + 4);
        q += 8;
        if ((uint64_t)(end - q) < 4ull * W) return -1;
        gr = BitRd{q, W, 0, 0, 0};
        q += 4ull * W;
    } else {
        if (end - q < 4) return -1;
        N = rd32(q);
        q += 4;
    }
    if ((uint64_t)(end - q) < N || N > cap) return -1;
    const uint8_t *gpos = q;
    q += N;
    // char sub-stream header (huffman_decode_char 930-984, my_huffman_decode_char 1107-1187)
    const uint32_t avail = (uint32_t)(end - q);
    if (avail < 1) return -1;
    const uint32_t ts = q[0], nbm = (2 * ts + 7) / 8, hdr = 1 + nbm + 2 * ts;
    if (avail < hdr + 4) return -1;
    // the char tree is walked bit by bit: copy it to LDS (tpairs / tbm) first
    for (uint32_t k = 0; k < 2 * ts; k++) tpairs[k] = q[1 + nbm + k];
    for (uint32_t k = 0; k < nbm; k++) tbm[k] = q[1 + k];
    const uint8_t *bm = tbm, *pairs = tpairs;
    const uint32_t nw = rd32(q + hdr);
    if ((uint64_t)hdr + 4 + 4ull * nw > avail) return -1;
    BitRd cr{q + hdr + 4, nw, 0, 0, 0};
    const uint32_t real = ts + 1;
    bool gdone = false, cdone = false;   // a stream that runs out yields zeros from then on
    uint64_t o = 0;
    for (uint32_t t = 0; t < N; t++) {
        uint32_t g = 0;
        if (G > 1 && !gdone) {   // huffman_decode_idxGroup (3009-3054): root = simple node G-2
            uint32_t node = G - 2;
            for (;;) {
                const int bit = gr.next();
                if (bit < 0) { gdone = true; g = 0; break; }
                uint32_t nx = bit ? grc[node] : glc[node];
                if (nx < G) { g = nx; break; }
                nx -= G;
                if (nx + 1 >= G) return -1;
                node = nx;
            }
        }
        uint32_t ch = 0;
        if (ts > 0 && !cdone) {
            uint32_t node = ts - 1;
            for (;;) {
                const int bit = cr.next();
                if (bit < 0) { cdone = true; ch = 0; break; }
                const uint32_t k = 2 * node + (uint32_t)bit;
                const uint32_t v = pairs[k];
                if (!((bm[k >> 3] >> (k & 7)) & 1)) { ch = v; break; }
                const uint32_t nx = v - (256 - real);
                if (v < 256 - real || nx >= ts) return -1;
                node = nx;
            }
        }
        const uint32_t r = (G > 1 ? g * 256u : 0u) + gpos[t];   // 3586-3595
        if (r >= wcnt) return -1;
        const uint32_t ix = pindex[r];
        uint32_t L = 0;
        if (ix != 0) {   // my_LZ78_decompress (1901-1934): phrase[ix - 1] + c
            if (ix > t) return -1;
            L = plen[ix - 1];
            if (o + L + 1 > cap) return -1;
            const uint8_t *src = out + pstart[ix - 1];
            for (uint32_t k = 0; k < L; k++) out[o + k] = src[k];
        }
        if (o + L + 1 > cap) return -1;
        out[o + L] = (uint8_t)ch;
        pstart[t] = (uint32_t)o;
        plen[t] = L + 1;
        o += L + 1;
    }
    if (o > 0 && out[o - 1] == 0) o--;   // 3701-3703
    return (int64_t)o;
}

constexpr uint32_t kDecGmax = FCX_MAX_BLOCK_BYTES / 256 + 4;   // groups of a <= 1 MiB block

__global__ __launch_bounds__(64) void k78_decode(Dec78 D) {   // one wave per record, lane 0 decodes
    const uint32_t b = blockIdx.x;
    // group tree children (2 x Gmax) and the char tree live in LDS for the bit walks
    __shared__ uint32_t gtree[2 * kDecGmax];
    __shared__ uint8_t tpairs[512], tbm[64];
    if (b >= D.nb || threadIdx.x != 0) return;
    const uint64_t B = D.B;
    const int64_t r = dec_block(D.in + D.roff[b], D.rlen[b], D.out + b * B, B, D.pindex + b * (B + 2),
                                D.pstart + b * B, D.plen + b * B, gtree, kDecGmax, tpairs, tbm);
    D.dlen[b] = r < 0 ? ~0ull : (uint64_t)r;
}

__global__ __launch_bounds__(256) void k78_pack_out(Dec78 D, const uint64_t *__restrict__ doff,
                                                    uint8_t *__restrict__ dst) {
    const uint32_t b = blockIdx.y;
    const uint64_t n = D.dlen[b], o = doff[b];
    const uint8_t *src = D.out + (uint64_t)b * D.B;
    for (uint64_t p = blockIdx.x * 256 + threadIdx.x; p < n; p += gridDim.x * 256) dst[o + p] = src[p];
}

}  // namespace fcx78

namespace {
constexpr uint32_t kDecBatch = 1024;   // records decoded concurrently (one walker each; ~13 MB of scratch per record)

struct DevBuf {
    void *p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

// decodes `nrec` records whose payloads sit at host `in` + roff[i] (rlen[i] bytes);
// writes the decoded bytes densely to host `out`
int lz78_decode_records(const uint8_t *in, uint64_t in_len, const std::vector<uint64_t> &roff,
                        const std::vector<uint32_t> &rlen, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    const uint32_t nrec = (uint32_t)roff.size();
    *out_len = 0;
    if (nrec == 0) return FCX_OK;
    const uint32_t B = FCX_MAX_BLOCK_BYTES + 8, Gmax = 1;   // group trees live in LDS (k78_decode)
    const uint32_t nb = std::min(nrec, kDecBatch);
    DevBuf din, dscr;
    H78(hipMalloc(&din.p, in_len ? in_len : 16));
    H78(hipMemcpy(din.p, in, in_len, hipMemcpyHostToDevice));
    const uint64_t nbl = nb;
    const uint64_t sz[] = {nbl * 8, nbl * 4, nbl * B, nbl * (B + 2) * 4, nbl * B * 4, nbl * B * 4,
                           nbl * 2 * Gmax * 4, nbl * 8, nbl * 8, std::min<uint64_t>(cap, nbl * B) + 16};
    constexpr int K = sizeof(sz) / sizeof(sz[0]);
    uint64_t offs[K], tot = 0;
    for (int i = 0; i < K; i++) {
        offs[i] = tot;
        tot += (sz[i] + 255) & ~255ull;
    }
    H78(hipMalloc(&dscr.p, tot));
    char *m = (char *)dscr.p;
    Dec78 D;
    D.B = B;
    D.Gmax = Gmax;
    D.in = (const uint8_t *)din.p;
    uint64_t *d_roff = (uint64_t *)(m + offs[0]);
    uint32_t *d_rlen = (uint32_t *)(m + offs[1]);
    D.roff = d_roff;
    D.rlen = d_rlen;
    D.out = (uint8_t *)(m + offs[2]);
    D.pindex = (uint32_t *)(m + offs[3]);
    D.pstart = (uint32_t *)(m + offs[4]);
    D.plen = (uint32_t *)(m + offs[5]);
    D.lc = (uint32_t *)(m + offs[6]);
    D.dlen = (uint64_t *)(m + offs[7]);
    uint64_t *d_doff = (uint64_t *)(m + offs[8]);
    uint8_t *d_dst = (uint8_t *)(m + offs[9]);
    std::vector<uint64_t> dl(nb), doff(nb);
    uint64_t o = 0;
    for (uint32_t r0 = 0; r0 < nrec; r0 += nb) {
        D.nb = std::min(nb, nrec - r0);
        H78(hipMemcpy(d_roff, roff.data() + r0, 8ull * D.nb, hipMemcpyHostToDevice));
        H78(hipMemcpy(d_rlen, rlen.data() + r0, 4ull * D.nb, hipMemcpyHostToDevice));
        k78_decode<<<D.nb, 64>>>(D);
        H78(hipGetLastError());
        H78(hipMemcpy(dl.data(), D.dlen, 8ull * D.nb, hipMemcpyDeviceToHost));
        uint64_t bo = 0;
        for (uint32_t i = 0; i < D.nb; i++) {
            if (dl[i] == ~0ull)
                return fail78(FCX_ERR_FORMAT, "fcx_lz78: malformed record " + std::to_string(r0 + i + 1));
            doff[i] = bo;
            bo += dl[i];
        }
        if (o + bo > cap) return fail78(FCX_ERR_CAPACITY, "fcx_lz78: decoded output exceeds capacity");
        H78(hipMemcpy(d_doff, doff.data(), 8ull * D.nb, hipMemcpyHostToDevice));
        k78_pack_out<<<dim3(64, D.nb), 256>>>(D, d_doff, d_dst);
        H78(hipGetLastError());
        H78(hipMemcpy(out + o, d_dst, bo, hipMemcpyDeviceToHost));
        o += bo;
    }
    *out_len = o;
    return FCX_OK;
}
}  // namespace

extern "C" {

int64_t fcx_lz78_decompress_block(const uint8_t *in, uint32_t len, uint8_t *out, uint64_t cap) {
    if (!in || !out) return fail78(FCX_ERR_ARG, "fcx_lz78_decompress_block: NULL argument");
    std::vector<uint64_t> roff{0};
    std::vector<uint32_t> rlen{len};
    uint64_t n = 0;
    if (int rc = lz78_decode_records(in, len, roff, rlen, out, cap, &n)) return rc;
    return (int64_t)n;
}

int fcx_lz78_decompress_host(const uint8_t *in, uint64_t in_len, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    if (!in || !out_len || (cap && !out)) return fail78(FCX_ERR_ARG, "fcx_lz78_decompress_host: NULL argument");
    // header check as main() (4140-4159): "FCX" magic, anything but '7' selects LZ78
    if (in_len < FCX_HEADER_BYTES || memcmp(in, "FCX", 3) != 0 || in[3] == '7')
        return fail78(FCX_ERR_FORMAT, "fcx_lz78_decompress_host: not an FCX8 (LZ78) stream");
    uint16_t nblk;
    memcpy(&nblk, in + 8, 2);
    std::vector<uint64_t> roff;
    std::vector<uint32_t> rlen;
    uint64_t q = FCX_HEADER_BYTES;
    for (uint32_t b = 0; b < nblk; b++) {
        if (q + 4 > in_len) return fail78(FCX_ERR_FORMAT, "fcx_lz78: truncated record length");
        uint32_t sz;
        memcpy(&sz, in + q, 4);
        q += 4;
        if (q + sz > in_len) return fail78(FCX_ERR_FORMAT, "fcx_lz78: truncated record");
        roff.push_back(q);
        rlen.push_back(sz);
        q += sz;
    }
    // bytes after the block_num counted records are ignored, as main() does (4162-4201: it reads
    // block_num records and judges the result by size).  The u16 count wraps past 65535
    // blocks (:105), so such a file decodes to its counted blocks and the CLI reports FAIL
    // on the size, like the reference.
    return lz78_decode_records(in, in_len, roff, rlen, out, cap, out_len);
}

}  // extern "C"
