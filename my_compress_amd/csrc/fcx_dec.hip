// fcx_dec.hip — GPU decoder of FCX7 / LZ77 block records (gfx950).
//
// Replaces my_decompress_file_lz77 (my_compress.cpp:2255-2393) with its callees
// my_huffman_decode_char (1107-1187), golomb_rice_decode (309-358),
// decombine_bits (1315-1338) and my_LZ77_decompress (1716-1735), for a whole
// device-resident run of block records ([u32 len][payload]..., the file minus
// its 10-byte header).  The decoded bytes equal the reference decoder's,
// including its quirks: a single-symbol Huffman sub-stream (ts = 0, W = 0)
// decodes as zeros, symbols the words run out of stay zero, and the block stops
// at the first match token it has no (p, l) for (2331-2335).
//
//   k_dindex  one thread walks the record lengths (a sequential chain of u32s);
//   k_dhead   one thread per block parses the payload header: N, the four
//             sub-stream headers (tree, W, words), pCnt, G; bounds-checked;
//   k_dscan   block offsets of the decoded symbols, golomb values and tokens;
//   k_dtable  one wave per sub-stream: parent links from the serialized tree,
//             codes (root->leaf paths, LSB-first) and a 1024-entry lookup table
//             (codes <= 10 bits resolve in one probe, longer ones continue from
//             their depth-10 node);
//   k_dsyms   one workgroup per sub-stream: the bit stream is cut into 1024-bit
//             segments, one per lane; lanes agree on each segment's first code
//             boundary by a Jacobi fixed point (Huffman codes resynchronise
//             within a few symbols), scan their symbol counts and decode again
//             into place.  The same machinery decodes the Golomb-Rice lengths;
//   k_dlen    one workgroup per block: the early-stop token, sum of lengths =
//             decoded block size; k_dscan_out: output offsets;
//   k_dlz     one workgroup per block walks its tokens in steps: each step takes
//             the tokens whose output fits an LDS tile, scatters literal bytes
//             and copy links (x -> x - p), and resolves the links by pointer
//             jumping against the tile and the 2 KiB history before it.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fcx.h"
#include "fcx_device.h"

namespace fcx {
void set_last_error(const std::string &m);

// device error bits of the decoder
constexpr uint32_t kDErrRecord = 1, kDErrHeader = 2, kDErrTree = 4, kDErrGolomb = 8, kDErrDist = 16,
                   kDErrOutCap = 32, kDErrScratch = 64;

constexpr uint32_t kDSymThreads = 1024;
constexpr uint32_t kDLzThreads = 1024;
constexpr uint32_t kDLzTile = 8192;              // output bytes resolved per LDS step
constexpr uint32_t kDLzTPT = 4;                  // tokens read per lane and step
constexpr uint32_t kDTblBits = 10;
constexpr uint32_t kMaxTokensPerBlock = FCX_MAX_BLOCK_BYTES;

struct DStream {         // one Huffman sub-stream (or the raw flags byte)
    uint64_t words_bit;  // absolute bit offset of the code words in the input
    uint64_t pairs_off;  // byte offset of the (l, r) pairs; bitmap is just before
    uint64_t dst;        // byte offset of the decoded symbols in the symbol scratch
    uint32_t nbits;      // 32 W
    uint32_t count;      // symbols to produce
    uint32_t ts;         // internal nodes (0: single symbol, decodes as zeros)
    uint32_t raw;        // 1: no Huffman stream, `rawv` is the one flags byte (nb <= 1)
    uint32_t rawv;
    uint32_t pad;
};

struct DBlock {
    uint64_t payload_off;   // byte offset of the payload in the input
    uint64_t sym_off;       // symbol scratch: [flags nb][chars N][P bytes][golomb 4G], 4-aligned parts
    uint64_t glen_off;      // index of this block's first golomb value
    uint64_t out_off;       // output byte offset
    uint32_t payload_len;
    uint32_t N, pcnt, G, nb, pbytes;
    uint32_t n_eff, pc_eff; // tokens decoded (early stop) and matches among them
    uint32_t out_len;
    uint32_t glen_got;      // golomb values decoded
    uint32_t pad[2];
};

__device__ inline uint32_t ld_u32le(const uint8_t *p, uint64_t off) {
    return p[off] | (p[off + 1] << 8) | (p[off + 2] << 16) | ((uint32_t)p[off + 3] << 24);
}

// ---------------------------------------------------------------------------
__global__ void k_dindex(const uint8_t *in, uint64_t in_len, uint32_t nblocks, DBlock *blk, uint32_t *err) {
    uint64_t off = 0;
    for (uint32_t b = 0; b < nblocks; b++) {
        if (off + 4 > in_len) { atomicOr(err, kDErrRecord); return; }
        const uint32_t len = ld_u32le(in, off);
        if (len > in_len - off - 4) { atomicOr(err, kDErrRecord); return; }
        blk[b].payload_off = off + 4;
        blk[b].payload_len = len;
        off += 4 + (uint64_t)len;
    }
}

struct HCursor {
    const uint8_t *in;
    uint64_t p, end;
    bool ok;
    __device__ uint32_t u32() {
        if (p + 4 > end) { ok = false; return 0; }
        const uint32_t v = ld_u32le(in, p);
        p += 4;
        return v;
    }
    __device__ uint64_t take(uint64_t n) {
        if (n > end - p) { ok = false; return p; }
        const uint64_t q = p;
        p += n;
        return q;
    }
};

__device__ bool parse_sub(HCursor &c, DStream &s, uint32_t count) {
    const uint64_t tsb = c.take(1);
    if (!c.ok) return false;
    const uint32_t ts = c.in[tsb];
    const uint32_t nbm = (2 * ts + 7) / 8;
    c.take(nbm);
    s.pairs_off = c.take(2ull * ts);
    const uint32_t W = c.u32();
    const uint64_t wo = c.take(4ull * W);
    if (!c.ok || W > (1u << 26)) return false;
    s.words_bit = 8 * wo;
    s.nbits = 32 * W;
    s.ts = ts;
    s.count = count;
    s.raw = 0;
    s.rawv = 0;
    return true;
}

// one thread per block: payload header (my_decompress_file_lz77 2255-2330)
__global__ void k_dhead(const uint8_t *in, uint32_t nblocks, DBlock *blk, DStream *ds, uint64_t *symb,
                        uint32_t *err) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblocks) return;
    if (*err & kDErrRecord) return;
    DBlock &B = blk[b];
    HCursor c{in, B.payload_off, B.payload_off + B.payload_len, true};
    DStream *s = ds + 4ull * b;
    const uint32_t N = c.u32();
    bool ok = c.ok && N <= kMaxTokensPerBlock;
    const uint32_t nb = (N + 7) / 8;
    if (ok) {
        if (nb > 1) ok = parse_sub(c, s[0], nb);
        else {
            const uint64_t r = c.take(nb);
            s[0] = DStream{};
            s[0].raw = 1;
            s[0].count = nb;
            s[0].rawv = (c.ok && nb) ? c.in[r] : 0u;
            ok = c.ok;
        }
    }
    if (ok) ok = parse_sub(c, s[1], N);
    uint32_t pcnt = 0, pbytes = 0, G = 0;
    if (ok) {
        pcnt = c.u32();
        ok = c.ok && pcnt <= N;
    }
    if (ok) {
        pbytes = (kPBits * pcnt) / 8 + 1;   // :2311
        ok = parse_sub(c, s[2], pbytes);
    }
    if (ok) {
        G = c.u32();
        // a Golomb code is <= 67 bits (l <= 257): more words than that cannot be valid
        ok = c.ok && (uint64_t)G <= (67ull * pcnt + 31) / 32 + 1;
    }
    if (ok) {
        if (G > 0) ok = parse_sub(c, s[3], 4 * G);
        else { s[3] = DStream{}; s[3].count = 0; s[3].raw = 1; }
    }
    if (!ok) {
        atomicOr(err, kDErrHeader);
        B.N = B.nb = B.pcnt = B.G = B.pbytes = 0;
        for (int q = 0; q < 4; q++) { s[q] = DStream{}; s[q].raw = 1; }
        symb[b] = 0;
        return;
    }
    B.N = N; B.nb = nb; B.pcnt = pcnt; B.G = G; B.pbytes = pbytes;
    auto a4 = [](uint64_t x) { return (x + 3) & ~3ull; };
    symb[b] = a4(nb) + a4(N) + a4(pbytes) + 4ull * G;
}

// exclusive scans over blocks (one workgroup, sequential chunks): symbol bytes,
// golomb values; sets DStream.dst and DBlock.sym_off / glen_off; totals out
__global__ void k_dscan(uint32_t nblocks, DBlock *blk, DStream *ds, const uint64_t *symb, uint64_t *totals) {
    __shared__ uint64_t sh[2][1024 / 64];
    __shared__ uint64_t carry[2];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) { carry[0] = 0; carry[1] = 0; }
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nblocks; b0 += blockDim.x) {
        const uint32_t b = b0 + tid;
        uint64_t v[2] = {b < nblocks ? symb[b] : 0, b < nblocks ? (uint64_t)blk[b].pcnt : 0};
        uint64_t inc[2];
        for (int q = 0; q < 2; q++) {
            inc[q] = v[q];
            for (int o = 1; o < 64; o <<= 1) {
                const uint64_t t = __shfl_up(inc[q], o, 64);
                if (lane >= (uint32_t)o) inc[q] += t;
            }
            if (lane == 63) sh[q][wv] = inc[q];
        }
        __syncthreads();
        uint64_t pre[2], tot[2];
        for (int q = 0; q < 2; q++) {
            uint64_t p = 0, a = 0;
            for (uint32_t w = 0; w < blockDim.x / 64; w++) {
                if (w < wv) p += sh[q][w];
                a += sh[q][w];
            }
            pre[q] = carry[q] + p + inc[q] - v[q];
            tot[q] = a;
        }
        if (b < nblocks) {
            DBlock &B = blk[b];
            B.sym_off = pre[0];
            B.glen_off = pre[1];
            auto a4 = [](uint64_t x) { return (x + 3) & ~3ull; };
            DStream *s = ds + 4ull * b;
            s[0].dst = pre[0];
            s[1].dst = pre[0] + a4(B.nb);
            s[2].dst = s[1].dst + a4(B.N);
            s[3].dst = s[2].dst + a4(B.pbytes);
        }
        __syncthreads();
        if (tid == 0) { carry[0] += tot[0]; carry[1] += tot[1]; }
        __syncthreads();
    }
    if (tid == 0) { totals[0] = carry[0]; totals[1] = carry[1]; }   // the host sizes the scratch from these
}

// ---------------------------------------------------------------------------
// decode tables: one wave per (block, stream) with a tree.
// tbl[1024] u16: bit 15 clear: symbol | len << 8 (len <= 10); bit 15 set: continue
// the tree walk from internal node (entry & 0x1FF) after 10 bits; 0xFFFF: invalid.
// child[2 * 256] u16: < 256 leaf symbol, 256 + k internal node k.
__global__ __launch_bounds__(64) void k_dtable(const uint8_t *in, uint32_t nblocks, const DStream *ds,
                                               uint16_t *tbl, uint16_t *child, uint32_t *err) {
    __shared__ uint16_t ch[512];
    __shared__ uint16_t par[256];    // parent node | side << 15; 0xFFFF = none
    __shared__ uint8_t dep[256];
    __shared__ uint32_t code[256];
    __shared__ uint32_t bad;
    const uint32_t q = blockIdx.x, lane = threadIdx.x;
    if (q >= 4 * nblocks) return;
    const DStream s = ds[q];
    if (s.raw || s.ts == 0 || s.count == 0) return;
    const uint32_t ts = s.ts, real = ts + 1;
    const uint64_t bm_off = s.pairs_off - (2 * ts + 7) / 8;
    if (lane == 0) bad = 0;
    for (uint32_t k = lane; k < 256; k += 64) par[k] = 0xFFFF;
    __syncthreads();
    // children (1042-1057: an internal child k is stored as (256 - real) + k)
    for (uint32_t x = lane; x < 2 * ts; x += 64) {
        const bool internal = (in[bm_off + (x >> 3)] >> (x & 7)) & 1;
        uint32_t v = in[s.pairs_off + x];
        if (internal) {
            const uint32_t k = v - (256 - real);
            // a child is created before its parent: k < x / 2 keeps the tree acyclic
            if (v < 256 - real || k >= x / 2) { bad = 1; v = 0; }
            else v = 256 + k;
        }
        ch[x] = (uint16_t)v;
    }
    __syncthreads();
    for (uint32_t x = lane; x < 2 * ts; x += 64)
        if (ch[x] >= 256) {
            const uint32_t k = ch[x] - 256;
            if (par[k] != 0xFFFF) bad = 1;   // two parents
            par[k] = (uint16_t)((x >> 1) | ((x & 1) << 15));
        }
    __syncthreads();
    // depth and code of every internal node by walking to the root (ts - 1)
    for (uint32_t k = lane; k < ts; k += 64) {
        // gathered leaf-up, the branch at depth i ends in bit i (root first, LSB-first)
        uint32_t d = 0, cd = 0, n = k;
        while (n != ts - 1) {
            const uint32_t pv = par[n];
            if (pv == 0xFFFF || d >= 31) { bad = 1; break; }
            cd = (cd << 1) | (pv >> 15);
            n = pv & 0x7FFF;
            d++;
        }
        dep[k] = (uint8_t)d;
        code[k] = cd;
    }
    __syncthreads();
    uint16_t *T = tbl + 1024ull * q;
    uint16_t *C = child + 512ull * q;
    for (uint32_t x = lane; x < 1024; x += 64) T[x] = 0xFFFF;
    for (uint32_t x = lane; x < 2 * ts; x += 64) C[x] = ch[x];
    __syncthreads();
    __threadfence_block();
    for (uint32_t x = lane; x < 2 * ts; x += 64) {
        const uint32_t node = x >> 1, side = x & 1;
        const uint32_t d = dep[node] + 1u;
        if (d > 32) { bad = 1; continue; }
        const uint32_t cd = code[node] | (side << dep[node]);
        if (ch[x] < 256) {
            if (d <= kDTblBits) {
                const uint16_t e = (uint16_t)(ch[x] | (d << 8));
                for (uint32_t sfx = 0; sfx < (1u << (kDTblBits - d)); sfx++) T[cd | (sfx << d)] = e;
            }
        } else if (d == kDTblBits) {
            T[cd] = (uint16_t)(0x8000u | (ch[x] - 256));
        }
    }
    __syncthreads();
    if (lane == 0 && bad) atomicOr(err, kDErrTree);
}

// ---------------------------------------------------------------------------
// LSB-first sequential bit reader: a 64-bit register buffer fed from a queue of
// four dwords (one 16-B load), with the next 16-B load in flight: the wait for a
// load falls every 128 bits consumed, one load behind.  The byte buffer of `len`
// bytes starts at bit `bit0` of its 16-B-aligned base.
struct BitBuf {
    const uint32_t *w;   // 16-B-aligned base
    uint64_t nw;         // dwords that hold valid bytes
    uint64_t buf, ni;    // ni: next 16-B unit to load
    uint32_t nbuf, qn, q0, q1, q2, q3;
    uint4 nxt;
    __device__ uint4 load4(uint64_t i) const {
        if (4 * i + 4 <= nw) return ((const uint4 *)w)[i];
        uint4 v;
        v.x = 4 * i < nw ? w[4 * i] : 0u;
        v.y = 4 * i + 1 < nw ? w[4 * i + 1] : 0u;
        v.z = 4 * i + 2 < nw ? w[4 * i + 2] : 0u;
        v.w = 4 * i + 3 < nw ? w[4 * i + 3] : 0u;
        return v;
    }
    __device__ uint32_t pop() {
        const uint32_t v = q0;
        q0 = q1; q1 = q2; q2 = q3;
        if (--qn == 0) {
            q0 = nxt.x; q1 = nxt.y; q2 = nxt.z; q3 = nxt.w;
            qn = 4;
            nxt = load4(ni++);
        }
        return v;
    }
    __device__ void refill() {
        if (nbuf <= 32) { buf |= (uint64_t)pop() << nbuf; nbuf += 32; }
    }
    __device__ void seek(uint64_t absbit) {   // afterwards >= 33 bits are buffered
        const uint64_t wi = absbit >> 5, i4 = wi >> 2;
        const uint4 c = load4(i4);
        nxt = load4(i4 + 1);
        ni = i4 + 2;
        const uint32_t skip = (uint32_t)(wi & 3);
        q0 = c.x; q1 = c.y; q2 = c.z; q3 = c.w;
        qn = 4;
        for (uint32_t k = 0; k < skip; k++) (void)pop();
        buf = pop();
        nbuf = 32;
        buf >>= (absbit & 31);
        nbuf -= (uint32_t)(absbit & 31);
        refill();
    }
    __device__ uint32_t peek() const { return (uint32_t)buf; }
    __device__ void drop(uint32_t n) { buf >>= n; nbuf -= n; refill(); }   // n <= 32
};

__device__ inline BitBuf make_bits(const uint8_t *buf, uint64_t len, uint64_t &bit0) {
    const uintptr_t a = (uintptr_t)buf;
    BitBuf s;
    s.w = (const uint32_t *)(a & ~(uintptr_t)15);
    bit0 = 8 * (a & 15);
    s.nw = ((a & 15) + len + 3) / 4;
    s.buf = 0; s.ni = 0; s.nbuf = 0; s.qn = 0; s.q0 = s.q1 = s.q2 = s.q3 = 0;
    s.nxt = make_uint4(0, 0, 0, 0);
    return s;
}

// one Huffman symbol from the low bits of a 32-bit window; len = 0 if none
__device__ inline uint32_t huff_sym(uint32_t win, const uint16_t *T, const uint16_t *C, uint32_t &len) {
    const uint32_t e = T[win & ((1u << kDTblBits) - 1)];
    if (!(e & 0x8000u)) { len = (e >> 8) & 0x1Fu; return e & 0xFFu; }
    len = 0;
    if (e == 0xFFFFu) return 0;
    uint32_t node = e & 0x1FFu;
    win >>= kDTblBits;
    for (uint32_t d = kDTblBits + 1; d <= 32; d++) {   // codes are <= 32 bits (k_dtable)
        const uint32_t nx = C[2 * node + (win & 1u)];
        win >>= 1;
        if (nx < 256) { len = d; return nx; }
        node = nx - 256;
    }
    return 0;
}

// one code at relative bit `pos` (the reader is positioned there); false if the
// stream cannot supply it.  Golomb-Rice (golomb_rice_decode 309-358): q ones, a
// zero, r in 2 bits, value 4q + r.
template <bool GOLOMB>
__device__ inline bool code_step(BitBuf &bb, uint32_t &pos, uint32_t nbits, const uint16_t *T, const uint16_t *C,
                                 uint32_t &v) {
    if (!GOLOMB) {
        uint32_t len;
        v = huff_sym(bb.peek(), T, C, len);
        if (len == 0 || pos + len > nbits) return false;
        bb.drop(len);
        pos += len;
        return true;
    }
    uint32_t q = 0;
    for (;;) {
        const uint32_t w = bb.peek();
        if (w == 0xFFFFFFFFu) {
            q += 32;
            pos += 32;
            if (pos + 3 > nbits) return false;
            bb.drop(32);
            continue;
        }
        const uint32_t ones = (uint32_t)__builtin_ctz(~w);
        q += ones;
        pos += ones;
        if (pos + 3 > nbits) return false;
        bb.drop(ones);
        v = 4 * q + ((bb.peek() >> 1) & 3u);
        bb.drop(3);
        pos += 3;
        return true;
    }
}

// Segment decoder: one workgroup decodes `count` symbols of an nbits stream at
// absolute bit sb.  Lane i owns bits [i S, (i+1) S) (S = nbits / lanes, a multiple
// of 32) and decodes the codes that START there.  The first code boundary in each
// segment is agreed by a Jacobi fixed point, start_{i+1} = exit of segment i
// walked from start_i; only lanes whose start moved walk again.  Huffman codes
// resynchronise within a few symbols, so this settles in 2-3 rounds; past
// kDMaxRounds the lanes walk one after another (exact, serial).  Then a scan of
// the counts and a second walk that stores the symbols.  Returns symbols produced.
constexpr uint32_t kDMaxRounds = 12;
constexpr uint32_t kDMinSegBits = 256;
constexpr uint32_t kDRetryScale = 16;   // an unsettled stream retries with segments this much longer

template <bool GOLOMB>
__device__ uint32_t seg_decode(const BitBuf &src, uint64_t sb, uint32_t nbits, uint32_t count, const uint16_t *T,
                               const uint16_t *C, uint8_t *dst8, uint32_t *dst32, uint32_t *st, uint32_t *cnt,
                               uint32_t *flag, uint64_t *stats) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    constexpr uint32_t kW = kDSymThreads / 64;
    // segments of >= kDMinSegBits (Jacobi needs room to resynchronise), a multiple of 32
    const uint32_t S0 = max(kDMinSegBits, ((nbits + kDSymThreads - 1) / kDSymThreads + 31) & ~31u);
    uint32_t seg_lo = 0, seg_hi = 0;
    auto walk = [&](uint32_t start, uint32_t &ex) -> uint32_t {
        BitBuf bb = src;
        uint32_t pos = start, n = 0, v;
        bool ok = true;
        if (pos < seg_hi) bb.seek(sb + pos);
        while (pos < seg_hi) {
            if (!code_step<GOLOMB>(bb, pos, nbits, T, C, v)) { ok = false; break; }
            n++;
        }
        ex = ok ? pos : nbits;   // a code that cannot complete ends the stream
        return n;
    };
    bool settled = false;
    uint32_t rounds = 0, mine = 0, ex = 0, n = 0;
    // codes that resynchronise slowly (near fixed-length, e.g. the packed distance
    // bytes) may not settle within short segments: a second attempt uses longer ones
    for (uint32_t attempt = 0; attempt < 2 && !settled; attempt++) {
        const uint64_t S = attempt == 0 ? S0 : (uint64_t)S0 * kDRetryScale;
        seg_lo = (uint32_t)min<uint64_t>(tid * S, nbits);
        seg_hi = (uint32_t)min<uint64_t>(seg_lo + S, nbits);
        __syncthreads();
        st[tid] = seg_lo;
        if (tid == 0) { flag[0] = 0; flag[1] = 0; }
        __syncthreads();
        mine = seg_lo;
        n = walk(mine, ex);
        for (uint32_t round = 0; round < kDMaxRounds; round++) {
            if (tid == 0) flag[(round + 1) & 1] = 0;
            if (tid + 1 < kDSymThreads && st[tid + 1] != ex) { st[tid + 1] = ex; flag[round & 1] = 1; }
            __syncthreads();
            rounds++;
            if (!flag[round & 1]) { settled = true; break; }
            if (st[tid] != mine) { mine = st[tid]; n = walk(mine, ex); }
            __syncthreads();
        }
    }
    if (!settled) {   // serial fallback over the long segments: every start exact before its lane walks
        const uint32_t active = (uint32_t)min<uint64_t>(kDSymThreads, (nbits + (uint64_t)S0 * kDRetryScale - 1) /
                                                                         ((uint64_t)S0 * kDRetryScale));
        for (uint32_t i = 0; i < active; i++) {
            if (tid == i) {
                mine = st[i];
                n = walk(mine, ex);
                if (i + 1 < kDSymThreads) st[i + 1] = ex;
            }
            __syncthreads();
        }
        mine = st[tid];
        if (tid >= active) n = 0;
    }
    if (tid == 0 && stats) {   // Jacobi rounds, serial fallbacks
        atomicAdd((unsigned long long *)stats, (unsigned long long)rounds);
        if (!settled) atomicAdd((unsigned long long *)stats + 1, 1ull);
        if (!settled && !GOLOMB) atomicAdd((unsigned long long *)stats + 4 + (blockIdx.x & 3), 1ull);
    }
    // exclusive scan of the per-lane counts
    uint32_t inc = n;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += t;
    }
    if (lane == 63) cnt[wv] = inc;
    __syncthreads();
    uint32_t idx = inc - n, tot = 0;
    for (uint32_t w = 0; w < kW; w++) {
        if (w < wv) idx += cnt[w];
        tot += cnt[w];
    }
    // walk again and store
    if (mine < seg_hi && idx < count) {
        BitBuf bb = src;
        uint32_t pos = mine, v;
        bb.seek(sb + pos);
        const uint32_t stop = min(count, idx + n);
        if (GOLOMB) {
            while (idx < stop && code_step<GOLOMB>(bb, pos, nbits, T, C, v)) dst32[idx++] = v;
        } else {
            // whole dwords inside this lane's range are stored at once; the partial
            // dwords at its two ends (shared with neighbours) byte by byte
            const uint32_t first = idx;
            uint32_t acc = 0;
            while (idx < stop && code_step<GOLOMB>(bb, pos, nbits, T, C, v)) {
                acc |= v << (8 * (idx & 3));
                if ((idx & 3) == 3) {
                    if (idx - 3 >= first) ((uint32_t *)dst8)[idx >> 2] = acc;
                    else
                        for (uint32_t q = first; q <= idx; q++) dst8[q] = (uint8_t)(acc >> (8 * (q & 3)));
                    acc = 0;
                }
                idx++;
            }
            if (idx & 3)
                for (uint32_t q = max(first, idx & ~3u); q < idx; q++) dst8[q] = (uint8_t)(acc >> (8 * (q & 3)));
        }
    }
    __syncthreads();
    return min(tot, count);
}

// one workgroup per sub-stream: Huffman symbols into the symbol scratch.  64 VGPRs (a few
// spilled) for two workgroups per CU: the serial code walks are latency-bound, and twice
// the waves took text's symbol streams from 15.1 to 9.9 ms per GiB
__global__ __launch_bounds__(kDSymThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_dsyms(const uint8_t *in, uint64_t in_len, uint32_t nblocks,
                                                        const DStream *ds, const uint16_t *tbl, const uint16_t *child,
                                                        uint8_t *sym, const uint32_t *err, uint64_t *stats) {
    __shared__ uint16_t T[1u << kDTblBits];
    __shared__ uint16_t C[512];
    __shared__ uint32_t st[kDSymThreads + 1];
    __shared__ uint32_t cnt[kDSymThreads / 64];
    __shared__ uint32_t flag[2];
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    if (q >= 4 * nblocks || (*err & (kDErrRecord | kDErrHeader | kDErrTree | kDErrScratch))) return;
    const DStream s = ds[q];
    uint8_t *dst = sym + s.dst;
    if (s.raw) {
        if (tid == 0 && s.count) dst[0] = (uint8_t)s.rawv;
        return;
    }
    uint32_t got = 0;
    if (s.ts != 0 && s.count != 0) {
        for (uint32_t x = tid; x < (1u << kDTblBits); x += kDSymThreads) T[x] = tbl[(1ull << kDTblBits) * q + x];
        for (uint32_t x = tid; x < 2 * s.ts; x += kDSymThreads) C[x] = child[512ull * q + x];
        __syncthreads();
        // every code 8 bits long (a complete depth-8 tree: the chars of random data): the
        // codes are the stream's bytes (the words start on a byte), so symbol i is T[byte i]
        // - a byte substitution, no segment agreement
        static_assert(kDSymThreads == (1u << kDTblBits), "one table entry per lane");
        const uint32_t e = T[tid];
        if (__syncthreads_and(!(e & 0x8000u) && ((e >> 8) & 0x1Fu) == 8u)) {
            got = min(s.count, s.nbits / 8);
            const uintptr_t a = (uintptr_t)(in + (s.words_bit >> 3)), aw = a & ~(uintptr_t)3;
            const uint32_t sh = (uint32_t)(a & 3);
            const uint32_t *w = (const uint32_t *)aw;
            const uint64_t vlim = (uint64_t)((uintptr_t)in + in_len - aw);   // valid bytes from w
            const uint64_t wlim = vlim / 4;                                   // whole dwords from w
            const uint32_t ndw = (got + 3) / 4;
            uint32_t *d32 = (uint32_t *)dst;
            // output dword j = lane + 1024 i: consecutive lanes touch consecutive dwords (loads
            // and stores coalesce); kU dwords per lane and step, all loads in flight together
            auto ld = [&](uint64_t wi) -> uint32_t {
                if (wi < wlim) return w[wi];
                uint32_t x = 0;   // the buffer's last partial dword, byte by byte
                for (uint32_t q = 0; q < 4; q++)
                    if (4 * wi + q < vlim) x |= (uint32_t)((const uint8_t *)aw)[4 * wi + q] << (8 * q);
                return x;
            };
            constexpr uint32_t kU = 4;
            for (uint32_t j00 = tid; j00 < ndw; j00 += kDSymThreads * kU) {
                uint32_t v0[kU], v1[kU];
#pragma unroll
                for (uint32_t u = 0; u < kU; u++) {
                    const uint32_t j = j00 + kDSymThreads * u;
                    v0[u] = j < ndw ? ld(j) : 0u;
                    v1[u] = j < ndw ? ld((uint64_t)j + 1) : 0u;
                }
#pragma unroll
                for (uint32_t u = 0; u < kU; u++) {
                    const uint32_t j = j00 + kDSymThreads * u;
                    if (j >= ndw) break;
                    const uint32_t c = __builtin_amdgcn_alignbyte(v1[u], v0[u], sh);
                    uint32_t o = 0;
#pragma unroll
                    for (uint32_t q = 0; q < 4; q++)
                        if (4 * j + q < got) o |= (uint32_t)(T[(c >> (8 * q)) & 0xFFu] & 0xFFu) << (8 * q);
                    d32[j] = o;   // (bytes past `got` are zero, as the tail below writes them)
                }
            }
        } else {
            uint64_t bit0;
            const BitBuf src = make_bits(in, in_len, bit0);
            got = seg_decode<false>(src, bit0 + s.words_bit, s.nbits, s.count, T, C, dst, nullptr, st, cnt, flag, stats);
        }
    }
    // symbols the words do not cover stay zero (the reference memsets, 1107-1187)
    for (uint32_t x = got + tid; x < s.count; x += kDSymThreads) dst[x] = 0;
}

// one workgroup per block: the pCnt Golomb-Rice lengths from the decoded golomb bytes
__global__ __launch_bounds__(kDSymThreads) void k_dgolomb(uint32_t nblocks, DBlock *blk, const DStream *ds,
                                                          const uint8_t *sym, uint32_t *glen, uint32_t *err,
                                                          uint64_t *stats) {
    __shared__ uint32_t st[kDSymThreads + 1];
    __shared__ uint32_t cnt[kDSymThreads / 64];
    __shared__ uint32_t flag[2];
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    if (b >= nblocks || (*err & (kDErrRecord | kDErrHeader | kDErrTree | kDErrScratch))) return;
    DBlock &B = blk[b];
    const uint32_t pcnt = B.pcnt;
    uint32_t got = 0;
    if (pcnt > 0) {
        const DStream s = ds[4ull * b + 3];
        const uint64_t nbytes = 4ull * B.G;
        uint64_t bit0;
        const BitBuf src = make_bits(sym + s.dst, nbytes, bit0);
        got = seg_decode<true>(src, bit0, (uint32_t)(8 * nbytes), pcnt, nullptr, nullptr, nullptr,
                               glen + B.glen_off, st, cnt, flag, stats + 2);
    }
    if (tid == 0) {
        B.glen_got = got;
        if (got < pcnt) atomicOr(err, kDErrGolomb);   // golomb stream too short: FORMAT
    }
}

// ---------------------------------------------------------------------------
// block-wide exclusive scan (blockDim.x threads, <= 16 waves); returns the prefix, total in *tot
__device__ inline uint32_t block_xscan(uint32_t v, uint32_t *sh, uint32_t *tot) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t inc = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += t;
    }
    if (lane == 63) sh[wv] = inc;
    __syncthreads();
    uint32_t pre = inc - v, all = 0;
    for (uint32_t w = 0; w < nw; w++) {
        const uint32_t x = sh[w];
        if (w < wv) pre += x;
        all += x;
    }
    __syncthreads();
    *tot = all;
    return pre;
}

// one workgroup per block: tokens decoded (the reference stops at the first match
// token past pCnt, 2331-2335), matches among them, decoded length
__global__ __launch_bounds__(256) void k_dlen(uint32_t nblocks, DBlock *blk, const uint8_t *sym,
                                              const uint32_t *glen, uint32_t *err) {
    __shared__ uint32_t sh[4];
    __shared__ uint64_t sh64[4];
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    if (b >= nblocks) return;
    DBlock &B = blk[b];
    if (*err & (kDErrRecord | kDErrHeader | kDErrTree | kDErrScratch | kDErrGolomb)) {
        if (tid == 0) B.out_len = 0;
        return;
    }
    const uint8_t *fl = sym + B.sym_off;
    const uint32_t N = B.N, pcnt = B.pcnt;
    uint32_t z = 0;
    for (uint32_t x = tid; x < B.nb; x += 256) {
        const uint32_t valid = min(8u, N - 8 * x);
        z += (uint32_t)__builtin_popcount(~(uint32_t)fl[x] & ((1u << valid) - 1u));
    }
    uint32_t Z;
    (void)block_xscan(z, sh, &Z);
    uint32_t n_eff = N, pc_eff = Z;
    if (Z > pcnt) {   // more match flags than distances: stop at the (pcnt+1)-th match token
        pc_eff = pcnt;
        if (tid == 0) {
            uint32_t seen = 0, t = 0;
            for (; t < N; t++)
                if (!((fl[t >> 3] >> (t & 7)) & 1)) {
                    if (seen == pcnt) break;
                    seen++;
                }
            sh[0] = t;
        }
        __syncthreads();
        n_eff = sh[0];
        __syncthreads();
    }
    // the reference encoder emits l in [3, 257] (1459-1462); a longer length is malformed
    // here (it could not fit an LZ step), the only stream the host decoder would take
    uint64_t s = 0;
    bool longl = false;
    for (uint32_t i = tid; i < pc_eff; i += 256) {
        const uint32_t l = glen[B.glen_off + i];
        longl = longl || l >= kMaxL;
        s += l;
    }
    if (longl) atomicOr(err, kDErrHeader);
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((tid & 63) == 0) sh64[tid >> 6] = s;
    __syncthreads();
    if (tid == 0) {
        const uint64_t tot = (uint64_t)n_eff + sh64[0] + sh64[1] + sh64[2] + sh64[3];
        B.n_eff = n_eff;
        B.pc_eff = pc_eff;
        if (tot > 0xFFFFFFFFull) { atomicOr(err, kDErrHeader); B.out_len = 0; }
        else B.out_len = (uint32_t)tot;
    }
}

// output offsets of the blocks; total into words[0]; capacity check
__global__ void k_dscan_out(uint32_t nblocks, DBlock *blk, uint64_t cap, uint64_t *words, uint32_t *err) {
    __shared__ uint64_t sh[16];
    __shared__ uint64_t carry;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nblocks; b0 += blockDim.x) {
        const uint32_t b = b0 + tid;
        const uint64_t v = b < nblocks ? blk[b].out_len : 0;
        uint64_t inc = v;
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t t = __shfl_up(inc, o, 64);
            if (lane >= (uint32_t)o) inc += t;
        }
        if (lane == 63) sh[wv] = inc;
        __syncthreads();
        uint64_t pre = carry + inc - v, all = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; w++) {
            if (w < wv) pre += sh[w];
            all += sh[w];
        }
        if (b < nblocks) blk[b].out_off = pre;
        __syncthreads();
        if (tid == 0) carry += all;
        __syncthreads();
    }
    if (tid == 0) {
        words[0] = carry;
        if (carry > cap) atomicOr(err, kDErrOutCap);
    }
}

// one workgroup per block: tokens -> bytes (my_LZ77_decompress 1716-1735).  64 VGPRs and
// four tokens per lane (74 KB of LDS): two workgroups per CU hide the steps' barriers and
// loads (rand 5.3 -> 4.2 ms per GiB, text 8.2 -> 5.7)
constexpr uint32_t kRes = 0x80000000u;   // lk entry: resolved byte (low 8 bits), else link (LDS index)
constexpr uint32_t kHist = 2048;

__device__ inline uint32_t block_xmax(uint32_t v, uint32_t *sh) {   // exclusive running max over threads
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t inc = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc = max(inc, t);
    }
    if (lane == 63) sh[wv] = inc;
    uint32_t ex = __shfl_up(inc, 1, 64);
    if (lane == 0) ex = 0;
    __syncthreads();
    for (uint32_t w = 0; w < wv && w < nw; w++) ex = max(ex, sh[w]);
    __syncthreads();
    return ex;
}

__global__ __launch_bounds__(kDLzThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_dlz(uint32_t nblocks, const DBlock *blk, const DStream *ds,
                                                     const uint8_t *sym, const uint32_t *glen, uint8_t *out,
                                                     uint32_t *err) {
    __shared__ uint8_t ob[kHist + kDLzTile];              // [history | this step's bytes]
    __shared__ __attribute__((aligned(16))) uint32_t lk[kDLzTile];   // token marks, then links / bytes
    __shared__ uint2 tr[kDLzTPT * kDLzThreads];                 // this step's tokens: off | L << 13 | ism << 22 | ok << 23, P | c << 16
    __shared__ uint32_t sh[16];
    __shared__ uint32_t s_any[2];
    __shared__ uint32_t s_used;
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    if (b >= nblocks || *err) return;
    const DBlock B = blk[b];
    const uint8_t *fl = sym + B.sym_off;
    const uint8_t *ch = sym + ds[4ull * b + 1].dst;
    const uint8_t *pb = sym + ds[4ull * b + 2].dst;
    const uint32_t *gl = glen + B.glen_off;
    uint8_t *o = out + B.out_off;
    const uint32_t n_eff = B.n_eff;
    uint32_t tc = 0, mc = 0, oc = 0;
    uint32_t window = kDLzTPT * kDLzThreads;   // tokens read per step, adapted to the token length seen
    bool bad = false;
    while (tc < n_eff) {
        const uint32_t limit = min(n_eff, tc + window);
        uint32_t len[kDLzTPT], L[kDLzTPT], P[kDLzTPT], c[kDLzTPT];
        bool ism[kDLzTPT], valid[kDLzTPT];
        uint32_t nm = 0;
#pragma unroll
        for (uint32_t u = 0; u < kDLzTPT; u++) {
            const uint32_t t = tc + kDLzTPT * tid + u;
            valid[u] = t < limit;
            ism[u] = valid[u] && !((fl[t >> 3] >> (t & 7)) & 1u);
            c[u] = valid[u] ? ch[t] : 0u;
            nm += ism[u] ? 1u : 0u;
        }
        uint32_t mtot;
        uint32_t rank = mc + block_xscan(nm, sh, &mtot);
        if (mtot == 0) {
            // literal tokens only (random data): the bytes are the chars, one per token
            const uint32_t cnt = limit - tc;
#pragma unroll
            for (uint32_t u = 0; u < kDLzTPT; u++)
                if (valid[u]) o[oc + kDLzTPT * tid + u] = (uint8_t)c[u];
            // history = the last 2 KiB of [history | these bytes]
            uint8_t h[kHist / kDLzThreads];
#pragma unroll
            for (uint32_t q = 0; q < kHist / kDLzThreads; q++) {
                const uint32_t j = cnt + tid + q * kDLzThreads;   // index in [history | bytes]
                h[q] = j < kHist ? ob[j] : ch[tc + j - kHist];
            }
            __syncthreads();
#pragma unroll
            for (uint32_t q = 0; q < kHist / kDLzThreads; q++) ob[tid + q * kDLzThreads] = h[q];
            __syncthreads();
            oc += cnt;
            tc += cnt;
            window = kDLzTPT * kDLzThreads;
            continue;
        }
        uint32_t lsum = 0;
#pragma unroll
        for (uint32_t u = 0; u < kDLzTPT; u++) {
            L[u] = 0; P[u] = 0;
            if (ism[u]) {
                L[u] = gl[rank];
                const uint32_t bit = kPBits * rank, k = bit >> 3;
                P[u] = ((pb[k] | (pb[k + 1] << 8) | (pb[k + 2] << 16)) >> (bit & 7)) & 0x7FFu;   // decombine_bits
                rank++;
            }
            len[u] = valid[u] ? (ism[u] ? L[u] + 1 : 1u) : 0u;
            lsum += len[u];
        }
        uint32_t ltot;
        uint32_t off = block_xscan(lsum, sh, &ltot);
        // clear the token marks of this step's tile (8 slots per lane, two 16-B stores)
        ((uint4 *)lk)[2 * tid] = make_uint4(0, 0, 0, 0);
        ((uint4 *)lk)[2 * tid + 1] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        // the tokens whose output fits the tile (a prefix): record + mark at their first byte
        uint32_t taken = 0, mtaken = 0, end = 0;
#pragma unroll
        for (uint32_t u = 0; u < kDLzTPT; u++) {
            if (valid[u] && off + len[u] <= kDLzTile) {
                taken++;
                // a distance before the block start is malformed (reference: Fatal Error,
                // :1727); its bytes resolve to 0 and the error is reported
                const bool okp = !ism[u] || (P[u] != 0 && P[u] <= oc + off);
                bad = bad || !okp;
                mtaken += ism[u] ? 1u : 0u;
                tr[kDLzTPT * tid + u] = make_uint2(off | (L[u] << 13) | ((ism[u] ? 1u : 0u) << 22) | ((okp ? 1u : 0u) << 23),
                                             P[u] | (c[u] << 16));
                lk[off] = kDLzTPT * tid + u + 1;
                end = off + len[u];
            }
            off += len[u];
        }
        uint32_t ttot, mt2;
        (void)block_xscan(taken, sh, &ttot);
        (void)block_xscan(mtaken, sh, &mt2);
        uint32_t umax = end;
        for (int o2 = 32; o2 > 0; o2 >>= 1) umax = max(umax, __shfl_xor(umax, o2, 64));
        if (tid == 0) s_used = 0;
        __syncthreads();
        if ((tid & 63) == 0) atomicMax(&s_used, umax);
        // every position finds its token: running max of the marks over positions
        const uint4 m0 = ((const uint4 *)lk)[2 * tid], m1 = ((const uint4 *)lk)[2 * tid + 1];
        uint32_t mk[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
        uint32_t run = 0;
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) { run = max(run, mk[j]); mk[j] = run; }
        const uint32_t carry = block_xmax(run, sh);
        const uint32_t used = s_used;
        uint32_t val[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const uint32_t x = 8 * tid + j;
            val[j] = 0;
            if (x < used) {
                const uint2 r = tr[max(carry, mk[j]) - 1];
                const uint32_t toff = r.x & 0x1FFFu, tl = (r.x >> 13) & 0x1FFu;
                const uint32_t k = x - toff;
                if (!((r.x >> 22) & 1u) || k == tl) val[j] = kRes | (r.y >> 16);
                else if (!((r.x >> 23) & 1u)) val[j] = kRes;
                else {
                    const uint32_t li = kHist + x - (r.y & 0xFFFFu);
                    val[j] = li < kHist ? (kRes | ob[li]) : li;
                }
            }
        }
        __syncthreads();   // all marks read before the links replace them
        ((uint4 *)lk)[2 * tid] = make_uint4(val[0], val[1], val[2], val[3]);
        ((uint4 *)lk)[2 * tid + 1] = make_uint4(val[4], val[5], val[6], val[7]);
        __syncthreads();
        // pointer jumping: lk[x] <- lk[lk[x]] until every byte is resolved (links point back)
        for (uint32_t r = 0;; r++) {
            if (tid == 0) s_any[r & 1] = 0;
            __syncthreads();
            bool any = false;
            for (uint32_t x = tid; x < used; x += kDLzThreads) {
                const uint32_t v = lk[x];
                if (!(v & kRes)) {
                    const uint32_t w = v < kHist ? (kRes | ob[v]) : lk[v - kHist];
                    lk[x] = w;
                    any = any || !(w & kRes);
                }
            }
            if (any) s_any[r & 1] = 1;
            __syncthreads();
            if (!s_any[r & 1]) break;
        }
        for (uint32_t x = tid; x < used; x += kDLzThreads) {
            const uint8_t v = (uint8_t)lk[x];
            ob[kHist + x] = v;
            o[oc + x] = v;
        }
        __syncthreads();
        // history = the last 2 KiB of [history | step bytes]
        const uint8_t h0 = ob[used + tid], h1 = ob[used + tid + kDLzThreads];
        __syncthreads();
        ob[tid] = h0;
        ob[tid + kDLzThreads] = h1;
        __syncthreads();
        oc += used;
        tc += ttot;
        mc += mt2;
        if (ttot == 0) { bad = true; break; }   // cannot happen for l <= 257 (k_dlen)
        // next window: enough tokens for about 1.25 tiles at this step's mean length
        window = min(kDLzTPT * kDLzThreads, max(256u, (uint32_t)(5ull * kDLzTile * ttot / (4ull * max(used, 1u)))));
    }
    if (bad) atomicOr(err, kDErrDist);
}

void dec_launch(const uint8_t *d_in, uint64_t in_len, uint32_t nblocks, uint8_t *d_out, uint64_t cap, DBlock *blk,
                DStream *ds, uint64_t *symb, uint16_t *tbl, uint16_t *child, uint8_t *sym, uint32_t *glen,
                uint64_t *words, uint32_t *err, int phase, hipStream_t st, hipEvent_t *ev) {
    if (phase == 0) {
        hipLaunchKernelGGL(k_dindex, dim3(1), dim3(1), 0, st, d_in, in_len, nblocks, blk, err);
        hipLaunchKernelGGL(k_dhead, dim3((nblocks + 255) / 256), dim3(256), 0, st, d_in, nblocks, blk, ds, symb, err);
        hipLaunchKernelGGL(k_dscan, dim3(1), dim3(1024), 0, st, nblocks, blk, ds, symb, words + 2);
        return;
    }
    auto mark = [&](int i) { if (ev) (void)hipEventRecord(ev[i], st); };
    mark(0);
    hipLaunchKernelGGL(k_dtable, dim3(4 * nblocks), dim3(64), 0, st, d_in, nblocks, ds, tbl, child, err);
    mark(1);
    hipLaunchKernelGGL(k_dsyms, dim3(4 * nblocks), dim3(kDSymThreads), 0, st, d_in, in_len, nblocks, ds, tbl, child, sym, err,
                       words + 4);
    mark(2);
    hipLaunchKernelGGL(k_dgolomb, dim3(nblocks), dim3(kDSymThreads), 0, st, nblocks, blk, ds, sym, glen, err, words + 4);
    mark(3);
    hipLaunchKernelGGL(k_dlen, dim3(nblocks), dim3(256), 0, st, nblocks, blk, sym, glen, err);
    hipLaunchKernelGGL(k_dscan_out, dim3(1), dim3(1024), 0, st, nblocks, blk, cap, words, err);
    mark(4);
    hipLaunchKernelGGL(k_dlz, dim3(nblocks), dim3(kDLzThreads), 0, st, nblocks, blk, ds, sym, glen, d_out, err);
    mark(5);
}

}  // namespace fcx

// ---------------------------------------------------------------------------
// C ABI (include/fcx.h): decoder context, device and host entry points
using namespace fcx;

namespace {
int dfail(int code, const std::string &m) {
    set_last_error(m);   // fcx_last_error() (fcx_capi.hip)
    return code;
}
#define DHIP(expr)                                                                             \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) return dfail(FCX_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
const char *kDStageNames[] = {"tables", "symbols", "golomb", "lengths", "lz"};
constexpr int kDStages = 5;
}  // namespace

struct fcx_dctx {
    int device = 0;
    uint32_t cap_blocks = 0;
    uint64_t sym_cap = 0, glen_cap = 0;
    DBlock *blk = nullptr;
    DStream *ds = nullptr;
    uint64_t *symb = nullptr;
    uint16_t *tbl = nullptr, *child = nullptr;
    uint8_t *sym = nullptr;
    uint32_t *glen = nullptr;
    uint64_t *words = nullptr;        // [0] total out, [1] error bits, [2] symbol bytes, [3] golomb values,
                                      // [4..7] Jacobi rounds / serial fallbacks (symbols, golomb)
    uint64_t *host_words = nullptr;
    bool profiling = false, timed = false;
    hipEvent_t ev[kDStages + 1] = {};
};

namespace {
template <typename T>
int dgrow(T **p, uint64_t &have, uint64_t need, const char *what) {
    if (need <= have && *p) return FCX_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    have = 0;
    hipError_t e = hipMalloc((void **)p, need ? need : 16);
    if (e != hipSuccess) return dfail(FCX_ERR_NOMEM, std::string("hipMalloc ") + what + ": " + hipGetErrorString(e));
    have = need;
    return FCX_OK;
}
}  // namespace

extern "C" {

int fcx_dctx_create(fcx_dctx **out, int device) {
    if (!out) return dfail(FCX_ERR_ARG, "fcx_dctx_create: NULL");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return dfail(FCX_ERR_HIP, "no HIP device: the GPU decoder needs one");
    if (device < 0 || device >= ndev) return dfail(FCX_ERR_ARG, "bad device index");
    DHIP(hipSetDevice(device));
    fcx_dctx *c = new fcx_dctx();
    c->device = device;
    if (hipHostMalloc((void **)&c->host_words, 128, hipHostMallocDefault) != hipSuccess ||
        hipMalloc((void **)&c->words, 128) != hipSuccess) {
        fcx_dctx_destroy(c);
        return dfail(FCX_ERR_NOMEM, "fcx_dctx_create: allocation failed");
    }
    for (auto &e : c->ev) (void)hipEventCreate(&e);
    *out = c;
    return FCX_OK;
}

void fcx_dctx_destroy(fcx_dctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    void *ptrs[] = {c->blk, c->ds, c->symb, c->tbl, c->child, c->sym, c->glen, c->words};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    if (c->host_words) (void)hipHostFree(c->host_words);
    for (auto &e : c->ev)
        if (e) (void)hipEventDestroy(e);
    delete c;
}

int fcx_dctx_set_profiling(fcx_dctx *c, int enable) {
    if (!c) return dfail(FCX_ERR_ARG, "NULL ctx");
    c->profiling = enable != 0;
    return FCX_OK;
}

int fcx_dctx_stage_count(fcx_dctx *c) { return c && c->timed ? kDStages : 0; }

int fcx_dctx_stage(fcx_dctx *c, int i, const char **name, float *ms) {
    if (!c || i < 0 || i >= kDStages || !c->timed) return dfail(FCX_ERR_ARG, "bad stage / not profiled");
    DHIP(hipEventSynchronize(c->ev[kDStages]));
    float v = 0;
    DHIP(hipEventElapsedTime(&v, c->ev[i], c->ev[i + 1]));
    if (name) *name = kDStageNames[i];
    if (ms) *ms = v;
    return FCX_OK;
}

int fcx_decompress_shard(fcx_dctx *c, const uint8_t *d_in, uint64_t in_len, uint32_t nblocks, uint8_t *d_out,
                         uint64_t cap, uint64_t *out_len, void *stream) {
    if (!c || (in_len && !d_in) || (cap && !d_out)) return dfail(FCX_ERR_ARG, "fcx_decompress_shard: NULL argument");
    hipStream_t st = (hipStream_t)stream;
    DHIP(hipSetDevice(c->device));
    c->timed = false;
    if (nblocks == 0) {
        if (out_len) *out_len = 0;
        return FCX_OK;
    }
    if (nblocks > c->cap_blocks) {
        uint64_t h = 0;
        int r;
        if (c->blk) (void)hipFree(c->blk);
        if (c->ds) (void)hipFree(c->ds);
        if (c->symb) (void)hipFree(c->symb);
        if (c->tbl) (void)hipFree(c->tbl);
        if (c->child) (void)hipFree(c->child);
        c->blk = nullptr; c->ds = nullptr; c->symb = nullptr; c->tbl = nullptr; c->child = nullptr;
        c->cap_blocks = 0;
        if ((r = dgrow(&c->blk, h = 0, sizeof(DBlock) * (uint64_t)nblocks, "blocks"))) return r;
        if ((r = dgrow(&c->ds, h = 0, sizeof(DStream) * 4ull * nblocks, "streams"))) return r;
        if ((r = dgrow(&c->symb, h = 0, 8ull * nblocks, "symb"))) return r;
        if ((r = dgrow(&c->tbl, h = 0, 2048ull * 4 * nblocks, "tables"))) return r;
        if ((r = dgrow(&c->child, h = 0, 1024ull * 4 * nblocks, "children"))) return r;
        c->cap_blocks = nblocks;
    }
    uint32_t *err = (uint32_t *)(c->words + 1);
    DHIP(hipMemsetAsync(c->words, 0, 128, st));
    dec_launch(d_in, in_len, nblocks, d_out, cap, c->blk, c->ds, c->symb, c->tbl, c->child, c->sym, c->glen, c->words,
               err, 0, st, nullptr);
    // k_dscan left the scratch totals next to the error bits
    DHIP(hipMemcpyAsync(c->host_words, c->words, 32, hipMemcpyDeviceToHost, st));
    DHIP(hipStreamSynchronize(st));
    if ((uint32_t)c->host_words[1] & (kDErrRecord | kDErrHeader))
        return dfail(FCX_ERR_FORMAT, "malformed block records / headers");
    int r;
    if ((r = dgrow(&c->sym, c->sym_cap, c->host_words[2] + 64, "symbols"))) return r;
    if ((r = dgrow(&c->glen, c->glen_cap, 4 * c->host_words[3] + 64, "golomb values"))) return r;
    hipEvent_t *ev = c->profiling ? c->ev : nullptr;
    c->timed = ev != nullptr;
    dec_launch(d_in, in_len, nblocks, d_out, cap, c->blk, c->ds, c->symb, c->tbl, c->child, c->sym, c->glen, c->words,
               err, 1, st, ev);
    DHIP(hipGetLastError());
    DHIP(hipMemcpyAsync(c->host_words, c->words, 128, hipMemcpyDeviceToHost, st));
    DHIP(hipStreamSynchronize(st));
    static const bool dbg = getenv("FCX_DEC_DEBUG") != nullptr;
    if (dbg)
        fprintf(stderr, "fcx decode: symbol streams rounds %llu fallbacks %llu (flags %llu chars %llu p %llu golomb %llu)"
                " | golomb rounds %llu fallbacks %llu\n",
                (unsigned long long)c->host_words[4], (unsigned long long)c->host_words[5],
                (unsigned long long)c->host_words[8], (unsigned long long)c->host_words[9],
                (unsigned long long)c->host_words[10], (unsigned long long)c->host_words[11],
                (unsigned long long)c->host_words[6], (unsigned long long)c->host_words[7]);
    const uint32_t e = (uint32_t)c->host_words[1];
    if (e & kDErrOutCap) return dfail(FCX_ERR_CAPACITY, "output capacity too small");
    if (e) return dfail(FCX_ERR_FORMAT, "malformed stream (decoder error bits " + std::to_string(e) + ")");
    if (out_len) *out_len = c->host_words[0];
    return FCX_OK;
}

int fcx_dctx_device(fcx_dctx *c, int *device) {
    if (!c) return dfail(FCX_ERR_ARG, "NULL ctx");
    if (device) *device = c->device;
    return FCX_OK;
}

}  // extern "C"
