// fcx_device.h — constants, batch layout and wave helpers shared by the gfx950
// kernels of the FCX7 LZ77 + Huffman compress path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fcx {

// ---- format constants (my_compress.cpp:1261-1277, 222-224) ----------------
constexpr uint32_t kWin = 2047;     // SLIDE_WIN_LEN
constexpr uint32_t kMaxL = 258;     // CUR_BUFF_LEN: match length cap is min(258, len-i) - 1
constexpr uint32_t kMinL = 3;       // MIN_MATCH_LEN
constexpr uint32_t kPBits = 11;     // P_BITS

// ---- device work decomposition --------------------------------------------
constexpr uint32_t kTile = 4096;            // positions per match-kernel workgroup
constexpr uint32_t kMatchThreads = 512;
constexpr uint32_t kSubSeg = kTile / kMatchThreads;  // 8 positions per lane in the tile parse
constexpr uint32_t kHashBits = 12;
constexpr uint32_t kHalo = kWin;                     // left halo of a tile
constexpr uint32_t kLookAhead = 260;                 // right look-ahead bytes (>= 257)
constexpr uint32_t kTileBytes = 6464;                // >= kHalo + kTile + kLookAhead, x64
constexpr uint32_t kMaxChainSteps = 96;              // per-position candidate budget before "unknown"
constexpr uint32_t kDenseUnknowns = 512;             // tile gives up all-position search past this
constexpr uint32_t kChunk = 8192;                    // symbols per histogram / encode workgroup
constexpr uint32_t kStreams = 4;                     // flags, chars, p-bits, golomb words
constexpr uint32_t kHuffHdrStride = 576;             // >= 1 + 64 + 510 bytes of tree header
constexpr uint32_t kLazyWindow = 16384;              // stitch kernel's LDS data window

// m[i] packs the match at position i: bits 0..10 distance p, bits 11..19 length L (0 = literal)
constexpr uint32_t kUnknown = 0xFFFFFFFFu;
__host__ __device__ inline uint32_t m_pack(uint32_t L, uint32_t p) { return (L << 11) | p; }
__host__ __device__ inline uint32_t m_len(uint32_t m) { return m >> 11; }
__host__ __device__ inline uint32_t m_dist(uint32_t m) { return m & 0x7FFu; }

constexpr uint32_t kTileLazy = 1u;   // tile_flags: spec parse unavailable, stitch walks it

// per-block results of the parse/emit stage
struct BlockInfo {
    uint32_t len;          // input bytes of the block
    uint32_t ntok;         // N
    uint32_t nmatch;       // pCnt
    uint32_t gbits;        // golomb bits
    uint32_t slen[kStreams];   // stream lengths in bytes
    uint32_t hdrlen[kStreams]; // Huffman tree header bytes (0 = stream absent / raw)
    uint32_t nwords[kStreams]; // Huffman code words W
    uint32_t words_rel[kStreams]; // byte offset of stream words inside the block record
    uint32_t rec_bytes;    // 4 + payload
    uint32_t lazy_evals;   // statistics
    uint32_t lazy_tiles;
    uint32_t pad;
};

struct Layout {
    uint64_t n;            // input bytes of the shard
    uint32_t B;            // block bytes
    uint32_t nblocks;
    uint32_t tpb;          // tiles per block
    uint32_t wpb;          // 64-bit chain words per block
    uint32_t sstride[kStreams];   // per-block stride of each stream buffer (bytes, x16)
    uint32_t cpb[kStreams];       // chunks per block per stream
    uint32_t cpb_total;           // sum of cpb
    uint32_t pad;
};

// ---- wave64 helpers --------------------------------------------------------
__device__ inline uint32_t lane_id() { return __lane_id(); }

__device__ inline uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t t = __shfl_xor(v, o, 64);
        v = v > t ? v : t;
    }
    return v;
}

__device__ inline uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ inline uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t lo = __shfl_xor((uint32_t)v, o, 64);
        uint32_t hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}

// inclusive prefix sum across the 64 lanes
__device__ inline uint32_t wave_incl_scan(uint32_t v) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(v, o, 64);
        if (lane >= (uint32_t)o) v += t;
    }
    return v;
}

// unaligned 4-byte little-endian read from an LDS byte image backed by u32 words
__device__ inline uint32_t lds_ld4(const uint32_t *w, uint32_t pos) {
    uint32_t lo = w[pos >> 2], hi = w[(pos >> 2) + 1];
    return __builtin_amdgcn_alignbyte(hi, lo, pos & 3);
}
__device__ inline uint32_t lds_ld1(const uint32_t *w, uint32_t pos) {
    return (w[pos >> 2] >> ((pos & 3) * 8)) & 0xFFu;
}
__device__ inline uint32_t lds_key3(const uint32_t *w, uint32_t pos) { return lds_ld4(w, pos) & 0xFFFFFFu; }

// common-prefix length of the byte images at a and b, starting at `from`, capped at cap
__device__ inline uint32_t lds_match_len(const uint32_t *w, uint32_t a, uint32_t b, uint32_t from, uint32_t cap) {
    uint32_t L = from;
    while (L + 4 <= cap) {
        uint32_t x = lds_ld4(w, a + L) ^ lds_ld4(w, b + L);
        if (x) return L + (__builtin_ctz(x) >> 3);
        L += 4;
    }
    while (L < cap && lds_ld1(w, a + L) == lds_ld1(w, b + L)) L++;
    return L;
}

__device__ inline uint32_t hash3(uint32_t key) { return (key * 2654435761u) >> (32 - kHashBits); }

}  // namespace fcx
