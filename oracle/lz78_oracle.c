/*
 * lz78_oracle.c — CPU restatement of the reference's `-c lz78` block codec
 * (FCX8), written from the algorithm, not copied.
 *
 * TEST INFRASTRUCTURE ONLY (the checker, never the product): loaded by tests/
 * through oracle/__init__.py.  Pinned in tests/test_lz78.py against oracle/_ref
 * (the reference compiled in place: my_compress_file_lz78 / my_LZ78_compress /
 * my_decompress_file_lz78), the textbook string of the reference's own LZ78
 * self-test (my_compress.cpp:3977-3988), and tests/golden/golden_lz78.json.
 *
 * Reference line map (my_compress.cpp, lines counted by '\n'):
 *   my_LZ78_compress 1832-1899 (hash-map dictionary 1758-1796, BKDRHash 1799)
 *   my_LZ78_decompress 1901-1934
 *   block encoder my_compress_file_lz78 3127-3476: sort by idx 2888-2925,
 *     distinct idx 3102-3125, idx bitmap 3180-3212, groups of 256 ranks
 *     3214-3257, group Huffman tree 3258-3307 (create_huffman_tree 535-617),
 *     group codes huffman_encode_idxGroup 2927-3006, in-group positions
 *     3352-3360, char sub-stream 3362-3471 (= my_huffman_encode_char 987-1104)
 *   block decoder my_decompress_file_lz78 3478-3710 (+ huffman_decode_idxGroup
 *     3009-3054, huffman_decode_char 930-984)
 *
 * The dictionary of the reference is a set of exact strings (the BKDR key only
 * buckets them; 1774-1775 compares length and bytes), so the parse is the
 * textbook LZ78 trie walk: the phrase is the longest dictionary prefix plus one
 * byte, the token is (index of that prefix or 0, the byte), and the phrase
 * enters the dictionary under the next index (1-based).  When the rest of the
 * block is a dictionary string the last token is (its index, '\0') and nothing
 * is added (1858-1863).
 */
#include "fcx_oracle.h"
#include <stdlib.h>
#include <string.h>

static inline void put_u32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static inline uint32_t get_u32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }

/* ---- trie: open addressing on (parent, byte) -> child index ---------------- */
typedef struct {
    uint64_t *slot;   /* 0 = empty, else key << 24 | child  (key = (parent << 8 | byte) + 1) */
    uint64_t mask;
} trie_t;

static inline uint64_t trie_hash(uint64_t key) { return (key * 0x9E3779B97F4A7C15ull) >> 17; }

static uint32_t trie_get(const trie_t *t, uint32_t parent, uint32_t byte) {
    const uint64_t key = (((uint64_t)parent << 8) | byte) + 1;
    for (uint64_t h = trie_hash(key) & t->mask;; h = (h + 1) & t->mask) {
        const uint64_t s = t->slot[h];
        if (s == 0) return 0;
        if ((s >> 24) == key) return (uint32_t)(s & 0xFFFFFFu);
    }
}

static void trie_put(trie_t *t, uint32_t parent, uint32_t byte, uint32_t child) {
    const uint64_t key = (((uint64_t)parent << 8) | byte) + 1;
    uint64_t h = trie_hash(key) & t->mask;
    while (t->slot[h] != 0) h = (h + 1) & t->mask;
    t->slot[h] = (key << 24) | child;
}

/* my_LZ78_compress (1832-1899): tokens (idx[t], c[t]); capacity >= len; returns N */
uint32_t orc_lz78_parse(const uint8_t *in, uint32_t len, uint32_t *idx, uint8_t *c) {
    if (!in || len == 0) return 0;
    uint64_t cap = 1024;
    while (cap < 2ull * len + 2) cap <<= 1;
    trie_t t = {(uint64_t *)calloc(cap, sizeof(uint64_t)), cap - 1};
    uint32_t N = 0, next = 1, pos = 0;
    while (pos < len) {
        uint32_t node = 0;
        while (pos < len) {   /* extend while the prefix is a dictionary string (1848-1856) */
            const uint32_t ch = trie_get(&t, node, in[pos]);
            if (!ch) break;
            node = ch;
            pos++;
        }
        if (pos == len) {     /* whole remainder found: (index, '\0'), nothing added (1858-1863) */
            idx[N] = node; c[N] = 0; N++;
            break;
        }
        trie_put(&t, node, in[pos], next++);   /* 1866-1875 */
        idx[N] = node; c[N] = in[pos]; N++;    /* 1877-1886 */
        pos++;
    }
    free(t.slot);
    return N;
}

/* ---- LSB-first continuous bit writer (huffman_encode_idxGroup 2976-3002) --- */
typedef struct { uint8_t *words; uint32_t nw; uint32_t bit; uint32_t cur; } bitw_t;
static void bw_put(bitw_t *w, uint32_t code, uint32_t len) {   /* code bit k = k-th emitted */
    for (uint32_t k = 0; k < len; k++) {
        if (w->bit == 32) { put_u32(w->words + 4 * (size_t)w->nw++, w->cur); w->cur = 0; w->bit = 0; }
        w->cur |= ((code >> k) & 1u) << w->bit;
        w->bit++;
    }
}
static void bw_flush(bitw_t *w) {
    if (w->bit) { put_u32(w->words + 4 * (size_t)w->nw++, w->cur); w->cur = 0; w->bit = 0; }
}

/* my_compress_file_lz78 (3127-3476); returns payload bytes (0 on NULL / empty) */
uint32_t orc_lz78_compress_block(const uint8_t *in, uint32_t len, uint8_t *out) {
    if (!in || !out || len == 0) return 0;
    uint32_t *idx = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)len + 1));
    uint8_t *c = (uint8_t *)malloc((size_t)len + 1);
    const uint32_t N = orc_lz78_parse(in, len, idx, c);
    uint8_t *o = out;
    /* distinct indices, ascending (sort 3162 + filter 3102-3125) -> bitmap (3180-3206) */
    uint32_t maxi = 0;
    for (uint32_t t = 0; t < N; t++) if (idx[t] > maxi) maxi = idx[t];
    const uint32_t nbm = maxi / 8 + 1;
    uint8_t *bm = (uint8_t *)calloc(nbm, 1);
    for (uint32_t t = 0; t < N; t++) bm[idx[t] >> 3] |= (uint8_t)(1u << (idx[t] & 7));
    /* rank of an index among the distinct ones (mapIdx 3216-3219) */
    uint32_t *rank_at = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)maxi + 1));
    uint32_t wcnt = 0;
    for (uint32_t v = 0; v <= maxi; v++) {
        rank_at[v] = wcnt;
        if ((bm[v >> 3] >> (v & 7)) & 1) wcnt++;
    }
    put_u32(o, wcnt); o += 4;
    memcpy(o, bm, nbm); o += nbm;
    /* groups of 256 ranks: group id and position per token (3224-3254) */
    const uint32_t G = wcnt / 256 + (wcnt % 256 ? 1 : 0);
    uint32_t *gcnt = (uint32_t *)calloc(G ? G : 1, sizeof(uint32_t));
    uint32_t *grp = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)N + 1));
    uint8_t *gpos = (uint8_t *)malloc((size_t)N + 1);
    for (uint32_t t = 0; t < N; t++) {
        const uint32_t r = rank_at[idx[t]];
        grp[t] = r / 256;
        gpos[t] = (uint8_t)(r % 256);
        gcnt[grp[t]]++;
    }
    put_u32(o, G); o += 4;   /* G >= 1 (3280-3301) */
    int ok = 1;
    if (G > 1) {
        uint32_t *nodes = (uint32_t *)malloc(sizeof(uint32_t) * 4 * (2 * (size_t)G - 1));
        orc_huffman_tree(gcnt, G, nodes);
        for (uint32_t j = 0; j + 1 < G; j++) {   /* stHuffmanTreeNodeSimple of node j + G (3273-3287) */
            put_u32(o, nodes[4 * (j + G) + 2]); o += 4;
            put_u32(o, nodes[4 * (j + G) + 3]); o += 4;
        }
        /* codes: parent walk leaf -> root, emitted root first (2947-2992) */
        uint32_t *code = (uint32_t *)calloc(G, sizeof(uint32_t)), *clen = (uint32_t *)calloc(G, sizeof(uint32_t));
        for (uint32_t g = 0; g < G; g++) {
            uint32_t depth = 0, cur = g, par = nodes[4 * g + 1], bits = 0;
            while (par < 2 * G - 1 && par != 0) {
                if (depth == 32) { ok = 0; break; }
                bits = (bits << 1) | (nodes[4 * par + 2] == cur ? 0u : 1u);
                depth++;
                cur = par;
                par = nodes[4 * par + 1];
            }
            code[g] = bits;   /* bit k = edge at depth k (root edge in bit 0) */
            clen[g] = depth;
        }
        put_u32(o, N); o += 4;
        bitw_t w = {o + 4, 0, 0, 0};
        for (uint32_t t = 0; ok && t < N; t++) bw_put(&w, code[grp[t]], clen[grp[t]]);
        bw_flush(&w);
        put_u32(o, w.nw);
        o += 4 + 4 * (size_t)w.nw;
        free(code); free(clen); free(nodes);
    } else {
        put_u32(o, N); o += 4;
    }
    if (ok) {
        memcpy(o, gpos, N); o += N;             /* 3352-3357 */
        o += orc_huffman_stream(c, N, o);       /* 3362-3471 == my_huffman_encode_char */
    }
    free(idx); free(c); free(bm); free(rank_at); free(gcnt); free(grp); free(gpos);
    return ok ? (uint32_t)(o - out) : 0;
}

/* my_decompress_file_lz78 (3478-3710) into memory; -1 on a malformed stream.
 * Keeps the reference's tail rule (3701-3703): a block whose decoded bytes end
 * in 0x00 loses that byte. */
int64_t orc_lz78_decompress_block(const uint8_t *in, uint32_t len, uint8_t *out, uint64_t cap) {
    int64_t ret = -1;
    const uint8_t *q = in, *end = in + len;
    uint32_t *pindex = NULL, *grp = NULL, *lc = NULL, *rc = NULL, *pstart = NULL, *plen = NULL;
    uint8_t *cc = NULL;
    uint32_t N = 0, G = 0;
    const uint8_t *gpos = NULL;
    uint64_t o = 0;
    if (!in || len < 4) return -1;
    const uint32_t wcnt = get_u32(q); q += 4;
    if (wcnt == 0) return -1;   /* the reference reads pIndex[-1] (3502) */
    pindex = (uint32_t *)malloc(sizeof(uint32_t) * wcnt);
    {   /* 3494-3500: indices of the set bits, ascending */
        uint32_t i = 0;
        for (uint64_t v = 0; i < wcnt; v++) {
            if ((uint64_t)(end - q) <= (v >> 3)) goto done;
            if ((q[v >> 3] >> (v & 7)) & 1) pindex[i++] = (uint32_t)v;
        }
    }
    q += pindex[wcnt - 1] / 8 + 1;
    if (end - q < 4) goto done;
    G = get_u32(q); q += 4;
    if (G > 1) {
        if ((uint64_t)(end - q) < 8ull * (G - 1) + 8) goto done;
        lc = (uint32_t *)malloc(sizeof(uint32_t) * G);
        rc = (uint32_t *)malloc(sizeof(uint32_t) * G);
        for (uint32_t j = 0; j + 1 < G; j++) { lc[j] = get_u32(q); rc[j] = get_u32(q + 4); q += 8; }
        N = get_u32(q); q += 4;
        const uint32_t W = get_u32(q); q += 4;
        if ((uint64_t)(end - q) < 4ull * W) goto done;
        grp = (uint32_t *)calloc((size_t)N + 1, sizeof(uint32_t));
        /* huffman_decode_idxGroup (3009-3054): root = simple node G-2; a child < G is
         * a leaf, else child - G is a simple node */
        uint32_t node = G - 2, j = 0;
        for (uint32_t i = 0; i < W && j < N; i++) {
            uint32_t wv = get_u32(q + 4ull * i);
            for (int b = 0; b < 32; b++, wv >>= 1) {
                uint32_t nx = (wv & 1) ? rc[node] : lc[node];
                if (nx < G) {
                    grp[j++] = nx;
                    node = G - 2;
                    if (j >= N) break;
                } else {
                    nx -= G;
                    if (nx + 1 >= G) goto done;
                    node = nx;
                }
            }
        }
        q += 4ull * W;
    } else {
        if (end - q < 4) goto done;
        N = get_u32(q); q += 4;
    }
    if ((uint64_t)(end - q) < N) goto done;
    gpos = q;
    q += N;
    cc = (uint8_t *)calloc((size_t)N + 1, 1);
    if (!orc_huffman_stream_decode(q, (uint32_t)(end - q), cc, N)) goto done;
    /* my_LZ78_decompress (1901-1934): phrase t = phrase[idx - 1] + c, dictionary index t + 1 */
    pstart = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)N + 1));
    plen = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)N + 1));
    for (uint32_t t = 0; t < N; t++) {
        const uint32_t r = (G > 1 ? grp[t] * 256u : 0u) + gpos[t];   /* 3586-3595 */
        if (r >= wcnt) goto done;
        const uint32_t ix = pindex[r];
        uint32_t L = 0;
        if (ix != 0) {
            if (ix > t) goto done;
            L = plen[ix - 1];
            if (o + L + 1 > cap) goto done;
            memmove(out + o, out + pstart[ix - 1], L);
        }
        if (o + L + 1 > cap) goto done;
        out[o + L] = cc[t];
        pstart[t] = (uint32_t)o;
        plen[t] = L + 1;
        o += L + 1;
    }
    if (o > 0 && out[o - 1] == 0) o--;   /* 3701-3703 */
    ret = (int64_t)o;
done:
    free(pindex); free(grp); free(lc); free(rc); free(pstart); free(plen); free(cc);
    return ret;
}

/* main() 4073-4136 with -c lz78: "FCX8" header, [u32 len][payload] per block */
uint64_t orc_lz78_compress_file(const uint8_t *in, uint64_t n, uint32_t block_bytes, uint8_t *out, uint64_t cap) {
    if (cap < 10 || block_bytes == 0) return 0;
    const uint64_t nblk = (n + block_bytes - 1) / block_bytes;
    memcpy(out, "FCX8", 4);
    put_u32(out + 4, (uint32_t)n);
    const uint16_t nb16 = (uint16_t)nblk;
    memcpy(out + 8, &nb16, 2);
    uint64_t o = 10;
    uint8_t *tmp = (uint8_t *)malloc(5 * (size_t)block_bytes + 65536);
    for (uint64_t b = 0; b < nblk; b++) {
        const uint64_t off = b * block_bytes;
        const uint32_t len = (uint32_t)(n - off < block_bytes ? n - off : block_bytes);
        const uint32_t sz = orc_lz78_compress_block(in + off, len, tmp);
        if (sz == 0 || o + 4 + sz > cap) { free(tmp); return 0; }
        put_u32(out + o, sz);
        memcpy(out + o + 4, tmp, sz);
        o += 4 + sz;
    }
    free(tmp);
    return o;
}

/* main() 4137-4204 for an FCX8 file */
int64_t orc_lz78_decompress_file(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap) {
    if (n < 10 || memcmp(in, "FCX", 3) != 0 || in[3] == '7') return -1;
    uint16_t nblk;
    memcpy(&nblk, in + 8, 2);
    uint64_t q = 10, o = 0;
    for (uint32_t b = 0; b < nblk; b++) {
        if (q + 4 > n) return -1;
        const uint32_t sz = get_u32(in + q);
        q += 4;
        if (q + sz > n) return -1;
        const int64_t r = orc_lz78_decompress_block(in + q, sz, out + o, cap - o);
        if (r < 0) return -1;
        o += (uint64_t)r;
        q += sz;
    }
    return (int64_t)o;
}
