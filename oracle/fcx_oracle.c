/*
 * fcx_oracle.c — CPU restatement of the reference's `-c lz77` compress path and
 * its decoder, written from the algorithm, not copied.
 *
 * TEST INFRASTRUCTURE ONLY (the checker, never the product): loaded by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Parity of this file
 * is pinned in tests/test_oracle.py against (a) the reference's own KATs
 * (Sunday, my_compress.cpp:3749-3759; the disabled self-tests 3779-3867) and
 * (b) oracle/_ref, the reference compiled in place, on the golden inputs.
 *
 * Reference line map (my_compress.cpp, lines counted by '\n'):
 *   Sunday_Search 1407-1443, longest_match_sunday 1446-1514, parse 1675-1714,
 *   constants 1261-1277, golomb 222-304 / 309-358, combine_bits 1292-1338,
 *   Huffman tree 458-617, char coder 849-984 / 987-1187, block codec
 *   2073-2393, container 101-113 / 4073-4204.
 */
#include "fcx_oracle.h"
#include <stdlib.h>
#include <string.h>

#define SLIDE_WIN_LEN 2047   /* my_compress.cpp:1262 */
#define CUR_BUFF_LEN 258     /* my_compress.cpp:1263 */
#define P_BITS 11            /* my_compress.cpp:1264 */
#define MIN_MATCH_LEN 3      /* my_compress.cpp:1265 */
#define GOLOMB_M 4           /* my_compress.cpp:222-224 (M=4, Q_BITS=2) */
#define GOLOMB_QBITS 2

static inline void put_u32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static inline uint32_t get_u32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }

/* ------------------------------------------------------------------------- */
/* Sunday search, my_compress.cpp:1407-1443.  May read text[text_len] (one past
 * the text) exactly like the reference (1429); callers keep slack there.      */
int32_t orc_sunday_search(const uint8_t *text, int32_t text_len, const uint8_t *pat, int32_t pat_len) {
    int32_t shift[256];
    memset(shift, 0, sizeof(shift));
    for (int32_t i = 0; i < pat_len; i++) shift[pat[i]] = pat_len - i;
    int32_t s = 0, k = 0;
    while (s + pat_len <= text_len) {
        if (text[s + k] == pat[k]) {
            if (++k == pat_len) return s;
        } else {
            int32_t sh = shift[text[s + pat_len]];
            s += sh ? sh : pat_len + 1;
            k = 0;
        }
    }
    return -1;
}

/* ------------------------------------------------------------------------- */
/* Match finder A: restatement of longest_match_sunday (1446-1514).  This has
 * the reference's cost profile and is the "port" CPU baseline.               */
static void match_sunday(const uint8_t *d, uint32_t len, uint32_t cur, uint32_t *p, uint32_t *l, uint8_t *c) {
    *p = 0; *l = 0; *c = d[cur];
    if (cur == 0) return;
    uint32_t end = cur + ((cur + CUR_BUFF_LEN <= len) ? CUR_BUFF_LEN : (len - cur));
    uint32_t win = cur > SLIDE_WIN_LEN ? cur - SLIDE_WIN_LEN : 0;
    uint32_t next = win;
    int32_t cap = (int32_t)(end - cur) - 1;
    if (cap < MIN_MATCH_LEN) return;
    for (int32_t ml = MIN_MATCH_LEN; ml <= cap; ml++) {
        int32_t text_len = (int32_t)(cur - win) + ml - 1;
        int32_t hit = orc_sunday_search(d + next, text_len, d + cur, ml);
        if (hit == -1 || next + (uint32_t)hit == cur) return;
        next += (uint32_t)hit;
        if (next >= cur) break;
        while (d[next + ml] == d[cur + ml] && ml < cap) ml++;
        *p = cur - next; *l = (uint32_t)ml; *c = d[cur + ml];
        /* Sunday skip for the next (longer) pattern length (1491-1503) */
        int32_t shift[256];
        memset(shift, 0, sizeof(shift));
        for (int32_t i = 0; i < ml + 1; i++) shift[d[cur + i]] = ml + 1 - i;
        int32_t sh = shift[d[next + ml + 1]];
        next += sh ? (uint32_t)sh : (uint32_t)(ml + 2);
        if (next >= cur) break;
    }
}

/* Match finder B: same result, computed directly from the semantics the
 * Sunday loop implements — the LEFTMOST j in [max(0,i-2047), i) reaching the
 * MAXIMUM common-prefix length L, L capped at min(258, len-i)-1, literal when
 * L < 3.  Position-ordered hash chains give every candidate with an equal
 * 3-byte prefix; they are scanned oldest-first with an early exit at the cap. */
typedef struct {
    int32_t *head;   /* 1<<16 buckets: most recent position, -1 = empty */
    int32_t *prev;   /* previous position with the same bucket */
    int32_t *cand;   /* scratch for the window's candidates */
    uint32_t inserted;
} chains_t;

static inline uint32_t key3(const uint8_t *q) { return (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16); }
static inline uint32_t hash3(uint32_t k) { return (k * 2654435761u) >> 16; }

static void match_exhaustive(const uint8_t *d, uint32_t len, uint32_t cur, chains_t *ch, uint32_t *p, uint32_t *l, uint8_t *c) {
    for (; ch->inserted < cur; ch->inserted++) {
        uint32_t j = ch->inserted;
        if (j + 3 > len) continue;
        uint32_t h = hash3(key3(d + j));
        ch->prev[j] = ch->head[h];
        ch->head[h] = (int32_t)j;
    }
    *p = 0; *l = 0; *c = d[cur];
    if (cur == 0 || len - cur < 4) return;
    uint32_t cap = (len - cur < CUR_BUFF_LEN ? len - cur : CUR_BUFF_LEN) - 1;
    int32_t lo = cur > SLIDE_WIN_LEN ? (int32_t)(cur - SLIDE_WIN_LEN) : 0;
    uint32_t k = key3(d + cur);
    int nc = 0;
    for (int32_t j = ch->head[hash3(k)]; j >= lo; j = ch->prev[j])
        if (key3(d + j) == k) ch->cand[nc++] = j;
    uint32_t best = MIN_MATCH_LEN - 1, bestj = 0;
    for (int q = nc - 1; q >= 0; q--) {          /* oldest (leftmost) first */
        uint32_t j = (uint32_t)ch->cand[q];
        if (best >= MIN_MATCH_LEN && d[j + best] != d[cur + best]) continue;
        uint32_t L = MIN_MATCH_LEN;
        while (L < cap && d[j + L] == d[cur + L]) L++;
        if (L > best) { best = L; bestj = j; if (best == cap) break; }
    }
    if (best >= MIN_MATCH_LEN) { *p = cur - bestj; *l = best; *c = d[cur + best]; }
}

/* Greedy parse, my_LZ77_compress 1675-1714: cursor += l + 1. */
uint32_t orc_lz77_parse(const uint8_t *in, uint32_t len, int finder, uint32_t *p, uint32_t *l, uint8_t *c) {
    /* zero slack after the block: the Sunday loop may read past it (1429) */
    uint8_t *d = (uint8_t *)calloc((size_t)len + 1024, 1);
    memcpy(d, in, len);
    chains_t ch = {0};
    if (finder == ORC_FINDER_EXHAUSTIVE) {
        ch.head = (int32_t *)malloc(sizeof(int32_t) << 16);
        memset(ch.head, 0xff, sizeof(int32_t) << 16);
        ch.prev = (int32_t *)malloc(sizeof(int32_t) * ((size_t)len + 1));
        ch.cand = (int32_t *)malloc(sizeof(int32_t) * (SLIDE_WIN_LEN + 1));
    }
    uint32_t n = 0, cur = 0;
    while (cur < len) {
        if (finder == ORC_FINDER_EXHAUSTIVE) match_exhaustive(d, len, cur, &ch, &p[n], &l[n], &c[n]);
        else match_sunday(d, len, cur, &p[n], &l[n], &c[n]);
        cur += l[n] + 1;
        n++;
    }
    free(ch.head); free(ch.prev); free(ch.cand);
    free(d);
    return n;
}

/* ------------------------------------------------------------------------- */
/* Golomb-Rice k=2, golomb_rice_encode 258-304: per value q=v>>2 one-bits, a
 * zero bit, then the 2 bits of r=v&3 LSB first; one continuous LSB-first u32
 * stream, final partial word flushed (the 273-291 word-spill logic is a plain
 * continuous pack).                                                           */
uint32_t orc_golomb_encode(const uint32_t *vals, uint32_t n, uint32_t *words) {
    uint32_t nw = 0, acc = 0, pos = 0;
#define PUTBIT(b) do { if (b) acc |= 1u << pos; if (++pos == 32) { words[nw++] = acc; acc = 0; pos = 0; } } while (0)
    for (uint32_t i = 0; i < n; i++) {
        uint32_t q = vals[i] >> GOLOMB_QBITS, r = vals[i] & (GOLOMB_M - 1);
        for (uint32_t k = 0; k < q; k++) PUTBIT(1);
        PUTBIT(0);
        PUTBIT(r & 1);
        PUTBIT((r >> 1) & 1);
    }
#undef PUTBIT
    if (pos) words[nw++] = acc;
    return nw;
}

/* golomb_rice_decode 309-358 */
static uint32_t golomb_decode(const uint32_t *words, uint32_t nw, uint32_t *out, uint32_t need) {
    uint32_t n = 0, q = 0, r = 0, rb = 0;
    int after_sep = 0;
    if (need == 0) return 0;
    for (uint32_t i = 0; i < nw; i++) {
        uint32_t w = words[i];
        for (int b = 0; b < 32; b++, w >>= 1) {
            uint32_t bit = w & 1;
            if (!after_sep) {
                if (bit) q++; else after_sep = 1;
            } else {
                r |= bit << rb;
                if (++rb >= GOLOMB_QBITS) {
                    out[n++] = q * GOLOMB_M + r;
                    after_sep = 0; rb = 0; q = 0; r = 0;
                    if (n >= need) return n;
                }
            }
        }
    }
    return n;
}

/* combine_bits 1292-1313: low `bits` of each value, LSB-first, into a zeroed
 * buffer of (bits*n)/8 + 1 bytes. */
void orc_combine_bits(const uint32_t *vals, uint32_t n, uint32_t bits, uint8_t *out) {
    memset(out, 0, (size_t)(bits * n) / 8 + 1);
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; i++)
        for (uint32_t b = 0; b < bits; b++, pos++)
            if ((vals[i] >> b) & 1) out[pos >> 3] |= (uint8_t)(1u << (pos & 7));
}

/* decombine_bits 1315-1338 */
static void decombine_bits(const uint8_t *in, uint32_t n, uint32_t bits, uint32_t *out) {
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t v = 0;
        for (uint32_t b = 0; b < bits; b++, pos++)
            if ((in[pos >> 3] >> (pos & 7)) & 1) v |= 1u << b;
        out[i] = v;
    }
}

/* ------------------------------------------------------------------------- */
/* Huffman tree, create_huffman_tree 535-617 (+ merge sort 458-498).
 * Leaves = symbols with weight>0 in symbol order, stably sorted by weight.
 * Internal node k lives at n + (n - real) + k.  Each step merges list[s]
 * (left) and list[s+1] (right) and re-inserts the sum AFTER every entry of
 * weight <= sum (strict '<' at 588).                                          */
uint32_t orc_huffman_tree(const uint32_t *w, uint32_t n, uint32_t *nodes) {
    if (n <= 1) return 0;
    uint32_t m = 2 * n - 1;
    memset(nodes, 0, sizeof(uint32_t) * 4 * m);
    uint32_t *lw = (uint32_t *)malloc(sizeof(uint32_t) * n), *li = (uint32_t *)malloc(sizeof(uint32_t) * n);
    uint32_t real = 0;
    for (uint32_t i = 0; i < n; i++)
        if (w[i] > 0) { nodes[4 * i] = w[i]; lw[real] = w[i]; li[real] = i; real++; }
    /* stable sort by weight (insertion sort == stable merge sort result) */
    for (uint32_t a = 1; a < real; a++) {
        uint32_t kw = lw[a], ki = li[a];
        int32_t b = (int32_t)a - 1;
        while (b >= 0 && lw[b] > kw) { lw[b + 1] = lw[b]; li[b + 1] = li[b]; b--; }
        lw[b + 1] = kw; li[b + 1] = ki;
    }
    uint32_t s = 0;
    for (uint32_t node = n + (n - real); node < m; node++, s++) {
        uint32_t left = li[s], right = li[s + 1];
        uint32_t sum = nodes[4 * left] + nodes[4 * right];
        nodes[4 * node + 0] = sum;
        nodes[4 * node + 2] = left;
        nodes[4 * node + 3] = right;
        nodes[4 * left + 1] = node;
        nodes[4 * right + 1] = node;
        uint32_t j = s + 2;
        for (; j < real && lw[j] <= sum; j++) { lw[j - 1] = lw[j]; li[j - 1] = li[j]; }
        lw[j - 1] = sum; li[j - 1] = node;
    }
    free(lw); free(li);
    return real;
}

/* One Huffman sub-stream, my_huffman_encode_char 987-1104 (+ 849-928):
 * [u8 ts][ceil(2ts/8) B child-is-internal bitmap][ts x (u8 l, u8 r)]
 * [u32 W][W x u32 codes, root->leaf path bits LSB-first, W = ceil(bits/32)]. */
uint32_t orc_huffman_stream(const uint8_t *src, uint32_t n, uint8_t *out) {
    if (n == 0) return 0;  /* 989-990 */
    uint32_t hist[256] = {0};
    for (uint32_t i = 0; i < n; i++) hist[src[i]]++;
    uint32_t *nodes = (uint32_t *)malloc(sizeof(uint32_t) * 4 * 511);
    uint32_t real = orc_huffman_tree(hist, 256, nodes);
    uint32_t ts = real > 1 ? real - 1 : 0;
    uint32_t nbm = (2 * ts + 7) / 8;
    uint8_t *o = out;
    *o++ = (uint8_t)ts;
    uint8_t *bm = o;
    memset(bm, 0, nbm);
    o += nbm;
    for (uint32_t j = 0; j < ts; j++) {
        uint32_t node = j + 256 + (256 - real);
        uint32_t lc = nodes[4 * node + 2], rc = nodes[4 * node + 3];
        if (lc >= 256) bm[(2 * j) >> 3] |= (uint8_t)(1u << ((2 * j) & 7));
        if (rc >= 256) bm[(2 * j + 1) >> 3] |= (uint8_t)(1u << ((2 * j + 1) & 7));
        *o++ = (uint8_t)(lc >= 256 ? lc - 256 : lc);
        *o++ = (uint8_t)(rc >= 256 ? rc - 256 : rc);
    }
    /* code of each symbol: walk leaf -> root (878-892), emit root-first */
    uint32_t code[256], clen[256];
    for (uint32_t sym = 0; sym < 256; sym++) {
        uint32_t bits = 0, depth = 0, cur = sym, par = nodes[4 * sym + 1];
        uint32_t path[256];
        while (par < 511 && par != 0) {
            path[depth++] = (nodes[4 * par + 2] == cur) ? 0u : 1u;
            cur = par;
            par = nodes[4 * par + 1];
        }
        for (uint32_t k = 0; k < depth; k++) bits |= path[depth - 1 - k] << k; /* depth <= 32 asserted below */
        code[sym] = bits;
        clen[sym] = depth;
    }
    uint8_t *wptr = o + 4;
    uint32_t nw = 0;
    uint64_t acc = 0;
    uint32_t pos = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t L = clen[src[i]];
        if (L > 32) { free(nodes); return 0; } /* unreachable for blocks <= 1 MiB */
        acc |= (uint64_t)code[src[i]] << pos;
        pos += L;
        while (pos >= 32) { put_u32(wptr + 4 * nw++, (uint32_t)acc); acc >>= 32; pos -= 32; }
    }
    if (pos) put_u32(wptr + 4 * nw++, (uint32_t)acc);
    put_u32(o, nw);
    o = wptr + 4 * nw;
    free(nodes);
    return (uint32_t)(o - out);
}

/* decode one sub-stream (my_huffman_decode_char 1107-1187 + 930-984);
 * returns bytes consumed or 0 on malformed input */
static uint32_t huffman_stream_decode(const uint8_t *in, uint32_t avail, uint8_t *dst, uint32_t count) {
    if (avail < 1) return 0;
    uint32_t ts = in[0], nbm = (2 * ts + 7) / 8;
    uint32_t hdr = 1 + nbm + 2 * ts;
    if (avail < hdr + 4) return 0;
    const uint8_t *bm = in + 1, *pairs = in + 1 + nbm;
    uint32_t nw = get_u32(in + hdr);
    if ((uint64_t)hdr + 4 + 4ull * nw > avail) return 0;
    const uint8_t *words = in + hdr + 4;
    uint32_t real = ts + 1;
    /* children: < 256 leaf symbol, else internal node index (value + 256) */
    uint32_t lc[256], rc[256];
    for (uint32_t j = 0; j < ts; j++) {
        lc[j] = pairs[2 * j] + (((bm[(2 * j) >> 3] >> ((2 * j) & 7)) & 1) ? 256u : 0u);
        rc[j] = pairs[2 * j + 1] + (((bm[(2 * j + 1) >> 3] >> ((2 * j + 1) & 7)) & 1) ? 256u : 0u);
    }
    memset(dst, 0, count);  /* ts == 0: the symbol is not stored, output stays 0 */
    if (ts > 0 && count > 0) {
        uint32_t root = ts - 1, node = root, j = 0;
        for (uint32_t i = 0; i < nw && j < count; i++) {
            uint32_t w = get_u32(words + 4 * i);
            for (int b = 0; b < 32; b++, w >>= 1) {
                uint32_t nx = (w & 1) ? rc[node] : lc[node];
                if (nx < 256) {
                    dst[j++] = (uint8_t)nx;
                    node = root;
                    if (j >= count) break;
                } else {
                    nx = nx - 256 - (256 - real);
                    if (nx >= ts) return 0;
                    node = nx;
                }
            }
        }
    }
    return hdr + 4 + 4 * nw;
}

uint32_t orc_huffman_stream_decode(const uint8_t *in, uint32_t avail, uint8_t *dst, uint32_t count) {
    return huffman_stream_decode(in, avail, dst, count);
}

/* ------------------------------------------------------------------------- */
/* Block codec, my_compress_file_lz77 2115-2253 + make_bitMap_table 2073-2113 */
uint32_t orc_compress_block(const uint8_t *in, uint32_t len, uint8_t *out, int finder) {
    if (!in || !out) return 0;
    uint32_t *p = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)len + 1));
    uint32_t *l = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)len + 1));
    uint8_t *c = (uint8_t *)malloc((size_t)len + 1);
    uint32_t N = orc_lz77_parse(in, len, finder, p, l, c);
    uint8_t *o = out;
    put_u32(o, N); o += 4;
    /* flags: bit t = token t is a literal; Huffman-coded when > 1 byte */
    uint32_t nb = (N + 7) / 8;
    uint8_t *flags = (uint8_t *)calloc(nb + 1, 1);
    for (uint32_t t = 0; t < N; t++) if (l[t] == 0) flags[t >> 3] |= (uint8_t)(1u << (t & 7));
    if (nb > 1) o += orc_huffman_stream(flags, nb, o);
    else { memcpy(o, flags, nb); o += nb; }
    free(flags);
    /* chars of every token */
    o += orc_huffman_stream(c, N, o);
    /* distances and lengths of the matches */
    uint32_t pc = 0;
    for (uint32_t t = 0; t < N; t++) if (l[t] != 0) { p[pc] = p[t]; l[pc] = l[t]; pc++; }
    put_u32(o, pc); o += 4;
    uint32_t pbytes = (P_BITS * pc) / 8 + 1;
    uint8_t *pb = (uint8_t *)malloc(pbytes);
    orc_combine_bits(p, pc, P_BITS, pb);
    o += orc_huffman_stream(pb, pbytes, o);
    free(pb);
    uint32_t *gw = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)pc * 3 + 1));
    uint32_t G = orc_golomb_encode(l, pc, gw);
    put_u32(o, G); o += 4;
    o += orc_huffman_stream((const uint8_t *)gw, 4 * G, o);  /* LE host */
    free(gw); free(p); free(l); free(c);
    return (uint32_t)(o - out);
}

/* my_decompress_file_lz77 2255-2393 + my_LZ77_decompress 1716-1735 */
int64_t orc_decompress_block(const uint8_t *in, uint32_t len, uint8_t *out, uint64_t cap) {
    int64_t ret = -1;
    if (len < 4) return -1;
    const uint8_t *q = in, *end = in + len;
    uint32_t N = get_u32(q); q += 4;
    uint32_t nb = (N + 7) / 8;
    uint8_t *flags = (uint8_t *)calloc((size_t)nb + 1, 1);
    uint8_t *c = (uint8_t *)calloc((size_t)N + 1, 1);
    uint32_t *p = NULL, *l = NULL, *gw = NULL;
    uint8_t *pb = NULL;
    uint32_t u;
    if (nb > 1) { if (!(u = huffman_stream_decode(q, (uint32_t)(end - q), flags, nb))) goto done; q += u; }
    else { if ((uint32_t)(end - q) < nb) goto done; memcpy(flags, q, nb); q += nb; }
    if (!(u = huffman_stream_decode(q, (uint32_t)(end - q), c, N))) goto done;
    q += u;
    if (end - q < 4) goto done;
    uint32_t pc = get_u32(q); q += 4;
    if (pc > N) goto done;
    uint32_t pbytes = (P_BITS * pc) / 8 + 1;
    pb = (uint8_t *)calloc(pbytes, 1);
    if (!(u = huffman_stream_decode(q, (uint32_t)(end - q), pb, pbytes))) goto done;
    q += u;
    p = (uint32_t *)calloc((size_t)pc + 1, 4);
    l = (uint32_t *)calloc((size_t)pc + 1, 4);
    decombine_bits(pb, pc, P_BITS, p);
    if (end - q < 4) goto done;
    uint32_t G = get_u32(q); q += 4;
    gw = (uint32_t *)calloc((size_t)G + 1, 4);
    if (G > 0) {
        if (!(u = huffman_stream_decode(q, (uint32_t)(end - q), (uint8_t *)gw, 4 * G))) goto done;
        q += u;
    }
    if (golomb_decode(gw, G, l, pc) != pc) goto done;
    uint64_t o = 0;
    uint32_t mi = 0;
    for (uint32_t t = 0; t < N; t++) {
        int lit = (flags[t >> 3] >> (t & 7)) & 1;
        if (!lit) {
            if (mi >= pc) break;   /* reference: "Fatal Error", stops building tokens (2331-2335) */
            uint32_t dist = p[mi], L = l[mi++];
            if (dist == 0 || dist > o || o + L + 1 > cap) goto done;
            for (uint32_t k = 0; k < L; k++, o++) out[o] = out[o - dist];
        }
        if (o + 1 > cap) goto done;
        out[o++] = c[t];
    }
    ret = (int64_t)o;
done:
    free(flags); free(c); free(p); free(l); free(gw); free(pb);
    return ret;
}

/* ------------------------------------------------------------------------- */
/* container, main() 4073-4136: "FCX7", u32 total (mod 2^32), u16 blocks
 * (mod 2^16), then [u32 len][payload] per block.                             */
uint64_t orc_compress_file(const uint8_t *in, uint64_t n, uint32_t block_bytes, uint8_t *out,
                           uint64_t cap, int finder) {
    if (cap < 10) return 0;
    uint64_t nblk = (n + block_bytes - 1) / block_bytes;
    memcpy(out, "FCX7", 4);
    put_u32(out + 4, (uint32_t)n);
    uint16_t nb16 = (uint16_t)nblk;
    memcpy(out + 8, &nb16, 2);
    uint64_t o = 10;
    uint8_t *tmp = (uint8_t *)malloc(2 * (size_t)block_bytes + 4096);
    for (uint64_t b = 0; b < nblk; b++) {
        uint64_t off = b * block_bytes;
        uint32_t len = (uint32_t)(n - off < block_bytes ? n - off : block_bytes);
        uint32_t sz = orc_compress_block(in + off, len, tmp, finder);
        if (o + 4 + sz > cap) { free(tmp); return 0; }
        put_u32(out + o, sz);
        memcpy(out + o + 4, tmp, sz);
        o += 4 + sz;
    }
    free(tmp);
    return o;
}

/* main() 4137-4204 */
int64_t orc_decompress_file(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap) {
    if (n < 10 || memcmp(in, "FCX", 3) != 0 || in[3] != '7') return -1;
    uint16_t nblk;
    memcpy(&nblk, in + 8, 2);
    uint64_t q = 10, o = 0;
    for (uint32_t b = 0; b < nblk; b++) {
        if (q + 4 > n) return -1;
        uint32_t sz = get_u32(in + q);
        q += 4;
        if (q + sz > n) return -1;
        int64_t r = orc_decompress_block(in + q, sz, out + o, cap - o);
        if (r < 0) return -1;
        o += (uint64_t)r;
        q += sz;
    }
    return (int64_t)o;
}
