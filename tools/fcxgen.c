/*
 * fcxgen — synthetic input generators for the FCX7 / LZ77 benchmark configs.
 *
 * Not part of the compress path and not part of the oracle: this is the input
 * specification of SURVEY.md §8(d) / Appendix B.2, shared by tests, bench.py
 * and the golden-vector script.  The reference's only RNG idiom is
 * `srand(seed); rand() % k` (随机数的生成.cpp:35-38); glibc's TYPE_3 additive
 * generator is embedded here so the bytes do not depend on the host libc.
 *
 *   rand : byte = rand() % 256
 *   zeros: all 0x00
 *   runs : repeat { b = rand()%4; r = 1 + rand()%64; append r x b }
 *   text : 4096-word vocabulary over "etaoinshrdlcumwfgypbvkjxqz" with
 *          letter = A[min(rand()%26, rand()%26)], sentences of 8..20 words,
 *          word index r1 % (1 + rand()%V) with r1 drawn FIRST, a capitalised
 *          first word, ". " sentence ends and '\n' after every 4th sentence.
 *
 * Every generator is streaming: gen_*(state, out, n) appends the next n bytes,
 * so a caller can produce a multi-GiB input in pieces (fcxgen_fill).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---- glibc random_r TYPE_3 (deg 31, sep 3) -------------------------------- */
typedef struct {
    int32_t r[34];   /* ring of the last 34 outputs of the recurrence */
    uint32_t k;      /* ring slot (0..33) of the next value */
} glibc_rand_t;

static void grand_seed(glibc_rand_t *g, uint32_t seed) {
    int32_t r[344 + 34];
    if (seed == 0) seed = 1;
    r[0] = (int32_t)seed;
    for (int i = 1; i < 31; i++) {
        /* r[i] = (16807 * r[i-1]) % 2147483647 via Schrage's method */
        int32_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
        int32_t w = 16807 * lo - 2836 * hi;
        if (w < 0) w += 2147483647;
        r[i] = w;
    }
    for (int i = 31; i < 34; i++) r[i] = r[i - 31];
    for (int i = 34; i < 344 + 34; i++) r[i] = (int32_t)((uint32_t)r[i - 31] + (uint32_t)r[i - 3]);
    /* keep the 34 most recent values: sequence indices 344 .. 377 */
    for (int i = 0; i < 34; i++) g->r[i] = r[344 + i];
    g->k = 0; /* next rand() returns r[344 + 0] >> 1 */
}

/* the k-th rand() returns r[344+k] >> 1; the ring holds the 34 raw values
 * r[344+k .. 344+k+34) and slot g->k holds r[344+k]. */
static inline int32_t grand_next(glibc_rand_t *g) {
    uint32_t slot = g->k;
    g->k = slot == 33 ? 0 : slot + 1;
    int32_t v = g->r[slot];
    /* value for index 344+k+34 = r[344+k+3] + r[344+k+31] */
    uint32_t s3 = slot + 3 >= 34 ? slot + 3 - 34 : slot + 3;
    uint32_t s31 = slot + 31 >= 34 ? slot + 31 - 34 : slot + 31;
    g->r[slot] = (int32_t)((uint32_t)g->r[s3] + (uint32_t)g->r[s31]);
    return (int32_t)((uint32_t)v >> 1);
}

/* ---- generator state ------------------------------------------------------ */
enum { GEN_RAND = 0, GEN_ZEROS = 1, GEN_RUNS = 2, GEN_TEXT = 3, GEN_DNA = 4 };

#define TEXT_V 4096
typedef struct {
    int kind;
    glibc_rand_t g;
    /* runs: pending run */
    uint32_t run_left; uint8_t run_byte;
    /* text */
    char *vocab;            /* TEXT_V words of <= 10 letters, each 11 bytes */
    uint8_t wlen[TEXT_V];
    uint32_t in_sent, sent_len, sents;
    uint8_t pend[16]; uint32_t pend_n, pend_pos; /* bytes of the current word + separator */
} fcxgen_t;

static const char *ALPHA = "etaoinshrdlcumwfgypbvkjxqz";

static void text_next_word(fcxgen_t *s) {
    int32_t r1 = grand_next(&s->g);
    int32_t k = 1 + grand_next(&s->g) % TEXT_V;
    int32_t idx = r1 % k;
    uint32_t n = 0;
    memcpy(s->pend, s->vocab + 11 * idx, s->wlen[idx]);
    n = s->wlen[idx];
    if (s->in_sent == 0) s->pend[0] = (uint8_t)(s->pend[0] - 32);
    s->in_sent++;
    if (s->in_sent >= s->sent_len) {
        s->pend[n++] = '.';
        s->pend[n++] = ' ';
        s->in_sent = 0;
        s->sent_len = 8 + grand_next(&s->g) % 13;
        if (++s->sents % 4 == 0) s->pend[n++] = '\n';
    } else {
        s->pend[n++] = ' ';
    }
    s->pend_n = n;
    s->pend_pos = 0;
}

void *fcxgen_create(int kind, uint32_t seed) {
    fcxgen_t *s = (fcxgen_t *)calloc(1, sizeof(fcxgen_t));
    if (!s) return NULL;
    s->kind = kind;
    grand_seed(&s->g, seed);
    if (kind == GEN_TEXT) {
        s->vocab = (char *)calloc(TEXT_V, 11);
        for (int i = 0; i < TEXT_V; i++) {
            int L = 1 + grand_next(&s->g) % 10;
            for (int j = 0; j < L; j++) {
                int a = grand_next(&s->g) % 26;
                int b = grand_next(&s->g) % 26;
                s->vocab[11 * i + j] = ALPHA[a < b ? a : b];
            }
            s->wlen[i] = (uint8_t)L;
        }
        s->in_sent = 0;
        s->sent_len = 8 + grand_next(&s->g) % 13;
        s->sents = 0;
        s->pend_n = s->pend_pos = 0;
    }
    return s;
}

void fcxgen_destroy(void *h) {
    fcxgen_t *s = (fcxgen_t *)h;
    if (!s) return;
    free(s->vocab);
    free(s);
}

/* append the next n bytes of the stream to out */
void fcxgen_fill(void *h, uint8_t *out, uint64_t n) {
    fcxgen_t *s = (fcxgen_t *)h;
    uint64_t i = 0;
    switch (s->kind) {
    case GEN_RAND:
        for (; i < n; i++) out[i] = (uint8_t)(grand_next(&s->g) % 256);
        break;
    case GEN_ZEROS:
        memset(out, 0, n);
        break;
    case GEN_DNA:   /* "ACGT"[rand() % 4]: a 4-letter alphabet, 64 distinct 3-byte keys */
        for (; i < n; i++) out[i] = (uint8_t)"ACGT"[grand_next(&s->g) % 4];
        break;
    case GEN_RUNS:
        while (i < n) {
            if (s->run_left == 0) {
                s->run_byte = (uint8_t)(grand_next(&s->g) % 4);
                s->run_left = 1 + grand_next(&s->g) % 64;
            }
            uint64_t take = s->run_left < n - i ? s->run_left : n - i;
            memset(out + i, s->run_byte, take);
            i += take;
            s->run_left -= (uint32_t)take;
        }
        break;
    case GEN_TEXT:
        while (i < n) {
            if (s->pend_pos == s->pend_n) text_next_word(s);
            uint32_t avail = s->pend_n - s->pend_pos;
            uint64_t take = avail < n - i ? avail : n - i;
            memcpy(out + i, s->pend + s->pend_pos, take);
            s->pend_pos += (uint32_t)take;
            i += take;
        }
        break;
    }
}

/* ---- jump-ahead for the rand kind ------------------------------------------
 * r[i] = r[i-31] + r[i-3] (mod 2^32) is linear: with s = r[j..j+31) the state at
 * the next output index j, one step maps s -> (s[1..30], s[0] + s[28]).  Skipping
 * k outputs applies M^k (31x31 over Z/2^32) by binary powering: O(31^3 log k).
 * Lets rank r of a multi-GPU run start at byte r*shard of one seeded stream
 * (BASELINE config 4: 8 GiB rand seed 4 sharded over 8 GPUs).                 */
typedef struct { uint32_t a[31][31]; } mat31;

static void mat_mul(const mat31 *x, const mat31 *y, mat31 *z) {
    for (int i = 0; i < 31; i++)
        for (int j = 0; j < 31; j++) {
            uint32_t acc = 0;
            for (int k = 0; k < 31; k++) acc += x->a[i][k] * y->a[k][j];
            z->a[i][j] = acc;
        }
}

int fcxgen_skip(void *h, uint64_t k) {
    fcxgen_t *s = (fcxgen_t *)h;
    if (!s || (s->kind != GEN_RAND && s->kind != GEN_DNA)) return -1;
    uint32_t st[31], nst[31];
    for (int i = 0; i < 31; i++) st[i] = (uint32_t)s->g.r[(s->g.k + i) % 34u];
    mat31 base, res, tmp;
    memset(&base, 0, sizeof(base));
    for (int i = 0; i < 30; i++) base.a[i][i + 1] = 1;
    base.a[30][0] = 1;
    base.a[30][28] = 1;
    memset(&res, 0, sizeof(res));
    for (int i = 0; i < 31; i++) res.a[i][i] = 1;
    uint64_t e = k;
    while (e) {
        if (e & 1) { mat_mul(&res, &base, &tmp); res = tmp; }
        mat_mul(&base, &base, &tmp);
        base = tmp;
        e >>= 1;
    }
    for (int i = 0; i < 31; i++) {
        uint32_t acc = 0;
        for (int j = 0; j < 31; j++) acc += res.a[i][j] * st[j];
        nst[i] = acc;
    }
    /* rebuild the 34-entry ring for the new position */
    s->g.k = (uint32_t)((s->g.k + k) % 34u);
    uint32_t vals[34];
    for (int i = 0; i < 31; i++) vals[i] = nst[i];
    for (int i = 31; i < 34; i++) vals[i] = vals[i - 31] + vals[i - 3];
    for (int i = 0; i < 34; i++) s->g.r[(s->g.k + i) % 34u] = (int32_t)vals[i];
    return 0;
}

/* one-shot convenience: n bytes of `kind` with `seed` */
int fcxgen_generate(int kind, uint32_t seed, uint8_t *out, uint64_t n) {
    void *h = fcxgen_create(kind, seed);
    if (!h) return -1;
    fcxgen_fill(h, out, n);
    fcxgen_destroy(h);
    return 0;
}

/* first n raw rand() values (for checking the embedded generator) */
void fcxgen_rand_values(uint32_t seed, int32_t *out, int n) {
    glibc_rand_t g;
    grand_seed(&g, seed);
    for (int i = 0; i < n; i++) out[i] = grand_next(&g);
}
