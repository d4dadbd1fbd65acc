/*
 * fcx_oracle.h — CPU restatement of the reference's LZ77 + Huffman block codec.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this; the product (my_compress_amd/) never links it.
 * Pinned against the reference's own KATs and against oracle/_ref (the
 * reference compiled in place) — see tests/test_oracle.py.
 *
 * All integers are little-endian; all functions are reentrant.
 */
#ifndef FCX_ORACLE_H
#define FCX_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_FINDER_SUNDAY = 0, ORC_FINDER_EXHAUSTIVE = 1 };

/* Sunday_Search (my_compress.cpp:1407-1443): leftmost occurrence or -1 */
int32_t orc_sunday_search(const uint8_t *text, int32_t text_len, const uint8_t *pat, int32_t pat_len);

/* greedy LZ77 parse (my_compress.cpp:1675-1714); p/l/c capacity >= len; returns N */
uint32_t orc_lz77_parse(const uint8_t *in, uint32_t len, int finder, uint32_t *p, uint32_t *l, uint8_t *c);

/* golomb_rice_encode k=2 (my_compress.cpp:258-304); returns word count */
uint32_t orc_golomb_encode(const uint32_t *vals, uint32_t n, uint32_t *words);

/* combine_bits (my_compress.cpp:1292-1313): writes (bits*n)/8+1 bytes */
void orc_combine_bits(const uint32_t *vals, uint32_t n, uint32_t bits, uint8_t *out);

/* create_huffman_tree (my_compress.cpp:535-617): nodes = (2n-1) x {w,parent,l,r};
 * returns realLeafNum */
uint32_t orc_huffman_tree(const uint32_t *weights, uint32_t n, uint32_t *nodes);

/* my_huffman_encode_char (my_compress.cpp:987-1104); returns bytes written */
uint32_t orc_huffman_stream(const uint8_t *src, uint32_t n, uint8_t *out);

/* my_compress_file_lz77 (my_compress.cpp:2115-2253); returns payload bytes */
uint32_t orc_compress_block(const uint8_t *in, uint32_t len, uint8_t *out, int finder);

/* my_decompress_file_lz77 (my_compress.cpp:2255-2393); returns decoded bytes,
 * or -1 on a malformed stream */
int64_t orc_decompress_block(const uint8_t *in, uint32_t len, uint8_t *out, uint64_t cap);

/* main() compress loop (my_compress.cpp:4073-4136) over an in-memory input;
 * returns total bytes (10-byte header + sum(4 + payload)), or 0 if cap is short */
uint64_t orc_compress_file(const uint8_t *in, uint64_t n, uint32_t block_bytes, uint8_t *out,
                           uint64_t cap, int finder);

/* main() decompress loop (my_compress.cpp:4137-4204); returns decoded bytes or -1 */
int64_t orc_decompress_file(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap);

/* one Huffman sub-stream decoder (huffman_decode_char 930-984 / my_huffman_decode_char
 * 1107-1187); returns bytes consumed, 0 on malformed input */
uint32_t orc_huffman_stream_decode(const uint8_t *in, uint32_t avail, uint8_t *dst, uint32_t count);

/* ---- -c lz78 (lz78_oracle.c) ---------------------------------------------- */
/* my_LZ78_compress (my_compress.cpp:1832-1899): tokens (idx, c); returns N */
uint32_t orc_lz78_parse(const uint8_t *in, uint32_t len, uint32_t *idx, uint8_t *c);
/* my_compress_file_lz78 (my_compress.cpp:3127-3476); returns payload bytes */
uint32_t orc_lz78_compress_block(const uint8_t *in, uint32_t len, uint8_t *out);
/* my_decompress_file_lz78 (my_compress.cpp:3478-3710); decoded bytes or -1 */
int64_t orc_lz78_decompress_block(const uint8_t *in, uint32_t len, uint8_t *out, uint64_t cap);
/* main() with -c lz78: "FCX8" file; total bytes or 0 */
uint64_t orc_lz78_compress_file(const uint8_t *in, uint64_t n, uint32_t block_bytes, uint8_t *out, uint64_t cap);
int64_t orc_lz78_decompress_file(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap);

#ifdef __cplusplus
}
#endif
#endif
