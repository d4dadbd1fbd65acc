/*
 * fcx.h — C ABI of the MI355X-native LZ77 + Huffman compressor (FCX7 format).
 *
 * The reference (YuBinRen/my_compress) has no plugin/FFI surface; its only seam
 * is the per-block function pair main() calls.  Each entry point below names
 * the reference interface it replaces (my_compress.cpp, lines counted by '\n'):
 *
 *   fcx_compress_block    <- uInt32 my_compress_file_lz77(void*, uInt32, uInt8*)   :2115 (called at :4099)
 *   fcx_decompress_block  <- uInt32 my_decompress_file_lz77(void*, uInt32, FILE*) :2255 (called at :4182)
 *   fcx_write_header      <- stCmpFileHead fwrite/rewrite in main()                :101-111, :4079-4086, :4128-4129
 *   fcx_parse_header      <- header read + "FCX" magic check in main()            :4140-4159
 *   fcx_compress_shard    <- main()'s per-block compress loop                      :4090-4122
 *                            (batched: every block of a device-resident shard in one
 *                             launch sequence, emitting [u32 len][payload]...)
 *   fcx_decompress_shard  <- main()'s per-block decompress loop, my_decompress_file_lz77
 *                            per record                                            :4160-4204, :2255
 *                            (GPU decoder: every record of a device-resident run)
 *   fcx_decompress_host   <- the whole decompress mode of main() on host buffers  :4137-4204
 *   fcx_dist_*            <- main()'s compress loop (:4090-4122) with the blocks spread over
 *                            several GPUs: contiguous block ranges per GPU, the segments
 *                            concatenated in block order over RCCL (the reference writes the
 *                            blocks to one file in order, :4112-4114)
 *
 * Conventions: plain pointers and sizes, no exceptions cross the ABI, every
 * function returns FCX_OK (0) or a negative FCX_ERR_* code unless stated; the
 * message of the last error on the calling thread is fcx_last_error().  One
 * host thread per context; functions are reentrant across contexts.
 * The compress path is GPU-only: without a usable HIP device every compress
 * entry point fails with FCX_ERR_HIP (there is no CPU fallback).
 */
#ifndef FCX_H
#define FCX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FCX_OK 0
#define FCX_ERR_ARG (-1)       /* NULL pointer, zero/oversize block, bad value */
#define FCX_ERR_CAPACITY (-2)  /* output buffer too small */
#define FCX_ERR_HIP (-3)       /* HIP runtime error / no device */
#define FCX_ERR_FORMAT (-4)    /* malformed compressed stream */
#define FCX_ERR_INTERNAL (-5)  /* device-side invariant violated */
#define FCX_ERR_NOMEM (-6)
#define FCX_ERR_RCCL (-7)      /* RCCL (collective) error */

#define FCX_HEADER_BYTES 10u                 /* "FCX7" + u32 total + u16 blocks (:101-109) */
#define FCX_DEFAULT_BLOCK_BYTES (1u << 20)  /* BLOCK_BYTES (:113) */
#define FCX_MAX_BLOCK_BYTES (1u << 20)      /* reference decoder buffer limit (:2373) */

typedef struct fcx_ctx fcx_ctx;

/* ---- per-block drop-in (host buffers) ------------------------------------ */

/* Same contract as my_compress_file_lz77 (:2115): compresses `len` bytes at `in`
 * (len <= FCX_MAX_BLOCK_BYTES) and writes the block payload to `out`, which the
 * caller sizes at >= 2*len + 1024 (the reference allots 2 MiB per 1 MiB block,
 * :4088).  Returns payload bytes, or 0 if a pointer is NULL (:2122-2123) or on
 * error (see fcx_last_error).  len == 0 is a valid block, as in the reference: its
 * 17-byte payload (N = 0, pCnt = 0, HUFF of one zero byte, G = 0) is written without
 * touching the device.  Runs on the current HIP device through a lazily created
 * per-thread context. */
uint32_t fcx_compress_block(const void *in, uint32_t len, uint8_t *out);

/* Same contract as my_decompress_file_lz77 (:2255) but into memory: decodes one
 * block payload of `len` bytes into `out` (capacity `cap`).  Returns decoded
 * bytes, or a negative FCX_ERR_* code.  Host decoder. */
int64_t fcx_decompress_block(const uint8_t *in, uint32_t len, uint8_t *out, uint64_t cap);

/* ---- container -------------------------------------------------------------- */

/* writes the 10-byte header: "FCX7", u32 total_in mod 2^32, u16 nblocks mod 2^16 */
int fcx_write_header(uint8_t *out10, uint64_t total_in, uint64_t nblocks);
/* parses a header; kind receives '7' (LZ77) or '8' (LZ78); FCX_ERR_FORMAT if not "FCX" */
int fcx_parse_header(const uint8_t *in10, uint32_t *total_in, uint16_t *nblocks, char *kind);
/* worst-case bytes of fcx_compress_shard's output for n input bytes */
uint64_t fcx_shard_bound(uint64_t n, uint32_t block_bytes);

/* ---- batched device path ---------------------------------------------------- */

/* Creates a context on HIP device `device` for blocks of `block_bytes`
 * (1 <= block_bytes <= FCX_MAX_BLOCK_BYTES) and shards up to `max_shard_bytes`;
 * scratch grows on demand if a later call is larger. */
int fcx_ctx_create(fcx_ctx **ctx, int device, uint32_t block_bytes, uint64_t max_shard_bytes);
void fcx_ctx_destroy(fcx_ctx *ctx);

/* Compresses the n device-resident bytes at d_in as consecutive blocks of the
 * context's block size and writes, contiguously at d_out (device, capacity cap),
 * [u32 payload_len][payload] for every block in order (no file header).  Work
 * is enqueued on `stream` (a hipStream_t; NULL = default stream).  If out_len is
 * non-NULL the call synchronises the stream and stores the byte count there;
 * the count is always also left in device memory (fcx_ctx_device_out_len). */
int fcx_compress_shard(fcx_ctx *ctx, const uint8_t *d_in, uint64_t n, uint8_t *d_out, uint64_t cap,
                       uint64_t *out_len, void *stream);
/* device address of the u64 output length written by the last fcx_compress_shard */
const uint64_t *fcx_ctx_device_out_len(fcx_ctx *ctx);
/* waits for the device and reads that length (and the device error bits) */
int fcx_ctx_read_out_len(fcx_ctx *ctx, uint64_t *out_len);

/* Host-to-host convenience: compresses host memory in shards of the context's
 * shard size through the pipelined stream path below and writes the same
 * [u32 len][payload]... stream to host `out` (capacity cap). */
int fcx_compress_host(fcx_ctx *ctx, const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap,
                      uint64_t *out_len);
/* device, block size and shard capacity of a context (any pointer may be NULL) */
int fcx_ctx_info(fcx_ctx *ctx, int *device, uint32_t *block_bytes, uint64_t *shard_bytes);

/* ---- pipelined host I/O (main()'s read / code / write loop, :4073-4204) ----- */

/* read: fill up to cap bytes, return the count (0 = end of input) or < 0 on error;
 * write: consume n bytes, return 0 or < 0 on error */
typedef int64_t (*fcx_read_fn)(void *user, uint8_t *buf, uint64_t cap);
typedef int (*fcx_write_fn)(void *user, const uint8_t *buf, uint64_t n);

/* Streams input through the GPU in shards of shard_bytes (rounded down to whole
 * blocks): two pinned/device slots, H2D / compute / D2H on separate streams, the
 * next shard read and the previous shard's records written while the GPU
 * compresses.  Emits the [u32 len][payload]... records (no file header; the
 * caller writes it from *total_in and *nblocks). */
int fcx_compress_stream(fcx_ctx *ctx, fcx_read_fn read, fcx_write_fn write, void *user, uint64_t shard_bytes,
                        uint64_t *total_in, uint64_t *total_out, uint64_t *nblocks);

/* ---- introspection ---------------------------------------------------------- */

/* Enables per-kernel hipEvent timing of subsequent fcx_compress_shard calls. */
int fcx_ctx_set_profiling(fcx_ctx *ctx, int enable);
/* Testing: forces how the match search runs in later calls — 0 auto (default: every
 * tile goes to the match unit its own sampled bytes call for, fcx_ctx_route_stats), 1 the
 * general kernel with the bucket search for every tile (unknown positions via the run table /
 * the stitch), 2 the general kernel with the run table for whole tiles, 3 the general kernel,
 * 4 the 4-byte-key unit, 5 the unit without the repeat filter, 6 the unit with the run-mode
 * walk inlined, 7 the unit without the bucket search — modes 1-7 unrouted, every tile of the
 * call through that one kernel.  The output is identical in every mode; only the speed
 * differs. */
int fcx_ctx_set_match_mode(fcx_ctx *ctx, int mode);
/* Pipelined launch: fcx_compress_shard splits the shard's blocks into `groups` groups
 * (0 = automatic, currently one group; at most 8, at least 64 blocks each) and launches
 * consecutive groups on two internal streams, so one group's kernels overlap the next
 * group's.  The output is identical for every setting. */
int fcx_ctx_set_groups(fcx_ctx *ctx, int groups);
/* After a profiled call: number of stages, and stage i's name and device ms (summed over
 * the call's block groups). */
int fcx_ctx_stage_count(fcx_ctx *ctx);
int fcx_ctx_stage(fcx_ctx *ctx, int i, const char **name, float *ms);
/* statistics of the last call (device counters copied back on request):
 * tokens, matches, lazily evaluated positions, lazy tiles, total tiles */
int fcx_ctx_stats(fcx_ctx *ctx, uint64_t *tokens, uint64_t *matches, uint64_t *lazy_evals,
                  uint64_t *lazy_tiles, uint64_t *tiles);
/* The match kernel the last fcx_compress_shard call ran (routed: the unit given the most
 * tiles): 0 general, 1 4-byte keys (small alphabets), 2 without the repeat filter
 * (match-dense data), 3 run-mode walk inlined (long matches), 4 without the bucket search
 * (few matches), 5 the uniform unit (one byte value over the window); -1 for a NULL ctx. */
int fcx_ctx_match_kernel(fcx_ctx *ctx);
/* Routing of the last (routed) call, after a device synchronize: out[0..3] tiles filed to the
 * sparse, runs, 4-byte-key and no-filter units (the runs and no-filter counts include the tiles
 * handed on to them), out[4] tiles handed on (sparse / runs units to the no-filter unit, the
 * uniform unit to the runs unit), out[5] tiles with bytes, out[6] tiles past the units' grids
 * (searched by the units' looped remainder kernels), out[7] 1 when the call waited for its own
 * counts (a context's first call), out[8] tiles filed to the uniform unit (one byte value over
 * the window: closed form).  Writes min(n, FCX_ROUTE_STATS) values; FCX_ERR_ARG when the last
 * call had a forced unit (fcx_ctx_set_match_mode). */
#define FCX_ROUTE_STATS 9
int fcx_ctx_route_stats(fcx_ctx *ctx, uint64_t *out, int n);

/* ---- GPU decoder ------------------------------------------------------------ */

typedef struct fcx_dctx fcx_dctx;

/* Decoder context on HIP device `device`; scratch grows on demand. */
int fcx_dctx_create(fcx_dctx **ctx, int device);
void fcx_dctx_destroy(fcx_dctx *ctx);

/* Decodes `nblocks` consecutive block records ([u32 len][payload]..., an FCX7
 * file without its 10-byte header) of in_len device-resident bytes at d_in into
 * d_out (device, capacity cap), blocks back to back in order.  The bytes equal
 * the reference decoder's (my_decompress_file_lz77 :2255), including its
 * single-symbol sub-stream and early-stop behaviour.  Synchronises `stream` (a
 * hipStream_t; NULL = default) once after the header pass (to size scratch) and
 * once at the end; stores the decoded byte count in *out_len.  FCX_ERR_FORMAT
 * for malformed input, FCX_ERR_CAPACITY if cap is too small. */
int fcx_decompress_shard(fcx_dctx *ctx, const uint8_t *d_in, uint64_t in_len, uint32_t nblocks, uint8_t *d_out,
                         uint64_t cap, uint64_t *out_len, void *stream);
/* Host-to-host: a whole FCX7 file (header included) into `out` (capacity cap),
 * through fcx_decompress_stream. */
int fcx_decompress_host(fcx_dctx *ctx, const uint8_t *in, uint64_t in_len, uint8_t *out, uint64_t cap,
                        uint64_t *out_len);
/* Streams an FCX7 file (header first) through the GPU decoder in groups of up
 * to 256 whole records; max_in (0 = unknown) bounds the staging buffers.
 * Reports the header's total (mod 2^32), the decoded bytes and the records. */
int fcx_decompress_stream(fcx_dctx *ctx, fcx_read_fn read, fcx_write_fn write, void *user, uint64_t max_in,
                          uint32_t *hdr_total, uint64_t *total_out, uint64_t *nblocks);
int fcx_dctx_device(fcx_dctx *ctx, int *device);
/* per-stage hipEvent timing of subsequent fcx_decompress_shard calls */
int fcx_dctx_set_profiling(fcx_dctx *ctx, int enable);
int fcx_dctx_stage_count(fcx_dctx *ctx);
int fcx_dctx_stage(fcx_dctx *ctx, int i, const char **name, float *ms);

/* ---- -c lz78 (FCX8): the reference's second block codec ---------------------
 *   fcx_lz78_compress_block  <- uInt32 my_compress_file_lz78(void*, uInt32, uInt8*)  :3127 (called at :4106)
 *   fcx_lz78_compress_shard  <- main()'s per-block loop with -c lz78                 :4090-4122
 *   fcx_lz78_compress_host   <- the whole -c lz78 compress mode of main()            :4073-4136
 * Same record framing as FCX7 ([u32 len][payload] per block); the payload layout is
 * my_compress_file_lz78's.  GPU-only like the LZ77 path (FCX_ERR_HIP without a device).
 * Compress scratch (~40 B per input byte of a batch of <= 1 GiB) is kept per device
 * between calls; calls on one device are serialised; fcx_lz78_release() frees it. */
/* d_in / d_out device pointers; writes the records (no header) and their length. */
int fcx_lz78_compress_shard(const uint8_t *d_in, uint64_t n, uint32_t block_bytes, uint8_t *d_out, uint64_t cap,
                            uint64_t *out_len, void *stream);
/* host buffers; writes the "FCX8" header (total mod 2^32, u16 block count) + records. */
int fcx_lz78_compress_host(const uint8_t *in, uint64_t n, uint32_t block_bytes, uint8_t *out, uint64_t cap,
                           uint64_t *out_len);
/* frees the current device's LZ78 compress scratch */
int fcx_lz78_release(void);
/* one block: payload bytes (no length prefix), 0 on NULL / error; out >= 10*len + 4096. */
uint32_t fcx_lz78_compress_block(const void *in, uint32_t len, uint8_t *out);
/*   fcx_lz78_decompress_block <- my_decompress_file_lz78(void*, uInt32, FILE*)       :3478 (called at :4189)
 *   fcx_lz78_decompress_host  <- the whole decompress mode of main() for FCX8        :4137-4204
 * GPU decoder, one lane per record; keeps the reference's quirks (a block whose decoded
 * bytes end in 0x00 loses that byte, 3701-3703; a one-symbol char stream decodes as
 * zeros).  decompress_block returns decoded bytes or a negative FCX_ERR_*. */
int64_t fcx_lz78_decompress_block(const uint8_t *in, uint32_t len, uint8_t *out, uint64_t cap);
int fcx_lz78_decompress_host(const uint8_t *in, uint64_t in_len, uint8_t *out, uint64_t cap, uint64_t *out_len);

/* ---- multi-GPU: block ranges per GPU + RCCL over xGMI -------------------------
 * Blocks are independent (the window and the parse restart per block, :1675-1703), so
 * rank r of N compresses the contiguous block range fcx_dist_block_range(nb, r, N) of the
 * input and the only exchange is the concatenation of the per-rank segments
 * ([u32 len][payload]... each) in rank order: an all-gather of the u64 segment sizes,
 * then either a gather to rank 0 (grouped point-to-point receives, every xGMI link at
 * once, 1/N of the all-gather's traffic) or an all-gather-v (one broadcast per source
 * rank with its exact size), straight into the output buffer at each segment's offset.
 * The 10-byte header is the caller's (fcx_write_header from the global totals). */
typedef struct fcx_dist fcx_dist;
#define FCX_DIST_ID_BYTES 128u   /* ncclUniqueId */
#define FCX_DIST_GATHER 0        /* concat to rank 0 only */
#define FCX_DIST_ALLGATHER 1     /* concat on every rank */

/* contiguous block range [b0, b1) of rank r of n (the partition of my_compress_amd.dist) */
void fcx_dist_block_range(uint64_t nblocks, int rank, int nranks, uint64_t *b0, uint64_t *b1);
/* gather-aware partition: rank 0 (the receiver) takes floor(nblocks * share0_ppm / 10^6)
 * blocks first, ranks 1..N-1 split the rest near-evenly (share0_ppm 0 = the even split
 * above).  Equals my_compress_amd.dist.block_range(nblocks, rank, N, share0_ppm). */
void fcx_dist_block_range_w(uint64_t nblocks, int rank, int nranks, uint32_t share0_ppm, uint64_t *b0,
                            uint64_t *b1);
/* a fresh RCCL unique id (rank 0 creates it; the caller hands it to every rank) */
int fcx_dist_unique_id(uint8_t *id);
/* one rank of an N-process job (one process per GPU, on HIP device `device`) */
int fcx_dist_init_rank(fcx_dist **d, int nranks, int rank, const uint8_t *id, int device);
/* one process driving ndev devices (rank i on devices[i]; ncclCommInitAll) */
int fcx_dist_init_local(fcx_dist **d, int ndev, const int *devices);
void fcx_dist_destroy(fcx_dist *d);
/* ranks of the job and ranks driven by this process */
int fcx_dist_size(fcx_dist *d, int *nranks, int *nlocal);
/* Concatenates the segments of every rank in rank order (process-per-GPU form: local
 * index 0).  d_seg/seg_len: this rank's segment (device); d_out/cap: the destination
 * (device; on rank 0 for FCX_DIST_GATHER it may be the buffer d_seg lives in, with
 * d_seg == d_out).  *total receives the concatenated length on every rank.  Enqueued on
 * `stream` (a hipStream_t of the rank's device) and synchronised. */
int fcx_dist_concat(fcx_dist *d, int local, const uint8_t *d_seg, uint64_t seg_len, uint8_t *d_out, uint64_t cap,
                    uint64_t *total, int mode, void *stream);
/* The strong-scaling step of one rank, compress and concatenation overlapped (process-per-GPU
 * form).  Every rank passes rank_bytes[0..N) (each rank's input bytes, e.g. from
 * fcx_dist_block_range_w; the same array everywhere) and its own n = rank_bytes[rank] device
 * bytes at d_in.  A peer (rank > 0) compresses its range as `nsub` sub-batches of whole blocks
 * (1 <= nsub <= FCX_DIST_MAX_SUB), each at its bound offset of d_out (capacity >=
 * fcx_dist_gather_bound(n, block, nsub)), and sends each piece to rank 0 as soon as it is done
 * (its u64 length and error word, then its bytes) while the next piece compresses.  Rank 0
 * compresses its range into d_out at offset 0 while the pieces arrive in a staging buffer the
 * handle keeps, then moves them behind its own segment: d_out[0, *total) on rank 0 is every
 * rank's [u32 len][payload] records in block order (capacity >= fcx_shard_bound of the whole
 * input).  A peer whose compress fails sends failure words instead of pieces, so rank 0 always
 * completes the exchange; rank 0 then sends the job's verdict to every peer, so every rank
 * returns an error when any rank failed.  *total: the concatenation on rank 0, the bytes sent on
 * a peer.  Collective over the job; `stream` is the compress stream; returns after both streams
 * are synchronised. */
#define FCX_DIST_MAX_SUB 64u
int fcx_dist_compress_gather(fcx_dist *d, fcx_ctx *ctx, const uint8_t *d_in, uint64_t n, const uint64_t *rank_bytes,
                             uint32_t nsub, uint8_t *d_out, uint64_t cap, uint64_t *total, void *stream);
/* d_out capacity fcx_dist_compress_gather needs for n input bytes in nsub sub-batches */
uint64_t fcx_dist_gather_bound(uint64_t n, uint32_t block_bytes, uint32_t nsub);
/* The whole job in one process (fcx_dist_init_local): host input, rounds of up to
 * round_bytes per device (0 = 1 GiB) split into block ranges, every device compresses
 * its range with one host thread each, the segments are gathered to local rank 0 over
 * RCCL and copied to `out` ([u32 len][payload] records, no header); *out_len = bytes. */
int fcx_dist_compress_host(fcx_dist *d, const uint8_t *in, uint64_t n, uint32_t block_bytes, uint64_t round_bytes,
                           uint8_t *out, uint64_t cap, uint64_t *out_len);
/* name of the transport under a handle: "rccl" or "loopback" */
const char *fcx_dist_transport(fcx_dist *d);

/* ---- loopback transport: the protocols above between thread ranks of one process ------
 * The multi-rank protocols (fcx_dist_concat, fcx_dist_compress_gather, fcx_dist_compress_host)
 * talk to a transport seam (group start/end, send/recv of device bytes, all-gather,
 * broadcast); RCCL is the product transport.  The loopback transport runs the same protocol
 * code between host threads of one process on one device -- each thread rank with its own
 * fcx_dist, fcx_ctx and streams -- so the N > 1 exchange runs on a one-GPU box: a matched
 * send/recv pair is one device-to-device copy on the hub's stream, ordered after both sides'
 * stream positions, and both streams wait for it.  An operation left unmatched for
 * timeout_ms (0 = 60 s) aborts the hub, and every rank then fails instead of hanging. */
typedef struct fcx_loop fcx_loop;
int fcx_loop_create(fcx_loop **hub, int nranks, int device, uint32_t timeout_ms);
/* drops the creator's reference; the hub lives until its last fcx_dist is destroyed */
void fcx_loop_destroy(fcx_loop *hub);
/* rank `rank` of the hub's job, one rank per handle (the fcx_dist_init_rank form) */
int fcx_dist_init_loop(fcx_dist **d, fcx_loop *hub, int rank);
/* every rank of an nranks job in one handle on one device (the fcx_dist_init_local form) */
int fcx_dist_init_loop_local(fcx_dist **d, int nranks, int device, uint32_t timeout_ms);
/* Rank 0 of the last fcx_dist_compress_gather: device ms of its final moves of the peers' bytes
 * behind its own segment (N - 1 copies, hipEvents on its stream); -1 on a peer or before any. */
int fcx_dist_gather_copy_ms(fcx_dist *d, float *ms);
/* Testing: a peer of fcx_dist_compress_gather treats sub-batch `piece` as failed after the
 * earlier pieces are queued (as device error bits would); -1 = off. */
int fcx_dist_debug_fail(fcx_dist *d, int piece);

const char *fcx_last_error(void);
const char *fcx_version(void);

#ifdef __cplusplus
}
#endif
#endif /* FCX_H */
