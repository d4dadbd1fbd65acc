// cli.cpp — the my_compress command line (main(), my_compress.cpp:3726-4213),
// compress path on the GPU through the C ABI.
//
//   my_compress -i IN [-o OUT] -c lz77     compress (FCX7, 1 MiB blocks)
//   my_compress -i IN [-o OUT]             decompress
//
// Same flags, default output "./out" (4040-4042) and byte stream as the
// reference.  Both directions stream through the GPU (fcx_compress_stream /
// fcx_decompress_stream: file reads and writes overlap the device work); without
// a HIP device, compress fails and decompress uses the host decoder.  Superset:
// -b/--block BYTES (<= 1 MiB; the reference fixes 1 MiB, BLOCK_BYTES :113) and
// -d/--device N and -g/--gpus N (-c lz77 over N GPUs of this node, devices d .. d+N-1:
// contiguous block ranges per GPU, segments gathered over RCCL, byte-identical
// output).  `-c lz78` runs the LZ78 codec (FCX8) on the GPU: 256 MiB shards
// through fcx_lz78_compress_host / fcx_lz78_decompress_host (whole files in host
// memory for decompress).
#include <getopt.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "fcx.h"

static int usage() {
    fprintf(stderr,
            "usage: ./my_compress -i[or --file_in] <input file name> [-o[or --file_out] <output file name>] "
            "[-c (or --compress) <lz77/lz78>] [-b (or --block) <bytes>] [-d (or --device) <hip device>] "
            "[-g (or --gpus) <count>]\n");
    return -1;
}

static int64_t file_read(void *u, uint8_t *buf, uint64_t cap) {
    FILE *f = (FILE *)u;
    const size_t n = fread(buf, 1, (size_t)cap, f);
    return ferror(f) ? -1 : (int64_t)n;
}

struct Files {
    FILE *in, *out;
};
static int64_t files_read(void *u, uint8_t *buf, uint64_t cap) { return file_read(((Files *)u)->in, buf, cap); }
static int files_write(void *u, const uint8_t *buf, uint64_t n) {
    return fwrite(buf, 1, (size_t)n, ((Files *)u)->out) == n ? 0 : -1;
}

static int do_compress(FILE *fin, FILE *fout, uint32_t block, int device) {
    // 256 MiB shards through the pipelined stream path: the next shard is read and the
    // previous one written while the GPU compresses (main()'s loop, 4073-4136)
    const uint64_t shard = (256ull << 20) / block * block;
    fcx_ctx *ctx = nullptr;
    if (fcx_ctx_create(&ctx, device, block, shard)) {
        fprintf(stderr, "fcx: %s\n", fcx_last_error());
        return -1;
    }
    uint8_t hdr[FCX_HEADER_BYTES];
    fcx_write_header(hdr, 0, 0);  // placeholder, rewritten at the end (4079-4086, 4128-4129)
    fwrite(hdr, 1, sizeof(hdr), fout);
    uint64_t total_in = 0, total_out = 0, nblocks = 0;
    Files io{fin, fout};
    auto t0 = std::chrono::steady_clock::now();
    const int r = fcx_compress_stream(ctx, files_read, files_write, &io, shard, &total_in, &total_out, &nblocks);
    if (r) {
        fprintf(stderr, "fcx: %s\n", fcx_last_error());
        fcx_ctx_destroy(ctx);
        return -1;
    }
    fcx_write_header(hdr, total_in, nblocks);
    fseek(fout, 0, SEEK_SET);
    fwrite(hdr, 1, sizeof(hdr), fout);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("<Final>: LZ77 totalBytes = %llu, compress total bytes=%llu, compress rate: %.2f%%\n",
           (unsigned long long)total_in, (unsigned long long)total_out,
           total_in ? 100.0 * (double)total_out / (double)total_in : 0.0);
    printf("[***TIME***]  All block compress spend %.0f ms!!!\n", ms);
    if (nblocks > 65535) fprintf(stderr, "warning: %llu blocks exceed the u16 block count of the format\n",
                                 (unsigned long long)nblocks);
    fcx_ctx_destroy(ctx);
    return 0;
}

// -c lz77 over ngpus devices (fcx_dist_compress_host): the file in rounds of up to
// 1 GiB per GPU, each round's block ranges compressed in parallel and gathered to the
// first device over RCCL, records written in block order (4090-4122)
static int do_compress_dist(FILE *fin, FILE *fout, uint32_t block, int device, int ngpus) {
    std::vector<int> devs(ngpus);
    for (int i = 0; i < ngpus; i++) devs[i] = device + i;
    fcx_dist *d = nullptr;
    if (fcx_dist_init_local(&d, ngpus, devs.data())) {
        fprintf(stderr, "fcx: %s\n", fcx_last_error());
        return -1;
    }
    const uint64_t per = (1ull << 30) / block * block;
    std::vector<uint8_t> buf(per * (uint64_t)ngpus), out(fcx_shard_bound(buf.size(), block));
    uint8_t hdr[FCX_HEADER_BYTES];
    fcx_write_header(hdr, 0, 0);
    fwrite(hdr, 1, sizeof(hdr), fout);
    uint64_t total_in = 0, total_out = 0, nblocks = 0;
    auto t0 = std::chrono::steady_clock::now();
    int rc = 0;
    for (;;) {
        const size_t n = fread(buf.data(), 1, buf.size(), fin);
        if (n == 0) break;
        uint64_t got = 0;
        if (fcx_dist_compress_host(d, buf.data(), n, block, per, out.data(), out.size(), &got)) {
            fprintf(stderr, "fcx: %s\n", fcx_last_error());
            rc = -1;
            break;
        }
        fwrite(out.data(), 1, (size_t)got, fout);
        total_in += n;
        total_out += got;
        nblocks += (n + block - 1) / block;
    }
    fcx_dist_destroy(d);
    if (rc) return rc;
    fcx_write_header(hdr, total_in, nblocks);
    fseek(fout, 0, SEEK_SET);
    fwrite(hdr, 1, sizeof(hdr), fout);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("<Final>: LZ77 totalBytes = %llu, compress total bytes=%llu, compress rate: %.2f%% (%d GPUs)\n",
           (unsigned long long)total_in, (unsigned long long)total_out,
           total_in ? 100.0 * (double)total_out / (double)total_in : 0.0, ngpus);
    printf("[***TIME***]  All block compress spend %.0f ms!!!\n", ms);
    if (nblocks > 65535) fprintf(stderr, "warning: %llu blocks exceed the u16 block count of the format\n",
                                 (unsigned long long)nblocks);
    return 0;
}

// the reference compares sizes only (4198-4201)
static int report(uint64_t got_total, uint32_t total) {
    const bool ok = (uint32_t)got_total == total;
    printf("All block decompress total bytes = %llu, Compress Before bytes = %u [%s]\n",
           (unsigned long long)got_total, total, ok ? "SUCCESS" : "FAIL");
    return ok ? 0 : 1;
}

// host decoder, used when no HIP device is present
static int decompress_host(FILE *fin, FILE *fout, uint32_t total, uint16_t nblocks) {
    std::vector<uint8_t> payload, plain(FCX_MAX_BLOCK_BYTES + 8);
    uint64_t got_total = 0;
    for (uint32_t b = 0; b < nblocks; b++) {
        uint32_t sz = 0;
        if (fread(&sz, 4, 1, fin) != 1) return -1;
        payload.resize(sz);
        if (fread(payload.data(), 1, sz, fin) != sz) return -1;
        int64_t n = fcx_decompress_block(payload.data(), sz, plain.data(), plain.size());
        if (n < 0) {
            fprintf(stderr, "block %u: %s\n", b + 1, n == FCX_ERR_FORMAT ? "malformed" : "decode error");
            return -1;
        }
        fwrite(plain.data(), 1, (size_t)n, fout);
        got_total += (uint64_t)n;
    }
    return report(got_total, total);
}

// FCX8 (-c lz78): 256 MiB shards of whole blocks, each through the GPU codec
static int compress_lz78(FILE *fin, FILE *fout, uint32_t block) {
    const uint64_t shard = (256ull << 20) / block * block;
    std::vector<uint8_t> buf(shard), out;
    uint8_t hdr[FCX_HEADER_BYTES];
    memcpy(hdr, "FCX8", 4);
    memset(hdr + 4, 0, 6);
    fwrite(hdr, 1, sizeof(hdr), fout);   // placeholder, rewritten at the end (4079-4086)
    uint64_t total_in = 0, total_out = 0, nblocks = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const size_t n = fread(buf.data(), 1, buf.size(), fin);
        if (n == 0) break;
        out.resize(FCX_HEADER_BYTES + 10 * n + 4096 * (n / block + 1));
        uint64_t got = 0;
        if (fcx_lz78_compress_host(buf.data(), n, block, out.data(), out.size(), &got)) {
            fprintf(stderr, "fcx: %s\n", fcx_last_error());
            return -1;
        }
        fwrite(out.data() + FCX_HEADER_BYTES, 1, got - FCX_HEADER_BYTES, fout);
        total_in += n;
        total_out += got - FCX_HEADER_BYTES;
        nblocks += (n + block - 1) / block;
    }
    const uint32_t t32 = (uint32_t)total_in;
    const uint16_t nb16 = (uint16_t)nblocks;
    memcpy(hdr + 4, &t32, 4);
    memcpy(hdr + 8, &nb16, 2);
    fseek(fout, 0, SEEK_SET);
    fwrite(hdr, 1, sizeof(hdr), fout);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("<Final>: LZ78 totalBytes = %llu, compress total bytes=%llu, compress rate: %.2f%%\n",
           (unsigned long long)total_in, (unsigned long long)total_out,
           total_in ? 100.0 * (double)total_out / (double)total_in : 0.0);
    printf("[***TIME***]  All block compress spend %.0f ms!!!\n", ms);
    if (nblocks > 65535) fprintf(stderr, "warning: %llu blocks exceed the u16 block count of the format\n",
                                 (unsigned long long)nblocks);
    (void)fcx_lz78_release();   // the codec's cached device scratch
    return 0;
}

static int decompress_lz78(FILE *fin, FILE *fout, uint32_t total) {
    rewind(fin);
    std::vector<uint8_t> blob;
    uint8_t tmp[1 << 16];
    size_t n;
    while ((n = fread(tmp, 1, sizeof(tmp), fin)) > 0) blob.insert(blob.end(), tmp, tmp + n);
    uint16_t nblocks;
    memcpy(&nblocks, blob.data() + 8, 2);
    // decoded bytes <= the header's total (mod 2^32; the reference decoder never adds
    // bytes, it may drop a trailing 0x00 per block): size by it, and only when that
    // fails on capacity (a total that wrapped) by the decoder's per-block bound (:2373)
    std::vector<uint8_t> out((uint64_t)total + 64ull * nblocks + 64);
    uint64_t got = 0;
    int r = fcx_lz78_decompress_host(blob.data(), blob.size(), out.data(), out.size(), &got);
    if (r == FCX_ERR_CAPACITY) {
        out.assign((uint64_t)nblocks * (FCX_MAX_BLOCK_BYTES + 8) + 1, 0);
        r = fcx_lz78_decompress_host(blob.data(), blob.size(), out.data(), out.size(), &got);
    }
    if (r) {
        fprintf(stderr, "fcx: %s\n", fcx_last_error());
        return -1;
    }
    fwrite(out.data(), 1, (size_t)got, fout);
    return report(got, total);
}

static int do_decompress(FILE *fin, FILE *fout, int device) {
    uint8_t hdr[FCX_HEADER_BYTES];
    if (fread(hdr, 1, sizeof(hdr), fin) != sizeof(hdr)) {
        fprintf(stderr, "Read file head infomation error!!!\n");
        return -1;
    }
    uint32_t total = 0;
    uint16_t nblocks = 0;
    char kind = 0;
    if (fcx_parse_header(hdr, &total, &nblocks, &kind)) {
        fprintf(stderr, "This file is not support to decompress!!!!\n");
        return -1;
    }
    if (kind != '7') return decompress_lz78(fin, fout, total);
    fcx_dctx *d = nullptr;
    if (fcx_dctx_create(&d, device) != FCX_OK) {
        fprintf(stderr, "fcx: %s; decoding on the host\n", fcx_last_error());
        return decompress_host(fin, fout, total, nblocks);
    }
    // GPU decoder over whole records (the stream path re-reads the header)
    rewind(fin);
    Files io{fin, fout};
    uint64_t got_total = 0, nrec = 0;
    uint32_t htotal = 0;
    const int r = fcx_decompress_stream(d, files_read, files_write, &io, 0, &htotal, &got_total, &nrec);
    fcx_dctx_destroy(d);
    if (r) {
        fprintf(stderr, "fcx: %s\n", fcx_last_error());
        return -1;
    }
    return report(got_total, total);
}

int main(int argc, char **argv) {
    static struct option long_options[] = {{"file_in", required_argument, nullptr, 'i'},
                                           {"file_out", required_argument, nullptr, 'o'},
                                           {"compress", required_argument, nullptr, 'c'},
                                           {"block", required_argument, nullptr, 'b'},
                                           {"device", required_argument, nullptr, 'd'},
                                           {"gpus", required_argument, nullptr, 'g'},
                                           {nullptr, 0, nullptr, 0}};
    std::string file_in, file_out = "./out";
    bool compress = false, lz77 = false;
    uint32_t block = FCX_DEFAULT_BLOCK_BYTES;
    int device = 0, ngpus = 1, opt;
    bool dist = false;   // -g given: the RCCL multi-GPU path (also at -g 1)
    if (argc < 3) return usage();
    while ((opt = getopt_long(argc, argv, "i:o:c:b:d:g:", long_options, nullptr)) != -1) {
        switch (opt) {
        case 'i': file_in = optarg; break;
        case 'o': file_out = optarg; break;
        case 'c':
            compress = true;
            lz77 = strncmp(optarg, "lz77", 4) == 0;  // any other value means LZ78 (4034-4038)
            break;
        case 'b': block = (uint32_t)strtoul(optarg, nullptr, 0); break;
        case 'd': device = atoi(optarg); break;
        case 'g': ngpus = atoi(optarg); dist = true; break;
        default: return usage();
        }
    }
    if (file_in.empty() || ngpus < 1) return usage();
    if (block == 0 || block > FCX_MAX_BLOCK_BYTES) {
        fprintf(stderr, "block size must be in [1, %u]\n", FCX_MAX_BLOCK_BYTES);
        return -1;
    }
    FILE *fin = fopen(file_in.c_str(), "rb");
    if (!fin) { printf("open: %s Fail!!\n", file_in.c_str()); return -1; }
    FILE *fout = fopen(file_out.c_str(), "wb");
    if (!fout) { printf("open: %s Fail!!\n", file_out.c_str()); fclose(fin); return -1; }
    if (!compress) (void)hipSetDevice(device);   // the FCX8 decoder runs on the current device
    if (compress && !lz77 && hipSetDevice(device) != hipSuccess) {
        fprintf(stderr, "fcx: no HIP device %d\n", device);
        return -1;
    }
    const int r = compress ? (lz77 ? (dist ? do_compress_dist(fin, fout, block, device, ngpus)
                                                                  : do_compress(fin, fout, block, device))
                                   : compress_lz78(fin, fout, block))
                           : do_decompress(fin, fout, device);
    fclose(fin);
    fclose(fout);
    return r;
}
