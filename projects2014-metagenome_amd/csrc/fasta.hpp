// fasta.hpp -- FASTA / FASTQ (optionally gzip) input, split into reads on the device.
//
// The reference parses every input file on the host with kseq (seq_io/sequence_io.cpp:364-405,
// read_fasta_file_critical), one OpenMP thread per file (cli/build.cpp:31-56), and hands the
// records to the constructor in batches of 1 MB / ~25 000 reads (BatchAccumulator,
// common/batch_accumulator.hpp:14-102).  Here the caller's thread only reads (and, for .gz,
// inflates) the file into pinned memory; at build time the raw bytes go to HBM in one copy and
// three tile kernels split them into the read buffer the extractor takes (each record's sequence,
// lines joined, followed by a '$' separator):
//   stats  -- per tile: position of its last newline (FASTA) / its newline count (FASTQ);
//   count  -- per tile, with the line state at its start known from the prefix max / sum: the
//             bytes it keeps and the records it starts;
//   write  -- the kept bytes at the tile's scanned offset, '$' for every record boundary, and the
//             read starts (for per-read counts).
// Record rules (kseq's kseq_read): FASTA -- a line starting with '>' or '@' is a header, every other
// line belongs to the current record's sequence, '\n' and a '\r' right before it are dropped (a
// '\r' inside a line stays a sequence byte, which breaks k-mer windows like any invalid char), bytes
// before the first header are skipped; a sequence line starting with '+' (kseq would read FASTQ
// quality lines there) is refused with an error.  FASTQ -- four-line records ('@' header, sequence,
// '+', quality) counted from the first '@' (blank lines before it are skipped).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <zlib.h>

#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include <fcntl.h>
#include <unistd.h>

#include "device_common.hpp"
#include "host_stage.hpp"

namespace mtg {

constexpr int FA_BLOCK = 256;
constexpr int FA_PER = 32;                      // bytes per thread
constexpr int FA_TILE = FA_BLOCK * FA_PER;      // bytes per tile

// one input file's bytes (decompressed) in pinned host memory
struct FastaInput {
    char *data = nullptr;
    uint64_t size = 0;
    bool fastq = false;
    uint64_t first_header = 0;  // FASTA: the first '>' at a line start; FASTQ: the first '@' (bytes
                                // before it are skipped)
    uint64_t lines_before = 0;  // FASTQ: newlines before first_header (the 4-line phase starts there)
    std::string path;
};

// read (and inflate) a file into pinned memory; throws with the reference's message style
inline FastaInput load_fasta_file(const std::string &path) {
    FastaInput in;
    in.path = path;
    uint64_t fsize = 0;
    bool gz = false;
    {
        const int fd = ::open(path.c_str(), O_RDONLY);
        if (fd < 0) throw std::runtime_error("ERROR: Cannot read from file " + path);
        const off_t end = ::lseek(fd, 0, SEEK_END);
        fsize = end > 0 ? (uint64_t)end : 0;
        unsigned char magic[2] = {0, 0};
        gz = fsize >= 2 && ::pread(fd, magic, 2, 0) == 2 && magic[0] == 0x1f && magic[1] == 0x8b;
        if (!gz) {
            // plain file: straight into a pinned block from the pool (steady-state builds pin
            // nothing new), large reads, no zlib copy
            char *buf = (char *)PinnedPool::get().take(fsize + 1);
            uint64_t size = 0;
            while (size < fsize) {
                const ssize_t got = ::pread(fd, buf + size, (size_t)std::min<uint64_t>(fsize - size, 1ull << 30), (off_t)size);
                if (got < 0) {
                    ::close(fd);
                    if (!PinnedPool::get().give(buf)) (void)hipHostFree(buf);
                    throw std::runtime_error("ERROR: Cannot read from file " + path);
                }
                if (got == 0) break;
                size += (uint64_t)got;
            }
            ::close(fd);
            in.data = buf;
            in.size = size;
        } else {
            ::close(fd);
        }
    }
    char *buf = in.data;
    uint64_t size = in.size;
    if (gz) {
    gzFile f = gzopen(path.c_str(), "rb");
    if (!f) throw std::runtime_error("ERROR: Cannot read from file " + path);
    gzbuffer(f, 1u << 20);
    uint64_t cap = std::max<uint64_t>(fsize + (1u << 16), 1u << 20);
    buf = nullptr;
    if (hipHostMalloc((void **)&buf, cap, hipHostMallocDefault) != hipSuccess) {
        gzclose(f);
        throw std::runtime_error("pinned host allocation failed for " + path);
    }
    size = 0;
    while (true) {
        if (size == cap) {  // compressed input: grow (x2) and keep what is read
            char *nb = nullptr;
            if (hipHostMalloc((void **)&nb, 2 * cap, hipHostMallocDefault) != hipSuccess) {
                (void)hipHostFree(buf);
                gzclose(f);
                throw std::runtime_error("pinned host allocation failed for " + path);
            }
            std::memcpy(nb, buf, size);
            (void)hipHostFree(buf);
            buf = nb;
            cap *= 2;
        }
        const unsigned want = (unsigned)std::min<uint64_t>(cap - size, 1u << 30);
        const int got = gzread(f, buf + size, want);
        if (got < 0) {
            (void)hipHostFree(buf);
            gzclose(f);
            throw std::runtime_error("ERROR: Cannot read from file " + path);
        }
        if (got == 0) break;
        size += (uint64_t)got;
    }
    gzclose(f);
    }
    in.data = buf;
    in.size = size;
    uint64_t i = 0;
    while (i < size && (buf[i] == '\n' || buf[i] == '\r' || buf[i] == ' ')) ++i;
    in.fastq = i < size && buf[i] == '@';
    if (in.fastq) {
        in.first_header = i;
        for (uint64_t p = 0; p < i; ++p) in.lines_before += buf[p] == '\n';
    } else {  // the first header: almost always byte 0, else a host scan
        uint64_t p = 0;
        while (p < size && !(buf[p] == '>' && (p == 0 || buf[p - 1] == '\n'))) {
            const void *nl = std::memchr(buf + p, '\n', size - p);
            p = nl ? (uint64_t)((const char *)nl - buf) + 1 : size;
        }
        in.first_header = p;
    }
    return in;
}

inline void free_fasta(FastaInput &in) {
    if (in.data && !PinnedPool::get().give(in.data)) (void)hipHostFree(in.data);
    in.data = nullptr;
}

// stats: tlast[t] = global index of the tile's last '\n' (-1: none); tnl[t] = its newline count
__global__ __launch_bounds__(FA_BLOCK) void fasta_stats_kernel(const uint8_t *__restrict__ raw, uint64_t n,
                                                               int64_t *__restrict__ tlast,
                                                               uint32_t *__restrict__ tnl) {
    __shared__ int64_t s_last[FA_BLOCK];
    __shared__ uint32_t s_scan[FA_BLOCK / 64 + 1];
    const uint64_t b0 = (uint64_t)blockIdx.x * FA_TILE + (uint64_t)threadIdx.x * FA_PER;
    int64_t last = -1;
    uint32_t cnt = 0;
    for (int j = 0; j < FA_PER; ++j) {
        const uint64_t i = b0 + j;
        if (i < n && raw[i] == '\n') {
            last = (int64_t)i;
            ++cnt;
        }
    }
    s_last[threadIdx.x] = last;
    uint32_t tot;
    block_exclusive_sum<FA_BLOCK>(cnt, s_scan, &tot);
    for (int s = FA_BLOCK / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) s_last[threadIdx.x] = max(s_last[threadIdx.x], s_last[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        tlast[blockIdx.x] = s_last[0];
        tnl[blockIdx.x] = tot;
    }
}

// exclusive prefix (max over tlast -> prev_nl, sum over u32 -> u64 offsets) by one workgroup
__global__ __launch_bounds__(1024) void fasta_prefix_kernel(const int64_t *__restrict__ tlast, const uint32_t *__restrict__ a,
                                                            const uint32_t *__restrict__ b, uint64_t nt,
                                                            int64_t *__restrict__ prev_nl, uint64_t *__restrict__ aoff,
                                                            uint64_t *__restrict__ boff) {
    __shared__ int64_t s_m[1024];
    __shared__ uint64_t s_a[1024], s_b[1024];
    __shared__ int64_t c_m;
    __shared__ uint64_t c_a, c_b;
    if (threadIdx.x == 0) {
        c_m = -1;
        c_a = 0;
        c_b = 0;
    }
    __syncthreads();
    for (uint64_t base = 0; base < nt; base += 1024) {
        const uint64_t i = base + threadIdx.x;
        s_m[threadIdx.x] = i < nt && tlast ? tlast[i] : -1;
        s_a[threadIdx.x] = i < nt && a ? a[i] : 0;
        s_b[threadIdx.x] = i < nt && b ? b[i] : 0;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {  // inclusive Hillis-Steele
            int64_t m = s_m[threadIdx.x];
            uint64_t x = s_a[threadIdx.x], y = s_b[threadIdx.x];
            if ((int)threadIdx.x >= off) {
                m = max(m, s_m[threadIdx.x - off]);
                x += s_a[threadIdx.x - off];
                y += s_b[threadIdx.x - off];
            }
            __syncthreads();
            s_m[threadIdx.x] = m;
            s_a[threadIdx.x] = x;
            s_b[threadIdx.x] = y;
            __syncthreads();
        }
        if (i < nt) {
            const int64_t em = threadIdx.x ? s_m[threadIdx.x - 1] : -1;
            const uint64_t ea = threadIdx.x ? s_a[threadIdx.x - 1] : 0, eb = threadIdx.x ? s_b[threadIdx.x - 1] : 0;
            if (prev_nl) prev_nl[i] = max(c_m, em);
            if (aoff) aoff[i] = c_a + ea;
            if (boff) boff[i] = c_b + eb;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            c_m = max(c_m, s_m[1023]);
            c_a += s_a[1023];
            c_b += s_b[1023];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (aoff) aoff[nt] = c_a;
        if (boff) boff[nt] = c_b;
    }
}

// a thread's FA_PER bytes as words (zero past n)
__device__ __forceinline__ void fa_load(const uint8_t *__restrict__ raw, uint64_t n, uint64_t b0, uint32_t (&w)[FA_PER / 4]) {
    if (b0 + FA_PER <= n) {
        const uint4 *p = reinterpret_cast<const uint4 *>(raw + b0);
#pragma unroll
        for (int q = 0; q < FA_PER / 16; ++q) {
            const uint4 v = p[q];
            w[4 * q] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < FA_PER / 4; ++q) {
            w[q] = 0;
            for (int bb = 0; bb < 4; ++bb)
                if (b0 + 4 * q + bb < n) w[q] |= (uint32_t)raw[b0 + 4 * q + bb] << (8 * bb);
        }
    }
}

/*
 * count (WRITE = false) and write passes over the same tiles.  Per byte: skipped before the first
 * header.  FASTA -- a header line writes '$' at its '>' / '@' (a record starts after it) and
 * nothing else; sequence lines write every byte but '\n' and a '\r' before '\n' (or at the end);
 * a sequence line starting with '+' raises *bad (count pass).  FASTQ -- line r = 1 (mod 4, counted
 * from the first '@' line) writes its bytes but a line-ending '\r', and '$' for its '\n'; the '\n'
 * of a header line (r = 0) starts a record.
 */
template <bool WRITE>
__global__ __launch_bounds__(FA_BLOCK) void fasta_split_kernel(
    const uint8_t *__restrict__ raw, uint64_t n, int fastq, uint64_t first_hdr, const int64_t *__restrict__ prev_nl,
    const uint64_t *__restrict__ nl_off, uint32_t *__restrict__ tkeep, uint32_t *__restrict__ tstart,
    const uint64_t *__restrict__ keep_off, const uint64_t *__restrict__ start_off, uint8_t *__restrict__ out,
    uint64_t out_base, uint64_t *__restrict__ rstarts, uint32_t *__restrict__ rcounts, uint64_t read_base,
    uint64_t line_base, uint32_t *__restrict__ bad) {
    constexpr int NW = FA_PER / 4;
    __shared__ int64_t s_last[FA_BLOCK];
    __shared__ uint32_t s_scan[FA_BLOCK / 64 + 1];
    __shared__ uint8_t s_out[WRITE ? FA_TILE : 1];
    const uint32_t tid = threadIdx.x;
    const uint64_t t = blockIdx.x;
    const uint64_t b0 = t * FA_TILE + (uint64_t)tid * FA_PER;
    uint32_t w[NW];
    fa_load(raw, n, b0, w);
    auto byte = [&](int j) -> uint32_t { return (w[j >> 2] >> (8 * (j & 3))) & 0xFFu; };
    int64_t last = -1;
    uint32_t nls = 0;
#pragma unroll
    for (int j = 0; j < FA_PER; ++j) {
        if (b0 + j < n && byte(j) == '\n') {
            last = (int64_t)(b0 + j);
            ++nls;
        }
    }
    // the last newline before this thread's bytes: prefix max over the tile's threads
    s_last[tid] = last;
    __syncthreads();
    for (int off = 1; off < FA_BLOCK; off <<= 1) {
        const int64_t v = tid >= (uint32_t)off ? s_last[tid - off] : -1;
        __syncthreads();
        s_last[tid] = max(s_last[tid], v);
        __syncthreads();
    }
    int64_t cur = max(prev_nl[t], tid ? s_last[tid - 1] : (int64_t)-1);
    uint32_t tot;
    const uint32_t nl_before = block_exclusive_sum<FA_BLOCK>(nls, s_scan, &tot);
    uint64_t line = fastq ? nl_off[t] + nl_before : 0;
    auto is_hdr = [](uint32_t ch) { return ch == '>' || ch == '@'; };
    bool hdr = !fastq && (uint64_t)(cur + 1) < n && is_hdr(raw[cur + 1]);  // the current line's kind
    bool plus = false;
    uint32_t ev[NW];
    uint32_t keep = 0, starts = 0, stmask = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) ev[q] = 0;
#pragma unroll
    for (int j = 0; j < FA_PER; ++j) {
        const uint64_t i = b0 + j;
        if (i >= n) break;
        const uint32_t ch = byte(j);
        uint32_t e = 0;
        bool st = false;
        // a '\r' that ends its line is dropped with the '\n'; any other '\r' is a sequence byte
        const bool cr_end = ch == '\r' && (j + 1 < FA_PER ? byte(j + 1) : (i + 1 < n ? (uint32_t)raw[i + 1] : (uint32_t)'\n')) == '\n';
        if (i < first_hdr) {
        } else if (fastq) {
            const uint64_t r = (line - line_base) & 3;
            if (r == 1) e = ch == '\n' ? (uint32_t)'$' : (cr_end ? 0u : ch);
            else if (r == 0 && ch == '\n') st = true;
        } else {
            if (hdr) {
                if (i == (uint64_t)(cur + 1)) {
                    e = '$';
                    st = true;
                }
            } else {
                if (ch == '+' && i == (uint64_t)(cur + 1)) plus = true;
                if (ch != '\n' && !cr_end) e = ch;
            }
        }
        ev[j >> 2] |= e << (8 * (j & 3));
        keep += e != 0;
        starts += st;
        stmask |= (uint32_t)st << j;
        if (ch == '\n') {
            cur = (int64_t)i;
            ++line;
            if (!fastq) hdr = i + 1 < n && is_hdr(j + 1 < FA_PER ? byte(j + 1) : (uint32_t)raw[i + 1]);
        }
    }
    uint32_t ktot, stot;
    const uint32_t koff = block_exclusive_sum<FA_BLOCK>(keep, s_scan, &ktot);
    const uint32_t soff = block_exclusive_sum<FA_BLOCK>(starts, s_scan, &stot);
    if constexpr (!WRITE) {
        if (plus && bad) atomicOr(bad, 1u);
        if (tid == 0) {
            tkeep[t] = ktot;
            tstart[t] = stot;
        }
    } else {
        const uint64_t ob = out_base + keep_off[t];
        uint32_t o = koff;
        uint64_t r = read_base + start_off[t] + soff;
#pragma unroll
        for (int j = 0; j < FA_PER; ++j) {
            const uint32_t e = (ev[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            if ((stmask >> j) & 1u) {
                if (rstarts) {
                    rstarts[r] = ob + o + (e ? 1 : 0);  // FASTA: after its '$'; FASTQ: the next kept byte
                    rcounts[r] = 1;
                }
                ++r;
            }
            if (e) s_out[o++] = (uint8_t)e;
        }
        __syncthreads();
        for (uint32_t q = tid; q < ktot; q += FA_BLOCK) out[ob + q] = s_out[q];
    }
}

}  // namespace mtg
