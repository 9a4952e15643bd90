// kmc.hpp -- KMC1 k-mer counter databases as build input (BASELINE config 5, `metagraph build`
// on a `.kmc_suf` / `.kmc_pre` pair).
//
// The reference reads them through the KMC API (seq_io/kmc_parser.cpp:27-62, CKMCFile in the
// KMC submodule, absent here) and hands every k-mer to the constructor as a one-k-mer sequence
// with its count (cli/parse_sequences.hpp:50-101), plus its reverse complement when the database
// counted canonical k-mers and the graph is not canonical.  Here the host only reads the two
// files; the records are decoded on the device, straight into the read buffer of the build
// (k bases + '$' per record, per-read counts), so the rest of the path is the FASTA path.
//
// KMC1 layout (decoded from the reference's fixtures, tests/data/transcripts_1000_kmc_counters*):
//   .kmc_pre  "KMCP" | u64 lut[4^lut_len] (first record of every prefix) | header | u32 header
//             size | "KMCP";  header = u32 k, mode, counter_size, lut_len, min_count, max_count,
//             u64 total, u32 flags (bit 0 = single strand: both_strands = !(flags & 1)), ...
//   .kmc_suf  "KMCS" | total records of (k - lut_len) / 4 suffix bytes (2-bit A,C,G,T, first base
//             in the high bits) + counter_size little-endian count bytes | "KMCS"
// A record's k-mer is its prefix (lut_len bases, the index into lut) followed by its suffix.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <functional>
#include <vector>

#include <fcntl.h>
#include <unistd.h>

#include "host_stage.hpp"

namespace mtg {

// a whole file in a pinned block of the pool (PinnedPool), so its host-to-device copy runs at DMA
// speed; returned to the pool when the owner goes away
struct PinnedFile {
    uint8_t *data = nullptr;
    uint64_t size = 0;
    PinnedFile() = default;
    PinnedFile(const PinnedFile &) = delete;
    PinnedFile &operator=(const PinnedFile &) = delete;
    PinnedFile(PinnedFile &&o) noexcept : data(o.data), size(o.size) { o.data = nullptr, o.size = 0; }
    PinnedFile &operator=(PinnedFile &&o) noexcept {
        if (this != &o) {
            release();
            data = o.data, size = o.size;
            o.data = nullptr, o.size = 0;
        }
        return *this;
    }
    ~PinnedFile() { release(); }
    void release() {
        if (data && !PinnedPool::get().give(data)) (void)hipHostFree(data);
        data = nullptr;
        size = 0;
    }
};

struct KmcInput {
    unsigned k = 0, lut_len = 0, counter_size = 0;
    uint32_t min_count = 0, max_count = 0;  // effective inclusive bounds
    bool both = false;                     // also emit the reverse complement
    uint64_t total = 0;
    uint64_t nlut = 0;                     // prefix-table entries (4^lut_len)
    PinnedFile pre, suf;                   // the two files as read
    const uint8_t *dpre = nullptr, *dsuf = nullptr;  // their device mirrors (DeviceMirror) or null
    const uint8_t *lut_bytes() const { return pre.data + 4; }  // u64 lut[nlut] after "KMCP"
    const uint8_t *records() const { return suf.data + 4; }    // after "KMCS"
    uint64_t record_bytes() const { return suf.size >= 8 ? suf.size - 8 : 0; }
};

static std::string kmc_strip(const std::string &p) {
    for (const char *suf : {".kmc_suf", ".kmc_pre"}) {
        const size_t n = strlen(suf);
        if (p.size() >= n && p.compare(p.size() - n, n, suf) == 0) return p.substr(0, p.size() - n);
    }
    return p;
}

// optional device copy of a file made while it is read: file byte j lands at device byte j + 4 (so
// the 8-byte prefix table after the 4-byte "KMCP" marker is 8-byte aligned), piece by piece on
// `stream` as each piece is read, so the host-to-device copy runs under the reading
struct DeviceMirror {
    std::function<uint8_t *(uint64_t bytes)> alloc;  // device buffer of `bytes` (file size + 8)
    hipStream_t stream = nullptr;
    int device = 0;
    uint8_t *out = nullptr;                           // the buffer, once read
};

// a file into a pinned pool block: large preads from several threads at once (a single reader
// copies out of the page cache at ~3.5 GB/s: 316 of the 561 ms of configs[4]'s file route went
// to reading the 1.1 GB suffix file into pageable memory, and its host-to-device copy then ran
// from pageable memory too)
static PinnedFile read_file_pinned(const std::string &path, unsigned threads, DeviceMirror *dm = nullptr) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("cannot open " + path);
    const off_t end = ::lseek(fd, 0, SEEK_END);
    PinnedFile f;
    const uint64_t n = end > 0 ? (uint64_t)end : 0;
    try {
        f.data = (uint8_t *)PinnedPool::get().take(n + 1);
    } catch (...) {
        ::close(fd);
        throw;
    }
    f.size = n;
    uint8_t *dst = nullptr;
    if (dm) {
        try {
            dst = dm->alloc(n + 8);
        } catch (...) {
            ::close(fd);
            throw;
        }
    }
    constexpr uint64_t PIECE = 64ull << 20;
    const unsigned nt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(threads, (n + PIECE - 1) / PIECE));
    std::atomic<uint64_t> next{0};
    std::atomic<bool> bad{false};
    auto work = [&]() {
        if (dst) (void)hipSetDevice(dm->device);
        while (!bad) {
            const uint64_t p0 = next.fetch_add(PIECE);
            if (p0 >= n) return;
            const uint64_t p1 = std::min(n, p0 + PIECE);
            for (uint64_t p = p0; p < p1;) {
                const ssize_t got = ::pread(fd, f.data + p, (size_t)(p1 - p), (off_t)p);
                if (got <= 0) {
                    bad = true;
                    return;
                }
                p += (uint64_t)got;
            }
            if (dst && hipMemcpyAsync(dst + 4 + p0, f.data + p0, p1 - p0, hipMemcpyHostToDevice, dm->stream) != hipSuccess) {
                bad = true;
                return;
            }
        }
    };
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < nt; ++t) pool.emplace_back(work);
    work();
    for (auto &t : pool) t.join();
    ::close(fd);
    if (bad) throw std::runtime_error("cannot read " + path);
    if (dm) dm->out = dst;
    return f;
}

// seq_io::read_kmers (kmc_parser.cpp:27-62): min/max as the reference passes them (max
// exclusive), combined with the database's own cut-offs as CKMCFile::SetMin/MaxCount do
static KmcInput kmc_open(const std::string &path, uint64_t min_count, uint64_t max_count,
                         bool call_both_from_canonical, unsigned threads = 8, DeviceMirror *dpre = nullptr,
                         DeviceMirror *dsuf = nullptr) {
    const std::string base = kmc_strip(path);
    auto bad = [&](const char *why) {
        return std::runtime_error("Error: Can't open KMC database " + base + " (" + why + ")");
    };
    KmcInput in;
    try {
        in.pre = read_file_pinned(base + ".kmc_pre", threads, dpre);
        in.suf = read_file_pinned(base + ".kmc_suf", threads, dsuf);
    } catch (const std::exception &) {
        throw bad("missing file");
    }
    if (dpre && dsuf) {
        in.dpre = dpre->out;
        in.dsuf = dsuf->out;
    }
    const PinnedFile &pre = in.pre, &suf = in.suf;
    if (pre.size < 16 || memcmp(pre.data, "KMCP", 4) || memcmp(pre.data + pre.size - 4, "KMCP", 4))
        throw bad("no KMCP markers");
    if (suf.size < 8 || memcmp(suf.data, "KMCS", 4) || memcmp(suf.data + suf.size - 4, "KMCS", 4))
        throw bad("no KMCS markers");
    uint32_t hsize;
    memcpy(&hsize, pre.data + pre.size - 8, 4);
    if (hsize < 36 || (uint64_t)hsize + 12 > (uint64_t)pre.size) throw bad("header size");
    const uint8_t *h = pre.data + pre.size - 8 - hsize;
    uint32_t f[6];
    memcpy(f, h, 24);
    in.k = f[0];
    in.counter_size = f[2];
    in.lut_len = f[3];
    memcpy(&in.total, h + 24, 8);
    uint32_t flags;
    memcpy(&flags, h + 32, 4);
    uint32_t version = 0;
    if (hsize >= 64) memcpy(&version, h + hsize - 4, 4);
    if (version != 0) throw bad("only the KMC1 database layout is supported");
    if (f[1] != 0) throw bad("quality-value (mode 1) databases are not supported");
    if (in.k == 0 || in.k > 256 || in.lut_len > 16 || in.lut_len > in.k || (in.k - in.lut_len) % 4 ||
        in.counter_size > 4)
        throw bad("layout");
    const uint64_t nlut = 1ull << (2 * in.lut_len);
    if (4 + nlut * 8 + hsize + 8 > pre.size) throw bad("prefix table");
    in.nlut = nlut;
    const uint64_t rec = (in.k - in.lut_len) / 4 + in.counter_size;
    if (suf.size - 8 != in.total * rec) throw bad("record count");
    const bool both_strands = (flags & 1) == 0;
    in.both = call_both_from_canonical && both_strands;
    // SetMinCount / SetMaxCount only narrow the database's own [min, max]
    const uint64_t lo = std::max<uint64_t>(min_count, f[4]);
    const uint64_t hi = max_count ? std::min<uint64_t>(max_count - 1, f[5]) : 0;
    in.min_count = (uint32_t)std::min<uint64_t>(lo, 0xFFFFFFFFull);
    in.max_count = (uint32_t)std::min<uint64_t>(hi, 0xFFFFFFFFull);
    if (min_count >= max_count) in.total = 0;  // read_kmers returns without reading
    return in;
}

/*
 * One thread per record: its prefix (binary search of the prefix table), suffix and count;
 * writes the k-mer as k ASCII bases + '$' (and its reverse complement after it when `both`),
 * and the per-read start / count.  Records outside [min, max] become k 'N's: no k-mer.
 */
__global__ void kmc_decode_kernel(const uint8_t *__restrict__ rec, const uint64_t *__restrict__ lut,
                                  uint64_t nlut, uint64_t total, unsigned k, unsigned lut_len,
                                  unsigned counter_size, uint32_t min_count, uint32_t max_count,
                                  int both, uint8_t *__restrict__ seq, uint64_t seq_base,
                                  uint64_t *__restrict__ starts, uint32_t *__restrict__ counts,
                                  uint64_t read_base) {
    const unsigned slen = (k - lut_len) / 4, rsize = slen + counter_size;
    const uint64_t stride = (uint64_t)(k + 1) * (both ? 2 : 1);
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < total; r += gs) {
        uint64_t lo = 0, hi = nlut;  // last prefix whose first record is <= r
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if (lut[mid] <= r) lo = mid; else hi = mid;
        }
        const uint8_t *p = rec + r * rsize;
        uint32_t cnt = 0;
        for (unsigned b = 0; b < counter_size; ++b) cnt |= (uint32_t)p[slen + b] << (8 * b);
        const bool keep = cnt >= min_count && cnt <= max_count;
        uint8_t *o = seq + seq_base + r * stride;
        const char *acgt = "ACGT";
        for (unsigned i = 0; i < lut_len; ++i) o[i] = keep ? acgt[(lo >> (2 * (lut_len - 1 - i))) & 3] : 'N';
        for (unsigned i = 0; i < k - lut_len; ++i)
            o[lut_len + i] = keep ? acgt[(p[i >> 2] >> (6 - 2 * (i & 3))) & 3] : 'N';
        o[k] = '$';
        if (both) {
            uint8_t *q = o + k + 1;
            for (unsigned i = 0; i < k; ++i) {
                const uint8_t c = o[k - 1 - i];
                q[i] = c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : c == 'T' ? 'A' : 'N';
            }
            q[k] = '$';
        }
        if (starts) {
            const uint64_t rr = read_base + r * (both ? 2 : 1);
            starts[rr] = seq_base + r * stride;
            counts[rr] = cnt;
            if (both) {
                starts[rr + 1] = seq_base + r * stride + k + 1;
                counts[rr + 1] = cnt;
            }
        }
    }
}

// ------------------------------------------------------------------------ KMC1 writer
//
// The builder's own k-mer counter output, for the KMC input of BASELINE config 5 (`metagraph
// build` on a KMC database of k = 31 counts): the counted k-mers of device reads, sorted in KMC's
// record order and written in the layout above, so the reference's KMC branch (and kmc_open here)
// reads them back.  KMC's order is lexicographic with the first base most significant, and its
// canonical form is the lexicographically smaller of a k-mer and its reverse complement
// (tests/test_kmc.py pins both on the reference's fixtures).

// 2-bit chars of a 64-bit word in reverse order (char i <-> char 31 - i)
__device__ __forceinline__ uint64_t rev_chars64(uint64_t x) {
    x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
    return __builtin_bswap64(x);
}

// in place: the 2-bit BOSS key of a K-mer a_1..a_K (kmer_boss.hpp:58-72: a_K in the low two bits,
// a_i at bit 2i) -> its KMC word sum a_i << 2 (K - i); canonical: min(word, word of the rc).  With
// p = sum a_i << 2 (i - 1) (the plain co-lex word), word = rev_K(p) and the rc's word = ~p.
__global__ void kmc_key_kernel(uint64_t *__restrict__ keys, uint64_t n, unsigned K, int canonical) {
    const uint64_t mask = K >= 32 ? ~0ull : (1ull << (2 * K)) - 1;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        const uint64_t b = keys[i];
        const uint64_t plain = (b >> 2) | ((b & 3ull) << (2 * (K - 1)));
        const uint64_t w = rev_chars64(plain) >> (64 - 2 * K);
        const uint64_t rc = ~plain & mask;
        keys[i] = canonical && rc < w ? rc : w;
    }
}

// the files: `<base>.kmc_pre` (prefix table + the 64-byte header) and `<base>.kmc_suf` (records)
// from keys[0..n) sorted in KMC order with their counts (saturated at the counter's maximum)
static void kmc_write_files(const std::string &base, const uint64_t *keys, const uint32_t *counts, uint64_t n,
                            unsigned k, unsigned lut_len, unsigned counter_size, bool canonical, unsigned threads) {
    if (k == 0 || k > 32 || lut_len > k || (k - lut_len) % 4 || counter_size < 1 || counter_size > 4 || lut_len > 16)
        throw std::runtime_error("KMC writer: unsupported layout");
    const unsigned slen = (k - lut_len) / 4, rsize = slen + counter_size;
    const uint64_t nlut = 1ull << (2 * lut_len);
    const unsigned sbits = 2 * (k - lut_len);
    const uint64_t cmax = counter_size >= 4 ? 0xFFFFFFFFull : (1ull << (8 * counter_size)) - 1;
    threads = std::max(1u, threads);
    std::vector<uint8_t> rec(4 + n * rsize + 4);
    memcpy(rec.data(), "KMCS", 4);
    memcpy(rec.data() + rec.size() - 4, "KMCS", 4);
    std::vector<uint64_t> lut(nlut + 1, 0);
    // records in parallel; the prefix table from the (sorted) prefixes: lut[p] = first record of
    // prefix p = the number of records with a smaller prefix
    std::vector<std::thread> pool;
    const uint64_t per = (n + threads - 1) / threads;
    for (unsigned t = 0; t < threads; ++t)
        pool.emplace_back([&, t] {
            const uint64_t r0 = std::min(n, t * per), r1 = std::min(n, r0 + per);
            for (uint64_t r = r0; r < r1; ++r) {
                uint8_t *o = rec.data() + 4 + r * rsize;
                const uint64_t suf = sbits >= 64 ? keys[r] : keys[r] & ((1ull << sbits) - 1);
                for (unsigned i = 0; i < slen; ++i) o[i] = (uint8_t)(suf >> (sbits - 8 * (i + 1)));
                const uint64_t c = std::min<uint64_t>(counts ? counts[r] : 1, cmax);
                for (unsigned b = 0; b < counter_size; ++b) o[slen + b] = (uint8_t)(c >> (8 * b));
                // prefix boundaries: record r starts every prefix in (prefix(r - 1), prefix(r)]
                const uint64_t pr = sbits >= 64 ? 0 : keys[r] >> sbits;
                const uint64_t pp = r ? (sbits >= 64 ? 0 : keys[r - 1] >> sbits) + 1 : 0;
                for (uint64_t q = pp; q <= pr && q < nlut; ++q) lut[q] = r;
            }
        });
    for (auto &th : pool) th.join();
    const uint64_t plast = n ? (sbits >= 64 ? 0 : keys[n - 1] >> sbits) + 1 : 0;
    for (uint64_t q = plast; q < nlut; ++q) lut[q] = n;  // prefixes past the last record
    // header (the fixtures' 64-byte layout): k, mode 0, counter size, prefix length, min count 1,
    // max count 10^9 (KMC's default cut-offs for a -ci1 run), total, flags (bit 0: single strand),
    // padding, version 0
    uint8_t h[64] = {0};
    const uint32_t f[6] = {k, 0, counter_size, lut_len, 1, 1000000000u};
    memcpy(h, f, 24);
    memcpy(h + 24, &n, 8);
    const uint32_t flags = canonical ? 0u : 1u;
    memcpy(h + 32, &flags, 4);
    auto put = [&](const std::string &path, const std::vector<const void *> &parts, const std::vector<size_t> &sizes) {
        FILE *fp = fopen(path.c_str(), "wb");
        if (!fp) throw std::runtime_error("KMC writer: cannot create " + path);
        bool ok = true;
        for (size_t i = 0; i < parts.size(); ++i) ok = ok && fwrite(parts[i], 1, sizes[i], fp) == sizes[i];
        ok = (fclose(fp) == 0) && ok;
        if (!ok) throw std::runtime_error("KMC writer: short write to " + path);
    };
    const uint32_t hsize = 64;
    put(base + ".kmc_pre", {"KMCP", lut.data(), h, &hsize, "KMCP"}, {4, nlut * 8, 64, 4, 4});
    put(base + ".kmc_suf", {rec.data()}, {rec.size()});
}

}  // namespace mtg
