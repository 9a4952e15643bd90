// host_stage.hpp -- host side of the drop-in boundary: the staged reads of one constructor and the
// pinned buffers the finished chunk is returned in.
//
// The reference's constructor takes reads through add_sequences from many OpenMP threads at once
// (cli/build.cpp:31-56 -> KmerCollector::add_sequences, kmer_collector.cpp:194-226, which enqueues
// the batch on a thread pool under a mutex).  Here a batch reserves its byte range under a short
// exclusive lock and is copied in under a shared lock, so concurrent adders copy in parallel and
// only a buffer growth serialises them.  The buffer is pinned host memory, and every adder thread
// hands each 32 MiB piece it has copied to a copy stream that DMAs it into a device mirror of the
// buffer, so the reads' host-to-device copy runs while later reads are still being staged (the
// build then only waits for the last pieces).
#pragma once

#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace mtg {

// sets the calling thread's HIP device for a scope and restores the previous one
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(device);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Pinned host blocks, recycled: a returned block is kept for the next request of at most its size
// (a steady stream of builds allocates no pinned memory; pinning is the slow part of a hipHostMalloc).
// The spare blocks are bounded -- at most kKeep blocks and kKeepBytes in total; a returned block
// bigger than that is unpinned at once -- so one large build (tens of GB of W and weights) does not
// hold unswappable host memory after its chunk is freed; trim() drops every spare block.
class PinnedPool {
  public:
    static PinnedPool &get() {
        static PinnedPool p;
        return p;
    }
    void *take(size_t bytes) {
        bytes = std::max<size_t>(bytes, 64);
        {
            std::lock_guard<std::mutex> lk(mu_);
            auto it = free_.lower_bound(bytes);
            if (it != free_.end() && it->first <= 2 * bytes + (64u << 20)) {
                void *p = it->second;
                spare_ -= it->first;
                free_.erase(it);
                return p;
            }
        }
        void *p = nullptr;
        if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess || !p) {
            trim();  // spare blocks may be what exhausted the pinnable memory: retry once without them
            if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess || !p)
                throw std::runtime_error("pinned host allocation of " + std::to_string(bytes) + " bytes failed");
        }
        std::lock_guard<std::mutex> lk(mu_);
        size_[p] = bytes;
        return p;
    }
    // false: not a pool block (the caller frees it some other way)
    bool give(void *p) {
        if (!p) return true;
        std::lock_guard<std::mutex> lk(mu_);
        auto it = size_.find(p);
        if (it == size_.end()) return false;
        const size_t bytes = it->second;
        if (bytes > kKeepBytes) {  // never kept
            size_.erase(it);
            (void)hipHostFree(p);
            return true;
        }
        free_.emplace(bytes, p);
        spare_ += bytes;
        while (free_.size() > kKeep || spare_ > kKeepBytes) {  // drop the smallest spare block
            auto f = free_.begin();
            spare_ -= f->first;
            size_.erase(f->second);
            (void)hipHostFree(f->second);
            free_.erase(f);
        }
        return true;
    }
    // unpin every spare block
    void trim() {
        std::lock_guard<std::mutex> lk(mu_);
        for (auto &f : free_) {
            size_.erase(f.second);
            (void)hipHostFree(f.second);
        }
        free_.clear();
        spare_ = 0;
    }
    size_t spare_bytes() {
        std::lock_guard<std::mutex> lk(mu_);
        return spare_;
    }

  private:
    static constexpr size_t kKeep = 16;
    static constexpr size_t kKeepBytes = size_t(4) << 30;
    std::mutex mu_;
    std::multimap<size_t, void *> free_;
    std::unordered_map<void *, size_t> size_;
    size_t spare_ = 0;
};

// copy `n` items with `threads` host threads (ranges of items; `fn(i0, i1)`)
template <typename Fn>
static void parallel_ranges(uint64_t n, unsigned threads, uint64_t min_per_thread, Fn fn) {
    const uint64_t want = std::max<uint64_t>(1, n / std::max<uint64_t>(min_per_thread, 1));
    const unsigned t = (unsigned)std::min<uint64_t>(std::max(1u, threads), want);
    if (t <= 1) {
        fn(0, n);
        return;
    }
    std::vector<std::thread> pool;
    pool.reserve(t);
    for (unsigned j = 0; j < t; ++j) pool.emplace_back(fn, n * j / t, n * (j + 1) / t);
    for (auto &th : pool) th.join();
}

// 32 read bytes -> 2-bit codes (A/a 0, C/c 1, G/g 2, T/t/U/u 3; char j at bits 2j) and the valid
// mask (bit j: byte j is one of ACGTUacgtu).  Every other byte (N, separators, ...) breaks k-mer
// windows the same way in the extractor (encode_dna, drag_and_mark_segments), so the code and the
// mask carry everything the device needs.
static inline void pack32_scalar(const char *p, unsigned n, uint64_t *codes, uint32_t *valid) {
    uint64_t cw = 0;
    uint32_t vw = 0;
    for (unsigned j = 0; j < n; ++j) {
        const unsigned x = (unsigned char)p[j] | 0x20u;
        unsigned code = 4;
        switch (x) {
            case 'a': code = 0; break;
            case 'c': code = 1; break;
            case 'g': code = 2; break;
            case 't': case 'u': code = 3; break;
            default: break;
        }
        if (code < 4) {
            cw |= (uint64_t)code << (2 * j);
            vw |= 1u << j;
        }
    }
    *codes = cw;
    *valid = vw;
}

__attribute__((target("avx2"))) static inline void pack32_avx2(const char *p, uint64_t *codes, uint32_t *valid) {
    const __m256i v = _mm256_loadu_si256((const __m256i *)p);
    const __m256i x = _mm256_or_si256(v, _mm256_set1_epi8(0x20));
    const __m256i ok = _mm256_or_si256(
        _mm256_or_si256(_mm256_cmpeq_epi8(x, _mm256_set1_epi8('a')), _mm256_cmpeq_epi8(x, _mm256_set1_epi8('c'))),
        _mm256_or_si256(_mm256_or_si256(_mm256_cmpeq_epi8(x, _mm256_set1_epi8('g')),
                                        _mm256_cmpeq_epi8(x, _mm256_set1_epi8('t'))),
                        _mm256_cmpeq_epi8(x, _mm256_set1_epi8('u'))));
    // low nibble: a 1, c 3, g 7, t 4, u 5 -> code
    const __m256i lut = _mm256_setr_epi8(0, 0, 0, 1, 3, 3, 0, 2, 0, 0, 0, 0, 0, 0, 0, 0,
                                         0, 0, 0, 1, 3, 3, 0, 2, 0, 0, 0, 0, 0, 0, 0, 0);
    __m256i c = _mm256_shuffle_epi8(lut, _mm256_and_si256(x, _mm256_set1_epi8(0x0F)));
    c = _mm256_and_si256(c, ok);
    // 4 codes -> one byte per dword: b0 + 4 b1 (16-bit), then + 16 (b2 + 4 b3) (32-bit)
    const __m256i w16 = _mm256_maddubs_epi16(c, _mm256_set1_epi16(0x0401));
    const __m256i w32 = _mm256_madd_epi16(w16, _mm256_set1_epi32(0x00100001));
    const __m256i by = _mm256_shuffle_epi8(w32, _mm256_setr_epi8(0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
                                                                  -1, -1, 0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1,
                                                                  -1, -1, -1, -1));
    const uint64_t lo = (uint32_t)_mm256_extract_epi32(by, 0), hi = (uint32_t)_mm256_extract_epi32(by, 4);
    *codes = lo | (hi << 32);
    *valid = (uint32_t)_mm256_movemask_epi8(ok);
}

// The reads of one constructor in pinned memory as 2-bit codes + a valid mask (3 bits per char
// instead of a byte: the host-to-device copy moves 0.375 B per char), each read followed by an
// invalid char (no k-mer window spans two reads), with the start offset and count of every read.
// Every adder thread packs a contiguous chunk that starts on a 32-char word, so threads never
// share a word; the gaps left by that alignment are invalid chars.  The device unpacks the
// buffer to one byte per char (unpack_reads_kernel) before the extractor reads it.
class HostStage {
  public:
    ~HostStage() {
        if (stream_) {
            DeviceGuard g(device_);
            (void)hipStreamSynchronize(stream_);
            (void)hipStreamDestroy(stream_);
        }
        if (dcodes_) (void)hipFree(dcodes_);
        if (codes_) (void)hipHostFree(codes_);
        if (valid_) (void)hipHostFree(valid_);
    }

    // copy staged pieces to a device mirror on `device` as they are written (see the header)
    void enable_mirror(int device) {
        device_ = device;
        mirror_ = true;
    }

    // n reads: read i is `lens[i]` bytes at ptrs[i]; counts may be null (all 1).
    // Per-read counts are kept as (start, count) runs: consecutive reads of one count share a run
    // (windows never span an invalid char, so a run maps each of its windows to the right count),
    // and a batch without counts is one run -- no per-read bookkeeping on the common path.
    void add(const char *const *ptrs, const uint64_t *lens, const uint64_t *counts, size_t n, unsigned threads) {
        add_reads(n, [&](size_t i) { return ptrs[i]; }, [&](size_t i) { return lens[i]; }, counts, threads, nullptr);
    }
    // n reads back to back in `data`, read i = [offsets[i], offsets[i + 1])
    void add_packed(const char *data, const uint64_t *offsets, const uint64_t *counts, size_t n, unsigned threads) {
        // reads back to back: a read's last partial block may load bytes of the next read (masked
        // off), up to the end of the last read
        add_reads(n, [&](size_t i) { return data + offsets[i]; },
                  [&](size_t i) { return offsets[i + 1] - offsets[i]; }, counts, threads, data + offsets[n]);
    }

    template <typename Ptr, typename Len>
    void add_reads(size_t n, Ptr ptr, Len len, const uint64_t *counts, unsigned threads, const char *load_end) {
        if (!n) return;
        // chunk c packs reads [n c / t, n (c + 1) / t) from char cbase[c] (a multiple of 32)
        const unsigned t = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(std::max(1u, threads), n / 4096));
        std::vector<uint64_t> cbase(t + 1, 0);
        parallel_ranges(t, t, 1, [&](uint64_t c0, uint64_t c1) {
            for (uint64_t c = c0; c < c1; ++c) {
                uint64_t sum = 0;
                for (uint64_t i = n * c / t; i < n * (c + 1) / t; ++i) sum += len(i) + 1;
                cbase[c + 1] = (sum + 31) & ~31ull;
            }
        });
        for (unsigned c = 0; c < t; ++c) cbase[c + 1] += cbase[c];
        const uint64_t total = cbase[t];
        uint64_t off;
        {
            std::unique_lock<std::shared_mutex> ex(grow_);
            if (size_ + total > cap_) grow(std::max<uint64_t>(size_ + total, cap_ + cap_ / 2));
            if (mirror_ && !mirror_ready()) {
                try {
                    grow_mirror();
                } catch (const std::exception &) {
                    mirror_ = false;  // no device memory for a mirror: the build copies the reads itself
                }
            }
            off = size_;
            size_ += total;
            if (!counts) {  // the whole batch is one run of count 1
                if (counts_.empty() || counts_.back() != 1u || run_end_ != off) {
                    starts_.push_back(off);
                    counts_.push_back(1u);
                }
                run_end_ = off + total;
            } else {
                for (unsigned c = 0; c < t; ++c) {
                    uint64_t pos = off + cbase[c];
                    for (uint64_t i = n * c / t; i < n * (c + 1) / t; ++i) {
                        const uint64_t cnt = counts[i];
                        const uint32_t c32 = cnt > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)cnt;
                        if (counts_.empty() || counts_.back() != c32 || run_end_ != pos) {
                            starts_.push_back(pos);
                            counts_.push_back(c32);
                        }
                        any_count_not_one_ |= c32 != 1;
                        pos += len(i) + 1;
                        run_end_ = pos;
                    }
                }
                run_end_ = off + total;  // the alignment gap of the last chunk joins the last run
            }
        }
        std::shared_lock<std::shared_mutex> sh(grow_);  // a growth waits for the packing
        const bool mirror = mirror_ready();
        const bool avx2 = __builtin_cpu_supports("avx2");
        parallel_ranges(t, t, 1, [&](uint64_t c0, uint64_t c1) {
            std::unique_ptr<DeviceGuard> g;
            if (mirror) g.reset(new DeviceGuard(device_));
            for (uint64_t c = c0; c < c1; ++c) {
                const uint64_t w0 = (off + cbase[c]) / 32, w1 = (off + cbase[c + 1]) / 32;
                uint64_t w = w0, piece = w0;
                uint64_t cw = 0;
                uint32_t vw = 0;
                unsigned o = 0;  // chars in the current word
                auto put = [&](uint64_t codes, uint32_t valid, unsigned nc) {  // nc <= 32 chars
                    cw |= codes << (2 * o);
                    vw |= valid << o;
                    if (o + nc >= 32) {
                        codes_[w] = cw;
                        valid_[w] = vw;
                        ++w;
                        cw = o ? codes >> (64 - 2 * o) : 0;
                        vw = o ? valid >> (32 - o) : 0;
                        o = o + nc - 32;
                    } else {
                        o += nc;
                    }
                };
                for (uint64_t i = n * c / t; i < n * (c + 1) / t; ++i) {
                    const char *p = ptr(i);
                    const uint64_t l = len(i);
                    uint64_t j = 0;
                    uint64_t codes;
                    uint32_t valid;
                    if (avx2) {
                        for (; j + 32 <= l; j += 32) {
                            pack32_avx2(p + j, &codes, &valid);
                            put(codes, valid, 32);
                        }
                        if (j < l && load_end && p + j + 32 <= load_end) {
                            // the tail straight from the buffer, masked, with the separator (an invalid
                            // char) in the same put: 3.3-4.3 -> 5.0-5.3 GB/s per thread on 150-char reads
                            const unsigned m = (unsigned)(l - j);
                            pack32_avx2(p + j, &codes, &valid);
                            put(codes & ((1ull << (2 * m)) - 1), valid & ((1u << m) - 1), m + 1);
                            goto next_read;
                        }
                        if (j < l) {  // the tail through a zero-padded copy (zero bytes are invalid)
                            const unsigned m = (unsigned)(l - j);
                            alignas(32) char tail[32] = {};
                            std::memcpy(tail, p + j, m);
                            pack32_avx2(tail, &codes, &valid);
                            put(codes & (m == 32 ? ~0ull : ((1ull << (2 * m)) - 1)), valid, m);
                            j = l;
                        }
                    }
                    for (; j < l; j += 32) {
                        const unsigned m = (unsigned)std::min<uint64_t>(32, l - j);
                        pack32_scalar(p + j, m, &codes, &valid);
                        put(codes, valid, m);
                    }
                    put(0, 0, 1);  // the separator
                next_read:
                    if (mirror && w - piece >= kPieceWords) {
                        send(piece, w - piece);
                        piece = w;
                    }
                }
                if (o) {  // the alignment gap: invalid chars
                    codes_[w] = cw;
                    valid_[w] = vw;
                    ++w;
                }
                if (mirror && w1 > piece) send(piece, w1 - piece);
            }
        });
    }

    uint64_t size() const { return size_; }              // chars (a multiple of 32)
    const uint64_t *codes() const { return codes_; }     // size() / 32 words
    const uint32_t *valid() const { return valid_; }     // size() / 32 words
    uint64_t n_reads() const { return starts_.size(); }  // count runs (see add)
    const std::vector<uint64_t> &starts() const { return starts_; }
    const std::vector<uint32_t> &counts() const { return counts_; }
    bool any_count_not_one() const { return any_count_not_one_; }

    // the device mirror holds (or has in flight) every staged word
    bool mirror_ready() const { return mirror_ && dcodes_ && dcap_ >= cap_; }
    // wait for the mirror's copies; the device copies of codes() and valid() (false: no mirror)
    bool mirror_wait(const uint64_t **dcodes, const uint32_t **dvalid) {
        if (!mirror_ready() || mirror_failed_) return false;
        DeviceGuard g(device_);
        if (hipStreamSynchronize(stream_) != hipSuccess || mirror_failed_) return false;
        *dcodes = dcodes_;
        *dvalid = dvalid_;
        return true;
    }
    // the build consumed the staged reads (the pinned buffers are kept for the next batch)
    void clear() {
        std::unique_lock<std::shared_mutex> ex(grow_);
        clear_locked();
    }
    // the same with grow_ already held exclusively by the caller (the build): no add can slip in
    // between the end of the build and the clear
    void clear_locked() {
        if (stream_) {
            DeviceGuard g(device_);
            (void)hipStreamSynchronize(stream_);
        }
        mirror_failed_ = false;
        size_ = 0;
        run_end_ = ~0ull;
        starts_.clear();
        counts_.clear();
        any_count_not_one_ = false;
    }
    std::shared_mutex &lock() { return grow_; }

  private:
    static constexpr uint64_t kPieceWords = 1ull << 20;  // 32 Mi chars (12 MiB) per mirror copy

    void send(uint64_t w0, uint64_t nw) {
        if (hipMemcpyAsync(dcodes_ + w0, codes_ + w0, nw * 8, hipMemcpyHostToDevice, stream_) != hipSuccess ||
            hipMemcpyAsync(dvalid_ + w0, valid_ + w0, nw * 4, hipMemcpyHostToDevice, stream_) != hipSuccess)
            mirror_failed_ = true;  // the build falls back to its own copy
    }

    // device mirror of the host capacity (under the exclusive lock); keeps the words staged so far
    void grow_mirror() {
        DeviceGuard g(device_);
        if (!stream_ && hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess)
            throw std::runtime_error("copy stream");
        const uint64_t nw = cap_ / 32;
        uint64_t *p = nullptr;
        if (hipMalloc((void **)&p, nw * 12 + 64) != hipSuccess) throw std::runtime_error("mirror allocation");
        uint32_t *pv = (uint32_t *)(p + nw);
        const uint64_t sw = size_ / 32;
        bool ok = hipStreamSynchronize(stream_) == hipSuccess;
        if (ok && sw) {
            if (dcodes_)
                ok = hipMemcpyAsync(p, dcodes_, sw * 8, hipMemcpyDeviceToDevice, stream_) == hipSuccess &&
                     hipMemcpyAsync(pv, dvalid_, sw * 4, hipMemcpyDeviceToDevice, stream_) == hipSuccess;
            else  // staged before the mirror existed
                ok = hipMemcpyAsync(p, codes_, sw * 8, hipMemcpyHostToDevice, stream_) == hipSuccess &&
                     hipMemcpyAsync(pv, valid_, sw * 4, hipMemcpyHostToDevice, stream_) == hipSuccess;
        }
        ok = ok && hipStreamSynchronize(stream_) == hipSuccess;
        if (!ok) {
            (void)hipFree(p);
            throw std::runtime_error("mirror copy");
        }
        if (dcodes_) (void)hipFree(dcodes_);
        dcodes_ = p;
        dvalid_ = pv;
        dcap_ = cap_;
    }

    void grow(uint64_t want) {
        want = (std::max<uint64_t>(want, 1u << 20) + 31) & ~31ull;
        if (stream_) {  // in-flight mirror copies read the old buffers
            DeviceGuard g(device_);
            (void)hipStreamSynchronize(stream_);
        }
        uint64_t *pc = nullptr;
        uint32_t *pv = nullptr;
        if (hipHostMalloc((void **)&pc, want / 4, hipHostMallocDefault) != hipSuccess || !pc ||
            hipHostMalloc((void **)&pv, want / 8, hipHostMallocDefault) != hipSuccess || !pv) {
            if (pc) (void)hipHostFree(pc);
            throw std::runtime_error("pinned host allocation of " + std::to_string(want * 3 / 8) + " bytes failed");
        }
        if (size_) {
            std::memcpy(pc, codes_, size_ / 4);
            std::memcpy(pv, valid_, size_ / 8);
        }
        if (codes_) (void)hipHostFree(codes_);
        if (valid_) (void)hipHostFree(valid_);
        codes_ = pc;
        valid_ = pv;
        cap_ = want;
    }

    std::shared_mutex grow_;
    int device_ = 0;
    bool mirror_ = false;
    std::atomic<bool> mirror_failed_{false};
    hipStream_t stream_ = nullptr;
    uint64_t *dcodes_ = nullptr;
    uint32_t *dvalid_ = nullptr;
    uint64_t dcap_ = 0;
    uint64_t *codes_ = nullptr;
    uint32_t *valid_ = nullptr;
    uint64_t size_ = 0, cap_ = 0;  // chars
    std::vector<uint64_t> starts_;
    std::vector<uint32_t> counts_;
    uint64_t run_end_ = ~0ull;  // char offset where the last run ends (a new batch may extend it)
    bool any_count_not_one_ = false;
};

}  // namespace mtg
