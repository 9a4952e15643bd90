// host_stage.hpp -- host side of the drop-in boundary: the staged reads of one constructor and the
// pinned buffers the finished chunk is returned in.
//
// The reference's constructor takes reads through add_sequences from many OpenMP threads at once
// (cli/build.cpp:31-56 -> KmerCollector::add_sequences, kmer_collector.cpp:194-226, which enqueues
// the batch on a thread pool under a mutex).  Here a batch reserves its byte range under a short
// exclusive lock and is copied in under a shared lock, so concurrent adders copy in parallel and
// only a buffer growth serialises them.  The buffer is pinned host memory, so the build's single
// host-to-device copy of the reads runs at PCIe/xGMI DMA speed instead of through a bounce buffer.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
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

// Pinned host blocks, recycled: a returned block is kept for the next request of at most its size
// (a steady stream of builds allocates no pinned memory; pinning is the slow part of a hipHostMalloc).
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
                free_.erase(it);
                return p;
            }
        }
        void *p = nullptr;
        if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess || !p)
            throw std::runtime_error("pinned host allocation of " + std::to_string(bytes) + " bytes failed");
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
        free_.emplace(it->second, p);
        while (free_.size() > kKeep) {  // drop the smallest spare block
            auto f = free_.begin();
            size_.erase(f->second);
            (void)hipHostFree(f->second);
            free_.erase(f);
        }
        return true;
    }

  private:
    static constexpr size_t kKeep = 8;
    std::mutex mu_;
    std::multimap<size_t, void *> free_;
    std::unordered_map<void *, size_t> size_;
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

// The reads of one constructor, back to back in pinned memory, each followed by a '$' separator
// (no k-mer window spans two reads), with the start offset and count of every read.
class HostStage {
  public:
    ~HostStage() {
        if (data_) (void)hipHostFree(data_);
    }

    // n reads: read i is `lens[i]` bytes at ptrs[i]; counts may be null (all 1).
    // Per-read counts are kept as (start, count) runs: consecutive reads of one count share a run
    // (windows never span a separator, so a run maps each of its windows to the right count), and
    // a batch without counts is one run -- no per-read bookkeeping on the common path.
    void add(const char *const *ptrs, const uint64_t *lens, const uint64_t *counts, size_t n, unsigned threads) {
        add_reads(n, [&](size_t i) { return ptrs[i]; }, [&](size_t i) { return lens[i]; }, counts, threads);
    }
    // n reads back to back in `data`, read i = [offsets[i], offsets[i + 1])
    void add_packed(const char *data, const uint64_t *offsets, const uint64_t *counts, size_t n, unsigned threads) {
        add_reads(n, [&](size_t i) { return data + offsets[i]; },
                  [&](size_t i) { return offsets[i + 1] - offsets[i]; }, counts, threads);
    }

    template <typename Ptr, typename Len>
    void add_reads(size_t n, Ptr ptr, Len len, const uint64_t *counts, unsigned threads) {
        if (!n) return;
        // the batch's byte offsets: per-chunk sums in parallel, then each chunk copies from its base
        const unsigned t = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(std::max(1u, threads), n / 4096));
        std::vector<uint64_t> cbase(t + 1, 0);
        parallel_ranges(t, t, 1, [&](uint64_t c0, uint64_t c1) {
            for (uint64_t c = c0; c < c1; ++c) {
                uint64_t sum = 0;
                for (uint64_t i = n * c / t; i < n * (c + 1) / t; ++i) sum += len(i) + 1;
                cbase[c + 1] = sum;
            }
        });
        for (unsigned c = 0; c < t; ++c) cbase[c + 1] += cbase[c];
        const uint64_t total = cbase[t];
        uint64_t off;
        {
            std::unique_lock<std::shared_mutex> ex(grow_);
            if (size_ + total > cap_) grow(std::max<uint64_t>(size_ + total, cap_ + cap_ / 2));
            off = size_;
            size_ += total;
            uint64_t pos = off;
            for (size_t i = 0; i < n; ++i) {
                const uint64_t cnt = counts ? counts[i] : 1;
                const uint32_t c32 = cnt > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)cnt;
                if (counts_.empty() || counts_.back() != c32 || run_end_ != pos) {
                    starts_.push_back(pos);
                    counts_.push_back(c32);
                }
                any_count_not_one_ |= c32 != 1;
                if (!counts) {  // the whole batch is one run of count 1
                    pos = off + total;
                    break;
                }
                pos += len(i) + 1;
            }
            run_end_ = pos;
        }
        std::shared_lock<std::shared_mutex> sh(grow_);  // a growth waits for the copy
        char *dst = data_ + off;
        parallel_ranges(t, t, 1, [&](uint64_t c0, uint64_t c1) {
            for (uint64_t c = c0; c < c1; ++c) {
                uint64_t o = cbase[c];
                for (uint64_t i = n * c / t; i < n * (c + 1) / t; ++i) {
                    const uint64_t l = len(i);
                    std::memcpy(dst + o, ptr(i), l);
                    dst[o + l] = '$';
                    o += l + 1;
                }
            }
        });
    }

    const char *data() const { return data_; }
    uint64_t size() const { return size_; }
    uint64_t n_reads() const { return starts_.size(); }  // count runs (see add)
    const std::vector<uint64_t> &starts() const { return starts_; }
    const std::vector<uint32_t> &counts() const { return counts_; }
    bool any_count_not_one() const { return any_count_not_one_; }
    // the build consumed the staged reads (the pinned buffer is kept for the next batch)
    void clear() {
        std::unique_lock<std::shared_mutex> ex(grow_);
        size_ = 0;
        run_end_ = ~0ull;
        starts_.clear();
        counts_.clear();
        any_count_not_one_ = false;
    }
    std::shared_mutex &lock() { return grow_; }

  private:
    void grow(uint64_t want) {
        want = std::max<uint64_t>(want, 1u << 20);
        char *p = nullptr;
        if (hipHostMalloc((void **)&p, want, hipHostMallocDefault) != hipSuccess || !p)
            throw std::runtime_error("pinned host allocation of " + std::to_string(want) + " bytes failed");
        if (size_) std::memcpy(p, data_, size_);
        if (data_) (void)hipHostFree(data_);
        data_ = p;
        cap_ = want;
    }

    std::shared_mutex grow_;
    char *data_ = nullptr;
    uint64_t size_ = 0, cap_ = 0;
    std::vector<uint64_t> starts_;
    std::vector<uint32_t> counts_;
    uint64_t run_end_ = ~0ull;  // byte offset where the last run ends (a new batch may extend it)
    bool any_count_not_one_ = false;
};

}  // namespace mtg
