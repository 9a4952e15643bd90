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
        if (stream_) {
            DeviceGuard g(device_);
            (void)hipStreamSynchronize(stream_);
            (void)hipStreamDestroy(stream_);
        }
        if (dmirror_) (void)hipFree(dmirror_);
        if (data_) (void)hipHostFree(data_);
    }

    // copy staged pieces to a device mirror on `device` as they are written (see the header)
    void enable_mirror(int device) {
        device_ = device;
        mirror_ = true;
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
            if (mirror_ && !mirror_ready()) {
                try {
                    grow_mirror();
                } catch (const std::exception &) {
                    mirror_ = false;  // no device memory for a mirror: the build copies the reads itself
                }
            }
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
        const bool mirror = mirror_ready();
        parallel_ranges(t, t, 1, [&](uint64_t c0, uint64_t c1) {
            std::unique_ptr<DeviceGuard> g;
            if (mirror) g.reset(new DeviceGuard(device_));
            for (uint64_t c = c0; c < c1; ++c) {
                uint64_t o = cbase[c], piece = o;
                for (uint64_t i = n * c / t; i < n * (c + 1) / t; ++i) {
                    const uint64_t l = len(i);
                    std::memcpy(dst + o, ptr(i), l);
                    dst[o + l] = '$';
                    o += l + 1;
                    if (mirror && o - piece >= kPiece) {
                        send(off + piece, o - piece);
                        piece = o;
                    }
                }
                if (mirror && o > piece) send(off + piece, o - piece);
            }
        });
    }

    // the device mirror holds (or has in flight) every staged byte
    bool mirror_ready() const { return mirror_ && dmirror_ && dcap_ >= cap_; }
    // wait for the mirror's copies; returns the device copy of data() (null: no mirror)
    const uint8_t *mirror_wait() {
        if (!mirror_ready() || mirror_failed_) return nullptr;
        DeviceGuard g(device_);
        if (hipStreamSynchronize(stream_) != hipSuccess || mirror_failed_) return nullptr;
        return dmirror_;
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
    static constexpr uint64_t kPiece = 32ull << 20;

    void send(uint64_t at, uint64_t bytes) {
        if (hipMemcpyAsync(dmirror_ + at, data_ + at, bytes, hipMemcpyHostToDevice, stream_) != hipSuccess)
            mirror_failed_ = true;  // the build falls back to its own copy
    }

    // device mirror of the host capacity (under the exclusive lock); keeps the bytes staged so far
    void grow_mirror() {
        DeviceGuard g(device_);
        if (!stream_ && hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess)
            throw std::runtime_error("copy stream");
        uint8_t *p = nullptr;
        if (hipMalloc((void **)&p, cap_ + 64) != hipSuccess) throw std::runtime_error("mirror allocation");
        if (hipStreamSynchronize(stream_) != hipSuccess ||
            (size_ && dmirror_ && hipMemcpyAsync(p, dmirror_, size_, hipMemcpyDeviceToDevice, stream_) != hipSuccess) ||
            hipStreamSynchronize(stream_) != hipSuccess) {
            (void)hipFree(p);
            throw std::runtime_error("mirror copy");
        }
        if (size_ && !dmirror_) {  // staged before the mirror existed
            if (hipMemcpyAsync(p, data_, size_, hipMemcpyHostToDevice, stream_) != hipSuccess) mirror_failed_ = true;
        }
        if (dmirror_) (void)hipFree(dmirror_);
        dmirror_ = p;
        dcap_ = cap_;
    }

    void grow(uint64_t want) {
        want = std::max<uint64_t>(want, 1u << 20);
        if (stream_) {  // in-flight mirror copies read the old buffer
            DeviceGuard g(device_);
            (void)hipStreamSynchronize(stream_);
        }
        char *p = nullptr;
        if (hipHostMalloc((void **)&p, want, hipHostMallocDefault) != hipSuccess || !p)
            throw std::runtime_error("pinned host allocation of " + std::to_string(want) + " bytes failed");
        if (size_) std::memcpy(p, data_, size_);
        if (data_) (void)hipHostFree(data_);
        data_ = p;
        cap_ = want;
    }

    std::shared_mutex grow_;
    int device_ = 0;
    bool mirror_ = false;
    std::atomic<bool> mirror_failed_{false};
    hipStream_t stream_ = nullptr;
    uint8_t *dmirror_ = nullptr;
    uint64_t dcap_ = 0;
    char *data_ = nullptr;
    uint64_t size_ = 0, cap_ = 0;
    std::vector<uint64_t> starts_;
    std::vector<uint32_t> counts_;
    uint64_t run_end_ = ~0ull;  // byte offset where the last run ends (a new batch may extend it)
    bool any_count_not_one_ = false;
};

}  // namespace mtg
