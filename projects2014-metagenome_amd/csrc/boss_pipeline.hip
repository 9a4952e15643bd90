// boss_pipeline.hip -- host orchestration of the device BOSS construction path and the C ABI
// declared in include/mtg_boss.h.
//
// Stage order follows construct_boss_chunk (boss_chunk_construct.cpp:248-356) preceded by the
// k-mer collector (kmer_collector.cpp:26-127, sorted_set.cpp:19-48):
//   K1 extract -> K2 sort -> K3 unique/count -> [K4 rc + sort] -> K5/K6 dummies (+ sort/unique)
//   -> K7 lift+merge -> K8 W/last/F/weights.
// Everything runs on one HIP stream; host syncs only to read sizes that size the next stage.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include <sys/types.h>
#include <unistd.h>

#include "../../include/mtg_boss.h"
#include "boss_kernels.hpp"
#include "comm.hpp"
#include "dbg_io.hpp"
#include "dist_kernels.hpp"
#include "superkmer.hpp"
#include "extract_partition.hpp"
#include "fasta.hpp"
#include "range_extract.hpp"
#include "suffix_extract.hpp"
#include "host_stage.hpp"
#include "kmc.hpp"
#include "msd_sort.hpp"
#include "radix_sort.hpp"

namespace mtg {

static thread_local std::string g_last_error;

static void set_error(const std::string &msg) { g_last_error = msg; }

#define HIP_CHECK(x)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess)                                                               \
            throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) +    \
                                     " at " #x);                                            \
    } while (0)

// growable device buffers, reused across builds
class Workspace {
  public:
    enum Slot {
        SEQ, STARTS, RCOUNTS, KA, KB, CA, CB, SUMS, DESC, HIST, STARTS_DIGIT, SMALL, BUCKETS,
        FLAGS, DA, DB, STREAM, SCOUNT, OW, OLAST, OWEIGHTS, MSD_COUNTS, MSD_BSTART,
        MSD_CURSOR, MSD_GSTART, MSD_UCOUNT, MSD_USTART, MSD_OVF, MSD_GLIST, FB_K, FB_V, RC_ALT, RC_ALTC, REAL, REALC, SPLITS, DTCNT, DTOFF, INFLAG, HIST1, HIST_ROWS,
        // multi-GPU build: exchange buffers, routing and the query join
        XA, XAC, XB, XBC, XHIST, XSTART_A, XSTART_B, XMAT, BOUNDS, RTCNT, RTOFF, XGATHER, QSEND, QRECV,
        QFLAG, QTCNT, QTOFF, DSRC, DSEND, DRECV, RUN_IDX, RUN_DELTA, RUN_OFF, KMC_LUT, KMC_REC, DUP_TABLE, FUSED_HIST, FUSED_CUR, STRIPE_CUR,
        LAST_BITS, DPOS, DWL, RANGE_BINS, MSD_GBUCKET, RC_CSTART, RC_COMB, RC_SENDC, PACKED, W4, FA_RAW, FA_TLAST, FA_PREV, FA_TA, FA_TB, FA_OA, FA_OB, FA_KOFF, RID_AT, BRUNS,
        SK_OWN, SK_TCNT, SK_TOFF, SK_WORDS, SK_LENS, SK_CNT, SK_RWORDS, SK_RLENS, SK_RCNT, SK_NW, SK_WOFF, SK_SEQ,
        SK_STARTS, SK_RID, CANON_IDX, SPEC_A, SPEC_B, SPEC_CAP, SPEC_CUR, GAP_BSTART, GAP_USTART, CANON, CANONC,
        FUSED_SEL, WN, SPEC_AC, SPEC_BC, SPEC1_CAPS, SPEC1_START, SPEC1_TV, QINDEX, DBITMAP, RC_L1START, RC_L1CUR, RC_TILEG,
        KA2, ROUND_DELTA, XA2, XAC2, CA2, SPEC_MID_TV, NSLOTS
    };
    ~Workspace() {
        // every device block once, by its base (a slot or kept entry may be a piece of one: carve)
        for (auto &r : roots_)
            if (r.base) (void)hipFree(r.base);
    }
    void *get(Slot s, size_t bytes, size_t keep = 0, hipStream_t stream = nullptr) {
        Buf &b = bufs_[s];
        bytes = std::max<size_t>(bytes, 256);
        if (b.cap < bytes) {
            size_t cap = 0;
            int root = -1;
            void *p = take_cached(bytes, &cap, &root);
            if (!p) {
                cap = bytes + std::min<size_t>(bytes / 8, 1ull << 30);
                const auto t0 = std::chrono::steady_clock::now();
                bool dropped = false, carved = false;
                if (carve_always) {
                    p = take_cached(bytes, &cap, &root, true);
                    carved = p != nullptr;
                }
                if (!p && !try_malloc(&p, cap, &root)) {
                    // no room for a new block: a piece carved off a kept block that holds the request (the
                    // rest stays kept: the later stages of a batched build fit in the blocks its rounds gave
                    // back instead of each taking a whole one), and only then kept blocks freed one at a
                    // time, largest first (freeing kept blocks is what costs: ~12 ms per GB while the driver
                    // clears them, 2.3 s a build at configs[2] when every failed allocation dropped the
                    // whole cache).  MTG_WS_CARVE=1 (tests): carve before any new block
                    p = take_cached(bytes, &cap, &root, true);
                    carved = p != nullptr;
                    while (!p && !cache_.empty() && drop_largest()) {
                        dropped = true;
                        cap = bytes + std::min<size_t>(bytes / 8, 1ull << 30);
                        if (!try_malloc(&p, cap, &root)) p = nullptr;
                    }
                    if (!p && !try_malloc(&p, cap, &root)) {
                        size_t fr = 0, tot = 0;
                        (void)hipMemGetInfo(&fr, &tot);
                        throw std::runtime_error("HIP error out of memory: workspace slot " + std::to_string((int)s) +
                                                 " wants " + std::to_string(cap >> 20) + " MiB (held " +
                                                 std::to_string(held() >> 20) + " MiB in all slots, this one " +
                                                 std::to_string(b.cap >> 20) + " MiB; free " + std::to_string(fr >> 20) +
                                                 " MiB)");
                    }
                }
                if (carved) ++carves_;
                if (trace && cap >= (1ull << 28))
                    fprintf(stderr, "[mtg trace] workspace slot %d: %s %lu MiB%s, %.1f ms (held %lu MiB, kept %lu MiB)\n",
                            (int)s, carved ? "carved" : "new", (unsigned long)(cap >> 20),
                            dropped ? " after dropping the kept blocks" : "",
                            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(),
                            (unsigned long)(held() >> 20), (unsigned long)(cached() >> 20));
            }
            if (keep && b.ptr) HIP_CHECK(hipMemcpyAsync(p, b.ptr, keep, hipMemcpyDeviceToDevice, stream));
            if (b.ptr) {
                HIP_CHECK(hipDeviceSynchronize());
                give_back(b);
            }
            b.ptr = p;
            b.cap = cap;
            b.root = root;
            ++gen_[s];
        }
        return b.ptr;
    }
    void swap(Slot a, Slot b) {
        std::swap(bufs_[a], bufs_[b]);
        ++gen_[a], ++gen_[b];
    }
    // the buffers a build's sort, rc, dummy and emit stages hold (not its input, look-back descriptors
    // or pass-A histograms): a build in rounds frees the previous build's before sizing its rounds
    void release_stage_buffers(bool keep_outputs = false) {
        // keep_outputs (mtg_boss_ctor_trim): the last build's device chunk arrays (W, last, weights) stay
        for (Slot sl : {KA, KB, CA, CB, SUMS, BUCKETS, FLAGS, DA, DB, STREAM, SCOUNT, OW, OLAST, OWEIGHTS, FB_K, FB_V,
                        RC_ALT, RC_ALTC, REAL, REALC, INFLAG, XA, XAC, XB, XBC, QSEND, QRECV, QFLAG, DSRC, DSEND,
                        DRECV, RC_SENDC, LAST_BITS, W4, WN, DPOS, DWL, CANON, CANONC, CANON_IDX, SPEC_A, SPEC_B,
                        SPEC_AC, SPEC_BC, KA2, XA2, XAC2, CA2})
            if (!keep_outputs || (sl != OW && sl != OLAST && sl != OWEIGHTS)) release(sl);
    }
    // a slot gives its buffer back (batched builds drop their round buffers before the later stages
    // grow).  The block is kept for the next get() of about its size rather than freed: freeing and
    // mapping again the ~200 GB of a configs[3] share cost seconds per build while the driver clears
    // the pages (and slowed the kernels running meanwhile).  A hipMalloc that fails frees the kept
    // blocks and tries again.
    void release(Slot s) {
        Buf &b = bufs_[s];
        if (b.ptr) {
            HIP_CHECK(hipDeviceSynchronize());
            give_back(b);
        }
        b.ptr = nullptr;
        b.cap = 0;
        b.root = -1;
        ++gen_[s];
    }
    // every byte the workspace holds, in slots and kept blocks
    uint64_t held() const {
        uint64_t t = cached();
        for (const auto &b : bufs_) t += b.cap;
        return t;
    }
    uint64_t cached() const {
        uint64_t t = 0;
        for (const auto &b : cache_) t += b.cap;
        return t;
    }
    // free HBM for new buffers: the device's free memory plus the kept blocks
    uint64_t free_bytes() const {
        size_t fr = 0, tot = 0;
        HIP_CHECK(hipMemGetInfo(&fr, &tot));
        return (uint64_t)fr + cached();
    }
    // the largest kept whole block freed (a block partly carved out to a slot stays); false: none
    bool drop_largest() {
        size_t big = cache_.size();
        for (size_t i = 0; i < cache_.size(); ++i)
            if (whole(cache_[i]) && (big == cache_.size() || cache_[i].cap > cache_[big].cap)) big = i;
        if (big == cache_.size()) return false;
        HIP_CHECK(hipDeviceSynchronize());
        free_root(cache_[big].root);
        cache_.erase(cache_.begin() + (long)big);
        return true;
    }
    void drop_cache() {
        if (cache_.empty()) return;
        HIP_CHECK(hipDeviceSynchronize());
        std::vector<Buf> keep;
        for (auto &b : cache_) {
            if (whole(b)) free_root(b.root);
            else keep.push_back(b);
        }
        cache_.swap(keep);
    }
    // end of a build: free the kept blocks no get() took during it (released in an earlier build and
    // idle since), so a big build's blocks do not pin HBM for the life of the constructor; the blocks
    // this build gave back stay for the next build of the same shape
    void end_build() {
        bool any = false;
        for (const auto &b : cache_) any |= b.age > 0 && whole(b);
        if (any) {
            HIP_CHECK(hipDeviceSynchronize());
            std::vector<Buf> keep;
            for (auto &b : cache_) {
                if (b.age > 0 && whole(b)) free_root(b.root);
                else keep.push_back(b);
            }
            cache_.swap(keep);
        }
        for (auto &b : cache_) b.age = 1;
    }
    uint64_t held_slot(Slot s) const { return bufs_[s].cap; }
    uint64_t carves() const { return carves_; }
    bool carve_always = false;  // MTG_WS_CARVE=1
    const void *peek(Slot s) const { return bufs_[s].ptr; }
    // bumped whenever the slot's buffer changes (regrown or released): a block given back may be
    // handed to another slot, so a pointer comparison alone cannot tell that the data is still there
    uint64_t generation(Slot s) const { return gen_[s]; }

  private:
    struct Buf {
        void *ptr = nullptr;
        size_t cap = 0;
        uint32_t age = 0;  // kept blocks: builds ended since it was given back (end_build)
        int root = -1;     // the device block (roots_) it is, or is a piece of
    };
    struct Root {
        void *base = nullptr;  // hipMalloc'ed, hipFree'd once when no piece of it is in use
        size_t cap = 0;
    };
    bool whole(const Buf &b) const { return b.root >= 0 && b.ptr == roots_[b.root].base && b.cap == roots_[b.root].cap; }
    bool try_malloc(void **p, size_t cap, int *root) {
        if (hipMalloc(p, cap) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        size_t i = 0;
        while (i < roots_.size() && roots_[i].base) ++i;
        if (i == roots_.size()) roots_.emplace_back();
        roots_[i] = Root{*p, cap};
        *root = (int)i;
        return true;
    }
    void free_root(int r) {
        (void)hipFree(roots_[r].base);
        roots_[r] = Root{};
    }
    // a slot's buffer back to the kept list, merged with the kept pieces of its block next to it (a
    // block whose pieces are all back is whole again: the next build of the same shape takes it whole)
    void give_back(Buf b) {
        b.age = 0;
        for (bool merged = true; merged;) {
            merged = false;
            for (size_t i = 0; i < cache_.size(); ++i) {
                Buf &o = cache_[i];
                if (o.root != b.root || b.root < 0) continue;
                if ((char *)o.ptr + o.cap == (char *)b.ptr) {
                    b.ptr = o.ptr, b.cap += o.cap;
                } else if ((char *)b.ptr + b.cap == (char *)o.ptr) {
                    b.cap += o.cap;
                } else {
                    continue;
                }
                cache_.erase(cache_.begin() + (long)i);
                merged = true;
                break;
            }
        }
        cache_.push_back(b);
    }
    // the smallest kept block of at least `bytes` and at most about twice that (a far bigger block
    // stays for the request it was made for); carve (the device has no room left): the smallest kept
    // block or piece that holds `bytes`, its front handed out and its rest kept when that is 256 MiB+
    void *take_cached(size_t bytes, size_t *cap, int *root, bool carve = false) {
        size_t best = cache_.size();
        for (size_t i = 0; i < cache_.size(); ++i)
            if (cache_[i].cap >= bytes && (carve || cache_[i].cap <= 2 * bytes + (64u << 20)) &&
                (best == cache_.size() || cache_[i].cap < cache_[best].cap))
                best = i;
        if (best == cache_.size()) return nullptr;
        Buf &k = cache_[best];
        void *p = k.ptr;
        *root = k.root;
        const size_t piece = (bytes + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);  // 2 MiB aligned
        if (carve && k.cap >= piece + (256u << 20)) {
            *cap = piece;
            k.ptr = (char *)k.ptr + piece;
            k.cap -= piece;
            k.age = 0;
            return p;
        }
        *cap = k.cap;
        cache_.erase(cache_.begin() + (long)best);
        return p;
    }
    Buf bufs_[NSLOTS];
    uint64_t gen_[NSLOTS] = {};
    std::vector<Root> roots_;
    uint64_t carves_ = 0;

  public:
    bool trace = false;  // MTG_TRACE: report every fresh allocation of 256 MiB or more

  private:
    std::vector<Buf> cache_;
};

struct Small {  // one device word block, zeroed per use
    unsigned long long total;
    unsigned long long totals[2];
    unsigned long long fhist[8];
    uint32_t counter;
    uint32_t skip;
    uint32_t root_same;
    uint32_t bad_dummy;
    uint32_t bruns;  // bucket_index: listed long runs
    uint32_t fasta_bad;  // fasta_split_kernel: a '+' sequence line
    uint32_t gidx_bad;   // group_gather_kernel: the output bucket index was abandoned
    uint32_t spec_ovf;   // msd_partition_kernel: a speculative bucket overflowed
    uint32_t wbad;       // window_reads_kernel: the input is not one window per read
    unsigned long long wcursor;  // window_reads_kernel: keys written
    uint32_t error;
};

class EventTimer {
  public:
    explicit EventTimer(hipStream_t s) : s_(s) {}
    ~EventTimer() {
        for (auto e : evs_) (void)hipEventDestroy(e);
    }
    int mark() {
        hipEvent_t e;
        HIP_CHECK(hipEventCreate(&e));
        HIP_CHECK(hipEventRecord(e, s_));
        evs_.push_back(e);
        return (int)evs_.size() - 1;
    }
    double ms(int a, int b) {
        float t = 0;
        HIP_CHECK(hipEventElapsedTime(&t, evs_[a], evs_[b]));
        return t;
    }

  private:
    hipStream_t s_;
    std::vector<hipEvent_t> evs_;
};

struct Ctx {
    Workspace ws;
    hipStream_t stream = nullptr;
    Small *small = nullptr;
    mtg_boss_timings timings{};
    uint32_t epoch = 0;           // look-back granule epoch of the last launch
    size_t desc_words = 0;        // zeroed capacity of the descriptor buffer
    // accumulated over the onesweep launches of the real-k-mer sorts of one build
    double radix_ms = 0, radix_bytes = 0;
    uint64_t radix_launches = 0;
    bool track_partition = false;  // time the msd_partition launches of the real-k-mer sorts
    bool use_lsd = false;          // MTG_SORT=lsd: LSD onesweep + unique instead of MSD (the fallback
                                   // sort of overflowing groups, selectable for the parity tests)
    bool emit_slow = false;        // MTG_EMIT=slow: always the compacting emit kernel (the redundant-sink path)
    bool debug = false;            // MTG_DEBUG=1: host-side checks between stages
    bool trace = false;            // MTG_TRACE=1: per-step wall times and sizes of the dist build
    bool fused = true;             // MTG_FUSED=0: K1 writes in window order, K2 partitions after
    uint64_t fused_min = 1ull << 22;  // MTG_FUSED_MIN: fewest window starts for the fused K1
    uint32_t force_ranges = 0;     // MTG_RANGES=P: collect in P key ranges (tests; else planned from memory)
    double mem_budget = 0;         // memory_preallocated (bytes; 0 = free HBM)
    bool disk = false;             // MTG_CONTAINER_VECTOR_DISK: the bounded-memory (range-batched) build
    bool host_output = false;      // the build's arrays go to the host (build_chunk): it may spill
    bool force_spill = false;      // MTG_SPILL=1: spill whenever the build runs in key ranges (tests)
    std::string swap_dir;          // spill files of the disk container (swap_dir of initialize)
    uint64_t disk_cap = 0;         // at most this many bytes of spill files (disk_cap_bytes); the rest in RAM
    std::vector<uint8_t> spill_W, spill_last;  // the spilled build's output rows (host)
    std::vector<uint32_t> spill_weights;
    uint64_t spilled_bytes = 0;    // bytes the last build kept outside HBM
    uint32_t hist_rows = 2048;     // MTG_HIST_ROWS: workgroups of the fused K1 histogram pass (tests
                                   // lower it so the grid-stride + prefetch loop runs on small inputs)
    double fused_ms = 0;           // device time of the last fused extract+partition launch
    bool fused_emit = true;        // MTG_FUSED_EMIT=0: K7 writes the lifted stream, K8 reads it (the
                                   // redundant-sink path)
    bool routed_min = false;       // MTG_ROUTED_CANON=min: the routed collect keeps min(fwd, rc)
    int dist_collect = 1;          // MTG_DIST_COLLECT: 1 routed keys (default), 0 super-k-mers
                                   // (=superkmer), 2 local collect + exchange of sorted runs (=local)
    unsigned fused_b1 = 0;         // MTG_FUSED_B1=n: the fused K1's level-1 digit forced to n bits (A/B runs)
    bool wide_b1 = true;           // MTG_WIDE_B1=0: no 10-bit level 1 (fused_plan)
    bool lu_fast = true;           // MTG_LU_FAST=0: local_unique_kernel's per-key list positions (A/B)
    bool fast2_ppt8 = true;        // MTG_FAST2_PPT8=0: the u128 packed-word pass B at 16 windows a thread (256 threads)
    bool rc_wide = true;           // MTG_RC_WIDE=0: the u128 rc sort planned like the unique (half-full merge groups)
    bool lu_wpe2 = true;           // MTG_LU_WPE2=0: the u128 local unique compiled for 1 wave per SIMD (no VGPR cap)
    bool fast2 = true;             // MTG_FAST2=0: the u128 rounds' pass B as the generic extract_partition_kernel
    int canon_mode = 1;            // the single-build extraction's canonical representative (cmode); the
                                   // super-k-mer owners of a multi-GPU build extract with 2
    uint32_t merge_it = 1;         // MTG_MERGE_IT: local_merge_kernel's least outputs per thread (A/B)
    bool range_scan = false;       // MTG_COLLECT=ranges: a build too big for one pass collects in key ranges
    bool kmc_mirror = true;  // add_kmc copies the first database to the device while reading it
                                   // that re-scan the reads (both strands) even where the canonical
                                   // rounds of the fused K1 apply (collect_rounds_fused)
    bool kspec = true;             // MTG_KSPEC=0: the fused K1 passes with K a runtime argument at K = 31 too
    bool dist_pull = true;         // MTG_DIST_SINKS=query: the multi-GPU sink join by routed queries
                                   // (target_split + query_join) instead of the pulled edge slices
    bool rc_fuse = true;           // MTG_RC_FUSE=0: the rc keys of a gapped canonical set written in canonical
                                   // order and partitioned by the rc sort's own level 1, not straight into
                                   // its level-1 buckets (rc_partition_gapped_kernel)
    bool dummy_bitmap = false;     // MTG_DUMMY_BITMAP=1: the source levels with few real chars as bits of a
                                   // bitmap (dummy_write_kernel) -- the sort gains 0.25 ms, the write pass
                                   // loses as much, so off by default
    bool dummy_ranks = true;       // MTG_DUMMY_SORT=lifted: sort the dummies as lifted keys, not as
                                   // dense u64 ranks (dummy_encode_kernel)
    // bucket index of the last msd_sort_unique's output over its final bucket bits, when every group
    // was one bucket (its group starts are that index): the fused rc merge reuses it for the canonical keys
    struct GroupIndex {
        const void *keys = nullptr;
        uint64_t n = 0;
        unsigned bits = 0, nbits = 0;
        const uint64_t *start = nullptr;
    } gidx;
    bool want_gidx = false;  // the next msd_sort_unique's output feeds the fused rc merge
    // a batched collect round's share of the canonical set's bucket index (collect_rounds_fused): the
    // speculative final level's gather writes entries [lo, hi) of `start` (2^bits buckets) as positions
    // + off in the whole set, and says so in `written`
    struct RoundIndex {
        uint64_t *start = nullptr;
        unsigned bits = 0;
        uint64_t off = 0, lo = 0, hi = 0;
        bool written = false;
    } ridx;
    bool round_index = true;  // MTG_ROUND_INDEX=0: the canonical set's index by a bucket_index pass
    // where the next msd_sort_unique's final gather writes its compact distinct keys (and counts) instead of
    // *keys (the exchange pieces append each piece's keys in place: routed_pieces); *keys then points there
    void *sort_out = nullptr;
    uint32_t *sort_out_vals = nullptr;
    uint64_t sort_out_cap = ~0ull;  // keys sort_out holds (more distinct keys: the usual gather into *keys)
    // the single build's canonical set left in the speculative level's bucket layout (no
    // group_gather_kernel): bucket g's keys at keys[bstart[g] ..), compact at ustart[g] ..
    // (ustart[g + 1] - ustart[g] keys).  rc_map and the fused rc merge read it there;
    // ensure_compact() writes the compact array to dst when anything else needs it.
    struct GappedSet {
        bool valid = false;
        const void *keys = nullptr;
        void *dst = nullptr;
        uint64_t u = 0, nb = 0;
        const uint64_t *bstart = nullptr, *ustart = nullptr;
    } gap;
    bool defer_gather_req = false;  // set around the single build's canonical collect
    bool defer_gather = true;       // MTG_DEFER_GATHER=0: the speculative level always gathers
    bool spec_rc = true;            // MTG_SPEC_RC=0: the rc sort's final level exact (tests the fallbacks)
    unsigned min_levels = 0;        // MTG_MSD_LEVELS=n: plan at least n MSD levels (tests the 3-level path)
    // MTG_SPEC3=0: the speculative final level only for 2-level plans.  (Sampled every 8th tile, the
    // level-3 buckets of level-2 buckets only a few tiles long were sized badly: at 20 M reads every
    // step overflowed into the exact level, sort 30.3 -> 38.9 ms; level 3 now samples every tile's
    // first eighth.)
    bool spec3 = true;
    // the speculative final level's local unique writes over its own buckets (each group is read whole
    // before it writes): one slack-sized buffer instead of two.  MTG_SPEC_INPLACE=0: two
    bool spec_inplace = true;
    // a free buffer the speculative final level of a 3-level sort may partition into (the batched
    // collect's level-1 array, sized for it, free once level 2 has moved the keys out): no third block
    void *spec_into = nullptr;
    uint64_t spec_into_bytes = 0;
    // a collect round whose keys are sparse in the plan's final buckets (it spans more level-1 buckets
    // than its share: canonical k-mers crowd the small prefixes) takes one final bit fewer, so its local
    // unique runs fuller groups (configs[3]'s second round: 2.95 M groups of ~390 distinct keys, 25.7 vs
    // 20.6 ms for the first round's 1.25 M).  MTG_ROUND_BITS=0: the plan's bits in every round
    bool round_bits = true;
    bool rounds_one_b = true;  // two collect rounds share one pass B (collect_rounds_fused); MTG_ROUNDS_ONE_B=0: not
    // MTG_DIST_PIECES=n: the routed multi-GPU collect sends exchange 1 in n pieces on the exchange stream,
    // each sorted by its owner while the next one is in flight (routed_pieces); 1 = one exchange, then the sort
    uint32_t dist_pieces = 4;
    bool dist_pieces_set = false;  // MTG_DIST_PIECES given: exactly that many (else fewer for small shares)
    hipStream_t xstream = nullptr;  // the multi-GPU exchange stream (created by the first distributed build)
    bool spec_final = true;  // MTG_SPEC=0: the exact final MSD level (histogram pass) instead of the
                             // sample-sized one (spec_final_level)
    bool spec_tiny = false;  // MTG_SPEC_CAPS=tiny: speculative buckets without slack (tests force the
                             // overflow fallback with it)
    bool spec_lu_fail = false;  // MTG_SPEC_LU_FAIL=1: the speculative level's local unique pass reports an
                                // overflow after it ran (tests the exact level after that late fallback)
    // MTG_SPEC_L1=0: the exact fused pass A (a histogram of every window) instead of the sampled one
    // and the speculative level-1 layout (fused_pass_b_spec), used from MTG_SPEC_L1_MIN windows on;
    // MTG_SPEC_L1_SAMPLE: pass A counts every n-th tile
    bool spec_l1 = true;
    bool spec_l1_tiny = false;  // MTG_SPEC_L1_CAPS=tiny: segments without slack (tests force its fallback)
    uint64_t spec_l1_min = 1ull << 28;
    uint32_t spec_l1_sample = 8;
    uint32_t spec_l1_stripes = 16;  // MTG_SPEC_L1_STRIPES: segments per level-1 bucket (a power of two <= 256)
    uint32_t spec_l1_slack = 16;    // MTG_SPEC_L1_SLACK: segment slack 1/n of the estimate (+ 3 sigma + 1024)
    // the speculative level-1 layout of the last fused K1 until the level-2 pass has read it: gap1_n
    // positions, tile t of the level-2 tiling holding keys in its first gap1_tv[t] positions
    uint64_t gap1_n = 0;
    const uint32_t *gap1_tv = nullptr;
    // the previous-level buckets a padded input's keys occupy, [gap1_lo, gap1_hi) (spec_mid_level; 0 / 0:
    // unknown, every bucket)
    uint64_t gap1_lo = 0, gap1_hi = 0;
    // a 3-level sort's speculative middle level (spec_mid_level) partitions into this buffer (the batched
    // collect's KB, sized for it); MTG_SPEC_MID=0: the exact middle level
    void *spec_mid_into = nullptr;
    uint64_t spec_mid_bytes = 0;
    bool spec_mid = true;
    // bucket index over the real edges, built by the dummy stage and reused by the split emit
    const void *bidx_keys = nullptr;
    uint64_t bidx_n = 0;
    const uint64_t *bidx = nullptr;
    unsigned bidx_shift = 0;
    uint64_t bidx_gen = 0;  // the BUCKETS slot's generation when the index was written
};

static inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// the extraction kernels' canonical argument: 0 basic, 1 min(fwd, rc), 2 the strand whose top 12 bits hash
// smaller (boss_kernels.hpp: take_rc) -- any one representative per {x, rc x} gives the same real edges and
// weights; 2 spreads the representatives over the key space (the multi-GPU collects, Ctx::canon_mode)
static inline int cmode(const Ctx &c, bool canonical) { return canonical ? c.canon_mode : 0; }

// The few environment switches, read once per constructor.  All but MTG_DEBUG / MTG_TRACE select
// alternate device paths that exist for correctness (fallbacks the parity tests force on small
// inputs), never a faster configuration.
static void load_knobs(Ctx &c) {
    auto is = [](const char *name, const char *val) {
        const char *e = getenv(name);
        return e && std::string(e) == val;
    };
    c.use_lsd = is("MTG_SORT", "lsd");
    c.emit_slow = is("MTG_EMIT", "slow");
    c.fused = !is("MTG_FUSED", "0");
    c.fused_emit = !is("MTG_FUSED_EMIT", "0");
    c.dummy_ranks = !is("MTG_DUMMY_SORT", "lifted");
    c.range_scan = is("MTG_COLLECT", "ranges");
    c.wide_b1 = !is("MTG_WIDE_B1", "0");
    c.kmc_mirror = !is("MTG_KMC_MIRROR", "0");
    c.lu_fast = !is("MTG_LU_FAST", "0");
    c.lu_wpe2 = !is("MTG_LU_WPE2", "0");
    c.rc_wide = !is("MTG_RC_WIDE", "0");
    c.fast2_ppt8 = !is("MTG_FAST2_PPT8", "0");
    c.fast2 = !is("MTG_FAST2", "0");
    if (const char *e = getenv("MTG_MERGE_IT")) c.merge_it = (uint32_t)std::max(1L, std::min(64L, atol(e)));
    if (const char *v = getenv("MTG_FUSED_B1")) c.fused_b1 = (unsigned)std::min(10, std::max(0, atoi(v)));
    c.spec_final = !is("MTG_SPEC", "0");
    c.defer_gather = !is("MTG_DEFER_GATHER", "0");
    c.spec_rc = !is("MTG_SPEC_RC", "0");
    c.spec3 = !is("MTG_SPEC3", "0");
    c.rounds_one_b = !is("MTG_ROUNDS_ONE_B", "0");
    c.ws.carve_always = is("MTG_WS_CARVE", "1");
    c.spec_inplace = !is("MTG_SPEC_INPLACE", "0");
    c.round_bits = !is("MTG_ROUND_BITS", "0");
    c.round_index = !is("MTG_ROUND_INDEX", "0");
    c.spec_mid = !is("MTG_SPEC_MID", "0");
    if (const char *e = getenv("MTG_DIST_PIECES")) {
        c.dist_pieces = (uint32_t)std::max(1L, std::min(16L, atol(e)));
        c.dist_pieces_set = true;
    }
    c.spec_tiny = is("MTG_SPEC_CAPS", "tiny");
    c.spec_lu_fail = is("MTG_SPEC_LU_FAIL", "1");
    c.spec_l1 = !is("MTG_SPEC_L1", "0");
    c.dist_pull = !is("MTG_DIST_SINKS", "query");
    c.kspec = !is("MTG_KSPEC", "0");
    c.dummy_bitmap = is("MTG_DUMMY_BITMAP", "1");
    c.rc_fuse = !is("MTG_RC_FUSE", "0");
    c.spec_l1_tiny = is("MTG_SPEC_L1_CAPS", "tiny");
    if (const char *e = getenv("MTG_SPEC_L1_STRIPES")) {
        const long v = atol(e);
        if (v >= 1 && v <= 256 && (v & (v - 1)) == 0) c.spec_l1_stripes = (uint32_t)v;
    }
    if (const char *e = getenv("MTG_SPEC_L1_SLACK")) c.spec_l1_slack = (uint32_t)std::max(2L, std::min(1024L, atol(e)));
    if (const char *e = getenv("MTG_SPEC_L1_MIN")) c.spec_l1_min = strtoull(e, nullptr, 10);
    if (const char *e = getenv("MTG_SPEC_L1_SAMPLE")) c.spec_l1_sample = (uint32_t)std::max(1L, std::min(64L, atol(e)));
    if (const char *v = getenv("MTG_MSD_LEVELS")) c.min_levels = (unsigned)std::min(3, std::max(0, atoi(v)));
    c.dist_collect = is("MTG_DIST_COLLECT", "superkmer") ? 0 : is("MTG_DIST_COLLECT", "local") ? 2 : 1;
    c.routed_min = is("MTG_ROUTED_CANON", "min");
    c.force_spill = is("MTG_SPILL", "1");
    c.debug = getenv("MTG_DEBUG") != nullptr;
    c.trace = getenv("MTG_TRACE") != nullptr;
    c.ws.trace = c.trace;
    if (const char *e = getenv("MTG_FUSED_MIN")) c.fused_min = strtoull(e, nullptr, 10);
    if (const char *e = getenv("MTG_RANGES")) c.force_ranges = (uint32_t)std::max(0L, std::min(4096L, atol(e)));
    if (const char *e = getenv("MTG_HIST_ROWS")) c.hist_rows = (uint32_t)std::max(1L, std::min(2048L, atol(e)));
}

// zero the per-stage words; the error word is sticky for the whole build (checked at the end)
static void reset_small(Ctx &c) {
    HIP_CHECK(hipMemsetAsync(c.small, 0, offsetof(Small, error), c.stream));
}

static uint64_t read_u64(Ctx &c, const unsigned long long *p) {
    unsigned long long v = 0;
    HIP_CHECK(hipMemcpyAsync(&v, p, sizeof(v), hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    return v;
}

// MTG_TRACE: host wall time since the previous trace point (stream drained first)
struct Tracer {
    Ctx &c;
    int rank;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void operator()(const char *what, uint64_t a = 0, uint64_t b = 0) {
        if (!c.trace) return;
        HIP_CHECK(hipStreamSynchronize(c.stream));
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[mtg trace r%d] %-22s %9.3f ms  %lu %lu\n", rank, what,
                std::chrono::duration<double, std::milli>(now - t).count(), (unsigned long)a, (unsigned long)b);
        t = now;
    }
};

static void check_error_word(Ctx &c) {
    uint32_t e = 0;
    HIP_CHECK(hipMemcpyAsync(&e, &c.small->error, sizeof(e), hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    if (e & 1u) throw std::runtime_error("device look-back timed out (error word " + std::to_string(e) + ")");
    if (e) throw std::runtime_error("device partition counts disagree with the histogram pass (error word " +
                                    std::to_string(e) + ")");
}

// Descriptor array for one look-back launch plus its epoch.  Granules of older epochs read as
// "not ready", so the array is zeroed only when it grows or the 16-bit epoch wraps.
static uint64_t *acquire_desc(Ctx &c, uint64_t words, uint32_t *epoch) {
    uint64_t *d = (uint64_t *)c.ws.get(Workspace::DESC, words * 8);
    if (words > c.desc_words || c.epoch >= 0xFFFF) {
        size_t cap = std::max<size_t>(words, c.desc_words);
        d = (uint64_t *)c.ws.get(Workspace::DESC, cap * 8);
        HIP_CHECK(hipMemsetAsync(d, 0, cap * 8, c.stream));
        c.desc_words = cap;
        c.epoch = 0;
    }
    *epoch = ++c.epoch;
    return d;
}

// bucket index of a sorted key array (boss_kernels.hpp: bucket_index_kernel + the grid-wide fill of
// its long empty runs)
constexpr uint32_t kBucketRuns = 4096;
template <int L>
static void bucket_index(Ctx &c, const Key<L> *keys, uint64_t n, unsigned shift, uint64_t nb, uint64_t *start) {
    uint64_t *runs = (uint64_t *)c.ws.get(Workspace::BRUNS, kBucketRuns * 24);
    HIP_CHECK(hipMemsetAsync(&c.small->bruns, 0, 4, c.stream));
    const uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(n + 1, 256), 8192));
    bucket_index_kernel<L><<<dim3((unsigned)g), dim3(256), 0, c.stream>>>(keys, n, shift, nb, start, runs,
                                                                         &c.small->bruns, kBucketRuns);
    HIP_CHECK(hipGetLastError());
    bucket_fill_kernel<<<dim3(1024), dim3(256), 0, c.stream>>>(runs, &c.small->bruns, kBucketRuns, start);
    HIP_CHECK(hipGetLastError());
}

// exclusive scans of the per-pass digit counts: block p scans hist[p * 256 ..] into start[p * 256 ..]
__global__ __launch_bounds__(256) void digit_starts_kernel(const unsigned long long *__restrict__ hist,
                                                           uint64_t *__restrict__ start) {
    __shared__ uint64_t s_wsum[4];
    const uint32_t t = threadIdx.x, p = blockIdx.x;
    const uint64_t v = hist[p * 256 + t];
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, 64);
        if ((t & 63) >= (uint32_t)o) x += y;
    }
    if ((t & 63) == 63) s_wsum[t >> 6] = x;
    __syncthreads();
    uint64_t before = 0;
    for (uint32_t w = 0; w < (t >> 6); ++w) before += s_wsum[w];
    start[p * 256 + t] = before + x - v;
}

// LSD radix sort of keys[0..n) (and vals) over the low nbits; result left in *keys / *vals
// (pointers swapped with *alt / *valt as passes ping-pong).  Passes whose digit is the same for every key
// are skipped.  spec_first: the lowest pass is launched before the histogram reaches the host (the digit
// starts are scanned on the device), so the copy and the host's look at it overlap that pass -- for
// inputs whose lowest digit is never constant (the dense dummy ranks); a constant one costs one pass.
template <int L, bool HAS_VAL>
static void radix_sort(Ctx &c, Key<L> **keys, Key<L> **alt, uint32_t **vals, uint32_t **valt,
                       uint64_t n, unsigned nbits, bool stats, bool spec_first = false) {
    if (n < 2) return;
    const int passes = (int)ceil_div(nbits, 8);
    auto *hist = (unsigned long long *)c.ws.get(Workspace::HIST, passes * 256 * 8);
    HIP_CHECK(hipMemsetAsync(hist, 0, passes * 256 * 8, c.stream));
    const uint64_t hgrid = std::min<uint64_t>(ceil_div(n, 256), 4096);
    radix_histogram_kernel<L><<<dim3((unsigned)hgrid), dim3(256), 0, c.stream>>>(*keys, n, passes, hist);
    HIP_CHECK(hipGetLastError());
    auto *dstart = (uint64_t *)c.ws.get(Workspace::STARTS_DIGIT, passes * 256 * 8);
    digit_starts_kernel<<<dim3((unsigned)passes), dim3(256), 0, c.stream>>>(hist, dstart);
    HIP_CHECK(hipGetLastError());
    std::vector<unsigned long long> h(passes * 256);
    HIP_CHECK(hipMemcpyAsync(h.data(), hist, h.size() * 8, hipMemcpyDeviceToHost, c.stream));
    constexpr int TILE = SortTraits<L>::TILE;
    const uint64_t tiles = ceil_div(n, TILE);
    if (tiles > 0xFFFFFFFFull) throw std::runtime_error("sort too large");
    EventTimer tm(c.stream);
    std::vector<int> done;
    auto launch = [&](int p) {
        uint32_t epoch;
        uint64_t *desc = acquire_desc(c, tiles * 256, &epoch);
        HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
        tm.mark();
        onesweep_kernel<L, HAS_VAL><<<dim3((unsigned)tiles), dim3(SortTraits<L>::BLOCK), 0, c.stream>>>(
            *keys, *alt, HAS_VAL ? *vals : nullptr, HAS_VAL ? *valt : nullptr, n, 8u * p,
            dstart + p * 256, desc, epoch, &c.small->counter, &c.small->error);
        HIP_CHECK(hipGetLastError());
        tm.mark();
        std::swap(*keys, *alt);
        if (HAS_VAL) std::swap(*vals, *valt);
        done.push_back(p);
    };
    if (spec_first) launch(0);
    HIP_CHECK(hipStreamSynchronize(c.stream));  // the histogram on the host (`h` is a local)
    for (int p = spec_first ? 1 : 0; p < passes; ++p) {
        bool trivial = false;
        for (int d = 0; d < 256; ++d)
            if (h[p * 256 + d] == n) trivial = true;
        if (!trivial) launch(p);
    }
    if (stats && !done.empty()) {
        HIP_CHECK(hipStreamSynchronize(c.stream));
        for (size_t i = 0; i < done.size(); ++i) c.radix_ms += tm.ms(2 * i, 2 * i + 1);
        c.radix_launches += done.size();
        c.radix_bytes += (double)done.size() * 2.0 * n * (sizeof(Key<L>) + (HAS_VAL ? 4 : 0));
    }
}

__global__ void set_u64_kernel(uint64_t *p, uint64_t a) { *p = a; }

// p[i] = v for i in [lo, hi)
__global__ __launch_bounds__(256) void fill_u64_kernel(uint64_t *__restrict__ p, uint64_t lo, uint64_t hi, uint64_t v) {
    const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += T) p[i] = v;
}

__global__ void set_pair_kernel(uint64_t *p, uint64_t a, uint64_t b) {
    p[0] = a;
    p[1] = b;
}

// Duplication estimate for the MSD plan: m evenly spaced sample keys go into a hash table of
// 64-bit fingerprints; the number of samples that find their fingerprint already present is
// C ~ m^2 / (2 n) * E_w[mult] (E_w: multiplicity seen by a random occurrence).  Reads arrive in
// random genome order, so evenly spaced samples are as good as random ones.
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    return x ^ (x >> 33);
}

template <int L>
__global__ void dup_sample_kernel(const Key<L> *__restrict__ keys, uint64_t n, uint32_t m,
                                  unsigned long long *__restrict__ table, uint32_t mask,
                                  unsigned long long *__restrict__ hits) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const Key<L> k = keys[(uint64_t)((double)j * ((double)n / m))];
    uint64_t h = 0x9e3779b97f4a7c15ull;
#pragma unroll
    for (int i = 0; i < L; ++i) h = mix64(h ^ k.w[i]);
    h |= 1;  // 0 marks an empty slot
    uint32_t slot = (uint32_t)(h >> 32) & mask;
    while (true) {
        const unsigned long long prev = atomicCAS(&table[slot], 0ull, (unsigned long long)h);
        if (prev == 0) return;
        if (prev == h) {
            atomicAdd(hits, 1ull);
            return;
        }
        slot = (slot + 1) & mask;
    }
}

// expected copies per distinct key of keys[0..n), conservative (it may err low, which costs a
// planned bit, never an overflowing plan); `fallback` below the sampling size
template <int L>
static double estimate_dup(Ctx &c, const Key<L> *keys, uint64_t n, double fallback) {
    constexpr uint32_t M = 1u << 20, SLOTS = 1u << 22;
    if (n < 8ull * M) return fallback;
    unsigned long long *table = (unsigned long long *)c.ws.get(Workspace::DUP_TABLE, (SLOTS + 1) * 8ull);
    HIP_CHECK(hipMemsetAsync(table, 0, (SLOTS + 1) * 8ull, c.stream));
    dup_sample_kernel<L><<<dim3(M / 256), dim3(256), 0, c.stream>>>(keys, n, M, table, SLOTS - 1, table + SLOTS);
    HIP_CHECK(hipGetLastError());
    const double hits = (double)read_u64(c, table + SLOTS);
    const double ew = 2.0 * (double)n * hits / ((double)M * M);  // E_w[multiplicity]
    const double dup = std::max(1.0, ew / 1.2);  // E_w / mean: 1.17 at 10x, 1.29 at 1.25x
    if (c.debug) fprintf(stderr, "[mtg debug] dup estimate n=%lu hits=%.0f E_w=%.2f -> %.2f\n", (unsigned long)n, hits, ew, dup);
    return dup;
}

// Sort + unique (+ saturating count merge) of keys[0..n) over their low nbits by MSD
// partitioning and per-group LDS hashing (msd_sort.hpp).  `dup` is the expected number of
// copies per distinct key, used only to plan the partition depth; a wrong guess costs time,
// never correctness (overflowing groups take another level or the LSD fallback).
// Result: sorted distinct keys in *keys (counts in *vals); returns their number.
struct MsdPlan {
    unsigned levels;
    unsigned digit_end[4];  // cumulative significant bits after each level
};

// partition depth: enough top bits T that an average final bucket holds <= LIMIT/3 distinct
// keys (canonical k-mers are up to 2x denser at small prefixes), in levels of <= max_digit
// bits (one full read + scatter each)
constexpr double kPlanDiv = 2.5;  // planned distinct keys per final bucket = LIMIT / kPlanDiv

template <int L>
static MsdPlan msd_plan(const Ctx &c, uint64_t n, unsigned nbits, double dup) {
    const double LIMIT = (double)LocalTraits<L>::LIMIT / 2;  // half-size LDS tables
    const unsigned dmax = MSD_DBITS;
    unsigned T = 0;
    while (T < nbits && T < 3 * dmax && (double)n / dup / (double)(1ull << T) > LIMIT / kPlanDiv)
        ++T;
    MsdPlan p{};
    p.levels = (T + dmax - 1) / dmax;
    if (c.min_levels > p.levels && T >= c.min_levels) p.levels = c.min_levels;  // (tests: MTG_MSD_LEVELS)
    for (unsigned l = 1; l <= p.levels; ++l) p.digit_end[l] = T * l / p.levels;
    return p;
}

static void note_bucket_index(Ctx &c, const void *keys, uint64_t n, const uint64_t *start, unsigned shift);

// The plan of the rc sort fused with the merge (and of the canonical set's bucket index it reads): u128 keys
// take one final bit fewer than the unique's plan, so a merge group holds ~480 rc + ~480 canonical keys in
// its 1024-key LDS arrays instead of ~240 + 240 -- the per-group cost (barriers, table setup) then spreads
// over twice the keys (configs[2]: 2.03e9 rc keys over 2^22 buckets, not 2^23)
template <int L>
static MsdPlan rc_plan(const Ctx &c, uint64_t n, unsigned nbits) {
    return msd_plan<L>(c, L == 2 && c.rc_wide ? std::max<uint64_t>(1, n / 2) : n, nbits, 1.0);
}

// the rc sort's local pass fused with the merge into the real edges (local_merge_kernel)
template <int L>
struct RcMerge {
    const Key<L> *ck;   // the sorted canonical set
    const uint32_t *cv;
    uint64_t nc;
    Key<L> *out;        // the real edges: merge(canonical, sorted rc)
    uint32_t *outc;
    bool done = false;  // set when the fused pass ran (else the caller merges)
    uint64_t *istart = nullptr;  // also the dummy stage's bucket index over the top ib bits of out
    unsigned ib = 0;
};

// bucket capacities of the speculative final level: the sampled count scaled up, 20 % + 512 keys
// of slack (a bucket of ~4600 keys overflows with probability ~1e-10 at a 1/8 sample)
// (buckets outside [blo, bhi) -- below the input's first or above its last previous-level prefix --
// hold no key and get no slack: a round of a batched collect fills a fraction of the buckets)
// align (a speculative middle level): capacities rounded up to whole tiles of the next level's tiling
__global__ void spec_caps_kernel(const uint32_t *__restrict__ sample, uint64_t nb, uint32_t stride,
                                 uint32_t *__restrict__ cap, bool tiny, uint64_t blo, uint64_t bhi,
                                 uint32_t align = 0) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    if (b < blo || b >= bhi) {
        cap[b] = 0;
        return;
    }
    uint32_t v = tiny ? (uint32_t)(((uint64_t)sample[b] * stride) / 2)
                      : (uint32_t)(((uint64_t)sample[b] * stride * 6) / 5) + 512u;
    if (align) v = (v + align - 1) / align * align;
    cap[b] = v;
}

// the tile fill of a speculative middle level's output (tile-aligned buckets [bstart[b], bstart[b + 1]),
// keys up to cur[b]): tile t holds keys in its first tv[t] positions -- the padded-input convention of
// the next level's kernels (Ctx::gap1_tv)
__global__ void spec_tile_fill_kernel(const uint64_t *__restrict__ bstart, const unsigned long long *__restrict__ cur,
                                      uint64_t nb, uint32_t tile, uint32_t *__restrict__ tv) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const uint64_t s = bstart[b], e = bstart[b + 1], k = cur[b];
    for (uint64_t t = s / tile; t < e / tile; ++t) {
        const uint64_t t0 = t * tile;
        tv[t] = (uint32_t)(k <= t0 ? 0 : min<uint64_t>(tile, k - t0));
    }
}

// The final MSD level of the main sort (level 2 after the fused K1's level 1) without its exact
// histogram pass (msd_hist_kernel reads all N keys: 1.68 ms at configs[1]): the buckets are sized
// from a histogram of every 8th tile with slack, the partition writes into them (a reservation past
// a bucket's end is refused and flagged), and every bucket is one local_unique group whose keys end
// where its cursor stopped.  Returns the distinct count with the sorted keys in *keys, or ~0 when
// it does not apply (too little free HBM for the two slack-sized buffers) or a bucket or a group
// overflowed -- then nothing the caller needs was touched and it runs the exact level.
// spec_counts_kernel: the keys each speculative bucket received (its cursor minus its start)
__global__ void spec_counts_kernel(const uint64_t *__restrict__ bstart, const unsigned long long *__restrict__ cur,
                                   uint64_t nb, uint32_t *__restrict__ cnt) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) cnt[b] = (uint32_t)(cur[b] - bstart[b]);
}

// one workgroup per bucket over buckets [lo, hi), in launches of at most 2^22 workgroups (a grid holds
// fewer than 2^32 work-items: 2^23 buckets of 512 threads do not launch at once)
template <typename F>
static void bucket_pieces(uint64_t lo, uint64_t hi, F &&launch) {
    constexpr uint64_t CH = 1ull << 22;
    for (uint64_t g0 = lo; g0 < hi; g0 += CH) launch(g0, (unsigned)std::min(CH, hi - g0));
}

// the deferred gather of a canonical set left in bucket layout (Ctx::gap), for a consumer that reads
// it compact
static void ensure_compact(Ctx &c) {
    if (!c.gap.valid) return;
    c.gap.valid = false;
    if (!c.gap.nb) return;
    bucket_pieces(0, c.gap.nb, [&](uint64_t g0, unsigned cnt) {
        group_gather_kernel<1, false><<<dim3(cnt), dim3(256), 0, c.stream>>>(
            (const Key<1> *)c.gap.keys, nullptr, c.gap.bstart, c.gap.ustart, (Key<1> *)c.gap.dst, nullptr, nullptr, 0,
            nullptr, nullptr, g0);
        HIP_CHECK(hipGetLastError());
    });
}

// rm (the rc sort fused with the merge, distinct input): the same buckets go to local_merge_kernel,
// one bucket per group, each group's output after the canonical keys before its bucket (cidx, the
// canonical sort's bucket index) and the rc keys the buckets before it received.
template <int L, bool COUNTED>
static uint64_t spec_final_level(Ctx &c, Key<L> **keys, uint32_t **vals, uint64_t n, unsigned nbits, unsigned bp,
                                 unsigned bb, uint32_t cmax, bool distinct, RcMerge<L> *rm,
                                 const Ctx::GroupIndex &cidx, bool fine = false, Key<L> *spare = nullptr) {
    // spare (c.spec_into, uncounted): a free buffer of c.spec_into_bytes the buckets may take instead of SPEC_A
    // COUNTED: the counts travel with their keys (SPEC_AC / SPEC_BC) and add with saturation in the
    // local pass, as in the exact level (configs[4]'s counted route)
    if constexpr (L != 1) {
        return ~0ull;
    } else {
        constexpr double KB = COUNTED ? 12.0 : 8.0;  // bytes of a key and its count
        if (distinct != (rm != nullptr)) return ~0ull;  // the plain unique, or the fused rc merge
        if (rm && !c.spec_rc) return ~0ull;
        if (rm && !(cidx.keys == (const void *)rm->ck && cidx.n == rm->nc && cidx.bits == bb && cidx.nbits == nbits &&
                    bb <= 32 && (!rm->istart || rm->ib >= bb)))
            return ~0ull;
        constexpr uint32_t SS = 8;
        constexpr int TILE = MsdTraits<L>::TILE;
        // after a speculative level-1 layout the input is the padded array (Ctx::gap1_n)
        const bool g1 = bp && c.gap1_n && !rm;
        const uint64_t npos = g1 ? c.gap1_n : n;
        const uint32_t *tv = g1 ? c.gap1_tv : nullptr;
        const uint64_t tiles = ceil_div(npos, TILE);
        if (c.use_lsd || !c.spec_final || tiles < 64 * SS || bb - bp > 9 || bb > 24) return ~0ull;
        // a padded input samples every tile: its tiles' fills differ (segment tails, empty tiles), so a
        // tile-granular sample sized the buckets badly (overflow at 2 M reads)
        if (g1) fine = true;
        const uint64_t nb = 1ull << bb;
        // the deferred gather (the fused rc merge follows) leaves the distinct keys in their own buckets
        // (SPEC_B); otherwise the local unique writes over its input buckets (in place: one buffer)
        const bool gap_out = !COUNTED && c.defer_gather_req && c.defer_gather && c.want_gidx;
        const bool inplace = !rm && c.spec_inplace && !gap_out;
        if (COUNTED) spare = nullptr;
        // the slack-sized buffers must fit next to everything else
        if (!spare) {
            const uint64_t fr = c.ws.free_bytes();
            if ((double)n * KB * 1.4 * (inplace ? 1.0 : 2.0) > 0.5 * (double)fr + (double)c.ws.held_slot(Workspace::SPEC_A) +
                                                  (double)c.ws.held_slot(Workspace::SPEC_B) +
                                                  (double)c.ws.held_slot(Workspace::SPEC_AC) +
                                                  (double)c.ws.held_slot(Workspace::SPEC_BC))
                return ~0ull;
        }
        uint32_t *h = (uint32_t *)c.ws.get(Workspace::MSD_COUNTS, nb * 4);
        HIP_CHECK(hipMemsetAsync(h, 0, nb * 4, c.stream));
        // 2 levels: every 8th tile (level-1 buckets span hundreds of tiles); 3 levels: the first 1/8 of every
        // tile (level-2 buckets can be only a few tiles long, and a tile-granular sample missed them)
        constexpr uint32_t GT = 8;  // fine sample: tiles per workgroup (one LDS window flush)
        msd_hist_kernel<L><<<dim3((unsigned)(fine ? ceil_div(tiles, GT) : ceil_div(tiles, SS))), dim3(MSD_BLOCK), 0,
                             c.stream>>>(*keys, npos, nbits, bb, bp, h, fine ? 1 : SS, fine ? SS : 1, fine ? GT : 1, tv);
        HIP_CHECK(hipGetLastError());
        // the buckets the keys can occupy: those under the previous level's first and last prefix
        // (a padded input's ends are not keys: every bucket)
        uint64_t blo = 0, bhi = nb;
        if (g1 && c.gap1_hi > c.gap1_lo) {  // a speculative middle level's output: its key range is known
            blo = c.gap1_lo << (bb - bp);
            bhi = std::min<uint64_t>(nb, c.gap1_hi << (bb - bp));
        } else if (bp && !g1) {
            Key<L> ends[2];
            HIP_CHECK(hipMemcpyAsync(&ends[0], *keys, sizeof(Key<L>), hipMemcpyDeviceToHost, c.stream));
            HIP_CHECK(hipMemcpyAsync(&ends[1], *keys + (n - 1), sizeof(Key<L>), hipMemcpyDeviceToHost, c.stream));
            HIP_CHECK(hipStreamSynchronize(c.stream));
            blo = (ends[0].w[0] >> (nbits - bp)) << (bb - bp);
            bhi = std::min<uint64_t>(nb, ((ends[1].w[0] >> (nbits - bp)) + 1) << (bb - bp));
        }
        uint32_t *cap = (uint32_t *)c.ws.get(Workspace::SPEC_CAP, nb * 4);
        spec_caps_kernel<<<dim3((unsigned)ceil_div(nb, 256)), dim3(256), 0, c.stream>>>(h, nb, SS, cap, c.spec_tiny,
                                                                                        blo, bhi);
        HIP_CHECK(hipGetLastError());
        uint64_t *bstart = (uint64_t *)c.ws.get(Workspace::MSD_BSTART, (nb + 1) * 8);
        {
            uint32_t ep;
            const uint64_t st = ceil_div(nb, 4096);
            uint64_t *desc = acquire_desc(c, st, &ep);
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(cap, nb, bstart, desc, ep,
                                                                              &c.small->counter, &c.small->error);
            HIP_CHECK(hipGetLastError());
        }
        const uint64_t C = read_u64(c, (const unsigned long long *)(bstart + nb));
        if (spare && C * sizeof(Key<L>) > c.spec_into_bytes) spare = nullptr;
        if (!spare) {  // the capacity is known now: both slack-sized buffers (one: fused rc merge, in place) must fit
            const uint64_t fr = c.ws.free_bytes();
            const double need = (double)C * KB * (rm || inplace ? 1.0 : 2.0);
            const double have = 0.9 * (double)fr + (double)c.ws.held_slot(Workspace::SPEC_A) +
                                (double)c.ws.held_slot(Workspace::SPEC_AC) +
                                (rm ? 0.0 : (double)c.ws.held_slot(Workspace::SPEC_B) +
                                                (double)c.ws.held_slot(Workspace::SPEC_BC));
            if (need > have) {
                if (c.debug) fprintf(stderr, "[mtg debug] speculative level: capacity %lu does not fit, exact level\n",
                                     (unsigned long)C);
                return ~0ull;
            }
        }
        Key<L> *sa = spare ? spare : (Key<L> *)c.ws.get(Workspace::SPEC_A, C * sizeof(Key<L>));
        uint32_t *sac = COUNTED ? (uint32_t *)c.ws.get(Workspace::SPEC_AC, C * 4) : nullptr;
        auto *cur = (unsigned long long *)c.ws.get(Workspace::SPEC_CUR, nb * 8);
        HIP_CHECK(hipMemcpyAsync(cur, bstart, nb * 8, hipMemcpyDeviceToDevice, c.stream));
        HIP_CHECK(hipMemsetAsync(&c.small->spec_ovf, 0, 4, c.stream));
        EventTimer tm(c.stream);
        tm.mark();
        msd_partition_kernel<L, COUNTED><<<dim3((unsigned)xcd_grid(tiles)), dim3(MSD_BLOCK), 0, c.stream>>>(
            *keys, sa, COUNTED ? *vals : nullptr, sac, npos, nbits, bb, bp, cur, 1,
            (const unsigned long long *)(bstart + 1), &c.small->spec_ovf, tv);
        HIP_CHECK(hipGetLastError());
        tm.mark();
        uint32_t povf = 0;
        HIP_CHECK(hipMemcpyAsync(&povf, &c.small->spec_ovf, 4, hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));
        if (c.track_partition && c.radix_launches == 0) {
            c.radix_ms += tm.ms(0, 1);
            c.radix_launches += 1;
            c.radix_bytes += 2.0 * n * KB;
        }
        if (povf) {
            if (c.debug) fprintf(stderr, "[mtg debug] speculative level: a bucket overflowed, exact level\n");
            c.radix_ms = 0, c.radix_launches = 0, c.radix_bytes = 0;
            ++c.timings.spec_fallbacks;
            return ~0ull;
        }
        // g1: the padded input stays marked (Ctx::gap1_n) until this level succeeds -- a local pass that
        // overflows below returns ~0 and the caller's exact level must read the padded array again
        auto consumed_gap1 = [&]() {
            if (g1) c.gap1_n = 0, c.gap1_tv = nullptr, c.gap1_lo = c.gap1_hi = 0;  // the buckets below are compact per bucket
        };
        if (rm) {  // the fused rc merge over the speculative buckets
            uint32_t *cnt = (uint32_t *)c.ws.get(Workspace::SPEC_CAP, nb * 4);
            spec_counts_kernel<<<dim3((unsigned)ceil_div(nb, 256)), dim3(256), 0, c.stream>>>(bstart, cur, nb, cnt);
            HIP_CHECK(hipGetLastError());
            uint64_t *gbase = (uint64_t *)c.ws.get(Workspace::MSD_USTART, (nb + 1) * 8);
            {
                uint32_t ep;
                const uint64_t st = ceil_div(nb, 4096);
                uint64_t *desc = acquire_desc(c, st, &ep);
                HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
                scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(cnt, nb, gbase, desc, ep,
                                                                                  &c.small->counter, &c.small->error);
                HIP_CHECK(hipGetLastError());
            }
            constexpr int CAP = MergeLocalTraits<L>::CAP;
            uint32_t *olist = (uint32_t *)c.ws.get(Workspace::MSD_OVF, nb * 4);  // the overflowing groups
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            uint64_t *istart = rm->istart;
            // the canonical keys where they are: compact, or still in their own bucket layout (c.gap,
            // whose compact index is cidx.start)
            const bool gapped = c.gap.valid && c.gap.dst == (const void *)rm->ck;
            const Key<L> *ck = gapped ? (const Key<L> *)c.gap.keys : rm->ck;
            const uint64_t *cgap = gapped ? c.gap.bstart : nullptr;
            // only the buckets either key set can occupy (a rank of a multi-GPU build owns ~1/P of them: the
            // other workgroups only wrote index entries, 0.8 ms a rank-step at P = 8); the index entries
            // outside them are 0 below and the merged count above
            uint64_t mlo = 0, mhi = nb;
            if (bp && !g1 && !gapped && rm->nc) {
                Key<L> e[4];
                HIP_CHECK(hipMemcpyAsync(&e[0], *keys, sizeof(Key<L>), hipMemcpyDeviceToHost, c.stream));
                HIP_CHECK(hipMemcpyAsync(&e[1], *keys + (n - 1), sizeof(Key<L>), hipMemcpyDeviceToHost, c.stream));
                HIP_CHECK(hipMemcpyAsync(&e[2], rm->ck, sizeof(Key<L>), hipMemcpyDeviceToHost, c.stream));
                HIP_CHECK(hipMemcpyAsync(&e[3], rm->ck + (rm->nc - 1), sizeof(Key<L>), hipMemcpyDeviceToHost, c.stream));
                HIP_CHECK(hipStreamSynchronize(c.stream));
                auto top = [&](const Key<L> &x) { return bits_at(shr(x, nbits - bp), 0, 32); };
                mlo = std::min(top(e[0]), top(e[2])) << (bb - bp);
                mhi = std::min<uint64_t>(nb, (std::max(top(e[1]), top(e[3])) + 1) << (bb - bp));
                if (istart && mlo < mhi) {
                    const uint64_t ilo = mlo << (rm->ib - bb), ihi = mhi << (rm->ib - bb), iend = 1ull << rm->ib;
                    if (ilo) fill_u64_kernel<<<dim3((unsigned)std::min<uint64_t>(ceil_div(ilo, 256), 4096)), dim3(256), 0,
                                               c.stream>>>(istart, 0, ilo, 0);
                    if (ihi < iend)
                        fill_u64_kernel<<<dim3((unsigned)std::min<uint64_t>(ceil_div(iend - ihi, 256), 4096)), dim3(256),
                                          0, c.stream>>>(istart, ihi, iend, n + rm->nc);
                    HIP_CHECK(hipGetLastError());
                } else if (mlo >= mhi) {
                    mlo = 0, mhi = nb;
                }
            }
            bucket_pieces(mlo, mhi, [&](uint64_t g0, unsigned cnt) {
                local_merge_kernel<L, COUNTED, CAP><<<dim3(cnt), dim3(512), 0, c.stream>>>(
                    sa, sac, bstart, nullptr, nullptr, ck, rm->cv, cidx.start, rm->out, rm->outc, olist,
                    &c.small->counter, bb, nbits, rm->ib, istart, cur, gbase, cgap, g0, c.merge_it);
                HIP_CHECK(hipGetLastError());
            });
            uint32_t novf = 0;
            HIP_CHECK(hipMemcpyAsync(&novf, &c.small->counter, 4, hipMemcpyDeviceToHost, c.stream));
            HIP_CHECK(hipStreamSynchronize(c.stream));
            if (novf) {  // the few big groups again with twice the LDS arrays, from the device-side list
                const uint32_t nlist = novf;
                HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
                bucket_pieces(0, nlist, [&](uint64_t g0, unsigned cnt) {
                    local_merge_kernel<L, COUNTED, 2 * CAP><<<dim3(cnt), dim3(512), 0, c.stream>>>(
                        sa, sac, bstart, nullptr, olist + g0, ck, rm->cv, cidx.start, rm->out, rm->outc, nullptr,
                        &c.small->counter, bb, nbits, rm->ib, istart, cur, gbase, cgap, 0, c.merge_it);
                    HIP_CHECK(hipGetLastError());
                });
                HIP_CHECK(hipMemcpyAsync(&novf, &c.small->counter, 4, hipMemcpyDeviceToHost, c.stream));
                HIP_CHECK(hipStreamSynchronize(c.stream));
            }
            if (novf) {
                if (c.debug) fprintf(stderr, "[mtg debug] speculative rc level: %u groups overflowed, exact level\n", novf);
                c.radix_ms = 0, c.radix_launches = 0, c.radix_bytes = 0;
                ++c.timings.spec_fallbacks;
                return ~0ull;
            }
            rm->done = true;
            ++c.timings.spec_levels;
            if (fine) ++c.timings.spec_fine_levels;
            if (gapped) c.gap.valid = false;  // merged: the canonical set is not needed compact
            if (istart) {  // index end = the merged count (a kernel argument: no host copy to wait for)
                const uint64_t R = n + rm->nc;
                set_u64_kernel<<<dim3(1), dim3(1), 0, c.stream>>>(istart + (1ull << rm->ib), R);
                HIP_CHECK(hipGetLastError());
                note_bucket_index(c, rm->out, R, istart, nbits - rm->ib);
            }
            if (c.debug)
                fprintf(stderr, "[mtg debug] speculative rc level: n=%lu capacity=%lu -> merged %lu\n", (unsigned long)n,
                        (unsigned long)C, (unsigned long)(n + rm->nc));
            return n;
        }
        // every bucket one group: [bstart[b], cur[b])
        Key<L> *sb = inplace ? sa : (Key<L> *)c.ws.get(Workspace::SPEC_B, C * sizeof(Key<L>));
        uint32_t *sbc = !COUNTED ? nullptr : inplace ? sac : (uint32_t *)c.ws.get(Workspace::SPEC_BC, C * 4);
        uint32_t *ucount = (uint32_t *)c.ws.get(Workspace::MSD_UCOUNT, (nb + 1) * 4);
        uint32_t *ovf = (uint32_t *)c.ws.get(Workspace::MSD_OVF, nb * 4);
        HIP_CHECK(hipMemsetAsync(ovf, 0, nb * 4, c.stream));
        HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
        const bool keycas = nbits < 64;
        constexpr int WPE = COUNTED ? 1 : MTG_LU_WPE;  // (the uncounted table fits 8 waves per SIMD at 64 VGPRs)
        // only the buckets the keys can occupy (blo, bhi above; a round of the batched collect fills a
        // fraction of them); the others count 0 keys
        HIP_CHECK(hipMemsetAsync(ucount, 0, (nb + 1) * 4, c.stream));
        bucket_pieces(blo, bhi, [&](uint64_t g0, unsigned cnt) {
            if (keycas && c.lu_fast)
                local_unique_kernel<1, COUNTED, true, 512, LocalTraits<1>::SLOTS / 2, false, WPE, true, false>
                    <<<dim3(cnt), dim3(512), 0, c.stream>>>(sa, sac, bstart, nullptr, nbits, bb, 0, sb, sbc, ucount, ovf,
                                                            &c.small->counter, cmax, cur, g0);
            else if (keycas)
                local_unique_kernel<1, COUNTED, true, 512, LocalTraits<1>::SLOTS / 2, false, WPE>
                    <<<dim3(cnt), dim3(512), 0, c.stream>>>(sa, sac, bstart, nullptr, nbits, bb, 0, sb, sbc, ucount, ovf,
                                                            &c.small->counter, cmax, cur, g0);
            else
                local_unique_kernel<1, COUNTED, false, 512, LocalTraits<1>::SLOTS / 2, false, 1>
                    <<<dim3(cnt), dim3(512), 0, c.stream>>>(sa, sac, bstart, nullptr, nbits, bb, 0, sb, sbc, ucount, ovf,
                                                            &c.small->counter, cmax, cur, g0);
            HIP_CHECK(hipGetLastError());
        });
        uint32_t novf = 0;
        HIP_CHECK(hipMemcpyAsync(&novf, &c.small->counter, 4, hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));
        if (c.spec_lu_fail) novf = 1;  // MTG_SPEC_LU_FAIL=1 (tests): as if a group had overflowed
        if (novf) {
            if (c.debug) fprintf(stderr, "[mtg debug] speculative level: %u groups overflowed, exact level\n", novf);
            c.radix_ms = 0, c.radix_launches = 0, c.radix_bytes = 0;
            ++c.timings.spec_fallbacks;
            return ~0ull;
        }
        uint64_t *ustart = (uint64_t *)c.ws.get(Workspace::MSD_USTART, (nb + 1) * 8);
        {
            uint32_t ep;
            const uint64_t st = ceil_div(nb, 4096);
            uint64_t *desc = acquire_desc(c, st, &ep);
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(ucount, nb, ustart, desc, ep,
                                                                              &c.small->counter, &c.small->error);
            HIP_CHECK(hipGetLastError());
        }
        if (!COUNTED && c.defer_gather_req && c.defer_gather && c.want_gidx) {
            // the fused rc merge follows: leave the distinct keys in their buckets (Ctx::gap); the
            // compact index of bucket g is ustart[g] (one bucket per group)
            uint64_t *gb = (uint64_t *)c.ws.get(Workspace::GAP_BSTART, (nb + 1) * 8);
            uint64_t *gu = (uint64_t *)c.ws.get(Workspace::GAP_USTART, (nb + 2) * 8);
            HIP_CHECK(hipMemcpyAsync(gb, bstart, (nb + 1) * 8, hipMemcpyDeviceToDevice, c.stream));
            HIP_CHECK(hipMemcpyAsync(gu, ustart, (nb + 1) * 8, hipMemcpyDeviceToDevice, c.stream));
            HIP_CHECK(hipMemcpyAsync(gu + nb + 1, ustart + nb, 8, hipMemcpyDeviceToDevice, c.stream));
            const uint64_t u = read_u64(c, (const unsigned long long *)(ustart + nb));
            c.gap = Ctx::GappedSet{true, sb, *keys, u, nb, gb, gu};
            consumed_gap1();
            ++c.timings.spec_levels;
            if (fine) ++c.timings.spec_fine_levels;
            c.gidx = Ctx::GroupIndex{*keys, u, bb, nbits, gu};
            if (c.debug)
                fprintf(stderr, "[mtg debug] speculative level: n=%lu capacity=%lu (%.2fx) -> %lu distinct, left in buckets\n",
                        (unsigned long)n, (unsigned long)C, (double)C / (double)n, (unsigned long)u);
            return u;
        }
        const bool index = c.want_gidx;
        // a collect round's share of the whole set's index (Ctx::ridx), its buckets 2^(bits - bb) a group
        const bool rindex = !index && c.ridx.start && bb <= c.ridx.bits;
        uint64_t *gi = index ? (uint64_t *)c.ws.get(Workspace::CANON_IDX, (nb + 2) * 8) : rindex ? c.ridx.start : nullptr;
        const unsigned ib = rindex ? c.ridx.bits : bb;
        if (index || rindex) HIP_CHECK(hipMemsetAsync(&c.small->gidx_bad, 0, 4, c.stream));
        if (c.sort_out && (c.sort_out_cap == ~0ull || read_u64(c, (const unsigned long long *)(ustart + nb)) <= c.sort_out_cap)) {
            *keys = (Key<L> *)c.sort_out;  // (the caller's destination: the input is no longer read)
            if (COUNTED) *vals = c.sort_out_vals;
        }
        bucket_pieces(0, nb, [&](uint64_t g0, unsigned cnt) {
            group_gather_kernel<L, COUNTED><<<dim3(cnt), dim3(256), 0, c.stream>>>(
                sb, sbc, bstart, ustart, *keys, COUNTED ? *vals : nullptr, nullptr, nbits - ib, gi, &c.small->gidx_bad,
                g0, ib - bb, rindex ? c.ridx.off : 0, rindex ? c.ridx.lo : 0, rindex ? c.ridx.hi : ~0ull);
            HIP_CHECK(hipGetLastError());
        });
        uint64_t u = 0;
        uint32_t ibad = 0;
        HIP_CHECK(hipMemcpyAsync(&u, ustart + nb, 8, hipMemcpyDeviceToHost, c.stream));
        if (index) {
            HIP_CHECK(hipMemcpyAsync(gi + nb, ustart + nb, 8, hipMemcpyDeviceToDevice, c.stream));
            HIP_CHECK(hipMemcpyAsync(gi + nb + 1, ustart + nb, 8, hipMemcpyDeviceToDevice, c.stream));
        }
        if (index || rindex) HIP_CHECK(hipMemcpyAsync(&ibad, &c.small->gidx_bad, 4, hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));
        if (index && !ibad) c.gidx = Ctx::GroupIndex{*keys, u, bb, nbits, gi};
        if (rindex) c.ridx.written = !ibad;
        consumed_gap1();
        ++c.timings.spec_levels;
        if (fine) ++c.timings.spec_fine_levels;
        if (c.debug)
            fprintf(stderr, "[mtg debug] speculative level: n=%lu capacity=%lu (%.2fx) -> %lu distinct\n",
                    (unsigned long)n, (unsigned long)C, (double)C / (double)n, (unsigned long)u);
        return u;
    }
}

// The middle level of a 3-level sort without its exact histogram pass (a 60 GB read per configs[3]
// round): the level-2 buckets are sized from a sample with slack and rounded up to whole tiles of the
// level-3 tiling, the keys go from *keys into them in *alt (the caller's buffer of c.spec_mid_bytes,
// Ctx::spec_mid_into), and the padded result is marked for level 3 as the speculative level-1 layout is
// for level 2 (Ctx::gap1_n / gap1_tv: tile t holds keys in its first tv[t] positions), with the
// level-2 prefix range of the keys (gap1_lo / gap1_hi) for level 3's bucket range.  False (nothing the
// caller needs touched) when it does not fit or a bucket overflowed: the exact level then.
template <int L, bool COUNTED>
static bool spec_mid_level(Ctx &c, Key<L> **keys, Key<L> **alt, uint64_t n, unsigned nbits, unsigned bp, unsigned bb) {
    if constexpr (L != 1 || COUNTED) {
        return false;
    } else {
        constexpr int TILE = MsdTraits<L>::TILE;
        constexpr uint32_t SS = 8;
        const uint64_t tiles = ceil_div(n, TILE);
        if (c.use_lsd || !c.spec_final || tiles < 64 * SS || bb - bp > 9 || bb > 24 || !bp) return false;
        const uint64_t nb = 1ull << bb;
        uint32_t *h = (uint32_t *)c.ws.get(Workspace::MSD_COUNTS, nb * 4);
        HIP_CHECK(hipMemsetAsync(h, 0, nb * 4, c.stream));
        // every 8th tile (level-1 buckets span hundreds of tiles here)
        msd_hist_kernel<L><<<dim3((unsigned)ceil_div(tiles, SS)), dim3(MSD_BLOCK), 0, c.stream>>>(*keys, n, nbits, bb, bp, h,
                                                                                                SS, 1, 1, nullptr);
        HIP_CHECK(hipGetLastError());
        Key<L> ends[2];
        HIP_CHECK(hipMemcpyAsync(&ends[0], *keys, sizeof(Key<L>), hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipMemcpyAsync(&ends[1], *keys + (n - 1), sizeof(Key<L>), hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));
        const uint64_t lo1 = ends[0].w[0] >> (nbits - bp), hi1 = ends[1].w[0] >> (nbits - bp);
        const uint64_t blo = lo1 << (bb - bp), bhi = std::min<uint64_t>(nb, (hi1 + 1) << (bb - bp));
        uint32_t *cap = (uint32_t *)c.ws.get(Workspace::SPEC_CAP, nb * 4);
        spec_caps_kernel<<<dim3((unsigned)ceil_div(nb, 256)), dim3(256), 0, c.stream>>>(h, nb, SS, cap, c.spec_tiny, blo,
                                                                                        bhi, (uint32_t)TILE);
        HIP_CHECK(hipGetLastError());
        uint64_t *bstart = (uint64_t *)c.ws.get(Workspace::MSD_BSTART, (nb + 1) * 8);
        {
            uint32_t ep;
            const uint64_t st = ceil_div(nb, 4096);
            uint64_t *desc = acquire_desc(c, st, &ep);
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(cap, nb, bstart, desc, ep,
                                                                              &c.small->counter, &c.small->error);
            HIP_CHECK(hipGetLastError());
        }
        const uint64_t C = read_u64(c, (const unsigned long long *)(bstart + nb));
        if (C * sizeof(Key<L>) > c.spec_mid_bytes) {
            if (c.debug) fprintf(stderr, "[mtg debug] speculative middle level: capacity %lu does not fit\n", (unsigned long)C);
            return false;
        }
        auto *cur = (unsigned long long *)c.ws.get(Workspace::SPEC_CUR, nb * 8);
        HIP_CHECK(hipMemcpyAsync(cur, bstart, nb * 8, hipMemcpyDeviceToDevice, c.stream));
        HIP_CHECK(hipMemsetAsync(&c.small->spec_ovf, 0, 4, c.stream));
        msd_partition_kernel<L, false><<<dim3((unsigned)xcd_grid(tiles)), dim3(MSD_BLOCK), 0, c.stream>>>(
            *keys, *alt, nullptr, nullptr, n, nbits, bb, bp, cur, 1, (const unsigned long long *)(bstart + 1),
            &c.small->spec_ovf, nullptr);
        HIP_CHECK(hipGetLastError());
        const uint64_t ntv = C / TILE;
        uint32_t *tv = (uint32_t *)c.ws.get(Workspace::SPEC_MID_TV, std::max<uint64_t>(ntv, 1) * 4);
        spec_tile_fill_kernel<<<dim3((unsigned)ceil_div(nb, 256)), dim3(256), 0, c.stream>>>(bstart, cur, nb, TILE, tv);
        HIP_CHECK(hipGetLastError());
        uint32_t povf = 0;
        HIP_CHECK(hipMemcpyAsync(&povf, &c.small->spec_ovf, 4, hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));
        if (povf) {
            if (c.debug) fprintf(stderr, "[mtg debug] speculative middle level: a bucket overflowed, exact level\n");
            ++c.timings.spec_fallbacks;
            return false;
        }
        std::swap(*keys, *alt);
        c.gap1_n = C;
        c.gap1_tv = tv;
        c.gap1_lo = blo, c.gap1_hi = bhi;
        ++c.timings.spec_levels;
        if (c.debug)
            fprintf(stderr, "[mtg debug] speculative middle level: n=%lu capacity=%lu (%.2fx)\n", (unsigned long)n,
                    (unsigned long)C, (double)C / (double)n);
        return true;
    }
}

template <int L, bool COUNTED>
static uint64_t msd_sort_unique(Ctx &c, Key<L> **keys, Key<L> **alt, uint32_t **vals,
                                uint32_t **valt, uint64_t n, unsigned nbits, uint32_t cmax,
                                double dup, const uint32_t *hist1 = nullptr, bool distinct = false,
                                const std::vector<uint64_t> *runs = nullptr, bool level1_done = false,
                                RcMerge<L> *rm = nullptr, const MsdPlan *force_plan = nullptr) {
    // level1_done: the producer already scattered the keys by the plan's level-1 digit
    // (extract_partition_kernel); hist1 holds that level's counts
    // hist1: counts of the top plan.digit_end[1] bits of the input, when its producer made them;
    // distinct: the input has no duplicates (the local pass skips its hash table);
    // runs: the input is runs->size() - 1 sorted runs at these offsets (one gather replaces
    // the partition passes)
    const Ctx::GroupIndex saved_gidx = c.gidx;  // the canonical sort's, for the fused rc merge below
    c.gidx = Ctx::GroupIndex{};
    if (n == 0) return 0;
    // *alt == nullptr (the single build after the speculative level-1 layout): the ping-pong buffer is taken
    // only by a path that needs it -- an exact level or the group passes -- never by the speculative level
    auto lazy_alt = [&]() {
        if (!*alt) *alt = (Key<L> *)c.ws.get(Workspace::KB, n * sizeof(Key<L>));
        if (COUNTED && !*valt) *valt = (uint32_t *)c.ws.get(Workspace::CB, n * 4);
    };
    constexpr uint32_t LIMIT = LocalTraits<L>::LIMIT;
    constexpr int TILE = MsdTraits<L>::TILE;
    const uint64_t tiles = ceil_div(n, TILE);
    // force_plan: the caller fixed the digits (the routed multi-GPU collect: level 1 is the routing digit)
    const MsdPlan plan = force_plan ? *force_plan : msd_plan<L>(c, n, nbits, dup);
    unsigned levels = plan.levels;
    unsigned digit_end[4] = {plan.digit_end[0], plan.digit_end[1], plan.digit_end[2], plan.digit_end[3]};
    unsigned b = 0;
    uint64_t *bstart = nullptr;
    uint64_t nbuckets = 1;
    auto run_level = [&](unsigned lev) {
        if (digit_end[lev] == 0) digit_end[lev] = std::min(nbits, digit_end[lev - 1] + 8);
        const unsigned bb = digit_end[lev], bp = digit_end[lev - 1];
        nbuckets = 1ull << bb;
        const uint32_t *cnt = hist1;
        // level 2 after a speculative level-1 layout reads the padded array (c.gap1_n positions), and so
        // does level 3 after a speculative middle level (spec_mid_level)
        const bool g1 = c.gap1_n && (lev == 2 ? level1_done : lev == 3);
        const uint64_t npos = g1 ? c.gap1_n : n, ltiles = g1 ? ceil_div(npos, TILE) : tiles;
        const uint32_t *tv = g1 ? c.gap1_tv : nullptr;
        if (lev != 1 || !hist1) {
            uint32_t *h = (uint32_t *)c.ws.get(Workspace::MSD_COUNTS, nbuckets * 4);
            HIP_CHECK(hipMemsetAsync(h, 0, nbuckets * 4, c.stream));
            if (bp == 0 && nbuckets <= 512) {
                const uint32_t nrows = (uint32_t)std::min<uint64_t>(tiles, 8192);
                uint32_t *rows = (uint32_t *)c.ws.get(Workspace::HIST_ROWS, (uint64_t)nrows * nbuckets * 4);
                msd_hist_rows_kernel<L><<<dim3(nrows), dim3(512), 0, c.stream>>>(*keys, n, nbits, bb, rows);
                HIP_CHECK(hipGetLastError());
                hist_rows_reduce_kernel<<<dim3(std::min<uint32_t>(nrows, 256), (unsigned)ceil_div(nbuckets, 256)),
                                          dim3(256), 0, c.stream>>>(rows, nrows, (uint32_t)nbuckets, h);
            } else {
                msd_hist_kernel<L><<<dim3((unsigned)ltiles), dim3(MSD_BLOCK), 0, c.stream>>>(*keys, npos, nbits, bb, bp,
                                                                                             h, 1, 1, 1, tv);
            }
            HIP_CHECK(hipGetLastError());
            cnt = h;
        }
        bstart = (uint64_t *)c.ws.get(Workspace::MSD_BSTART, (nbuckets + 1) * 8);
        uint32_t ep;
        const uint64_t st = ceil_div(nbuckets, 4096);
        uint64_t *desc = acquire_desc(c, st, &ep);
        HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
        scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(cnt, nbuckets, bstart, desc, ep,
                                                                      &c.small->counter, &c.small->error);
        HIP_CHECK(hipGetLastError());
        if (lev == 1 && level1_done) {
            b = bb;
            return;
        }
        lazy_alt();  // (a partition level writes *alt)
        auto *cur = (unsigned long long *)c.ws.get(Workspace::MSD_CURSOR, nbuckets * 8);
        HIP_CHECK(hipMemcpyAsync(cur, bstart, nbuckets * 8, hipMemcpyDeviceToDevice, c.stream));
        EventTimer tm(c.stream);
        tm.mark();
        // 512-thread tiles (8 K keys, two workgroups per CU) on XCD-contiguous tiles: 3.77 ms for the
        // cfg2 level-2 pass vs 4.09 with 1024-thread tiles (16 K keys, one per CU) -- before the XCD
        // mapping the longer runs of the big tiles won (4.65 vs 5.3 ms); nontemporal access measured
        // the same (tools/part_bench.hip)
        msd_partition_kernel<L, COUNTED><<<dim3((unsigned)xcd_grid(ltiles)), dim3(MSD_BLOCK), 0, c.stream>>>(
            *keys, *alt, COUNTED ? *vals : nullptr, COUNTED ? *valt : nullptr, npos, nbits, bb, bp, cur, 1, nullptr,
            nullptr, tv);
        HIP_CHECK(hipGetLastError());
        if (g1) c.gap1_n = 0, c.gap1_tv = nullptr, c.gap1_lo = c.gap1_hi = 0;  // compact from here on
        tm.mark();
        if (c.track_partition && c.radix_launches == 0) {  // first partition launch of the sort
            HIP_CHECK(hipStreamSynchronize(c.stream));
            c.radix_ms += tm.ms(0, 1);
            c.radix_launches += 1;
            c.radix_bytes += 2.0 * n * (sizeof(Key<L>) + (COUNTED ? 4 : 0));
        }
        std::swap(*keys, *alt);
        if (COUNTED) std::swap(*vals, *valt);
        b = bb;
    };
    if (runs && runs->size() >= 2 && runs->size() <= 129 && levels) {
        lazy_alt();
        // bucket layout of the top T bits straight from the runs' own order
        const unsigned T = digit_end[levels];
        const uint32_t P = (uint32_t)runs->size() - 1;
        nbuckets = 1ull << T;
        uint64_t *idx = (uint64_t *)c.ws.get(Workspace::RUN_IDX, (uint64_t)P * (nbuckets + 1) * 8);
        int64_t *delta = (int64_t *)c.ws.get(Workspace::RUN_DELTA, (uint64_t)P * nbuckets * 8);
        for (uint32_t j = 0; j < P; ++j) {
            const uint64_t r0 = (*runs)[j], rn = (*runs)[j + 1] - r0;
            bucket_index<L>(c, *keys + r0, rn, nbits - T, nbuckets, idx + (uint64_t)j * (nbuckets + 1));
        }
        bstart = (uint64_t *)c.ws.get(Workspace::MSD_BSTART, (nbuckets + 1) * 8);
        runs_delta_kernel<<<dim3((unsigned)std::min<uint64_t>(ceil_div(nbuckets + 1, 256), 16384)), dim3(256), 0,
                            c.stream>>>(idx, P, nbuckets, bstart, delta);
        HIP_CHECK(hipGetLastError());
        uint64_t *droff = (uint64_t *)c.ws.get(Workspace::RUN_OFF, (P + 1) * 8);
        HIP_CHECK(hipMemcpyAsync(droff, runs->data(), (P + 1) * 8, hipMemcpyHostToDevice, c.stream));
        runs_gather_kernel<L, COUNTED><<<dim3((unsigned)std::min<uint64_t>(ceil_div(n, 256), 65536)), dim3(256), 0,
                                         c.stream>>>(*keys, COUNTED ? *vals : nullptr, n, droff, P, delta,
                                                     nbuckets, nbits, T, *alt, COUNTED ? *valt : nullptr);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipStreamSynchronize(c.stream));  // `runs` is the caller's host vector
        std::swap(*keys, *alt);
        if (COUNTED) std::swap(*vals, *valt);
        b = T;
    } else {
        for (unsigned lev = 1; lev <= levels; ++lev) {
            // the last of 2 or 3 levels, the ones before it in place (3 levels: inputs over ~1.6e9 keys)
            // (any plain sort + unique too: configs[4]'s KMC records have no fused level 1)
            if (lev == levels && lev >= 2 && (lev == 2 || c.spec3) && (level1_done || (rm && distinct) || (!rm && !distinct))) {
                // the per-tile (fine) sample when the previous level's buckets span few tiles: 3 levels, or
                // a 10-bit level 1 on a small input (a tile-granular sample of ~30 tiles a bucket missed
                // by up to ~25 %)
                const bool fine = lev >= 3 || (n >> digit_end[lev - 1]) < 64ull * MsdTraits<L>::TILE;
                // the caller's spare buffer (c.spec_into) once level 2 has moved the keys out of it
                Key<L> *spare = lev >= 3 && c.spec_into && c.spec_into != (void *)*keys ? (Key<L> *)c.spec_into : nullptr;
                const uint64_t u = spec_final_level<L, COUNTED>(c, keys, vals, n, nbits, digit_end[lev - 1],
                                                                digit_end[lev], cmax, distinct, rm, saved_gidx, fine,
                                                                spare);
                if (u != ~0ull) return u;
            }
            // a 3-level sort's middle level without its histogram pass, into the caller's buffer
            if (lev == 2 && levels == 3 && level1_done && !c.gap1_n && c.spec_mid && c.spec3 && *alt &&
                c.spec_mid_into == (void *)*alt &&
                spec_mid_level<L, COUNTED>(c, keys, alt, n, nbits, digit_end[1], digit_end[2])) {
                b = digit_end[2];
                continue;
            }
            run_level(lev);
        }
    }

    lazy_alt();
    while (true) {
        // groups of consecutive buckets holding <= G keys; bigger buckets stand alone
        const uint64_t G = LIMIT / 4;
        uint64_t ngroups = 1;
        uint64_t *gstart;
        const uint64_t *gbucket_out = nullptr;
        if (b == 0) {
            gstart = (uint64_t *)c.ws.get(Workspace::MSD_GSTART, 16);
            set_pair_kernel<<<1, 1, 0, c.stream>>>(gstart, 0, n);
            HIP_CHECK(hipGetLastError());
        } else {
            uint32_t *gf = (uint32_t *)c.ws.get(Workspace::MSD_UCOUNT, (nbuckets + 1) * 4);
            const bool fuse = rm && distinct && b <= 32;
            uint64_t *cstart = nullptr;
            const uint64_t *gsize = bstart;
            if (fuse) {
                ensure_compact(c);  // this path reads the canonical keys compact
                // fused rc merge: the canonical keys of every bucket (bucket index of the sorted
                // set), and groups sized by rc + canonical keys together
                if (saved_gidx.keys == (const void *)rm->ck && saved_gidx.n == rm->nc && saved_gidx.bits == b &&
                    saved_gidx.nbits == nbits) {
                    cstart = const_cast<uint64_t *>(saved_gidx.start);  // the canonical sort's group starts
                } else {
                    cstart = (uint64_t *)c.ws.get(Workspace::RC_CSTART, (nbuckets + 2) * 8);
                    bucket_index<L>(c, rm->ck, rm->nc, nbits - b, nbuckets, cstart);
                }
                uint64_t *comb = (uint64_t *)c.ws.get(Workspace::RC_COMB, (nbuckets + 1) * 8);
                add_starts_kernel<<<dim3((unsigned)ceil_div(nbuckets + 1, 256)), dim3(256), 0, c.stream>>>(
                    bstart, cstart, nbuckets + 1, comb);
                HIP_CHECK(hipGetLastError());
                gsize = comb;
            }
            group_flags_kernel<<<dim3((unsigned)ceil_div(nbuckets, 256)), dim3(256), 0, c.stream>>>(
                gsize, nbuckets, G, gf);
            HIP_CHECK(hipGetLastError());
            uint64_t *gpos = (uint64_t *)c.ws.get(Workspace::MSD_USTART, (nbuckets + 1) * 8);
            uint32_t ep;
            const uint64_t st = ceil_div(nbuckets, 4096);
            uint64_t *desc = acquire_desc(c, st, &ep);
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(gf, nbuckets, gpos, desc, ep,
                                                                          &c.small->counter, &c.small->error);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipMemcpyAsync(&ngroups, gpos + nbuckets, 8, hipMemcpyDeviceToHost, c.stream));
            HIP_CHECK(hipStreamSynchronize(c.stream));
            gstart = (uint64_t *)c.ws.get(Workspace::MSD_GSTART, (ngroups + 1) * 8);
            // each group's bucket range: the fused rc merge's canonical ranges, or the output's bucket index
            uint64_t *gbucket = b <= 32 ? (uint64_t *)c.ws.get(Workspace::MSD_GBUCKET, (ngroups + 1) * 8) : nullptr;
            gbucket_out = gbucket;
            group_scatter_kernel<<<dim3((unsigned)ceil_div(nbuckets + 1, 256)), dim3(256), 0, c.stream>>>(
                bstart, gf, gpos, nbuckets, n, gstart, gbucket);
            HIP_CHECK(hipGetLastError());
            if (fuse && ngroups) {
                // sort the rc groups and merge them with the canonical keys in one pass
                constexpr int CAP = MergeLocalTraits<L>::CAP;
                uint32_t *olist = (uint32_t *)c.ws.get(Workspace::MSD_OVF, ngroups * 4);  // overflowing groups
                HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
                uint64_t *istart = rm->istart && rm->ib >= b ? rm->istart : nullptr;
                bucket_pieces(0, ngroups, [&](uint64_t g0, unsigned cnt) {
                    local_merge_kernel<L, COUNTED, CAP><<<dim3(cnt), dim3(512), 0, c.stream>>>(
                        *keys, COUNTED ? *vals : nullptr, gstart, gbucket, nullptr, rm->ck, rm->cv, cstart, rm->out,
                        rm->outc, olist, &c.small->counter, b, nbits, rm->ib, istart, nullptr, nullptr, nullptr, g0,
                        c.merge_it);
                    HIP_CHECK(hipGetLastError());
                });
                uint32_t novf = 0;
                HIP_CHECK(hipMemcpyAsync(&novf, &c.small->counter, 4, hipMemcpyDeviceToHost, c.stream));
                HIP_CHECK(hipStreamSynchronize(c.stream));
                if (novf) {  // the few big groups again with twice the LDS arrays, from the device-side list
                    const uint32_t nlist = novf;
                    HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
                    bucket_pieces(0, nlist, [&](uint64_t g0, unsigned cnt) {
                        local_merge_kernel<L, COUNTED, 2 * CAP><<<dim3(cnt), dim3(512), 0, c.stream>>>(
                            *keys, COUNTED ? *vals : nullptr, gstart, gbucket, olist + g0, rm->ck, rm->cv, cstart,
                            rm->out, rm->outc, nullptr, &c.small->counter, b, nbits, rm->ib, istart, nullptr, nullptr,
                            nullptr, 0, c.merge_it);
                        HIP_CHECK(hipGetLastError());
                    });
                    HIP_CHECK(hipMemcpyAsync(&novf, &c.small->counter, 4, hipMemcpyDeviceToHost, c.stream));
                    HIP_CHECK(hipStreamSynchronize(c.stream));
                    if (c.debug) fprintf(stderr, "[mtg debug] rc merge: %u big groups -> %u left\n", nlist, novf);
                }
                if (!novf) {
                    rm->done = true;
                    if (istart) {  // index end = the merged count (a kernel argument: no host copy to wait for)
                        const uint64_t R = n + rm->nc;
                        set_u64_kernel<<<dim3(1), dim3(1), 0, c.stream>>>(istart + (1ull << rm->ib), R);
                        HIP_CHECK(hipGetLastError());
                        note_bucket_index(c, rm->out, R, istart, nbits - rm->ib);
                    }
                    return n;  // the rc keys (distinct); rm->out holds U + n
                }
            }
        }
        uint32_t *ucount = (uint32_t *)c.ws.get(Workspace::MSD_UCOUNT, (ngroups + 1) * 4);
        uint32_t *ovf = (uint32_t *)c.ws.get(Workspace::MSD_OVF, ngroups * 4);
        HIP_CHECK(hipMemsetAsync(ovf, 0, ngroups * 4, c.stream));
        HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
        auto launch_local = [&](const uint32_t *glist, uint64_t count, unsigned sbits) {
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            auto go = [&](auto keycas, auto sl, auto nodup) {
                constexpr bool KC = decltype(keycas)::value;
                constexpr int SL = decltype(sl)::value;
                constexpr bool ND = decltype(nodup)::value;
                constexpr int WPE = (L == 1 && KC && !ND && !COUNTED) ? MTG_LU_WPE : 1;
                bucket_pieces(0, count, [&](uint64_t g0, unsigned cnt) {
                    if constexpr (KC && !ND) {
                        if (c.lu_fast && sbits == 0) {  // the first launch: no key-range slices
                            local_unique_kernel<L, COUNTED, KC, 512, SL, ND, WPE, true, false><<<dim3(cnt), dim3(512), 0, c.stream>>>(
                                *keys, COUNTED ? *vals : nullptr, gstart, glist ? glist + g0 : nullptr, nbits, b, sbits,
                                *alt, COUNTED ? *valt : nullptr, ucount, ovf, &c.small->counter, cmax, nullptr,
                                glist ? 0 : g0);
                            return;
                        }
                        if (c.lu_fast) {
                            local_unique_kernel<L, COUNTED, KC, 512, SL, ND, WPE, true><<<dim3(cnt), dim3(512), 0, c.stream>>>(
                                *keys, COUNTED ? *vals : nullptr, gstart, glist ? glist + g0 : nullptr, nbits, b, sbits,
                                *alt, COUNTED ? *valt : nullptr, ucount, ovf, &c.small->counter, cmax, nullptr,
                                glist ? 0 : g0);
                            return;
                        }
                    }
                    // u128 keys (configs[2]): the state-word table at <= 80 VGPRs, so three workgroups fit a CU
                    // (the LDS allows three; 93 VGPRs allowed two)
                    if constexpr (L == 2 && !KC && !ND && !COUNTED) {
                        if (c.lu_wpe2) {
                            local_unique_kernel<L, COUNTED, KC, 512, SL, ND, 6><<<dim3(cnt), dim3(512), 0, c.stream>>>(
                                *keys, COUNTED ? *vals : nullptr, gstart, glist ? glist + g0 : nullptr, nbits, b, sbits,
                                *alt, COUNTED ? *valt : nullptr, ucount, ovf, &c.small->counter, cmax, nullptr,
                                glist ? 0 : g0);
                            return;
                        }
                    }
                    local_unique_kernel<L, COUNTED, KC, 512, SL, ND, WPE><<<dim3(cnt), dim3(512), 0, c.stream>>>(
                        *keys, COUNTED ? *vals : nullptr, gstart, glist ? glist + g0 : nullptr, nbits, b, sbits, *alt,
                        COUNTED ? *valt : nullptr, ucount, ovf, &c.small->counter, cmax, nullptr, glist ? 0 : g0);
                });
            };
            using T_ = std::true_type;
            using F_ = std::false_type;
            using SHalf = std::integral_constant<int, LocalTraits<L>::SLOTS / 2>;
            const bool keycas = L == 1 && nbits < 64;
            if (distinct) go(F_{}, SHalf{}, T_{});
            else if (keycas) go(T_{}, SHalf{}, F_{});
            else go(F_{}, SHalf{}, F_{});
            HIP_CHECK(hipGetLastError());
            uint32_t nov = 0;
            HIP_CHECK(hipMemcpyAsync(&nov, &c.small->counter, 4, hipMemcpyDeviceToHost, c.stream));
            HIP_CHECK(hipStreamSynchronize(c.stream));
            return nov;
        };
        uint32_t novf = launch_local(nullptr, ngroups, 0);
        if (c.trace)
            fprintf(stderr, "[mtg trace] msd n=%lu levels=%u b=%u groups=%lu overflow=%u\n", (unsigned long)n, levels, b,
                    (unsigned long)ngroups, novf);
        if (c.debug)
            fprintf(stderr, "[mtg debug] msd n=%lu nbits=%u levels=%u b=%u buckets=%lu groups=%lu overflow=%u\n",
                    (unsigned long)n, nbits, levels, b, (unsigned long)nbuckets, (unsigned long)ngroups, novf);
        // overflowing one-bucket groups: rerun them alone in 2, 4, 8, 16 key-range slices
        std::vector<uint32_t> flags;
        std::vector<uint64_t> gs;
        for (unsigned sbits = 1; novf && b && sbits <= 4 && b + sbits <= nbits; ++sbits) {
            flags.resize(ngroups);
            HIP_CHECK(hipMemcpyAsync(flags.data(), ovf, ngroups * 4, hipMemcpyDeviceToHost, c.stream));
            HIP_CHECK(hipStreamSynchronize(c.stream));
            std::vector<uint32_t> list;
            for (uint64_t g = 0; g < ngroups; ++g)
                if (flags[g]) list.push_back((uint32_t)g);
            uint32_t *dlist = (uint32_t *)c.ws.get(Workspace::MSD_GLIST, list.size() * 4);
            HIP_CHECK(hipMemcpyAsync(dlist, list.data(), list.size() * 4, hipMemcpyHostToDevice, c.stream));
            novf = launch_local(dlist, list.size(), sbits);  // syncs: `list` outlives the copy
            if (c.debug) fprintf(stderr, "[mtg debug]   sliced rerun sbits=%u groups=%zu -> overflow=%u\n", sbits, list.size(), novf);
        }
        if (novf) {
            flags.resize(ngroups);
            gs.resize(ngroups + 1);
            HIP_CHECK(hipMemcpyAsync(flags.data(), ovf, ngroups * 4, hipMemcpyDeviceToHost, c.stream));
            HIP_CHECK(hipMemcpyAsync(gs.data(), gstart, (ngroups + 1) * 8, hipMemcpyDeviceToHost, c.stream));
            HIP_CHECK(hipStreamSynchronize(c.stream));
            uint64_t ovf_keys = 0;
            for (uint64_t g = 0; g < ngroups; ++g)
                if (flags[g]) ovf_keys += gs[g + 1] - gs[g];
            if (c.debug) {
                fprintf(stderr, "[mtg debug]   fallback: %u groups, %lu keys\n", novf, (unsigned long)ovf_keys);
                int shown = 0;
                for (uint64_t g = 0; g < ngroups && shown < 5; ++g)
                    if (flags[g]) {
                        fprintf(stderr, "[mtg debug]     group %lu [%lu, %lu)\n", (unsigned long)g,
                                (unsigned long)gs[g], (unsigned long)gs[g + 1]);
                        ++shown;
                    }
            }
            if (ovf_keys * 20 > n && levels < 3 && digit_end[levels] < nbits) {
                run_level(++levels);  // many overflows: one more level for everything
                continue;
            }
            // the rest: LSD radix sort + unique of each group in place
            for (uint64_t g = 0; g < ngroups; ++g) {
                if (!flags[g]) continue;
                const uint64_t g0 = gs[g], m = gs[g + 1] - gs[g];
                Key<L> *fk = (Key<L> *)c.ws.get(Workspace::FB_K, m * sizeof(Key<L>));
                uint32_t *fv = COUNTED ? (uint32_t *)c.ws.get(Workspace::FB_V, m * 4) : nullptr;
                Key<L> *ka = *keys + g0, *kb = fk;
                uint32_t *va = COUNTED ? *vals + g0 : nullptr, *vb = fv;
                radix_sort<L, COUNTED>(c, &ka, &kb, &va, &vb, m, nbits, false);
                reset_small(c);
                const uint64_t ut = ceil_div(m, 2048);
                uint32_t ep;
                uint64_t *desc = acquire_desc(c, ut, &ep);
                unsigned long long *sums = nullptr;
                if (COUNTED) {
                    sums = (unsigned long long *)c.ws.get(Workspace::SUMS, m * 8);
                    HIP_CHECK(hipMemsetAsync(sums, 0, m * 8, c.stream));
                }
                unique_kernel<L, COUNTED><<<dim3((unsigned)ut), dim3(256), 0, c.stream>>>(
                    ka, va, m, *alt + g0, sums, desc, ep, &c.small->counter, &c.small->total, &c.small->error);
                HIP_CHECK(hipGetLastError());
                const uint64_t u = read_u64(c, &c.small->total);
                if (COUNTED)
                    count_clamp_kernel<<<dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(u, 256), 4096))),
                                         dim3(256), 0, c.stream>>>(sums, u, cmax, *valt + g0);
                const uint32_t u32 = (uint32_t)u;
                HIP_CHECK(hipMemcpyAsync(ucount + g, &u32, 4, hipMemcpyHostToDevice, c.stream));
                HIP_CHECK(hipStreamSynchronize(c.stream));
            }
        }
        // pack: ustart = exclusive scan of ucount, gather tmp (= *alt) -> *keys
        uint64_t *ustart = (uint64_t *)c.ws.get(Workspace::MSD_USTART, (ngroups + 1) * 8);
        uint32_t ep;
        const uint64_t st = ceil_div(ngroups, 4096);
        uint64_t *desc = acquire_desc(c, st, &ep);
        HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
        scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(ucount, ngroups, ustart, desc, ep,
                                                                      &c.small->counter, &c.small->error);
        HIP_CHECK(hipGetLastError());
        // the output's bucket index over the top b bits comes out of the gather (the fused rc merge
        // of the canonical keys reuses it instead of a bucket_index pass: 0.44 ms at configs[1])
        // (only for the sorts the fused rc merge follows: c.want_gidx)
        const bool index = c.want_gidx && gbucket_out && b > 0;
        uint64_t *gi = index ? (uint64_t *)c.ws.get(Workspace::CANON_IDX, (nbuckets + 2) * 8) : nullptr;
        if (index) HIP_CHECK(hipMemsetAsync(&c.small->gidx_bad, 0, 4, c.stream));
        if (c.sort_out &&
            (c.sort_out_cap == ~0ull || read_u64(c, (const unsigned long long *)(ustart + ngroups)) <= c.sort_out_cap)) {
            *keys = (Key<L> *)c.sort_out;  // (the caller's destination: the gather reads *alt only)
            if (COUNTED) *vals = c.sort_out_vals;
        }
        bucket_pieces(0, ngroups, [&](uint64_t g0, unsigned cnt) {
            group_gather_kernel<L, COUNTED><<<dim3(cnt), dim3(256), 0, c.stream>>>(
                *alt, COUNTED ? *valt : nullptr, gstart, ustart, *keys, COUNTED ? *vals : nullptr, gbucket_out,
                nbits - b, gi, &c.small->gidx_bad, g0);
            HIP_CHECK(hipGetLastError());
        });
        uint64_t u = 0;
        uint32_t ibad = 0;
        HIP_CHECK(hipMemcpyAsync(&u, ustart + ngroups, 8, hipMemcpyDeviceToHost, c.stream));
        if (index) {  // entries nbuckets, nbuckets + 1 = the key count
            HIP_CHECK(hipMemcpyAsync(gi + nbuckets, ustart + ngroups, 8, hipMemcpyDeviceToDevice, c.stream));
            HIP_CHECK(hipMemcpyAsync(gi + nbuckets + 1, ustart + ngroups, 8, hipMemcpyDeviceToDevice, c.stream));
            HIP_CHECK(hipMemcpyAsync(&ibad, &c.small->gidx_bad, 4, hipMemcpyDeviceToHost, c.stream));
        }
        HIP_CHECK(hipStreamSynchronize(c.stream));
        if (index && !ibad) c.gidx = Ctx::GroupIndex{*keys, u, b, nbits, gi};
        return u;
    }
}

template <int L>
static unsigned bucket_bits(uint64_t n, unsigned keybits) {
    // ~4 keys a bucket; at most 2^26 buckets up to 2^30 keys (configs[1]: 5.5 a bucket), 2^29 above: at
    // configs[3]'s share (4.7e9 real edges) 2^26 buckets held 69 edges each, and the dummy sink join's
    // staged class ranges (whole buckets at both ends) outgrew its LDS and fell back to global searches
    const unsigned cap = n > (1ull << 30) ? 29 : 26;
    unsigned b = 1;
    while (b < cap && (1ull << (b + 2)) < n) ++b;
    return std::min(b, keybits);
}

struct BuildInput {
    const uint8_t *seq;
    uint64_t seq_len;
    const uint64_t *read_starts;
    const uint32_t *read_counts;
    uint64_t n_reads;
    const uint64_t *rid_at = nullptr;  // per-read counts: the read of every 4 K-position block
};

struct BuildOutput {
    uint8_t *W;
    uint8_t *last;
    uint32_t *weights;
    uint64_t n;
    uint64_t F[5];
    uint64_t n_real;
    uint64_t n_dummy;
    bool host = false;  // the spilled build (run_pipeline_spill): W / last / weights are host arrays
};

// MTG_DEBUG=1: host-side check that a device key array is strictly increasing
template <int L>
static void debug_check_sorted(Ctx &c, const char *what, const Key<L> *d, uint64_t n) {
    if (!c.debug || n == 0) return;
    std::vector<Key<L>> h(n);
    HIP_CHECK(hipMemcpyAsync(h.data(), d, n * sizeof(Key<L>), hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    uint64_t bad = 0;
    for (uint64_t i = 1; i < n; ++i) bad += !(h[i - 1] < h[i]);
    fprintf(stderr, "[mtg debug] %s: n=%lu, %lu order violations; first keys:", what,
            (unsigned long)n, (unsigned long)bad);
    for (uint64_t i = 0; i < std::min<uint64_t>(n, 8); ++i) fprintf(stderr, " %lx", (unsigned long)h[i].w[0]);
    fprintf(stderr, "\n");
}

// merge of two sorted arrays through the tiled merge-path kernels (boss_kernels.hpp)
template <int LO, int LA, bool LIFT, bool COUNTED, bool BCOUNTS>
static void merge_sorted(Ctx &c, const Key<LA> *a, const uint32_t *ac, uint64_t na,
                         const Key<LO> *b, const uint32_t *bc, uint64_t nb, unsigned K,
                         Key<LO> *out, uint32_t *oc, uint64_t off) {
    const uint64_t ntiles = ceil_div(na + nb, MergeTraits<LO>::TILE);
    if (!ntiles) return;
    uint64_t *splits = (uint64_t *)c.ws.get(Workspace::SPLITS, (ntiles + 1) * 8);
    merge_partition_kernel<LO, LA, LIFT><<<dim3((unsigned)ceil_div(ntiles + 1, 256)), dim3(256), 0, c.stream>>>(
        a, na, b, nb, K, ntiles, splits);
    HIP_CHECK(hipGetLastError());
    merge_kernel<LO, LA, LIFT, COUNTED, BCOUNTS><<<dim3((unsigned)ntiles), dim3(256), 0, c.stream>>>(
        a, ac, na, b, bc, nb, K, splits, out, oc, off);
    HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------- pipeline stages

// K1: extract (+ canonicalise) every valid k-mer window of the read buffer into *ka (count ->
// scan -> write over identical tiles).  Returns N.
template <int L2, bool COUNTED>
static uint64_t stage_extract(Ctx &c, unsigned K, bool canonical, uint32_t cmax, const BuildInput &in,
                              Key<L2> **ka, Key<L2> **kb, uint32_t **ca, uint32_t **cb) {
    using K2 = Key<L2>;
    const uint64_t npos = in.seq_len >= K ? in.seq_len - K + 1 : 0;
    c.timings.n_positions = npos;
    *ka = (K2 *)c.ws.get(Workspace::KA, npos * sizeof(K2));
    *kb = (K2 *)c.ws.get(Workspace::KB, npos * sizeof(K2));
    *ca = COUNTED ? (uint32_t *)c.ws.get(Workspace::CA, npos * 4) : nullptr;
    *cb = COUNTED ? (uint32_t *)c.ws.get(Workspace::CB, npos * 4) : nullptr;
    uint64_t N = 0;
    if (npos) {
        constexpr int TILE = ExtractTraits<L2>::TILE;
        const uint64_t tiles = ceil_div(npos, TILE);
        uint32_t *tcnt = (uint32_t *)c.ws.get(Workspace::DTCNT, (tiles + 1) * 4);
        uint64_t *toff = (uint64_t *)c.ws.get(Workspace::DTOFF, (tiles + 1) * 8);
        extract_kernel<L2, COUNTED, true><<<dim3((unsigned)tiles), dim3(256), 0, c.stream>>>(
            in.seq, in.seq_len, K, cmode(c, canonical), in.read_starts, in.read_counts, in.n_reads, in.rid_at, cmax,
            nullptr, nullptr, tcnt, nullptr, nullptr, 0);
        HIP_CHECK(hipGetLastError());
        uint32_t ep;
        const uint64_t st = ceil_div(tiles, 4096);
        uint64_t *desc = acquire_desc(c, st, &ep);
        HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
        scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(
            tcnt, tiles, toff, desc, ep, &c.small->counter, &c.small->error);
        HIP_CHECK(hipGetLastError());
        N = read_u64(c, (const unsigned long long *)(toff + tiles));
        extract_kernel<L2, COUNTED, false><<<dim3((unsigned)tiles), dim3(256), 0, c.stream>>>(
            in.seq, in.seq_len, K, cmode(c, canonical), in.read_starts, in.read_counts, in.n_reads, in.rid_at, cmax,
            *ka, *ca, nullptr, toff, nullptr, 0);
        HIP_CHECK(hipGetLastError());
    }
    c.timings.n_extracted = N;
    return N;
}

// Whether the reads may be one window each (K chars + a separator, read r at r * (K + 1): a KMC
// database decoded into reads); window_reads_kernel checks every read and says if not.
static bool window_layout(Ctx &c, unsigned K, const BuildInput &in) {
    if (!in.read_starts || in.n_reads == 0 || c.use_lsd) return false;
    const uint64_t n = in.n_reads, st = K + 1;
    if (in.seq_len < (n - 1) * st + K || in.seq_len > n * st) return false;
    uint64_t s[2] = {0, st};
    HIP_CHECK(hipMemcpyAsync(s, in.read_starts, (n >= 2 ? 2 : 1) * 8, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    return s[0] == 0 && (n < 2 || s[1] == st);
}

// K1 for one-window reads (boss_kernels.hpp: window_reads_kernel): every read's k-mer straight to *ka
// in any order.  False (nothing kept) when the layout does not hold.
template <int L2, bool COUNTED>
static bool stage_extract_windows(Ctx &c, unsigned K, bool canonical, uint32_t cmax, const BuildInput &in,
                                  Key<L2> **ka, Key<L2> **kb, uint32_t **ca, uint32_t **cb, uint64_t *N_out) {
    if (!window_layout(c, K, in)) return false;
    using K2 = Key<L2>;
    const uint64_t n = in.n_reads;
    *ka = (K2 *)c.ws.get(Workspace::KA, n * sizeof(K2));
    *kb = (K2 *)c.ws.get(Workspace::KB, n * sizeof(K2));
    *ca = COUNTED ? (uint32_t *)c.ws.get(Workspace::CA, n * 4) : nullptr;
    *cb = COUNTED ? (uint32_t *)c.ws.get(Workspace::CB, n * 4) : nullptr;
    HIP_CHECK(hipMemsetAsync(&c.small->wbad, 0, 4, c.stream));
    HIP_CHECK(hipMemsetAsync(&c.small->wcursor, 0, 8, c.stream));
    window_reads_kernel<L2, COUNTED><<<dim3((unsigned)ceil_div(n, 256 * 8)), dim3(256), 0, c.stream>>>(
        in.seq, in.seq_len, K, cmode(c, canonical), in.read_starts, in.read_counts, n, cmax, *ka,
        COUNTED ? *ca : nullptr, &c.small->wcursor, &c.small->wbad);
    HIP_CHECK(hipGetLastError());
    uint32_t bad = 0;
    unsigned long long N = 0;
    HIP_CHECK(hipMemcpyAsync(&bad, &c.small->wbad, 4, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipMemcpyAsync(&N, &c.small->wcursor, 8, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    if (bad) return false;
    if (c.debug) fprintf(stderr, "[mtg debug] one-window reads: %lu reads -> %llu k-mers\n", (unsigned long)n, N);
    c.timings.n_positions = in.seq_len >= K ? in.seq_len - K + 1 : 0;
    c.timings.n_extracted = N;
    *N_out = N;
    return true;
}

// The MSD plan of a fused K1's input.  Its level 1 is pass B's digit, which the VALU-bound pass B
// can take 10 bits wide (extract_partition_fast_kernel<512, 1024>: 8-key runs, its writes hidden
// behind the extraction): a plan of 19 bits -- ~2e9 k-mers, 15-20 M reads -- then runs 10 + 9
// instead of 6 + 6 + 7, one stand-alone partition pass instead of two.  `fast`: the uncounted pass
// B (the counted one keeps <= 9 bits).
static MsdPlan fused_plan(const Ctx &c, uint64_t N, unsigned nbits, double dup, bool fast) {
    MsdPlan p = msd_plan<1>(c, N, nbits, dup);
    if (!p.levels || !fast) return p;
    const unsigned T = p.digit_end[p.levels];
    unsigned b1 = 0;
    if (c.fused_b1) b1 = std::min(c.fused_b1, T);
    else if (c.wide_b1 && p.levels == 3 && !c.min_levels && T <= 10 + MSD_DBITS) b1 = 10;
    if (!b1) return p;
    MsdPlan q{};
    q.levels = 1 + (T - b1 + MSD_DBITS - 1) / MSD_DBITS;
    q.digit_end[1] = b1;
    for (unsigned l = 2; l <= q.levels; ++l) q.digit_end[l] = b1 + (T - b1) * (l - 1) / (q.levels - 1);
    return q;
}

// K1 fused with K2's first partition level (extract_partition.hpp), for 2-bit u64 keys on
// inputs big enough to have one: pass A (fused_pass_a, the histogram of the top FUSED_HB bits of
// every k-mer) then pass B (fused_pass_b, the k-mers scattered by their level-1 digit).
struct FusedA {
    uint64_t npos = 0, N = 0;
    double dup = 8.0;
    uint32_t nrows = 0, rps = 0, stripes = 0;
    uint64_t per_stripe = 0;
    uint32_t *rows = nullptr;  // per-row histograms (device), rps rows per stripe of pass-B tiles
    double sample_factor = 1.0;  // tiles per sampled tile of pass A (fused_pass_a with sample > 1)
    std::vector<uint32_t> h;   // their sum over the 2^FUSED_HB top-bit bins (host)
};

static bool fused_applies(const Ctx &c, unsigned K, uint64_t npos, unsigned kmax = 32) {
    return c.fused && !c.use_lsd && npos >= c.fused_min && npos >= 4096 && K - 1 >= FUSED_HB / 2 && K <= kmax;
}

// pass A over every window, and the duplication estimate from a sample of windows (on a side stream
// it overlapped pass A but measured no faster: 26.3 vs 26.2 ms per step)
// the fused passes with K = 31 compiled in (KC, extract_partition.hpp) unless MTG_KSPEC=0
// (K = 31 also takes the canonical mode cm as a template constant: extract_partition.hpp, CM)
template <bool OTHER, typename... A>
static void launch_hist_fast(const Ctx &c, unsigned K, dim3 g, dim3 b, const uint8_t *seq, uint64_t seq_len,
                             unsigned K_, int cm, A... a) {
    if (K == 31 && c.kspec && cm == 0) extract_hist_fast_kernel<OTHER, 31, 0><<<g, b, 0, c.stream>>>(seq, seq_len, K_, cm, a...);
    else if (K == 31 && c.kspec && cm == 1) extract_hist_fast_kernel<OTHER, 31, 1><<<g, b, 0, c.stream>>>(seq, seq_len, K_, cm, a...);
    else if (K == 31 && c.kspec && cm == 2) extract_hist_fast_kernel<OTHER, 31, 2><<<g, b, 0, c.stream>>>(seq, seq_len, K_, cm, a...);
    else extract_hist_fast_kernel<OTHER, 0><<<g, b, 0, c.stream>>>(seq, seq_len, K_, cm, a...);
}
template <int BLOCK, int NB, typename... A>
static void launch_part_fast(const Ctx &c, unsigned K, dim3 g, dim3 b, const uint8_t *seq, uint64_t seq_len,
                             unsigned K_, int cm, A... a) {
    if (K == 31 && c.kspec && cm == 0)
        extract_partition_fast_kernel<BLOCK, NB, 31, 0><<<g, b, 0, c.stream>>>(seq, seq_len, K_, cm, a...);
    else if (K == 31 && c.kspec && cm == 1)
        extract_partition_fast_kernel<BLOCK, NB, 31, 1><<<g, b, 0, c.stream>>>(seq, seq_len, K_, cm, a...);
    else if (K == 31 && c.kspec && cm == 2)
        extract_partition_fast_kernel<BLOCK, NB, 31, 2><<<g, b, 0, c.stream>>>(seq, seq_len, K_, cm, a...);
    else
        extract_partition_fast_kernel<BLOCK, NB, 0><<<g, b, 0, c.stream>>>(seq, seq_len, K_, cm, a...);
}

// sample > 1 (fused_pass_b_spec): every row counts every sample-th of its tiles, and the 2048 rows form
// c.spec_l1_stripes stripes (A->h, A->N are then estimates)
constexpr uint32_t kSpecRows = 2048;
static void fused_pass_a(Ctx &c, unsigned K, bool canonical, const BuildInput &in, FusedA *A, uint32_t sample = 1,
                         int fbk = 512) {
    // fbk: pass B's workgroup size (fused_block<L>: 512 for u64 keys, 256 for u128); K > 32: the wide
    // histogram kernel (u128 windows)
    const uint64_t npos = in.seq_len >= K ? in.seq_len - K + 1 : 0;
    constexpr uint32_t M = 1u << 19, SLOTS = 1u << 21;
    unsigned long long *table = (unsigned long long *)c.ws.get(Workspace::DUP_TABLE, (SLOTS + 2) * 8ull);
    HIP_CHECK(hipMemsetAsync(table, 0, (SLOTS + 2) * 8ull, c.stream));
    // (K > 32: the sampled k-mers need u128 words -- truncated to 64 bits, distinct k-mers collided and
    // the duplication estimate planned too few MSD bits for the u128 rounds)
    if (K > 32)
        dup_sample_reads_kernel<2><<<dim3(M / 256), dim3(256), 0, c.stream>>>(in.seq, in.seq_len, K, cmode(c, canonical),
                                                                              M, table, SLOTS - 1, table + SLOTS);
    else
        dup_sample_reads_kernel<1><<<dim3(M / 256), dim3(256), 0, c.stream>>>(in.seq, in.seq_len, K, cmode(c, canonical),
                                                                              M, table, SLOTS - 1, table + SLOTS);
    HIP_CHECK(hipGetLastError());
    constexpr int TILE = ExtractTraits<1>::TILE;
    const uint64_t tiles = ceil_div(npos, TILE);
    // rows in multiples of rps = pass-B tile / pass-A tile: rps consecutive rows count one stripe of
    // pass B's tiles (stripe_cursor_kernel).  Pass-B workgroup: 512 threads (8 K-window tiles, two
    // workgroups per CU).  With XCD-contiguous tiles and stripes the short runs of neighbouring tiles
    // meet in one L2: extract stage 6.97 -> 5.61 ms vs 1024-thread tiles (16 K windows), which won
    // before the XCD mapping (their longer runs: PMC writes 1.16 vs 1.30 x N w)
    const uint32_t rps = (uint32_t)(16 * fbk / TILE);
    // (stripe_cursor_kernel takes at most 1024 stripes: 2048 rows at rps = 2, 1024 at rps = 1)
    uint32_t nrows = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(tiles, c.hist_rows), 1024ull * rps);
    if (nrows >= rps) nrows -= nrows % rps;
    const unsigned hb = FUSED_HB;
    const uint32_t nbh = 1u << hb;
    uint32_t *rows = (uint32_t *)c.ws.get(Workspace::HIST_ROWS, (uint64_t)nrows * nbh * 4);
    uint32_t *h12 = (uint32_t *)c.ws.get(Workspace::FUSED_HIST, nbh * 4);
    HIP_CHECK(hipMemsetAsync(h12, 0, nbh * 4, c.stream));
    // stripes of pass B's tiles: S = nrows / rps stripes of per_stripe consecutive pass-B tiles
    // (= rps per_stripe pass-A tiles); pass-A row r counts the per_row pass-A tiles
    // [r per_row, (r + 1) per_row), so rows rps s .. rps s + rps - 1 cover stripe s.  One stripe
    // (fewer rows than rps) takes every row, each an equal share of the tiles.
    const uint64_t tiles_b = ceil_div(npos, (uint64_t)16 * fbk);
    uint32_t stripes = std::max<uint32_t>(1, nrows / rps);
    uint64_t per_stripe = ceil_div(tiles_b, stripes);
    uint64_t per_row = stripes == 1 ? ceil_div(tiles_b * rps, nrows) : per_stripe;
    uint32_t rps_out = rps;
    if (sample > 1) {
        // S stripes of kSpecRows / S rows: row r counts the pass-A tiles [r per_row, (r + 1) per_row),
        // so stripe s (pass-B tiles [s per_stripe, (s + 1) per_stripe), 2 pass-A tiles each) is rows
        // s rps .. + rps - 1
        const uint32_t S = c.spec_l1_stripes, srps = kSpecRows / S;
        nrows = kSpecRows;
        rows = (uint32_t *)c.ws.get(Workspace::HIST_ROWS, (uint64_t)nrows * nbh * 4);
        per_row = ceil_div(tiles, nrows);
        per_stripe = srps * per_row / 2;  // srps is even (S <= 256)
        stripes = (uint32_t)ceil_div(tiles_b, per_stripe);
        rps_out = srps;
    }
    if (K > 32) {
        if (K == 63 && c.kspec)
            extract_hist_wide_kernel<63><<<dim3(nrows), dim3(256), 0, c.stream>>>(in.seq, in.seq_len, K, cmode(c, canonical),
                                                                              tiles, per_row, rows, sample);
        else
            extract_hist_wide_kernel<0><<<dim3(nrows), dim3(256), 0, c.stream>>>(in.seq, in.seq_len, K, cmode(c, canonical),
                                                                             tiles, per_row, rows, sample);
    } else {
        launch_hist_fast<false>(c, K, dim3(nrows), dim3(256), in.seq, in.seq_len, K, cmode(c, canonical), tiles, per_row,
                                rows, (uint32_t *)nullptr, sample);
    }
    HIP_CHECK(hipGetLastError());
    hist_rows_reduce_kernel<<<dim3(std::min<uint32_t>(nrows, 256), (unsigned)ceil_div(nbh, 256)), dim3(256), 0,
                              c.stream>>>(rows, nrows, nbh, h12);
    HIP_CHECK(hipGetLastError());
    A->h.assign(nbh, 0);
    unsigned long long st[2];
    HIP_CHECK(hipMemcpyAsync(A->h.data(), h12, nbh * 4, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipMemcpyAsync(st, table + SLOTS, 16, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    uint64_t N = 0;
    for (uint32_t v : A->h) N += v;
    // a row samples ceil(per_row / sample) of its per_row tiles
    A->sample_factor = sample > 1 ? (double)per_row / (double)ceil_div(per_row, sample) : 1.0;
    N = (uint64_t)((double)N * A->sample_factor);
    const double mv = (double)std::max<unsigned long long>(st[1], 1);
    const double ew = 2.0 * (double)N * (double)st[0] / (mv * mv);
    A->npos = npos;
    A->N = N;
    A->dup = N >= 16ull * M ? std::max(1.0, ew / 1.2) : 8.0;
    A->nrows = nrows;
    A->rps = rps_out;
    A->stripes = stripes;
    A->per_stripe = per_stripe;
    A->rows = rows;
}

// a level-1 bucket mask of one collect round (extract_partition.hpp: FUSED_SEL_WORDS words)
struct BucketSel {
    uint32_t m[FUSED_SEL_WORDS] = {};
    bool has(uint32_t b) const { return (m[b >> 5] >> (b & 31)) & 1u; }
    void add(uint64_t lo, uint64_t hi) {
        for (uint64_t b = lo; b < hi; ++b) m[b >> 5] |= 1u << (b & 31);
    }
};

// the u128 pass B as the packed-word kernel (extract_partition_fast2_kernel): uncounted basic / canonical
template <int L, bool COUNTED>
static inline bool fast2_applies(const Ctx &c, unsigned K, bool canonical) {
    return L == 2 && !COUNTED && c.fast2 && K > 32 && K <= 64 && cmode(c, canonical) <= 1;
}

// pass B: the k-mers whose level-1 bucket (top b1 bits) is in `sel` (nullptr: every bucket)
// scattered into ka by that bucket; returns their number and their level-1 counts in *dh1 (device;
// zero outside `sel`)
template <int L, bool COUNTED>
static uint64_t fused_pass_b(Ctx &c, unsigned K, bool canonical, uint32_t cmax, const BuildInput &in,
                             const FusedA &A, unsigned b1, const BucketSel *sel, Key<L> *ka, uint32_t *ca,
                             const uint32_t **dh1_out, const long long *bdelta = nullptr) {
    // bdelta (the u64 pass B and the u128 packed-word one): per level-1 bucket, where its keys go relative
    // to ka (elements) -- the collect rounds' one pass B writes each round's buckets into that round's own
    // buffer
    const uint32_t nb1 = 1u << b1;
    const unsigned hb = FUSED_HB;
    if (sel && nb1 > 32 * FUSED_SEL_WORDS) throw std::runtime_error("collect round mask: level-1 digit too wide");
    std::vector<uint32_t> h1(nb1, 0);
    for (uint32_t i = 0; i < (1u << hb); ++i) {
        const uint32_t b = i >> (hb - b1);
        if (!sel || sel->has(b)) h1[b] += A.h[i];
    }
    uint32_t *dsel = nullptr;
    if (sel) {
        dsel = (uint32_t *)c.ws.get(Workspace::FUSED_SEL, sizeof(sel->m));
        HIP_CHECK(hipMemcpyAsync(dsel, sel->m, sizeof(sel->m), hipMemcpyHostToDevice, c.stream));
    }
    // level-1 bucket starts = the scatter cursors, then the bucket ends pass B checks its
    // reservations against
    std::vector<unsigned long long> cur(2 * nb1);
    unsigned long long acc = 0;
    for (uint32_t i = 0; i < nb1; ++i) {
        cur[i] = acc;
        acc += h1[i];
    }
    for (uint32_t i = 0; i < nb1; ++i) cur[nb1 + i] = cur[i] + h1[i];
    uint32_t *dh1 = (uint32_t *)c.ws.get(Workspace::HIST1, h1.size() * 4);
    unsigned long long *dcur = (unsigned long long *)c.ws.get(Workspace::FUSED_CUR, cur.size() * 8);
    HIP_CHECK(hipMemcpyAsync(dh1, h1.data(), h1.size() * 4, hipMemcpyHostToDevice, c.stream));
    HIP_CHECK(hipMemcpyAsync(dcur, cur.data(), cur.size() * 8, hipMemcpyHostToDevice, c.stream));
    // per-stripe cursors (stripe_cursor_kernel): pass-B tile t writes through stripe t / per_stripe
    static_assert(FusedTraits<COUNTED, 512>::TILE == 2 * ExtractTraits<1>::TILE, "a pass-B tile = 2 pass-A tiles");
    static_assert(FusedTraits<COUNTED, fused_block<2>()>::TILE == ExtractTraits<1>::TILE, "u128: a pass-B tile = 1 pass-A tile");
    auto *scur = (unsigned long long *)c.ws.get(Workspace::STRIPE_CUR, (size_t)A.stripes * nb1 * 16);
    unsigned long long *send = scur + (size_t)A.stripes * nb1;
    stripe_cursor_kernel<<<dim3(nb1), dim3(256), 0, c.stream>>>(A.rows, A.nrows, hb, b1, A.stripes, A.rps, dcur, scur,
                                                                 send, dsel);
    HIP_CHECK(hipGetLastError());
    EventTimer tm(c.stream);
    tm.mark();
    const bool fast_b = L == 1 && !COUNTED && K <= 32;
    if (bdelta && !fast_b && !fast2_applies<L, COUNTED>(c, K, canonical))
        throw std::runtime_error("per-bucket destinations need the u64 or the packed-word u128 pass B");
    if constexpr (L == 2) {
        // u128 windows (K <= 64): pass B on 256-thread tiles (A was made for them); uncounted canonical /
        // basic builds take the packed-word kernel (MTG_FAST2=0: the generic one)
        constexpr int B = fused_block<2>();
        if (b1 > 9) throw std::runtime_error("the u128 pass B takes at most 9 bits");
        const uint64_t ftiles = ceil_div(A.npos, FusedTraits<COUNTED, B>::TILE);
        if (fast2_applies<L, COUNTED>(c, K, canonical)) {
            // the same 4096-window tiles as 512 threads of 8 windows (twice the waves a CU at the same LDS)
            static_assert(FusedTraits<COUNTED, B>::TILE == 512 * 8, "a pass-B tile = 512 threads x 8 windows");
            if (c.fast2_ppt8 && K == 63 && c.kspec)
                extract_partition_fast2_kernel<512, 63, 8><<<dim3((unsigned)xcd_grid(ftiles)), dim3(512), 0, c.stream>>>(
                    in.seq, in.seq_len, K, cmode(c, canonical), b1, A.per_stripe, scur, send, (Key<2> *)ka, &c.small->error,
                    (const uint32_t *)dsel, bdelta);
            else if (c.fast2_ppt8)
                extract_partition_fast2_kernel<512, 0, 8><<<dim3((unsigned)xcd_grid(ftiles)), dim3(512), 0, c.stream>>>(
                    in.seq, in.seq_len, K, cmode(c, canonical), b1, A.per_stripe, scur, send, (Key<2> *)ka, &c.small->error,
                    (const uint32_t *)dsel, bdelta);
            else if (K == 63 && c.kspec)
                extract_partition_fast2_kernel<B, 63><<<dim3((unsigned)xcd_grid(ftiles)), dim3(B), 0, c.stream>>>(
                    in.seq, in.seq_len, K, cmode(c, canonical), b1, A.per_stripe, scur, send, (Key<2> *)ka, &c.small->error,
                    (const uint32_t *)dsel, bdelta);
            else
                extract_partition_fast2_kernel<B><<<dim3((unsigned)xcd_grid(ftiles)), dim3(B), 0, c.stream>>>(
                    in.seq, in.seq_len, K, cmode(c, canonical), b1, A.per_stripe, scur, send, (Key<2> *)ka, &c.small->error,
                    (const uint32_t *)dsel, bdelta);
        } else if (K == 63 && c.kspec)
            extract_partition_kernel<2, COUNTED, B, 63><<<dim3((unsigned)xcd_grid(ftiles)), dim3(B), 0, c.stream>>>(
                in.seq, in.seq_len, K, cmode(c, canonical), in.read_starts, in.read_counts, in.n_reads, in.rid_at, cmax, b1,
                A.per_stripe, scur, send, ka, COUNTED ? ca : nullptr, &c.small->error, dsel);
        else
            extract_partition_kernel<2, COUNTED, B><<<dim3((unsigned)xcd_grid(ftiles)), dim3(B), 0, c.stream>>>(
                in.seq, in.seq_len, K, cmode(c, canonical), in.read_starts, in.read_counts, in.n_reads, in.rid_at, cmax, b1,
                A.per_stripe, scur, send, ka, COUNTED ? ca : nullptr, &c.small->error, dsel);
    } else if (fast_b) {
        constexpr int B = 512;
        const dim3 g((unsigned)xcd_grid(ceil_div(A.npos, 16 * B)));
        if (b1 > 9)
            launch_part_fast<B, 1024>(c, K, g, dim3(B), in.seq, in.seq_len, K, cmode(c, canonical), b1, A.per_stripe, scur,
                                      send, ka, &c.small->error, (const uint32_t *)dsel, (uint32_t *)nullptr, bdelta);
        else
            launch_part_fast<B, 512>(c, K, g, dim3(B), in.seq, in.seq_len, K, cmode(c, canonical), b1, A.per_stripe, scur,
                                     send, ka, &c.small->error, (const uint32_t *)dsel, (uint32_t *)nullptr, bdelta);
    } else {
        if (b1 > 9) throw std::runtime_error("the counted pass B takes at most 9 bits");
        const uint64_t ftiles = ceil_div(A.npos, FusedTraits<COUNTED, 512>::TILE);
        extract_partition_kernel<1, COUNTED, 512><<<dim3((unsigned)xcd_grid(ftiles)), dim3(512), 0, c.stream>>>(
            in.seq, in.seq_len, K, cmode(c, canonical), in.read_starts, in.read_counts, in.n_reads, in.rid_at, cmax, b1,
            A.per_stripe, scur, send, (Key<1> *)ka, COUNTED ? ca : nullptr, &c.small->error, dsel);
    }
    HIP_CHECK(hipGetLastError());
    cursor_check_kernel<<<dim3((unsigned)ceil_div((uint64_t)A.stripes * nb1, 256)), dim3(256), 0, c.stream>>>(
        scur, send, A.stripes * nb1, &c.small->error);
    HIP_CHECK(hipGetLastError());
    tm.mark();
    HIP_CHECK(hipStreamSynchronize(c.stream));  // `h1` / `cur` / `sel` are host memory
    c.fused_ms = tm.ms(0, 1);
    *dh1_out = dh1;
    return acc;
}

// Pass B into the speculative level-1 layout (extract_partition.hpp: spec_l1_caps_kernel) after a
// sampled pass A (fused_pass_a with sample > 1): no exact histogram pass over every window (pass A:
// 1.29 ms at configs[1]).  Segments of (bucket, stripe) sized from the sample with slack, each a whole
// number of level-2 tiles; the level-2 pass reads the padded array through tvalid (c.gap1).  Returns
// the k-mer count with the exact level-1 counts in *dh1_out, or ~0 when a segment overflowed (nothing
// the caller needs was touched: it runs the exact passes).
static uint64_t fused_pass_b_spec(Ctx &c, unsigned K, bool canonical, const BuildInput &in, const FusedA &A,
                                  unsigned b1, Key<1> **ka, Key<1> **kb, const uint32_t **dh1_out) {
    const uint32_t nb1 = 1u << b1, S = A.stripes;
    constexpr uint32_t T2 = MsdTraits<1>::TILE;
    const uint64_t nseg = (uint64_t)nb1 * S;
    uint32_t *caps = (uint32_t *)c.ws.get(Workspace::SPEC1_CAPS, (nseg + 1) * 4);
    uint64_t *sst = (uint64_t *)c.ws.get(Workspace::SPEC1_START, (nseg + 1) * 8);
    spec_l1_caps_kernel<<<dim3(nb1), dim3(256), 0, c.stream>>>(A.rows, A.nrows, FUSED_HB, b1, S, A.rps,
                                                               (float)A.sample_factor, T2, caps, c.spec_l1_tiny,
                                                               c.spec_l1_slack);
    HIP_CHECK(hipGetLastError());
    {
        uint32_t ep;
        const uint64_t st = ceil_div(nseg, 4096);
        uint64_t *desc = acquire_desc(c, st, &ep);
        HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
        scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(caps, nseg, sst, desc, ep, &c.small->counter,
                                                                          &c.small->error);
        HIP_CHECK(hipGetLastError());
    }
    const uint64_t C1 = read_u64(c, (const unsigned long long *)(sst + nseg));
    if (C1 % T2) throw std::logic_error("spec level 1: segments not tile-aligned");
    {  // the padded array must fit next to everything else
        const uint64_t fr = c.ws.free_bytes();
        const double need = 8.0 * (double)C1, have = 0.9 * (double)fr + (double)c.ws.held_slot(Workspace::KA);
        if (need > have) return ~0ull;
    }
    *ka = (Key<1> *)c.ws.get(Workspace::KA, std::max<uint64_t>(C1, 1) * 8);
    // no ping-pong buffer: the speculative level 2 partitions into its own buckets (SPEC_A / SPEC_B); the
    // exact level, when the speculative one falls back, takes it then (msd_sort_unique: lazy_alt) -- 10.7 GB
    // less held at configs[1]; the rc stage takes KB at its own size (U keys)
    *kb = nullptr;
    auto *scur = (unsigned long long *)c.ws.get(Workspace::STRIPE_CUR, nseg * 16);
    unsigned long long *send = scur + nseg;
    spec_l1_cursor_kernel<<<dim3((unsigned)ceil_div(nseg, 256)), dim3(256), 0, c.stream>>>(sst, caps, nb1, S, scur,
                                                                                          send);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemsetAsync(&c.small->spec_ovf, 0, 4, c.stream));
    EventTimer tm(c.stream);
    tm.mark();
    constexpr int B = 512;
    const dim3 g((unsigned)xcd_grid(ceil_div(A.npos, 16 * B)));
    if (b1 > 9)
        launch_part_fast<B, 1024>(c, K, g, dim3(B), in.seq, in.seq_len, K, cmode(c, canonical), b1, A.per_stripe, scur, send,
                                  *ka, &c.small->error, (const uint32_t *)nullptr, &c.small->spec_ovf);
    else
        launch_part_fast<B, 512>(c, K, g, dim3(B), in.seq, in.seq_len, K, cmode(c, canonical), b1, A.per_stripe, scur, send,
                                 *ka, &c.small->error, (const uint32_t *)nullptr, &c.small->spec_ovf);
    HIP_CHECK(hipGetLastError());
    tm.mark();
    const uint64_t ntile2 = C1 / T2;
    uint32_t *dh1 = (uint32_t *)c.ws.get(Workspace::HIST1, nb1 * 4);
    uint32_t *tv = (uint32_t *)c.ws.get(Workspace::SPEC1_TV, std::max<uint64_t>(ntile2, 1) * 4);
    HIP_CHECK(hipMemsetAsync(dh1, 0, nb1 * 4, c.stream));
    HIP_CHECK(hipMemsetAsync(&c.small->total, 0, 8, c.stream));
    spec_l1_finish_kernel<<<dim3((unsigned)ceil_div(nseg, 256)), dim3(256), 0, c.stream>>>(sst, caps, scur, nb1, S, T2,
                                                                                          dh1, tv, &c.small->total);
    HIP_CHECK(hipGetLastError());
    uint32_t povf = 0;
    uint64_t N = 0;
    HIP_CHECK(hipMemcpyAsync(&povf, &c.small->spec_ovf, 4, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipMemcpyAsync(&N, &c.small->total, 8, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    c.fused_ms = tm.ms(0, 1);
    if (povf) {
        if (c.debug) fprintf(stderr, "[mtg debug] speculative level 1: a segment overflowed, exact passes\n");
        ++c.timings.spec_fallbacks;
        return ~0ull;
    }
    c.gap1_n = C1;
    c.gap1_tv = tv;
    c.timings.spec_l1 = 1;
    if (c.debug)
        fprintf(stderr, "[mtg debug] speculative level 1: N=%lu (sample %lu) padded %lu (%.3fx), %u stripes\n",
                (unsigned long)N, (unsigned long)A.N, (unsigned long)C1, (double)C1 / (double)std::max<uint64_t>(N, 1), S);
    *dh1_out = dh1;
    return N;
}

// Returns false (nothing done) when the fused path does not apply; else N, the duplication
// estimate, and the level-1 counts in *hist1 (device) with *ka scattered.
template <int L2, bool COUNTED>
static bool stage_extract_fused(Ctx &c, unsigned K, bool canonical, uint32_t cmax, const BuildInput &in,
                                Key<L2> **ka, Key<L2> **kb, uint32_t **ca, uint32_t **cb, uint64_t *N_out,
                                double *dup_out, const uint32_t **hist1_out, MsdPlan *plan_out) {
    if constexpr (L2 != 1) {
        return false;
    } else {
        const uint64_t npos = in.seq_len >= K ? in.seq_len - K + 1 : 0;
        if (!fused_applies(c, K, npos)) return false;
        FusedA A;
        // the speculative level-1 layout: uncounted single builds big enough that a sample sizes the
        // segments well (the rounds and the multi-GPU collect keep the exact passes)
        const bool spec1 = !COUNTED && K <= 32 && c.spec_l1 && npos >= c.spec_l1_min;
        c.gap1_n = 0;
        c.gap1_tv = nullptr;
        c.gap1_lo = c.gap1_hi = 0;
        if (spec1) {
            fused_pass_a(c, K, canonical, in, &A, c.spec_l1_sample);
            const MsdPlan plan = fused_plan(c, A.N, 2 * K, A.dup, true);
            if (plan.levels == 2) {
                const uint64_t N = fused_pass_b_spec(c, K, canonical, in, A, plan.digit_end[1], ka, kb, hist1_out);
                if (c.debug)
                    fprintf(stderr, "[mtg debug] fused extract (sampled) N=%lu dup=%.2f levels=%u digit1=%u\n",
                            (unsigned long)A.N, A.dup, plan.levels, plan.digit_end[1]);
                if (N != ~0ull) {
                    c.timings.n_positions = npos;
                    c.timings.n_extracted = N;
                    *ca = *cb = nullptr;
                    *N_out = N;
                    *dup_out = A.dup;
                    *plan_out = plan;
                    return true;
                }
            }
            A = FusedA{};
        }
        fused_pass_a(c, K, canonical, in, &A);
        const uint64_t N = A.N;
        const MsdPlan plan = fused_plan(c, N, 2 * K, A.dup, !COUNTED && K <= 32);
        if (c.debug)
            fprintf(stderr, "[mtg debug] fused extract N=%lu dup=%.2f levels=%u digit1=%u\n", (unsigned long)N, A.dup,
                    plan.levels, plan.levels ? plan.digit_end[1] : 0);
        if (!plan.levels) return false;  // nothing to partition: the plain extraction path
        const unsigned b1 = plan.digit_end[1];
        *ka = (Key<1> *)c.ws.get(Workspace::KA, std::max<uint64_t>(N, 1) * 8);
        *kb = (Key<1> *)c.ws.get(Workspace::KB, std::max<uint64_t>(N, 1) * 8);
        *ca = COUNTED ? (uint32_t *)c.ws.get(Workspace::CA, std::max<uint64_t>(N, 1) * 4) : nullptr;
        *cb = COUNTED ? (uint32_t *)c.ws.get(Workspace::CB, std::max<uint64_t>(N, 1) * 4) : nullptr;
        fused_pass_b<1, COUNTED>(c, K, canonical, cmax, in, A, b1, nullptr, *ka, COUNTED ? *ca : nullptr, hist1_out);
        c.timings.n_positions = npos;
        c.timings.n_extracted = N;
        *N_out = N;
        *dup_out = A.dup;
        *plan_out = plan;  // the sort runs this plan (its level 1 is pass B's digit)
        return true;
    }
}

// K2 + K3: sort + unique (saturating count merge) of *ka[0..N) -> *ka[0..U).  `dup` is the
// expected number of copies per distinct key (plans the MSD depth only).
template <int L2, bool COUNTED>
static uint64_t stage_collect(Ctx &c, unsigned K, uint32_t cmax, Key<L2> **ka, Key<L2> **kb,
                              uint32_t **ca, uint32_t **cb, uint64_t N, double dup, bool track,
                              const uint32_t *hist1 = nullptr, const MsdPlan *plan = nullptr) {
    // hist1 != nullptr: *ka is already scattered by the level-1 digit (stage_extract_fused)
    uint64_t U = 0;
    if (!hist1) c.gap1_n = 0, c.gap1_tv = nullptr, c.gap1_lo = c.gap1_hi = 0;
    if (c.use_lsd) {
        radix_sort<L2, COUNTED>(c, ka, kb, ca, cb, N, 2 * K, track);
        reset_small(c);
        if (N) {
            const uint64_t tiles = ceil_div(N, 2048);
            uint32_t desc_ep;
            uint64_t *desc = acquire_desc(c, tiles, &desc_ep);
            unsigned long long *sums = nullptr;
            if (COUNTED) {
                sums = (unsigned long long *)c.ws.get(Workspace::SUMS, N * 8);
                HIP_CHECK(hipMemsetAsync(sums, 0, N * 8, c.stream));
            }
            unique_kernel<L2, COUNTED><<<dim3((unsigned)tiles), dim3(256), 0, c.stream>>>(
                *ka, *ca, N, *kb, sums, desc, desc_ep, &c.small->counter, &c.small->total, &c.small->error);
            HIP_CHECK(hipGetLastError());
            U = read_u64(c, &c.small->total);
            if (COUNTED) {
                count_clamp_kernel<<<dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(U, 256), 4096))),
                                     dim3(256), 0, c.stream>>>(sums, U, cmax, *cb);
                HIP_CHECK(hipGetLastError());
            }
        }
        std::swap(*ka, *kb);
        std::swap(*ca, *cb);
    } else {
        c.track_partition = track;
        if (dup <= 0) dup = estimate_dup<L2>(c, *ka, N, 8.0);
        U = msd_sort_unique<L2, COUNTED>(c, ka, kb, ca, cb, N, 2 * K, cmax, dup, hist1, false, nullptr,
                                         hist1 != nullptr, nullptr, hist1 ? plan : nullptr);
        c.track_partition = false;
    }
    return U;
}

// ------------------------------------------------------------------- range-batched collection
//
// Inputs whose k-mers do not fit HBM at once (BASELINE configs[2]: 8.8e9 u128 windows) are
// collected one key range at a time, the bounded-memory role of the reference's disk container
// (SortedSetDisk + construct_boss_chunk_disk, boss_chunk_construct.cpp:664-933): every range
// re-scans the read buffer, extracts only the k-mers whose top chars fall in it, sorts and
// dedupes them (saturating counts), and appends them to the real-edge array.  The ranges are
// consecutive in BOSS order, so the appended array is sorted.  Canonical mode extracts BOTH
// strands: the real edges of CANONICAL_ONLY are exactly the k-mers of both strands (the canonical
// set plus add_reverse_complements, :179-222), and a palindrome window contributes its k-mer twice,
// the reference's doubled palindrome count.  Everything after the real edges (dummies, emit) is
// the single-pass pipeline's.

static std::vector<uint64_t> balanced_bounds(const uint64_t *hist, uint64_t nb, int P);

// number of key ranges for this input: 1 when the single-pass footprint fits the budget
// (memory_preallocated, else the free HBM plus what the workspace already holds)
template <int L2, bool COUNTED>
static uint32_t plan_ranges(Ctx &c, unsigned K, bool canonical, const BuildInput &in) {
    const uint64_t npos = in.seq_len >= K ? in.seq_len - K + 1 : 0;
    if (K < RB_CHARS + 1) return 1;  // at most 4^4 distinct k-mers: never worth a range
    if (c.force_ranges) return c.force_ranges;
    const double per_key = (double)sizeof(Key<L2>) + (COUNTED ? 4.0 : 0.0);
    double budget = c.mem_budget;
    if (budget <= 0) {
        size_t fr = 0, tot = 0;
        HIP_CHECK(hipMemGetInfo(&fr, &tot));
        budget = 0.9 * ((double)fr + (double)c.ws.held());
    }
    // single pass: KA + KB over every window, then the real edges, rc and dummy buffers
    if ((double)npos * per_key * 2.5 <= budget && !c.disk) return 1;
    const double keys = (double)npos * (canonical ? 2.0 : 1.0);
    uint32_t P = (uint32_t)std::ceil(keys * per_key * 2.0 / (0.4 * budget));
    P = std::max<uint32_t>(P, (uint32_t)std::ceil(keys / 2.0e9));  // <= 2e9 keys per range
    return std::min<uint32_t>(std::max<uint32_t>(P, 2), RB_BINS);
}

template <int L2, bool COUNTED>
static uint64_t collect_ranges(Ctx &c, unsigned K, bool canonical, uint32_t cmax, const BuildInput &in,
                               uint32_t P, Key<L2> **real, uint32_t **realc) {
    using K2 = Key<L2>;
    const uint64_t npos = in.seq_len >= K ? in.seq_len - K + 1 : 0;
    c.timings.n_positions = npos;
    const int both = canonical ? 1 : 0;
    constexpr int TILE = RangeTraits<L2>::TILE;
    const uint64_t tiles = ceil_div(npos, TILE);
    // count pass: per-tile counts of the 4^RB_CHARS top-char bins, and their column sums
    std::vector<uint64_t> hist(RB_BINS, 0);
    uint16_t *tbins = (uint16_t *)c.ws.get(Workspace::RANGE_BINS, std::max<uint64_t>(tiles, 1) * RB_BINS * 2);
    if (tiles) {
        auto *dh = (unsigned long long *)c.ws.get(Workspace::XHIST, RB_BINS * 8);
        HIP_CHECK(hipMemsetAsync(dh, 0, RB_BINS * 8, c.stream));
        range_count_kernel<L2><<<dim3((unsigned)tiles), dim3(256), 0, c.stream>>>(in.seq, in.seq_len, K, both, tbins);
        HIP_CHECK(hipGetLastError());
        range_bins_reduce_kernel<<<dim3((unsigned)std::min<uint64_t>(tiles, 2048)), dim3(RB_BINS), 0, c.stream>>>(
            tbins, tiles, dh);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(hist.data(), dh, RB_BINS * 8, hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));
    }
    uint64_t total = 0;
    for (uint64_t v : hist) total += v;
    P = std::min<uint32_t>(P, RB_BINS);
    const std::vector<uint64_t> bounds = balanced_bounds(hist.data(), RB_BINS, (int)P);
    c.timings.n_batches = P;
    uint64_t off = 0, cap = 0;
    *real = nullptr;
    *realc = nullptr;
    uint32_t *tcnt = (uint32_t *)c.ws.get(Workspace::DTCNT, (tiles + 1) * 4);
    uint64_t *toff = (uint64_t *)c.ws.get(Workspace::DTOFF, (tiles + 1) * 8);
    for (uint32_t j = 0; j < P; ++j) {
        const uint32_t lo = (uint32_t)bounds[j], hi = (uint32_t)bounds[j + 1];
        uint64_t nj = 0;
        for (uint32_t b = lo; b < hi; ++b) nj += hist[b];
        if (!nj) continue;
        K2 *ka = (K2 *)c.ws.get(Workspace::KA, nj * sizeof(K2));
        K2 *kb = (K2 *)c.ws.get(Workspace::KB, nj * sizeof(K2));
        uint32_t *ca = COUNTED ? (uint32_t *)c.ws.get(Workspace::CA, nj * 4) : nullptr;
        uint32_t *cb = COUNTED ? (uint32_t *)c.ws.get(Workspace::CB, nj * 4) : nullptr;
        BinSet sel{};
        sel.add(lo, hi);
        range_tile_counts_kernel<<<dim3((unsigned)ceil_div(tiles, 4)), dim3(256), 0, c.stream>>>(tbins, tiles, sel,
                                                                                                 tcnt);
        HIP_CHECK(hipGetLastError());
        uint32_t ep;
        const uint64_t st = ceil_div(tiles, 4096);
        uint64_t *desc = acquire_desc(c, st, &ep);
        HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
        scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(tcnt, tiles, toff, desc, ep,
                                                                          &c.small->counter, &c.small->error);
        HIP_CHECK(hipGetLastError());
        range_write_kernel<L2, COUNTED><<<dim3((unsigned)tiles), dim3(256), 0, c.stream>>>(
            in.seq, in.seq_len, K, both, in.read_starts, in.read_counts, in.n_reads, in.rid_at, cmax, sel, toff, ka, ca);
        HIP_CHECK(hipGetLastError());
        const uint64_t N = read_u64(c, (const unsigned long long *)(toff + tiles));
        if (N != nj) throw std::runtime_error("range extraction count differs from its histogram");
        // the range fills (hi - lo) / RB_BINS of the top-char space: plan the MSD depth as if its
        // keys were spread over all of it
        const double spread = (double)RB_BINS / (double)(hi - lo);
        const double dup = estimate_dup<L2>(c, ka, N, 8.0) / spread;
        c.track_partition = j == 0;  // the roofline's partition pass: the first range's first level
        const uint64_t U = msd_sort_unique<L2, COUNTED>(c, &ka, &kb, &ca, &cb, N, 2 * K, cmax, dup);
        c.track_partition = false;
        if (off + U > cap) {
            // first range: size the real edges from its distinct ratio (+25 %); later growth keeps
            // what is already appended
            const uint64_t want = off == 0 ? (uint64_t)((double)U / (double)N * (double)total * 1.25) + U
                                           : (off + U) + (off + U) / 4;
            cap = std::max(want, off + U);
            *real = (K2 *)c.ws.get(Workspace::REAL, cap * sizeof(K2), off * sizeof(K2), c.stream);
            if (COUNTED) *realc = (uint32_t *)c.ws.get(Workspace::REALC, cap * 4, off * 4, c.stream);
        }
        HIP_CHECK(hipMemcpyAsync(*real + off, ka, U * sizeof(K2), hipMemcpyDeviceToDevice, c.stream));
        if (COUNTED) HIP_CHECK(hipMemcpyAsync(*realc + off, ca, U * 4, hipMemcpyDeviceToDevice, c.stream));
        off += U;
    }
    if (!*real) {
        *real = (K2 *)c.ws.get(Workspace::REAL, sizeof(K2));
        if (COUNTED) *realc = (uint32_t *)c.ws.get(Workspace::REALC, 4);
    }
    c.timings.n_extracted = total / (canonical ? 2 : 1);  // valid windows (one k-mer per strand each)
    return off;
}

// ------------------------------------------------ canonical key rounds of the fused K1 (configs[3])
//
// configs[3]'s share of one GPU (125 M reads, 1.5e10 windows) does not fit one pass: its canonical
// k-mers alone are 120 GB, twice that with the sort's ping-pong buffer.  collect_ranges re-scans
// every read once per key range and extracts BOTH strands (19 ranges and 3.0e10 keys sorted there:
// 1.35 s of a 1.45 s step).  Here the fused K1's pass A runs once, and the canonical k-mers are
// collected in R rounds, each a contiguous interval of the level-1 buckets of the WHOLE input's MSD
// plan: pass B keeps only the round's buckets (extract_partition.hpp: a bucket mask), and the round's keys
// are sorted and deduplicated with that plan's later levels -- every final bucket has the size it
// has in a one-pass build -- and appended to the canonical set, in BOSS order since the rounds are.
// The rc stage, the dummies and the emit then run on the whole canonical set exactly as in the
// one-pass build (the role of SortedSetDisk's merged chunks, boss_chunk_construct.cpp:664-933).
// R is the fewest rounds whose sort buffers fit next to what the later stages hold
// (memory_preallocated, else the free HBM).  False (nothing kept) where the fused K1 does not apply.
template <int L, bool COUNTED>
static bool collect_rounds_fused(Ctx &c, unsigned K, bool canonical, uint32_t cmax, const BuildInput &in,
                                 Key<L> **out, uint32_t **outc, uint64_t *U_out) {
    // L = 2: u128 windows (32 < K <= 64, BASELINE configs[2]'s k = 63) -- the wide pass A and the generic
    // pass B on 256-thread tiles; the later levels are the MSD sort's exact ones
    using K2 = Key<L>;
    const uint64_t npos = in.seq_len >= K ? in.seq_len - K + 1 : 0;
    if (c.range_scan || c.disk || !fused_applies(c, K, npos, L == 1 ? 32 : 64)) return false;
    // a previous build's stage buffers would crowd out this build's rounds: they go now (and are
    // allocated again at the sizes this build needs)
    Tracer tr{c, 0};
    c.ws.release_stage_buffers();
    tr("rounds: release");
    FusedA A;
    fused_pass_a(c, K, canonical, in, &A, 1, fused_block<L>());
    tr("rounds: pass A", A.N, (uint64_t)(A.dup * 1000));
    const uint64_t N = A.N;
    MsdPlan plan = L == 1 ? fused_plan(c, N, 2 * K, A.dup, !COUNTED && K <= 32) : msd_plan<L>(c, N, 2 * K, A.dup);
    if (L == 2 && plan.levels && plan.digit_end[1] > 9) {
        // the u128 pass B takes at most 9 bits: level 1 of 9, the rest split over the later levels
        const unsigned T = plan.digit_end[plan.levels];
        MsdPlan q{};
        q.levels = 1 + (T - 9 + MSD_DBITS - 1) / MSD_DBITS;
        q.digit_end[1] = 9;
        for (unsigned l = 2; l <= q.levels; ++l) q.digit_end[l] = 9 + (T - 9) * (l - 1) / (q.levels - 1);
        plan = q;
    }
    if (!plan.levels) return false;
    const unsigned b1 = plan.digit_end[1];
    const uint32_t nb1 = 1u << b1;
    std::vector<uint64_t> h1(nb1, 0);
    for (uint32_t i = 0; i < (1u << FUSED_HB); ++i) h1[i >> (FUSED_HB - b1)] += A.h[i];
    // rounds: the later stages hold ~5 keys of 8 B per distinct canonical k-mer (the canonical set, the
    // real edges, the rc sort's two buffers) plus the rows; a round holds its keys twice (+ counts)
    uint32_t R = c.force_ranges;
    double budget = c.mem_budget;
    if (budget <= 0) {
        size_t fr = 0, tot = 0;
        HIP_CHECK(hipMemGetInfo(&fr, &tot));
        budget = 0.9 * ((double)fr + (double)c.ws.held());
    }
    const double u_est = std::min((double)N, (double)N / A.dup * 1.25);
    if (!R) {
        const double kb = (double)sizeof(K2);
        // (u128: the rounds hold only the growing canonical set beside their buffers, which are released
        // before the rc stage; reserving the later stages' 5 keys per distinct k-mer as well would plan
        // ~10 rounds at configs[2] instead of 2)
        const double per_u = L == 2 ? kb * 2 + 4.0 + (COUNTED ? 8.0 : 0.0)
                                    : kb * 5 + 4.0 + (COUNTED ? 4.0 * 5 + 8.0 : 0.0);
        const double per_key = 2 * kb + (COUNTED ? 8.0 : 0.0);
        const double avail = budget - per_u * u_est;
        R = avail > 0 ? (uint32_t)std::min<double>(std::ceil((double)N * per_key / avail), nb1) : nb1;
        R = std::max<uint32_t>(R, 2);
    }
    R = std::min(R, nb1);
    const std::vector<uint64_t> bb = balanced_bounds(h1.data(), nb1, (int)R);
    std::vector<uint64_t> nr(R, 0);
    uint64_t nmax = 1;
    for (uint32_t r = 0; r < R; ++r) {
        for (uint64_t b = bb[r]; b < bb[r + 1]; ++b) nr[r] += h1[b];
        nmax = std::max(nmax, nr[r]);
    }
    // two rounds of pass B (configs[3]'s share; configs[2]'s u128 rounds) become one when both rounds' keys fit beside the
    // partition buffer and the canonical set: the pass writes round 0's buckets into KA and round 1's into
    // KA2 (per-bucket destinations, bdelta), so the reads are scanned once (pass B 2 x 40 -> 45 ms).
    // MTG_ROUNDS_ONE_B=0: a pass B per round.  (Round 5 kept it off: the third ~64 GB block left the later
    // stages no room -- their 4-20 GB requests each took a whole idle 64 GB block -- until the workspace
    // learned to carve pieces off its kept blocks, Workspace::take_cached)
    bool one_b = false;
    // (u128, configs[2]: both rounds' keys, 141 GB, beside KB and the canonical set -- ~255 of the 309 GB)
    if (R == 2 && c.rounds_one_b && ((L == 1 && !COUNTED && K <= 32) || fast2_applies<L, COUNTED>(c, K, canonical))) {
        const double kb = (double)sizeof(K2);
        const double need = ((double)N + (double)nmax) * kb + u_est * 1.25 * kb + (double)(1ull << 30);
        one_b = need <= budget;
    }
    // a 3-level plan's speculative level 3 partitions into KA, which level 2 has emptied by then (the
    // round's keys in KB; with one pass B, round 1's in KA2): KA is sized for the level's slack-sized
    // buckets -- 1.2 n + 512 a bucket (spec_caps_kernel), +5 % -- when that fits the budget, so the level
    // needs no third round-sized block and its histogram pass goes (configs[3]'s share: levels 2 and 3
    // were both exact, a 60 GB read each per round)
    uint64_t ka_keys = one_b ? nr[0] : nmax;
    struct SpareGuard {  // never left set past this function (a thrown build included)
        Ctx &c;
        ~SpareGuard() { c.spec_into = nullptr, c.spec_into_bytes = 0, c.spec_mid_into = nullptr, c.spec_mid_bytes = 0; }
    } spare_guard{c};
    if (L == 1 && !COUNTED && plan.levels == 3 && c.spec3 && c.spec_final && c.spec_inplace && !c.use_lsd) {
        double fmax = 0;
        for (uint32_t r = 0; r < R; ++r) fmax = std::max(fmax, (double)(bb[r + 1] - bb[r]) / (double)nb1);
        const double cap = (1.2 * (double)nmax + 512.0 * (double)(1ull << plan.digit_end[3]) * fmax) * 1.05 + 65536.0;
        const double kb = (double)sizeof(K2);
        const double need = (cap + (one_b ? (double)nr[1] : 0.0) + (double)nmax) * kb + u_est * 1.25 * kb +
                            (double)(1ull << 30);
        if (cap > (double)ka_keys && need <= budget) ka_keys = (uint64_t)cap;
    }
    K2 *ka = (K2 *)c.ws.get(Workspace::KA, ka_keys * sizeof(K2));
    if (L == 1 && ka_keys > (one_b ? nr[0] : nmax)) c.spec_into = ka, c.spec_into_bytes = ka_keys * sizeof(K2);
    K2 *ka2 = one_b ? (K2 *)c.ws.get(Workspace::KA2, std::max<uint64_t>(nr[1], 1) * sizeof(K2)) : nullptr;
    // ... and the speculative middle level (spec_mid_level) partitions into KB: sized for its tile-aligned
    // slack buckets -- 1.2 n + 512 keys and up to one tile a bucket -- when that fits too
    uint64_t kb_keys = nmax;
    if (L == 1 && c.spec_into && c.spec_mid && plan.levels == 3) {
        double fmax = 0;
        for (uint32_t r = 0; r < R; ++r) fmax = std::max(fmax, (double)(bb[r + 1] - bb[r]) / (double)nb1);
        const double mcap = 1.2 * (double)nmax * 1.05 +
                            (512.0 + MsdTraits<L>::TILE) * (double)(1ull << plan.digit_end[2]) * fmax + 65536.0;
        const double kbb = (double)sizeof(K2);
        const double need = ((double)ka_keys + (one_b ? (double)nr[1] : 0.0) + mcap) * kbb + u_est * 1.25 * kbb +
                            (double)(1ull << 30);
        if (need <= budget) kb_keys = (uint64_t)mcap;
    }
    K2 *kb = (K2 *)c.ws.get(Workspace::KB, kb_keys * sizeof(K2));
    if (kb_keys > nmax) c.spec_mid_into = kb, c.spec_mid_bytes = kb_keys * sizeof(K2);
    uint32_t *ca = COUNTED ? (uint32_t *)c.ws.get(Workspace::CA, nmax * 4) : nullptr;
    uint32_t *cb = COUNTED ? (uint32_t *)c.ws.get(Workspace::CB, nmax * 4) : nullptr;
    tr("rounds: buffers", R, nmax);
    if (one_b) {
        // round 1's buckets start at nr[0] in the pass's layout and at ka2 in memory
        std::vector<long long> delta(nb1, 0);
        // (two allocations: their distance in elements from the addresses, not a pointer difference)
        const long long d1 = ((long long)(intptr_t)ka2 - (long long)(intptr_t)ka) / (long long)sizeof(K2) -
                             (long long)nr[0];
        for (uint32_t b = (uint32_t)bb[1]; b < nb1; ++b) delta[b] = d1;
        long long *dd = (long long *)c.ws.get(Workspace::ROUND_DELTA, nb1 * 8);
        HIP_CHECK(hipMemcpyAsync(dd, delta.data(), nb1 * 8, hipMemcpyHostToDevice, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));  // `delta` is a block-local host vector
        const uint32_t *dh1_all = nullptr;
        const uint64_t n = fused_pass_b<L, COUNTED>(c, K, canonical, cmax, in, A, b1, nullptr, ka, ca, &dh1_all, dd);
        if (n != N) throw std::runtime_error("the collect rounds' pass B differs from its histogram");
        tr("rounds: pass B (both rounds)", R, n);
    }
    std::vector<uint32_t> h1r(nb1);  // one_b: a round's level-1 counts (zero outside its buckets)
    if (c.debug)
        fprintf(stderr, "[mtg debug] canonical rounds: N=%lu dup=%.2f levels=%u digit1=%u rounds=%u largest=%lu\n",
                (unsigned long)N, A.dup, plan.levels, b1, R, (unsigned long)nmax);
    c.timings.n_positions = npos;
    c.timings.n_extracted = N;
    c.timings.n_batches = R;
    c.timings.collect_mode = 2;
    uint64_t off = 0, cap = 0;
    *out = nullptr;
    *outc = nullptr;
    bool first = true;
    // the canonical set sized from pass A's duplication estimate up front, so that every round's final
    // gather writes its distinct keys straight into it (c.sort_out) instead of into the round buffer and a
    // copy after (a 19 GB copy per configs[3] round); a round that finds more falls back to that copy
    if (R > 1 && !COUNTED) {
        cap = (uint64_t)u_est + 65536;
        *out = (K2 *)c.ws.get(Workspace::CANON, cap * sizeof(K2));
    }
    struct SortOutGuard {
        Ctx &c;
        ~SortOutGuard() { c.sort_out = nullptr, c.sort_out_vals = nullptr, c.sort_out_cap = ~0ull, c.ridx = Ctx::RoundIndex{}; }
    } sort_out_guard{c};
    // the rc stage reads the canonical set through a bucket index over the rc sort's final bits (its plan
    // for the set's size, estimated here from pass A's duplication): each round's speculative gather writes
    // its buckets' entries (Ctx::ridx) instead of a bucket_index pass over the whole set after the rounds
    // (5.6 ms at configs[3]'s share); a round that takes another path leaves it to that pass
    unsigned fb_est = 0;
    uint64_t *rgi = nullptr;
    bool rgi_ok = false;
    if (canonical && !COUNTED && c.round_index) {
        const MsdPlan rp = rc_plan<L>(c, std::max<uint64_t>(1, (uint64_t)((double)N / A.dup)), 2 * K);
        fb_est = rp.levels ? rp.digit_end[rp.levels] : 0;
        if (fb_est >= b1 && fb_est <= 26) {
            rgi = (uint64_t *)c.ws.get(Workspace::CANON_IDX, ((1ull << fb_est) + 2) * 8);
            rgi_ok = true;
        }
    }
    for (uint32_t r = 0; r < R; ++r) {
        if (rgi_ok && !nr[r]) {  // no keys: the round's index entries all point at the set's next position
            const uint64_t lo = bb[r] << (fb_est - b1), hi = bb[r + 1] << (fb_est - b1);
            if (lo < hi)
                fill_u64_kernel<<<dim3((unsigned)std::min<uint64_t>(ceil_div(hi - lo, 256), 4096)), dim3(256), 0, c.stream>>>(
                    rgi, lo, hi, off);
            HIP_CHECK(hipGetLastError());
        }
        if (!nr[r]) continue;
        const uint32_t *dh1 = nullptr;
        uint64_t n = 0;
        K2 *xa = ka, *xb = kb;
        uint32_t *xac = ca, *xbc = cb;
        if (one_b) {
            // this round's slice of the whole layout, and its level-1 counts
            for (uint32_t b = 0; b < nb1; ++b) h1r[b] = b >= bb[r] && b < bb[r + 1] ? (uint32_t)h1[b] : 0u;
            uint32_t *d = (uint32_t *)c.ws.get(Workspace::HIST1, nb1 * 4);
            HIP_CHECK(hipMemcpyAsync(d, h1r.data(), nb1 * 4, hipMemcpyHostToDevice, c.stream));
            HIP_CHECK(hipStreamSynchronize(c.stream));  // h1r is rewritten next round
            dh1 = d;
            n = nr[r];
            xa = r == 0 ? ka : ka2;
        } else {
            BucketSel sel;
            sel.add(bb[r], bb[r + 1]);
            n = fused_pass_b<L, COUNTED>(c, K, canonical, cmax, in, A, b1, &sel, ka, ca, &dh1);
            if (n != nr[r]) throw std::runtime_error("a collect round's k-mers differ from its histogram");
            tr("rounds: pass B", r, n);
        }
        c.track_partition = first;  // the roofline's partition pass: the first round's level 2
        MsdPlan rplan = plan;
        if (L == 1 && c.round_bits && plan.levels >= 2) {
            // keys per final bucket in this round against the whole input's average (Ctx::round_bits)
            const unsigned T = plan.digit_end[plan.levels], bp = plan.digit_end[plan.levels - 1];
            const double nbk = (double)(bb[r + 1] - bb[r]) * (double)(1ull << (T - b1));
            const double rho = ((double)n / nbk) / ((double)N / (double)(1ull << T));
            if (rho < 0.75 && T >= bp + 2) rplan.digit_end[plan.levels] = T - 1;
        }
        if (*out && off < cap && (!COUNTED || *outc)) {
            c.sort_out = *out + off, c.sort_out_cap = cap - off;
            c.sort_out_vals = COUNTED ? *outc + off : nullptr;  // (the counts travel with their keys)
        }
        if (rgi_ok) c.ridx = Ctx::RoundIndex{rgi, fb_est, off, bb[r] << (fb_est - b1), bb[r + 1] << (fb_est - b1), false};
        const uint64_t U = msd_sort_unique<L, COUNTED>(c, &xa, &xb, &xac, &xbc, n, 2 * K, cmax, A.dup, dh1, false,
                                                       nullptr, true, nullptr, &rplan);
        rgi_ok = rgi_ok && c.ridx.written;
        c.ridx = Ctx::RoundIndex{};
        c.sort_out = nullptr, c.sort_out_vals = nullptr, c.sort_out_cap = ~0ull;
        c.track_partition = false;
        first = false;
        tr("rounds: sort", r, U);
        if (off + U > cap) {
            // first round: size the canonical set from its distinct ratio (+25 %); later growth keeps
            // what is already appended
            const uint64_t want = off == 0 ? (uint64_t)((double)U / (double)n * (double)N * 1.25) + U
                                           : (off + U) + (off + U) / 4;
            cap = std::max(want, off + U);
            *out = (K2 *)c.ws.get(Workspace::CANON, cap * sizeof(K2), off * sizeof(K2), c.stream);
            if (COUNTED) *outc = (uint32_t *)c.ws.get(Workspace::CANONC, cap * 4, off * 4, c.stream);
        }
        if (xa != *out + off) {  // (gathered into the round buffer, not straight into the set)
            HIP_CHECK(hipMemcpyAsync(*out + off, xa, U * sizeof(K2), hipMemcpyDeviceToDevice, c.stream));
            if (COUNTED) HIP_CHECK(hipMemcpyAsync(*outc + off, xac, U * 4, hipMemcpyDeviceToDevice, c.stream));
        }
        off += U;
        if (c.debug)
            fprintf(stderr, "[mtg debug]   round %u: buckets [%lu, %lu) n=%lu -> %lu distinct\n", r,
                    (unsigned long)bb[r], (unsigned long)bb[r + 1], (unsigned long)n, (unsigned long)U);
    }
    if (!*out) {
        *out = (K2 *)c.ws.get(Workspace::CANON, sizeof(K2));
        if (COUNTED) *outc = (uint32_t *)c.ws.get(Workspace::CANONC, 4);
    }
    debug_check_sorted(c, "canonical rounds", *out, off);
    c.spec_into = nullptr, c.spec_into_bytes = 0, c.spec_mid_into = nullptr, c.spec_mid_bytes = 0;
    // the round buffers (sized for the largest round) go; the rc stage takes KB and SPEC_A again at
    // its own size
    for (auto sl : {Workspace::KA, Workspace::KA2, Workspace::CA, Workspace::KB, Workspace::CB, Workspace::SPEC_A,
                    Workspace::SPEC_B})
        c.ws.release(sl);
    // the fused rc merge reads the canonical keys through their bucket index over the rc sort's final
    // bits (a one-pass build gets it from its own sort's groups)
    c.gidx = Ctx::GroupIndex{};
    if (canonical && off && !COUNTED) {
        const MsdPlan rp = rc_plan<L>(c, off, 2 * K);
        const unsigned fb = rp.levels ? rp.digit_end[rp.levels] : 0;
        if (fb && fb <= 26) {
            const uint64_t nb = 1ull << fb;
            uint64_t *gi = (uint64_t *)c.ws.get(Workspace::CANON_IDX, (nb + 2) * 8);
            if (rgi_ok && fb == fb_est && gi == rgi) {  // written by the rounds' gathers: its two end entries
                fill_u64_kernel<<<dim3(1), dim3(256), 0, c.stream>>>(gi, nb, nb + 2, off);
                HIP_CHECK(hipGetLastError());
                if (c.debug) fprintf(stderr, "[mtg debug] canonical rounds: bucket index from the rounds' gathers\n");
            } else {
                bucket_index<L>(c, *out, off, 2 * K - fb, nb, gi);
                HIP_CHECK(hipMemcpyAsync(gi + nb + 1, gi + nb, 8, hipMemcpyDeviceToDevice, c.stream));
            }
            c.gidx = Ctx::GroupIndex{*out, off, fb, 2 * K, gi};

        }
    }
    *U_out = off;
    return true;
}

// K4: the reverse complements of a sorted canonical set ka[0..U) (add_reverse_complements,
// boss_chunk_construct.cpp:179-222), sorted on their own.  rc(x) of odd K is never x, so it is a
// 1:1 map; even K drops the palindromes and doubles their counts (rc_augment_kernel).  `buf`
// (+ `bufc`) takes the rc keys; the sorted result is in *rk / *rkc.  Returns their number.
template <int L2, bool COUNTED>
static uint64_t stage_rc(Ctx &c, unsigned K, unsigned cbits, uint32_t cmax, Key<L2> *ka,
                         uint32_t *ca, uint64_t U, Key<L2> *buf, uint32_t *bufc, Key<L2> **rk,
                         uint32_t **rkc, RcMerge<L2> *rm = nullptr, bool sort = true) {
    // rm: merge the sorted rc keys straight into rm->out (rm->done), when the MSD local pass can;
    // !sort: leave the rc keys unsorted in buf (the multi-GPU build routes them to their owners)
    using K2 = Key<L2>;
    uint64_t Urc = U;
    uint32_t *rc_hist = nullptr;
    bool rc_level1 = false;  // buf already partitioned by the rc sort's level-1 digit
    // the fused merge's plan (rc_plan: u128 merge groups twice as full); the plain sort plans its own
    const bool own_plan = rm && L2 == 2 && c.rc_wide;
    const MsdPlan rcp = own_plan ? rc_plan<L2>(c, U, 2 * K) : MsdPlan{};
    if (K & 1) {
        unsigned rc_hist_bits = 0;
        if (!c.use_lsd && sort) {
            const MsdPlan plan = own_plan ? rcp : msd_plan<L2>(c, U, 2 * K, 1.0);
            if (plan.levels) {
                rc_hist_bits = plan.digit_end[1];
                rc_hist = (uint32_t *)c.ws.get(Workspace::HIST1, (1u << rc_hist_bits) * 4);
                HIP_CHECK(hipMemsetAsync(rc_hist, 0, (1u << rc_hist_bits) * 4, c.stream));
            }
        }
        bool done = false;
        if constexpr (!COUNTED) {
            if (c.gap.valid && c.gap.dst == (const void *)ka && sort) {
                // the canonical set still in its speculative buckets (Ctx::gap): read it there
                const bool fuse = c.rc_fuse && rc_hist && rc_hist_bits <= 9 && c.gap1_n == 0 && U;
                const uint64_t tiles = ceil_div(U, RcPartTraits<L2>::TILE);
                // (fuse: the histogram only)
                rc_map_gapped_kernel<L2><<<dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(c.gap.nb, 16), 16384))),
                                           dim3(256), 0, c.stream>>>((const K2 *)c.gap.keys, c.gap.bstart, c.gap.ustart,
                                                                     c.gap.nb, fuse ? nullptr : buf, K, rc_hist, rc_hist_bits);
                HIP_CHECK(hipGetLastError());
                if (fuse) {
                    uint64_t *tile_g = (uint64_t *)c.ws.get(Workspace::RC_TILEG, tiles * 8);
                    rc_tile_bucket_kernel<<<dim3((unsigned)ceil_div(c.gap.nb, 256)), dim3(256), 0, c.stream>>>(
                        c.gap.ustart, c.gap.nb, RcPartTraits<L2>::TILE, tile_g);
                    HIP_CHECK(hipGetLastError());
                    // the histogram above gives the level-1 bucket starts; the rc keys are then written
                    // straight into their level-1 buckets (rc_partition_gapped_kernel)
                    const uint64_t nbk = 1ull << rc_hist_bits;
                    uint64_t *st = (uint64_t *)c.ws.get(Workspace::RC_L1START, (nbk + 1) * 8);
                    auto *cur = (unsigned long long *)c.ws.get(Workspace::RC_L1CUR, nbk * 8);
                    uint32_t ep;
                    uint64_t *desc = acquire_desc(c, 1, &ep);
                    HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
                    scan_counts_kernel<<<dim3(1), dim3(512), 0, c.stream>>>(rc_hist, nbk, st, desc, ep, &c.small->counter,
                                                                           &c.small->error);
                    HIP_CHECK(hipGetLastError());
                    HIP_CHECK(hipMemcpyAsync(cur, st, nbk * 8, hipMemcpyDeviceToDevice, c.stream));
                    rc_partition_gapped_kernel<L2><<<dim3((unsigned)xcd_grid(tiles)), dim3(512), 0, c.stream>>>(
                        (const K2 *)c.gap.keys, c.gap.bstart, c.gap.ustart, tile_g, c.gap.nb, U, K, rc_hist_bits, cur,
                        buf);
                    HIP_CHECK(hipGetLastError());
                    rc_level1 = true;
                }
                done = true;
            }
        }
        if (!done) {
            ensure_compact(c);
            rc_map_kernel<L2, COUNTED><<<dim3((unsigned)std::min<uint64_t>(ceil_div(U, 256 * 4), 16384)),
                                         dim3(256), 0, c.stream>>>(ka, ca, buf, bufc, U, K, rc_hist, rc_hist_bits);
            HIP_CHECK(hipGetLastError());
        }
    } else {
        ensure_compact(c);
        reset_small(c);
        const uint64_t tiles = ceil_div(U, 1024);
        uint32_t desc_ep;
        uint64_t *desc = acquire_desc(c, tiles, &desc_ep);
        rc_augment_kernel<L2, COUNTED><<<dim3((unsigned)tiles), dim3(256), 0, c.stream>>>(
            ka, ca, buf, bufc, U, K, cbits, cmax, desc, desc_ep,
            &c.small->counter, &c.small->total, &c.small->error);
        HIP_CHECK(hipGetLastError());
        Urc = read_u64(c, &c.small->total);
    }
    if (!sort) {
        *rk = buf;
        *rkc = bufc;
        return Urc;
    }
    K2 *ra = buf, *rb = (K2 *)c.ws.get(Workspace::RC_ALT, Urc * sizeof(K2));
    uint32_t *rca = bufc, *rcb = COUNTED ? (uint32_t *)c.ws.get(Workspace::RC_ALTC, Urc * 4) : nullptr;
    if (c.use_lsd) radix_sort<L2, COUNTED>(c, &ra, &rb, &rca, &rcb, Urc, 2 * K, false);
    else Urc = msd_sort_unique<L2, COUNTED>(c, &ra, &rb, &rca, &rcb, Urc, 2 * K, cmax, 1.0, rc_hist, true, nullptr,
                                            rc_level1, rm, own_plan && rcp.levels ? &rcp : nullptr);
    *rk = ra;
    *rkc = rca;
    return Urc;
}

// LSD sort + unique of the raw dummy k-mers da[0..Draw) (db is the ping-pong buffer); returns
// D and leaves the distinct dummies in *dk.  (An MSD sort of the dummies, planned for the 5-of-8
// value density of lifted chars and with a read-before-CAS hash for their repeated keys, measured
// 24.5 vs 7.5 ms per cfg2 step and 24.9 vs 0.51 s per cfg3 step: groups of the $-padded source
// levels overflow the LDS tables and fall back.)
// the dense-rank dummy sort (boss_kernels.hpp: dummy_rank): `ranks` (u64 view of one of the two
// Draw-key buffers xa / xb) sorted + deduplicated, the distinct ranks decoded to lifted keys in
// whichever buffer does not hold them (both hold Draw lifted keys); returns D, *dk = the keys
template <int L3, int LR = 1>
static uint64_t sort_unique_dummy_ranks(Ctx &c, unsigned kb, Key<L3> *xa, Key<L3> *xb, Key<LR> *ranks, uint64_t Draw,
                                        Key<L3> **dk) {
    static_assert(sizeof(Key<LR>) <= sizeof(Key<L3>), "the rank buffers are the lifted key buffers");
    Key<LR> *ra = ranks, *rb = (void *)ranks == (void *)xa ? (Key<LR> *)xb : (Key<LR> *)xa;
    uint32_t *nv = nullptr;
    const unsigned nbits = dummy_rank_bits(kb);
    // (the real k-mers' MSD partition + LDS-hash unique on these ranks: dummy stage 4.4 -> 6.8 ms)
    radix_sort<LR, false>(c, &ra, &rb, &nv, &nv, Draw, nbits, false, true);  // (dense ranks: the low digit varies)
    reset_small(c);
    const uint64_t ut = ceil_div(Draw, 2048);
    uint32_t udesc_ep;
    uint64_t *udesc = acquire_desc(c, ut, &udesc_ep);
    unique_kernel<LR, false><<<dim3((unsigned)ut), dim3(256), 0, c.stream>>>(
        ra, nullptr, Draw, rb, nullptr, udesc, udesc_ep, &c.small->counter, &c.small->total, &c.small->error);
    HIP_CHECK(hipGetLastError());
    Key<L3> *outk = (void *)rb == (void *)xa ? xb : xa;
    // (a block per 256 dummies up to 16384 blocks, each a contiguous chunk; the grid is sized for Draw and the
    // kernel reads D from the device, so the copy of D to the host overlaps the decode)
    dummy_decode_kernel<L3, LR><<<dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(Draw, 256), 16384))),
                                  dim3(256), 0, c.stream>>>(rb, 0, kb, outk, &c.small->total);
    HIP_CHECK(hipGetLastError());
    const uint64_t D = read_u64(c, &c.small->total);
    *dk = outk;
    return D;
}

// sort + unique of the lifted dummy keys da[0..Draw) (db is the ping-pong buffer); returns D and
// leaves the distinct dummies in *dk.  For k <= 30 they are sorted as dense u64 ranks (8 LSD passes
// of 8-byte keys instead of 12 of 16-byte ones); otherwise, or when a key is not of the dummy shape,
// by an LSD sort of the lifted keys.  (An MSD sort of the dummies, planned for the 5-of-8 value
// density of lifted chars and with a read-before-CAS hash for their repeated keys, measured 24.5 vs
// 7.5 ms per cfg2 step and 24.9 vs 0.51 s per cfg3 step: groups of the $-padded source levels
// overflow the LDS tables and fall back.)
template <int L3>
static uint64_t sort_unique_dummies(Ctx &c, unsigned K, Key<L3> *da, Key<L3> *db, uint64_t Draw,
                                    Key<L3> **dk) {
    uint64_t D = 0;
    uint32_t *nv = nullptr;
    const unsigned kb = K - 1;
    const int LR = dummy_rank_limbs(kb);
    if (c.dummy_ranks && kb >= 1 && LR && (LR == 1 || L3 >= 2) && Draw) {
        HIP_CHECK(hipMemsetAsync(&c.small->bad_dummy, 0, 4, c.stream));
        const unsigned g = (unsigned)std::min<uint64_t>(ceil_div(Draw, 256), 16384);
        if (LR == 1)
            dummy_encode_kernel<L3, 1><<<dim3(g), dim3(256), 0, c.stream>>>(da, Draw, kb, (Key<1> *)db, &c.small->bad_dummy);
        else
            dummy_encode_kernel<L3, 2><<<dim3(g), dim3(256), 0, c.stream>>>(da, Draw, kb, (Key<2> *)db, &c.small->bad_dummy);
        HIP_CHECK(hipGetLastError());
        uint32_t bad = 0;
        HIP_CHECK(hipMemcpyAsync(&bad, &c.small->bad_dummy, 4, hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));
        if (!bad) {
            if (LR == 1) return sort_unique_dummy_ranks<L3, 1>(c, kb, da, db, (Key<1> *)db, Draw, dk);
            if constexpr (L3 >= 2) return sort_unique_dummy_ranks<L3, 2>(c, kb, da, db, (Key<2> *)db, Draw, dk);
        }
        if (c.debug) fprintf(stderr, "[mtg debug] dummy keys outside the rank shape: lifted sort\n");
    }
    {
        radix_sort<L3, false>(c, &da, &db, &nv, &nv, Draw, 3 * K, false);
        reset_small(c);
        const uint64_t ut = ceil_div(Draw, 2048);
        uint32_t udesc_ep;
        uint64_t *udesc = acquire_desc(c, ut, &udesc_ep);
        unique_kernel<L3, false><<<dim3((unsigned)ut), dim3(256), 0, c.stream>>>(
            da, nullptr, Draw, db, nullptr, udesc, udesc_ep, &c.small->counter, &c.small->total,
            &c.small->error);
        HIP_CHECK(hipGetLastError());
        D = read_u64(c, &c.small->total);
    }
    *dk = db;
    return D;
}

// remember the bucket index over the real edges for the split emit's dummy ranks
static void note_bucket_index(Ctx &c, const void *keys, uint64_t n, const uint64_t *start, unsigned shift) {
    c.bidx_keys = keys;
    c.bidx_n = n;
    c.bidx = start;
    c.bidx_shift = shift;
    c.bidx_gen = c.ws.generation(Workspace::BUCKETS);
}

// the remembered bucket index still describes keys[0..n): the same array and count, and its entries still
// in the BUCKETS slot it was written to (a released or regrown slot may now hold another stage's data)
static bool bidx_valid(const Ctx &c, const void *keys, uint64_t n) {
    return c.bidx && c.bidx_keys == keys && c.bidx_n == n && (const void *)c.bidx == c.ws.peek(Workspace::BUCKETS) &&
           c.bidx_gen == c.ws.generation(Workspace::BUCKETS);
}

// K5/K6 on one device: dummy sinks and sources (all levels) of the sorted real edges ka[0..R)
template <int L2, int L3>
static uint64_t stage_dummies_local(Ctx &c, unsigned K, const Key<L2> *ka, uint64_t R, Key<L3> **dk) {
    using K3 = Key<L3>;
    const unsigned k = K - 1;
    const unsigned B = bucket_bits<L2>(R, 2 * K);
    const unsigned bshift = 2 * K - B;
    const uint64_t nb = 1ull << B;
    uint64_t *bstart = (uint64_t *)c.ws.get(Workspace::BUCKETS, (nb + 2) * 8);
    if (!(bidx_valid(c, ka, R) && c.bidx_shift == bshift && c.bidx == bstart)) {
        const uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(R + 1, 256), 8192));
        bucket_index_kernel<L2><<<dim3((unsigned)g), dim3(256), 0, c.stream>>>(ka, R, bshift, nb, bstart);
        HIP_CHECK(hipGetLastError());
        note_bucket_index(c, ka, R, bstart, bshift);
    }
    uint8_t *flags = (uint8_t *)c.ws.get(Workspace::FLAGS, R + 1);
    uint8_t *in_flag = (uint8_t *)c.ws.get(Workspace::INFLAG, R + 1);
    const uint64_t wtiles = ceil_div(R, DummyTraits<L2>::WTILE);
    uint32_t *tcnt = (uint32_t *)c.ws.get(Workspace::DTCNT, (wtiles + 1) * 4);
    uint64_t *toff = (uint64_t *)c.ws.get(Workspace::DTOFF, (wtiles + 1) * 8);
    uint64_t Draw = 0;
    // the dense-rank path writes the source levels with <= DUMMY_BITMAP_M real chars as bits of a bitmap
    // (dummy_write_kernel), so the count pass counts kbig levels per source
    const bool bitmap_path = L2 == 1 && c.dummy_ranks && c.dummy_bitmap && k >= 1 && k <= 30;
    const unsigned ks = std::min<unsigned>(k, DUMMY_BITMAP_M + 1), kbig = bitmap_path ? k - ks : k;
    if (R) {
        HIP_CHECK(hipMemsetAsync(in_flag, 0, R, c.stream));
        dummy_sink_kernel<L2><<<dim3((unsigned)ceil_div(R, DummyTraits<L2>::TILE)), dim3(256), 0,
                                c.stream>>>(ka, R, K, bstart, bshift, flags, in_flag);
        HIP_CHECK(hipGetLastError());
        dummy_count_kernel<<<dim3((unsigned)wtiles), dim3(256), 0, c.stream>>>(flags, in_flag, R, kbig, tcnt);
        HIP_CHECK(hipGetLastError());
        uint32_t ep;
        const uint64_t st = ceil_div(wtiles, 4096);
        uint64_t *desc = acquire_desc(c, st, &ep);
        HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
        scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(
            tcnt, wtiles, toff, desc, ep, &c.small->counter, &c.small->error);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(&Draw, toff + wtiles, 8, hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));
    }
    *dk = nullptr;
    if constexpr (L2 == 1) {
        if (bitmap_path) {  // written as dense ranks: no lifted keys until the decode
            const uint64_t nbits = dummy_bitmap_base(ks), nwords = ceil_div(nbits, 32);
            uint32_t *bm = (uint32_t *)c.ws.get(Workspace::DBITMAP, nwords * 4);
            HIP_CHECK(hipMemsetAsync(bm, 0, nwords * 4, c.stream));
            const uint64_t cap = Draw + nbits;  // u64 ranks: the written ones, then at most every bit
            K3 *da = (K3 *)c.ws.get(Workspace::DA, cap * sizeof(K3));
            K3 *db = (K3 *)c.ws.get(Workspace::DB, cap * sizeof(K3));
            if (R) {
                dummy_write_kernel<L2, L3, true><<<dim3((unsigned)wtiles), dim3(256), 0, c.stream>>>(
                    ka, flags, in_flag, R, K, toff, da, kbig, bm);
                HIP_CHECK(hipGetLastError());
            }
            HIP_CHECK(hipMemcpyAsync(&c.small->total, &Draw, 8, hipMemcpyHostToDevice, c.stream));
            dummy_bitmap_ranks_kernel<<<dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(nwords, 256), 4096))),
                                        dim3(256), 0, c.stream>>>(bm, nwords, k, ks, (uint64_t *)da, &c.small->total);
            HIP_CHECK(hipGetLastError());
            const uint64_t Dall = read_u64(c, &c.small->total);  // (also orders the copy of the host local)
            if (c.debug)
                fprintf(stderr, "[mtg debug] dummies: %lu written + %lu from the bitmap (%u levels per source)\n",
                        (unsigned long)Draw, (unsigned long)(Dall - Draw), ks);
            if (!Dall) return 0;
            return sort_unique_dummy_ranks<L3>(c, k, da, db, (Key<1> *)da, Dall, dk);
        }
    }
    if (!Draw) return 0;
    K3 *da = (K3 *)c.ws.get(Workspace::DA, Draw * sizeof(K3));
    K3 *db = (K3 *)c.ws.get(Workspace::DB, Draw * sizeof(K3));
    if constexpr (L2 == 1) {
        if (c.dummy_ranks && k <= 30) {  // written as dense ranks: no lifted keys until the decode
            dummy_write_kernel<L2, L3, true><<<dim3((unsigned)wtiles), dim3(256), 0, c.stream>>>(ka, flags, in_flag,
                                                                                                  R, K, toff, da);
            HIP_CHECK(hipGetLastError());
            return sort_unique_dummy_ranks<L3>(c, k, da, db, (Key<1> *)da, Draw, dk);
        }
    }
    if constexpr (L2 <= 2 && L3 >= 2) {
        if (c.dummy_ranks && dummy_rank_limbs(k) == 2) {  // 30 < k <= 62: dense u128 ranks (configs[2]: k = 62)
            dummy_write_kernel<L2, L3, true, 2><<<dim3((unsigned)wtiles), dim3(256), 0, c.stream>>>(ka, flags, in_flag,
                                                                                                     R, K, toff, da);
            HIP_CHECK(hipGetLastError());
            return sort_unique_dummy_ranks<L3, 2>(c, k, da, db, (Key<2> *)da, Draw, dk);
        }
    }
    dummy_write_kernel<L2, L3><<<dim3((unsigned)wtiles), dim3(256), 0, c.stream>>>(ka, flags, in_flag, R, K,
                                                                                    toff, da);
    HIP_CHECK(hipGetLastError());
    return sort_unique_dummies<L3>(c, K, da, db, Draw, dk);
}

template <int L3, bool COUNTED>
static void emit_stream(Ctx &c, unsigned k, uint32_t wmax, const Key<L3> *sk, const uint32_t *sc, uint64_t M,
                        uint64_t R, BuildOutput *out);

// K7 + K8: lift + merge the real edges with the sorted dummies (behind the main dummy row when
// `root`), then W / last / F / weights.  Rows go to out[1..]; out row 0 is the leading row.
template <int L2, int L3, bool COUNTED>
static void stage_merge_emit(Ctx &c, EventTimer &tm, int *ev_merge, unsigned k, unsigned bits,
                             const Key<L2> *real, const uint32_t *realc, uint64_t R, const Key<L3> *dk,
                             uint64_t D, bool root, BuildOutput *out) {
    using K3 = Key<L3>;
    const unsigned K = k + 1;
    const uint32_t wmax = bits >= 32 ? 0xFFFFFFFFu : (uint32_t)((1ull << bits) - 1);
    const uint64_t M = (root ? 1 : 0) + R + D;
    if (c.fused_emit && !c.emit_slow && M) {
        // K7 + K8 without the merged stream (split_emit_kernel): the dummies' output rows from
        // their ranks in A, then one pass over the output rows; a violated premise or a redundant
        // sink falls through to the exact unfused path below
        using SE = SplitEmitTraits<L2>;
        const uint64_t nout = M + 1;
        uint8_t *W = (uint8_t *)c.ws.get(Workspace::OW, nout);
        uint8_t *last = (uint8_t *)c.ws.get(Workspace::OLAST, nout);
        uint32_t *weights = COUNTED ? (uint32_t *)c.ws.get(Workspace::OWEIGHTS, nout * 4) : nullptr;
        uint64_t *pos = (uint64_t *)c.ws.get(Workspace::DPOS, D * 8);
        uint8_t *wl = (uint8_t *)c.ws.get(Workspace::DWL, D);
        const uint64_t ntiles = ceil_div(nout, SE::TILE);
        uint64_t *jsplit = (uint64_t *)c.ws.get(Workspace::SPLITS, (ntiles + 1) * 8);
        reset_small(c);
        if (D) {
            const bool idx = bidx_valid(c, real, R);
            dummy_rank_kernel<L2, L3><<<dim3((unsigned)ceil_div(D, 256)), dim3(256), 0, c.stream>>>(
                real, R, dk, D, K, idx ? c.bidx : nullptr, c.bidx_shift, root ? 2 : 1, pos, wl,
                &c.small->skip, &c.small->root_same);
            HIP_CHECK(hipGetLastError());
        }
        split_points_kernel<SE::TILE><<<dim3((unsigned)ceil_div(ntiles + 1, 256)), dim3(256), 0, c.stream>>>(
            pos, D, ntiles, jsplit);
        HIP_CHECK(hipGetLastError());
        split_emit_kernel<L2, COUNTED><<<dim3((unsigned)ntiles), dim3(SE::BLOCK), 0, c.stream>>>(
            real, realc, R, pos, wl, jsplit, nout, root ? 1 : 0, &c.small->root_same, wmax, W, last, weights);
        HIP_CHECK(hipGetLastError());
        f_bounds_split_kernel<L3, L2><<<1, 64, 0, c.stream>>>(real, R, dk, D, K, root ? 1 : 0, c.small->fhist);
        HIP_CHECK(hipGetLastError());
        *ev_merge = tm.mark();
        Small h;
        HIP_CHECK(hipMemcpyAsync(&h, c.small, sizeof(Small), hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));
        if (!h.skip) {
            for (int ch = 0; ch < 5; ++ch) out->F[ch] = h.fhist[ch];
            out->W = W;
            out->last = last;
            out->weights = weights;
            out->n = nout;
            out->n_real = R;
            out->n_dummy = M - R;
            return;
        }
    }
    K3 *sk = (K3 *)c.ws.get(Workspace::STREAM, M * sizeof(K3));
    uint32_t *sc = COUNTED ? (uint32_t *)c.ws.get(Workspace::SCOUNT, M * 4) : nullptr;
    if (root) {
        set_root_row_kernel<<<1, 1, 0, c.stream>>>((uint64_t *)sk, L3, COUNTED ? sc : nullptr);
        HIP_CHECK(hipGetLastError());
    }
    merge_sorted<L3, L2, true, COUNTED, false>(c, real, realc, R, dk, nullptr, D, K, sk, sc, root ? 1 : 0);
    debug_check_sorted(c, "merged stream", sk, M);
    *ev_merge = tm.mark();
    emit_stream<L3, COUNTED>(c, k, wmax, sk, sc, M, R, out);
}

// K8 over a sorted lifted stream sk[0..M) (+ counts): initialize_chunk (boss_chunk.cpp:32-133),
// rows to out[1..], compacted past redundant dummy sinks when there are any
template <int L3, bool COUNTED>
static void emit_stream(Ctx &c, unsigned k, uint32_t wmax, const Key<L3> *sk, const uint32_t *sc, uint64_t M,
                        uint64_t R, BuildOutput *out) {
    uint8_t *W = (uint8_t *)c.ws.get(Workspace::OW, M + 1);
    uint8_t *last = (uint8_t *)c.ws.get(Workspace::OLAST, M + 1);
    uint32_t *weights = COUNTED ? (uint32_t *)c.ws.get(Workspace::OWEIGHTS, (M + 1) * 4) : nullptr;
    HIP_CHECK(hipMemsetAsync(W, 0, 1, c.stream));
    HIP_CHECK(hipMemsetAsync(last, 0, 1, c.stream));
    if (COUNTED) HIP_CHECK(hipMemsetAsync(weights, 0, 4, c.stream));
    reset_small(c);
    uint64_t rows = M;
    bool slow = c.emit_slow;
    if (!slow && M) {
        emit_fast_kernel<L3, COUNTED><<<dim3((unsigned)ceil_div(M + 1, 256 * 8)), dim3(256), 0, c.stream>>>(
            sk, sc, M, k, wmax, W, last, weights, &c.small->skip);
        HIP_CHECK(hipGetLastError());
        f_bounds_kernel<L3><<<1, 64, 0, c.stream>>>(sk, M, k, c.small->fhist);
        HIP_CHECK(hipGetLastError());
        Small h;
        HIP_CHECK(hipMemcpyAsync(&h, c.small, sizeof(Small), hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));
        for (int ch = 0; ch < 5; ++ch) out->F[ch] = h.fhist[ch];
        slow = h.skip != 0;  // a redundant dummy sink: rows must be compacted
    } else if (!M) {
        for (int ch = 0; ch < 5; ++ch) out->F[ch] = 0;
        slow = false;
    }
    if (slow) {
        reset_small(c);
        const uint64_t tiles = ceil_div(M, 1024);
        uint32_t desc_ep;
        uint64_t *desc = acquire_desc(c, tiles, &desc_ep);
        emit_kernel<L3, COUNTED><<<dim3((unsigned)tiles), dim3(256), 0, c.stream>>>(
            sk, sc, M, k, wmax, W, last, weights, c.small->fhist, desc, desc_ep, &c.small->counter,
            &c.small->total, &c.small->error);
        HIP_CHECK(hipGetLastError());
        unsigned long long fh[8];
        HIP_CHECK(hipMemcpyAsync(fh, c.small->fhist, sizeof(fh), hipMemcpyDeviceToHost, c.stream));
        rows = read_u64(c, &c.small->total);
        uint64_t s = 0;
        for (int ch = 0; ch < 5; ++ch) {
            out->F[ch] = s;
            s += fh[ch];
        }
    }
    out->W = W;
    out->last = last;
    out->weights = weights;
    out->n = rows + 1;
    out->n_real = R;
    out->n_dummy = rows - R;
}

template <int L2, bool COUNTED>
static bool want_spill(Ctx &c, unsigned K, bool canonical, const BuildInput &in, uint32_t P);
template <int L2, int L3, bool COUNTED>
static void run_pipeline_spill(Ctx &c, unsigned k, bool canonical, unsigned bits, const BuildInput &in, uint32_t P,
                               BuildOutput *out);

template <int L2, int L3, bool COUNTED>
static void run_pipeline(Ctx &c, unsigned k, bool canonical, unsigned bits,
                         const BuildInput &in, BuildOutput *out) {
    using K2 = Key<L2>;
    const unsigned K = k + 1;
    const unsigned cbits = bits <= 8 ? 8 : bits <= 16 ? 16 : 32;
    const uint32_t cmax = cbits == 8 ? 0xFFu : cbits == 16 ? 0xFFFFu : 0xFFFFFFFFu;
    mtg_boss_timings &T = c.timings;
    T = mtg_boss_timings{};
    note_bucket_index(c, nullptr, 0, nullptr, 0);
    c.gap = Ctx::GappedSet{};
    T.world = 1;
    T.n_batches = 1;
    HIP_CHECK(hipMemsetAsync(c.small, 0, sizeof(Small), c.stream));
    EventTimer tm(c.stream);
    const int ev_start = tm.mark();
    Tracer tr{c, 0};

    // ---- K1 extract (fused with K2's first partition level when it applies)
    K2 *ka, *kb;
    uint32_t *ca, *cb;
    uint64_t N = 0;
    double dup = 0;
    const uint32_t *hist1 = nullptr;
    MsdPlan fplan{};
    c.radix_ms = 0;
    c.radix_bytes = 0;
    c.radix_launches = 0;
    const uint32_t P = plan_ranges<L2, COUNTED>(c, K, canonical, in);
    if (want_spill<L2, COUNTED>(c, K, canonical, in, P)) {  // not even the real edges fit: spill
        run_pipeline_spill<L2, L3, COUNTED>(c, k, canonical, bits, in, P, out);
        return;
    }
    uint64_t U = 0, R = 0;
    int ev_extract, ev_sort, ev_unique;
    bool rounds = false;  // the canonical set collected in rounds of the fused K1 (collect_rounds_fused)
    if (P > 1) {
        ev_extract = tm.mark();
        if constexpr (L2 <= 2) {
            rounds = collect_rounds_fused<L2, COUNTED>(c, K, canonical, cmax, in, &ka, &ca, &U);
            if (rounds) {
                R = U;
                kb = (K2 *)c.ws.get(Workspace::KB, std::max<uint64_t>(U, 1) * sizeof(K2));
                cb = COUNTED ? (uint32_t *)c.ws.get(Workspace::CB, std::max<uint64_t>(U, 1) * 4) : nullptr;
            }
        }
        if (!rounds) {
            // ---- K1-K4 one key range at a time (both strands in canonical mode): the real edges
            R = U = collect_ranges<L2, COUNTED>(c, K, canonical, cmax, in, P, &ka, &ca);
            T.collect_mode = 1;
        }
        ev_sort = ev_unique = tm.mark();
        T.n_unique = U;
    } else {
    if (stage_extract_windows<L2, COUNTED>(c, K, canonical, cmax, in, &ka, &kb, &ca, &cb, &N))
        dup = 1.0;  // one k-mer per record: distinct up to a strand
    else if (!stage_extract_fused<L2, COUNTED>(c, K, canonical, cmax, in, &ka, &kb, &ca, &cb, &N, &dup, &hist1,
                                                &fplan))
        N = stage_extract<L2, COUNTED>(c, K, canonical, cmax, in, &ka, &kb, &ca, &cb);
    ev_extract = tm.mark();

    // ---- K2 sort + K3 unique / saturating count merge (ka)
    c.want_gidx = canonical;  // the fused rc merge reads the canonical keys' bucket index
    c.defer_gather_req = canonical;  // ... and may read them in their speculative buckets (Ctx::gap)
    U = stage_collect<L2, COUNTED>(c, K, cmax, &ka, &kb, &ca, &cb, N, dup, true, hist1, &fplan);
    c.defer_gather_req = false;
    c.want_gidx = false;
    ev_sort = tm.mark();
    T.n_unique = U;
    if (c.debug) ensure_compact(c);
    debug_check_sorted(c, "collected k-mers", ka, U);
    ev_unique = tm.mark();

    // ---- K4 reverse complements (CANONICAL_ONLY): rc(x) of the sorted canonical set is sorted
    // on its own (no duplicates) and merged with it
    R = U;
    }
    if (canonical && U && (P == 1 || rounds)) {
        K2 *rk;
        uint32_t *rkc;
        // the real edges hold at most 2U keys (the palindromes of even K drop out of the rc set)
        K2 *real = (K2 *)c.ws.get(Workspace::REAL, 2 * U * sizeof(K2));
        uint32_t *realc = COUNTED ? (uint32_t *)c.ws.get(Workspace::REALC, 2 * U * 4) : nullptr;
        RcMerge<L2> rm{ka, ca, U, real, realc};
        // the dummy stage's bucket index (stage_dummies_local) comes out of the fused merge, sized
        // for R = 2U (odd K; even K loses its palindromes, and the dummy stage rebuilds the index
        // when that changes its size)
        rm.ib = bucket_bits<L2>(2 * U, 2 * K);
        rm.istart = (uint64_t *)c.ws.get(Workspace::BUCKETS, ((1ull << rm.ib) + 2) * 8);
        if (!kb) kb = (K2 *)c.ws.get(Workspace::KB, std::max<uint64_t>(U, 1) * sizeof(K2));  // (speculative layout)
        if (COUNTED && !cb) cb = (uint32_t *)c.ws.get(Workspace::CB, std::max<uint64_t>(U, 1) * 4);
        const uint64_t Urc = stage_rc<L2, COUNTED>(c, K, cbits, cmax, ka, ca, U, kb, cb, &rk, &rkc, &rm);
        R = U + Urc;
        if (!rm.done) {
            ensure_compact(c);
            merge_sorted<L2, L2, false, COUNTED, true>(c, ka, ca, U, rk, rkc, Urc, K, real, realc, 0);
        }
        ka = real;
        ca = realc;
        if (rounds) {
            // the canonical set and the rc sort's buffers are merged into REAL: give them back before the
            // dummy stage (configs[2]: 41 + 2 x 32 GB of u128 keys; with them held, the emit's last array
            // did not fit the 288 GB), and the dummy buffers take them from the workspace's kept blocks
            for (auto sl : {Workspace::CANON, Workspace::CANONC, Workspace::KB, Workspace::CB, Workspace::RC_ALT,
                            Workspace::RC_ALTC, Workspace::SPEC_A, Workspace::SPEC_B, Workspace::SPEC_AC,
                            Workspace::SPEC_BC})
                c.ws.release(sl);
            c.gidx = Ctx::GroupIndex{};  // it indexed the CANON block given back above
        }
    }
    ensure_compact(c);  // (a no-op unless the canonical set is still in buckets)
    T.n_real = R;
    tr("collect + rc", U, R);
    debug_check_sorted(c, "real k-mers", ka, R);
    const int ev_rc = tm.mark();

    // ---- K5/K6 dummy sinks and sources (all levels), sort + unique
    Key<L3> *dk = nullptr;
    const uint64_t D = stage_dummies_local<L2, L3>(c, K, ka, R, &dk);
    T.n_dummy = D + 1;
    tr("dummies", D);
    debug_check_sorted(c, "dummy k-mers", dk, D);
    const int ev_dummy = tm.mark();

    // ---- K7 lift + merge, K8 W / last / F / weights
    int ev_merge;
    stage_merge_emit<L2, L3, COUNTED>(c, tm, &ev_merge, k, bits, ka, ca, R, dk, D, true, out);
    const int ev_emit = tm.mark();
    tr("emit", out->n);
    check_error_word(c);
    HIP_CHECK(hipStreamSynchronize(c.stream));

    T.n_rows = out->n;
    T.extract_ms = tm.ms(ev_start, ev_extract);
    T.sort_ms = tm.ms(ev_extract, ev_sort);
    T.unique_ms = tm.ms(ev_sort, ev_unique);
    T.rc_ms = tm.ms(ev_unique, ev_rc);
    T.dummy_ms = tm.ms(ev_rc, ev_dummy);
    T.merge_ms = tm.ms(ev_dummy, ev_merge);
    T.emit_ms = tm.ms(ev_merge, ev_emit);
    T.total_ms = tm.ms(ev_start, ev_emit);
    T.radix_launches = c.radix_launches;
    T.radix_pass_ms = c.radix_launches ? c.radix_ms / c.radix_launches : 0;
    T.radix_bytes = c.radix_launches ? c.radix_bytes / c.radix_launches : 0;
    T.peak_bytes = c.ws.held();
}

// ------------------------------------------------------------------------ multi-GPU pipeline
//
// One rank per GPU builds the chunk of one range of BOSS order (dist_kernels.hpp):
//   K1-K3 on the rank's reads -> exchange 1: the sorted distinct k-mers by range (RCCL
//   all-to-all-v of contiguous slices) -> dedupe / saturating count merge of the P runs ->
//   [canonical: rc of the owned canonical k-mers, exchange 2 of both strands by the final
//   ranges, merge] -> exchange of the sink / in-edge queries -> sinks at the owner, sources
//   routed to theirs -> sort + unique -> lift + merge -> W / last / F / weights.
// The chunks concatenate in rank order with BOSS::Chunk::extend (boss_chunk.cpp:230-270).

// ranges over 4^m prefixes: bounds[j] = first prefix of rank j, balanced on `hist` (host)
static std::vector<uint64_t> balanced_bounds(const uint64_t *hist, uint64_t nb, int P) {
    std::vector<uint64_t> bounds(P + 1, nb);
    bounds[0] = 0;
    unsigned __int128 total = 0;
    for (uint64_t b = 0; b < nb; ++b) total += hist[b];
    unsigned __int128 cum = 0;
    int j = 1;
    for (uint64_t b = 0; b <= nb && j < P; ++b) {
        while (j < P && cum * (unsigned)P >= total * (unsigned)j) bounds[j++] = b;
        if (b < nb) cum += hist[b];
    }
    return bounds;
}

// the same ranges in lifted ($ACGT, 3 bits per char) prefixes; a bound past the last prefix
// becomes 8^m, above every lifted prefix
static std::vector<uint64_t> lifted_bounds(const std::vector<uint64_t> &b2, unsigned m) {
    std::vector<uint64_t> b3(b2.size());
    const uint64_t nb = 1ull << (2 * m);
    for (size_t j = 0; j < b2.size(); ++j) {
        if (b2[j] >= nb) {
            b3[j] = 1ull << (3 * m);
            continue;
        }
        uint64_t v = 0;
        for (unsigned i = 0; i < m; ++i) v |= (((b2[j] >> (2 * i)) & 3) + 1) << (3 * i);
        b3[j] = v;
    }
    return b3;
}

__global__ void gather_strided_kernel(const uint64_t *__restrict__ src, uint64_t stride, uint32_t cnt,
                                      uint64_t *__restrict__ dst) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < cnt) dst[j] = src[(uint64_t)j * stride];
}

struct Dist {
    Comm &comm;
    int P, me;
    unsigned m;       // prefix chars of the range partition
    unsigned shift2;  // 2-bit prefix = key >> shift2
    uint64_t nb;      // 4^m prefixes
    EventTimer *tm;
    std::vector<std::pair<int, int>> xev;  // event pairs around exchanges
    uint32_t coresident = 1;  // ranks on this rank's GPU (dist_coresident), the HBM they share
};

// a GPU's identity across hosts: FNV-1a of the host name and the device's PCI bus id (identical nodes
// repeat the same bus ids, so the bus id alone made every rank at the same slot of another node look
// co-resident -- ADVICE r5).  MTG_HOST_ID replaces the host name (the two-process tests play two hosts)
static uint64_t device_identity(const char *host, const char *bus) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const char *s) {
        for (const char *q = s; *q; ++q) h = (h ^ (uint8_t)*q) * 1099511628211ull;
    };
    mix(host);
    mix("|");
    mix(bus);
    return h;
}

static uint32_t coresident_count(const uint64_t *ids, int P, uint64_t mine) {
    uint32_t n = 0;
    for (int r = 0; r < P; ++r) n += ids[r] == mine;
    return std::max<uint32_t>(n, 1);
}

// the ranks that share this rank's GPU (threads of one process on its device, or several processes
// on one card): an all-gather of device_identity.  The rounds planners give each of them an equal
// share of the free HBM -- each planning for the whole free memory over-committed it (8 co-resident
// ranks of the round-4 simulation ran out of memory)
static uint32_t dist_coresident(Ctx &c, Dist &d) {
    if (d.P <= 1) return 1;
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    char bus[64] = {};
    if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, dev) != hipSuccess) {
        (void)hipGetLastError();
        snprintf(bus, sizeof(bus), "device %d", dev);
    }
    char host[256] = {};
    if (const char *e = getenv("MTG_HOST_ID")) snprintf(host, sizeof(host), "%s", e);
    else if (gethostname(host, sizeof(host) - 1) != 0) snprintf(host, sizeof(host), "?");
    const uint64_t h = device_identity(host, bus);
    uint64_t *dv = (uint64_t *)c.ws.get(Workspace::XMAT, (1 + (uint64_t)d.P) * 8);
    HIP_CHECK(hipMemcpyAsync(dv, &h, 8, hipMemcpyHostToDevice, c.stream));
    d.comm.allgather_u64(dv, dv + 1, 1, c.stream);
    std::vector<uint64_t> all(d.P);
    HIP_CHECK(hipMemcpyAsync(all.data(), dv + 1, (uint64_t)d.P * 8, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));  // `h` is a host local
    return coresident_count(all.data(), d.P, h);
}

// a rank's HBM budget for planning its rounds: memory_preallocated, else its share of the free HBM
// (the ranks on its GPU split it) plus what its workspace holds
static double dist_budget(const Ctx &c, const Dist &d) {
    if (c.mem_budget > 0) return c.mem_budget;
    size_t fr = 0, tot = 0;
    HIP_CHECK(hipMemGetInfo(&fr, &tot));
    return 0.9 * ((double)fr / (double)std::max<uint32_t>(d.coresident, 1) + (double)c.ws.held());
}

// prefix index of a sorted 2-bit array: start[p] = first key with prefix >= p, p in [0, nb]
template <int L2>
static uint64_t *prefix_index(Ctx &c, const Dist &d, Workspace::Slot slot, const Key<L2> *keys, uint64_t n) {
    uint64_t *st = (uint64_t *)c.ws.get(slot, (d.nb + 2) * 8);
    const uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(n + 1, 256), 8192));
    bucket_index_kernel<L2><<<dim3((unsigned)g), dim3(256), 0, c.stream>>>(keys, n, d.shift2, d.nb, st);
    HIP_CHECK(hipGetLastError());
    return st;
}

// global prefix histogram of the sorted arrays (summed over all ranks) -> balanced ranges;
// also returns every array's slice offsets for those ranges (host, P + 1 each)
template <int L2>
static std::vector<uint64_t> dist_ranges(Ctx &c, Dist &d, int na, const Key<L2> *const *arrs,
                                         const uint64_t *ns, std::vector<std::vector<uint64_t>> *soff,
                                         unsigned rc_K = 0) {
    // rc_K (canonical mode): also count the rc keys of arrs[0] (sampled), so the ranges balance
    // both strands of the real-edge set
    uint64_t *hist = (uint64_t *)c.ws.get(Workspace::XHIST, d.nb * 8);
    std::vector<std::vector<uint64_t>> starts(na);
    for (int a = 0; a < na; ++a) {
        uint64_t *st = prefix_index<L2>(c, d, a == 0 ? Workspace::XSTART_A : Workspace::XSTART_B, arrs[a], ns[a]);
        hist_from_starts_kernel<<<dim3((unsigned)ceil_div(d.nb, 256)), dim3(256), 0, c.stream>>>(st, d.nb, hist, a);
        HIP_CHECK(hipGetLastError());
        starts[a].resize(d.nb + 1);
        HIP_CHECK(hipMemcpyAsync(starts[a].data(), st, (d.nb + 1) * 8, hipMemcpyDeviceToHost, c.stream));
    }
    if (rc_K && ns[0]) {
        const uint64_t stride = std::max<uint64_t>(1, ns[0] >> 22);
        const uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(ceil_div(ns[0], stride), 256), 4096));
        rc_prefix_sample_kernel<L2><<<dim3((unsigned)g), dim3(256), 0, c.stream>>>(
            arrs[0], ns[0], rc_K, d.shift2, 2 * d.m, stride, (unsigned long long *)hist);
        HIP_CHECK(hipGetLastError());
    }
    const int e0 = d.tm->mark();
    d.comm.allreduce_sum_u64(hist, d.nb, c.stream);
    d.xev.push_back({e0, d.tm->mark()});
    std::vector<uint64_t> h(d.nb);
    HIP_CHECK(hipMemcpyAsync(h.data(), hist, d.nb * 8, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    std::vector<uint64_t> bounds = balanced_bounds(h.data(), d.nb, d.P);
    soff->assign(na, std::vector<uint64_t>(d.P + 1));
    for (int a = 0; a < na; ++a)
        for (int j = 0; j <= d.P; ++j) (*soff)[a][j] = starts[a][bounds[j]];
    return bounds;
}

// all-to-all-v of `na` arrays (slice offsets soff[a], P + 1 each) into one receive buffer laid
// out array-major then by source rank; returns the received element count
template <typename T>
static uint64_t exchange_runs(Ctx &c, Dist &d, int na, const T *const *arrs, const uint32_t *const *cnts,
                         const std::vector<std::vector<uint64_t>> &soff, Workspace::Slot rslot,
                         Workspace::Slot rcslot, T **recv, uint32_t **recvc,
                         std::vector<uint64_t> *runs = nullptr) {
    const int P = d.P;
    std::vector<uint64_t> scnt(na * P);
    for (int a = 0; a < na; ++a)
        for (int j = 0; j < P; ++j) scnt[a * P + j] = soff[a][j + 1] - soff[a][j];
    // every rank's counts -> the full matrix
    const size_t V = scnt.size();
    uint64_t *dm = (uint64_t *)c.ws.get(Workspace::XMAT, (V + V * P) * 8);
    HIP_CHECK(hipMemcpyAsync(dm, scnt.data(), V * 8, hipMemcpyHostToDevice, c.stream));
    const int e0 = d.tm->mark();
    d.comm.allgather_u64(dm, dm + V, V, c.stream);
    std::vector<uint64_t> mat(V * P);
    HIP_CHECK(hipMemcpyAsync(mat.data(), dm + V, V * P * 8, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    std::vector<uint64_t> rcnt(V), roff(V);
    uint64_t total = 0;
    for (int a = 0; a < na; ++a)
        for (int i = 0; i < P; ++i) {
            rcnt[a * P + i] = mat[(size_t)i * V + a * P + d.me];
            roff[a * P + i] = total;
            total += rcnt[a * P + i];
        }
    *recv = (T *)c.ws.get(rslot, total * sizeof(T));
    if (cnts) *recvc = (uint32_t *)c.ws.get(rcslot, total * 4);
    for (int a = 0; a < na; ++a) {
        d.comm.alltoallv(arrs[a], &scnt[a * P], soff[a].data(), *recv, &rcnt[a * P], &roff[a * P], sizeof(T),
                         c.stream);
        if (cnts)
            d.comm.alltoallv(cnts[a], &scnt[a * P], soff[a].data(), *recvc, &rcnt[a * P], &roff[a * P], 4,
                             c.stream);
        for (int j = 0; j < P; ++j)
            if (j != d.me) c.timings.n_sent += scnt[a * P + j];
    }
    HIP_CHECK(hipStreamSynchronize(c.stream));
    d.xev.push_back({e0, d.tm->mark()});
    if (runs) {  // where every received run starts (array-major, then source rank) + the end
        runs->assign(roff.begin(), roff.end());
        runs->push_back(total);
    }
    return total;
}

// route the keys produced by a kernel-side function (MODE, dist_kernels.hpp) to their owners:
// count -> scan -> write into the send buffer; returns slice offsets (P + 1)
template <int L, int MODE>
static std::vector<uint64_t> route(Ctx &c, const Dist &d, const Key<L> *in, uint64_t n, unsigned K,
                                   unsigned pshift, unsigned pbits, const std::vector<uint64_t> &bounds,
                                   Key<L> *out, const uint32_t *in_v = nullptr, uint32_t *out_v = nullptr) {
    const int P = d.P;
    if (P > MAX_ROUTE) throw std::runtime_error("more destinations than the routing kernels support");
    std::vector<uint64_t> soff(P + 1, 0);
    if (!n) return soff;
    const uint64_t ntiles = ceil_div(n, RT_TILE);
    uint64_t *db = (uint64_t *)c.ws.get(Workspace::BOUNDS, (P + 1) * 8);
    HIP_CHECK(hipMemcpyAsync(db, bounds.data(), (P + 1) * 8, hipMemcpyHostToDevice, c.stream));
    uint32_t *tcnt = (uint32_t *)c.ws.get(Workspace::RTCNT, (P * ntiles + 1) * 4);
    uint64_t *toff = (uint64_t *)c.ws.get(Workspace::RTOFF, (P * ntiles + 1) * 8);
    route_count_kernel<L, MODE><<<dim3((unsigned)ntiles), dim3(RT_BLOCK), 0, c.stream>>>(
        in, n, K, pshift, pbits, db, (uint32_t)P, tcnt, ntiles);
    HIP_CHECK(hipGetLastError());
    uint32_t ep;
    const uint64_t st = ceil_div(P * ntiles, 4096);
    uint64_t *desc = acquire_desc(c, st, &ep);
    HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
    scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(tcnt, P * ntiles, toff, desc, ep,
                                                                      &c.small->counter, &c.small->error);
    HIP_CHECK(hipGetLastError());
    route_write_kernel<L, MODE><<<dim3((unsigned)ntiles), dim3(RT_BLOCK), 0, c.stream>>>(
        in, n, K, pshift, pbits, db, (uint32_t)P, toff, ntiles, out, in_v, out_v);
    HIP_CHECK(hipGetLastError());
    uint64_t *g = (uint64_t *)c.ws.get(Workspace::XGATHER, (P + 1) * 8);
    gather_strided_kernel<<<dim3((unsigned)ceil_div(P + 1, 256)), 256, 0, c.stream>>>(toff, ntiles, (uint32_t)P + 1, g);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(soff.data(), g, (P + 1) * 8, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    return soff;
}

// ------------------------------------------------- multi-GPU: the bounded-memory (batched) collect
//
// A rank share too big for one pass (BASELINE configs[3]: 125 M reads = 1.5e10 windows per GPU)
// is collected in rounds.  The owner ranges are intervals of the range kernels' top-char bins
// (RB_CHARS node chars, range_extract.hpp), balanced on the global bin histogram; every owner range
// is cut into `rounds` consecutive batches balanced on the same histogram.  Round r: every rank
// extracts the k-mers of the r-th batch of every owner from its own reads (both strands in canonical
// mode: exactly the real-edge set, see collect_ranges), sorts and dedupes them, and sends each owner
// its slice; the owner merges the P sorted runs (saturating count addition, sorted_multiset.cpp:54-84)
// and appends them to its real edges.  The batches of one owner are consecutive in BOSS order, so
// the appended array is sorted, and no rc stage or second exchange is needed.  The reference bounds
// a multi-machine build by suffix instead (cli/build.cpp:106-148); this build keeps one exchange per
// round and one BOSS table.

// rounds of the batched collect: 1 (the single-pass dist path) when every rank's single-pass
// footprint fits its budget; else the most any rank needs (all ranks agree through an all-gather)
template <int L2, bool COUNTED>
static uint32_t plan_rounds_dist(Ctx &c, Dist &d, unsigned K, bool canonical, const BuildInput &in) {
    uint64_t want = 1;
    const uint64_t npos = in.seq_len >= K ? in.seq_len - K + 1 : 0;
    // bins of RB_CHARS node chars keep every emission group on one rank only for k - 1 >= RB_CHARS
    const bool can = K >= RB_CHARS + 2;
    if (can && c.force_ranges) {
        want = c.force_ranges;
    } else if (can) {
        const double per_key = (double)sizeof(Key<L2>) + (COUNTED ? 4.0 : 0.0);
        const double budget = dist_budget(c, d);
        // single pass: KA + KB over every window, the exchange buffers and the owned real edges
        if ((double)npos * per_key * 3.0 > budget || c.disk) {
            const double keys = (double)npos * (canonical ? 2.0 : 1.0);
            // a round holds its extracted keys twice (sort ping-pong), the received runs twice
            want = (uint64_t)std::ceil(keys * per_key * 4.0 / (0.4 * budget));
            want = std::max<uint64_t>(want, (uint64_t)std::ceil(keys / 2.0e9));
            want = std::max<uint64_t>(want, 2);
        }
    }
    uint64_t *dv = (uint64_t *)c.ws.get(Workspace::XMAT, (1 + (uint64_t)d.P) * 8);
    HIP_CHECK(hipMemcpyAsync(dv, &want, 8, hipMemcpyHostToDevice, c.stream));
    const int e0 = d.tm->mark();
    d.comm.allgather_u64(dv, dv + 1, 1, c.stream);
    d.xev.push_back({e0, d.tm->mark()});
    std::vector<uint64_t> all(d.P);
    HIP_CHECK(hipMemcpyAsync(all.data(), dv + 1, (uint64_t)d.P * 8, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));  // `want` is a host local
    uint64_t r = 1;
    for (uint64_t v : all) r = std::max(r, v);
    return (uint32_t)std::min<uint64_t>(r, RB_BINS);
}

template <int L2, bool COUNTED>
static uint64_t collect_ranges_dist(Ctx &c, Dist &d, unsigned K, bool canonical, uint32_t cmax,
                                    const BuildInput &in, uint32_t rounds, Key<L2> **real, uint32_t **realc,
                                    std::vector<uint64_t> *owner_bounds, Tracer &tr) {
    using K2 = Key<L2>;
    const uint64_t npos = in.seq_len >= K ? in.seq_len - K + 1 : 0;
    c.timings.n_positions = npos;
    c.timings.n_batches = rounds;
    const int both = canonical ? 1 : 0;
    constexpr int TILE = RangeTraits<L2>::TILE;
    const uint64_t tiles = ceil_div(npos, TILE);
    // count pass over this rank's reads, then the global bin histogram
    auto *dh = (unsigned long long *)c.ws.get(Workspace::XHIST, RB_BINS * 8);
    HIP_CHECK(hipMemsetAsync(dh, 0, RB_BINS * 8, c.stream));
    uint16_t *tbins = (uint16_t *)c.ws.get(Workspace::RANGE_BINS, std::max<uint64_t>(tiles, 1) * RB_BINS * 2);
    if (tiles) {
        range_count_kernel<L2><<<dim3((unsigned)tiles), dim3(256), 0, c.stream>>>(in.seq, in.seq_len, K, both, tbins);
        HIP_CHECK(hipGetLastError());
        range_bins_reduce_kernel<<<dim3((unsigned)std::min<uint64_t>(tiles, 2048)), dim3(RB_BINS), 0, c.stream>>>(
            tbins, tiles, dh);
        HIP_CHECK(hipGetLastError());
    }
    std::vector<uint64_t> local(RB_BINS), glob(RB_BINS);
    HIP_CHECK(hipMemcpyAsync(local.data(), dh, RB_BINS * 8, hipMemcpyDeviceToHost, c.stream));
    const int e0 = d.tm->mark();
    d.comm.allreduce_sum_u64((uint64_t *)dh, RB_BINS, c.stream);
    d.xev.push_back({e0, d.tm->mark()});
    HIP_CHECK(hipMemcpyAsync(glob.data(), dh, RB_BINS * 8, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    tr("range count", tiles);
    // owner intervals, then each cut into `rounds` batches
    const std::vector<uint64_t> ob = balanced_bounds(glob.data(), RB_BINS, d.P);
    std::vector<std::vector<uint64_t>> bb(d.P);
    for (int o = 0; o < d.P; ++o) {
        bb[o] = balanced_bounds(glob.data() + ob[o], ob[o + 1] - ob[o], (int)rounds);
        for (auto &v : bb[o]) v += ob[o];
    }
    *owner_bounds = ob;
    uint64_t own_total = 0;
    for (uint64_t b = ob[d.me]; b < ob[d.me + 1]; ++b) own_total += glob[b];
    uint32_t *tcnt = (uint32_t *)c.ws.get(Workspace::DTCNT, (tiles + 1) * 4);
    uint64_t *toff = (uint64_t *)c.ws.get(Workspace::DTOFF, (tiles + 1) * 8);
    uint64_t off = 0, cap = 0, extracted = 0;
    *real = nullptr;
    *realc = nullptr;
    for (uint32_t r = 0; r < rounds; ++r) {
        BinSet sel{};
        for (int o = 0; o < d.P; ++o) sel.add((uint32_t)bb[o][r], (uint32_t)bb[o][r + 1]);
        uint64_t nj = 0;
        for (uint32_t b = 0; b < RB_BINS; ++b)
            if (sel.has(b)) nj += local[b];
        K2 *ka = (K2 *)c.ws.get(Workspace::KA, std::max<uint64_t>(nj, 1) * sizeof(K2));
        K2 *kb = (K2 *)c.ws.get(Workspace::KB, std::max<uint64_t>(nj, 1) * sizeof(K2));
        uint32_t *ca = COUNTED ? (uint32_t *)c.ws.get(Workspace::CA, std::max<uint64_t>(nj, 1) * 4) : nullptr;
        uint32_t *cb = COUNTED ? (uint32_t *)c.ws.get(Workspace::CB, std::max<uint64_t>(nj, 1) * 4) : nullptr;
        uint64_t Ul = 0;
        if (nj) {
            range_tile_counts_kernel<<<dim3((unsigned)ceil_div(tiles, 4)), dim3(256), 0, c.stream>>>(tbins, tiles, sel,
                                                                                                     tcnt);
            HIP_CHECK(hipGetLastError());
            uint32_t ep;
            const uint64_t st = ceil_div(tiles, 4096);
            uint64_t *desc = acquire_desc(c, st, &ep);
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(tcnt, tiles, toff, desc, ep,
                                                                              &c.small->counter, &c.small->error);
            HIP_CHECK(hipGetLastError());
            range_write_kernel<L2, COUNTED><<<dim3((unsigned)tiles), dim3(256), 0, c.stream>>>(
                in.seq, in.seq_len, K, both, in.read_starts, in.read_counts, in.n_reads, in.rid_at, cmax, sel, toff, ka, ca);
            HIP_CHECK(hipGetLastError());
            const uint64_t N = read_u64(c, (const unsigned long long *)(toff + tiles));
            if (N != nj) throw std::runtime_error("range extraction count differs from its histogram");
            const double spread = (double)RB_BINS / (double)std::max<uint32_t>(1, sel.size());
            const double dup = estimate_dup<L2>(c, ka, N, 8.0) / spread;
            c.track_partition = r == 0;  // the roofline's partition pass: the first round's first level
            Ul = msd_sort_unique<L2, COUNTED>(c, &ka, &kb, &ca, &cb, N, 2 * K, cmax, dup);
            c.track_partition = false;
        }
        extracted += nj;
        tr("round collect", nj, Ul);
        // every owner's slice of the sorted local keys: the bin index of the keys at the owner bounds
        std::vector<std::vector<uint64_t>> soff(1, std::vector<uint64_t>(d.P + 1, 0));
        if (Ul) {
            uint64_t *st = prefix_index<L2>(c, d, Workspace::XSTART_A, ka, Ul);
            std::vector<uint64_t> starts(RB_BINS + 1);
            HIP_CHECK(hipMemcpyAsync(starts.data(), st, (RB_BINS + 1) * 8, hipMemcpyDeviceToHost, c.stream));
            HIP_CHECK(hipStreamSynchronize(c.stream));
            for (int j = 0; j <= d.P; ++j) soff[0][j] = starts[ob[j]];
        }
        K2 *xa = ka;
        uint32_t *xac = ca;
        uint64_t U = Ul;
        if (d.P > 1) {
            const K2 *arrs[1] = {ka};
            const uint32_t *cnts[1] = {ca};
            std::vector<uint64_t> runs;
            const uint64_t n1 = exchange_runs<K2>(c, d, 1, arrs, COUNTED ? cnts : nullptr, soff, Workspace::XA,
                                                  Workspace::XAC, &xa, &xac, &runs);
            U = n1;
            if (n1) {
                K2 *xb = (K2 *)c.ws.get(Workspace::XB, n1 * sizeof(K2));
                uint32_t *xbc = COUNTED ? (uint32_t *)c.ws.get(Workspace::XBC, n1 * 4) : nullptr;
                // the keys fill this owner's batch of the bins: plan as if spread over all of them
                const double spread = (double)RB_BINS / (double)std::max<uint64_t>(1, bb[d.me][r + 1] - bb[d.me][r]);
                const double dup1 = estimate_dup<L2>(c, xa, n1, 1.0) / spread;
                U = msd_sort_unique<L2, COUNTED>(c, &xa, &xb, &xac, &xbc, n1, 2 * K, cmax, dup1, nullptr, false,
                                                 &runs);
            }
            tr("round exchange + merge", n1, U);
        }
        if (off + U > cap) {
            // first filled round: size the owned real edges from its share of the owner's range
            uint64_t gr = 0;
            for (uint64_t b = bb[d.me][r]; b < bb[d.me][r + 1]; ++b) gr += glob[b];
            const uint64_t want = off == 0 && gr ? (uint64_t)((double)U / (double)gr * (double)own_total * 1.25) + U
                                                 : (off + U) + (off + U) / 4;
            cap = std::max(want, off + U);
            *real = (K2 *)c.ws.get(Workspace::REAL, cap * sizeof(K2), off * sizeof(K2), c.stream);
            if (COUNTED) *realc = (uint32_t *)c.ws.get(Workspace::REALC, cap * 4, off * 4, c.stream);
        }
        if (U) {
            HIP_CHECK(hipMemcpyAsync(*real + off, xa, U * sizeof(K2), hipMemcpyDeviceToDevice, c.stream));
            if (COUNTED) HIP_CHECK(hipMemcpyAsync(*realc + off, xac, U * 4, hipMemcpyDeviceToDevice, c.stream));
        }
        off += U;
    }
    if (!*real) {
        *real = (K2 *)c.ws.get(Workspace::REAL, sizeof(K2));
        if (COUNTED) *realc = (uint32_t *)c.ws.get(Workspace::REALC, 4);
    }
    c.timings.n_extracted = extracted / (canonical ? 2 : 1);  // valid windows (one k-mer per strand each)
    return off;
}

// ------------------------------------------ multi-GPU: the extraction routed straight to the owners
//
// The single build's fused K1 (extract_partition.hpp) already scatters every rank's k-mers by the
// top 9 bits of their key.  With the owner ranges drawn at 4-char (8-bit) boundaries -- unions of
// those buckets, balanced on the global histogram of pass A -- every owner's keys are one contiguous
// slice of the rank's scattered array: they go to the owner as extracted (exchange 1 moves every
// k-mer occurrence once), and the owner runs the single build's level-2 partition + LDS unique over
// the P received runs (the partition reads its input in any order), so each k-mer is sorted exactly
// once in the whole job.  The earlier design sorted and deduplicated each rank's k-mers locally,
// exchanged the distinct runs and deduplicated them again at the owner: at 1.25x local coverage
// (8 GPUs) the local dedupe keeps ~2/3 of the k-mers, so nearly every k-mer was sorted twice
// (DESIGN.md section 8).  Returns false when the fused extraction does not apply (the caller runs
// the local-collect path).
// the routed collect needs the fused K1 (u64 keys); MTG_COLLECT=ranges keeps the key-range collect
static bool routed_applies(const Ctx &c, unsigned K) {
    return c.fused && !c.use_lsd && K - 1 >= FUSED_HB / 2 && K <= 32 && !c.range_scan;
}

// one-window reads (KMC input) on every rank: cheaper through window_reads_kernel and the local
// collect than through the routed one.  Collective: the ranks share their layouts by an all-reduce.
static bool dist_window_input(Ctx &c, Dist &d, unsigned K, const BuildInput &in) {
    uint64_t *dv = (uint64_t *)c.ws.get(Workspace::XMAT, 8);
    const uint64_t win = window_layout(c, K, in) || in.seq_len == 0 ? 0 : 1;
    HIP_CHECK(hipMemcpyAsync(dv, &win, 8, hipMemcpyHostToDevice, c.stream));
    d.comm.allreduce_sum_u64(dv, 1, c.stream);
    uint64_t any_other = 0;
    HIP_CHECK(hipMemcpyAsync(&any_other, dv, 8, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));  // `win` is a host local
    return any_other == 0;
}

// Exchange 1 in pieces, hidden behind the owner sort.  Every owner's level-1 bucket interval is cut
// into Q consecutive sub-intervals balanced on the global histogram; piece q carries sub-interval q of
// every owner -- from each rank one contiguous slice of its scattered array per owner, at pass B's bucket
// cursors -- so the Q all-to-alls go out back to back on the exchange stream while the build stream
// sorts piece q - 1 (level 2 + LDS unique over its buckets, the single build's passes) and appends its
// distinct keys to the owned canonical set in BOSS order (the pieces are consecutive key ranges).  The
// reference has no runtime exchange (it shards by suffix, cli/build.cpp:106-148); the merge semantics are
// SortedMultiset's (sorted_multiset.cpp:54-84), the same as the one-exchange path.  The send counts of all
// pieces are known after pass B, so one all-gather sizes every receive before the first piece leaves.
// Returns the owned distinct keys (in the CANON slot); *hidden_ms = exchange time overlapped with sorting.
template <bool COUNTED>
static uint64_t routed_pieces(Ctx &c, Dist &d, unsigned K, uint32_t cmax, const Key<1> *ka, const uint32_t *ca,
                              const std::vector<unsigned long long> &cur, uint64_t nr, uint32_t nb1, unsigned B1,
                              unsigned OB, const std::vector<uint64_t> &bounds, const std::vector<uint64_t> &gh1,
                              const std::vector<uint64_t> &H, uint32_t Q, Key<1> **out, uint32_t **outc,
                              double *xspan_ms, double *hidden_ms, Tracer &tr) {
    using K2 = Key<1>;
    constexpr uint32_t NBH = 1u << FUSED_HB;
    const int P = d.P;
    std::vector<std::vector<uint64_t>> sub(P);
    for (int o = 0; o < P; ++o) {
        const uint64_t o0 = std::min<uint64_t>(bounds[o] << (B1 - OB), nb1);
        const uint64_t o1 = std::min<uint64_t>(bounds[o + 1] << (B1 - OB), nb1);
        sub[o] = balanced_bounds(gh1.data() + o0, o1 - o0, (int)Q);
        for (auto &v : sub[o]) v += o0;
    }
    auto at = [&](uint64_t b) -> uint64_t { return b >= nb1 ? nr : cur[b]; };
    // this rank's slices: piece-major, then owner; every rank's counts -> the matrix
    const size_t V = (size_t)Q * P;
    std::vector<uint64_t> scnt(V), soff(V);
    for (uint32_t q = 0; q < Q; ++q)
        for (int o = 0; o < P; ++o) {
            soff[q * P + o] = at(sub[o][q]);
            scnt[q * P + o] = at(sub[o][q + 1]) - soff[q * P + o];
        }
    uint64_t *dm = (uint64_t *)c.ws.get(Workspace::XMAT, (V + V * P) * 8);
    HIP_CHECK(hipMemcpyAsync(dm, scnt.data(), V * 8, hipMemcpyHostToDevice, c.stream));
    const int e0 = d.tm->mark();
    d.comm.allgather_u64(dm, dm + V, V, c.stream);
    d.xev.push_back({e0, d.tm->mark()});
    std::vector<uint64_t> mat(V * P);
    HIP_CHECK(hipMemcpyAsync(mat.data(), dm + V, V * P * 8, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    // receive layout: piece-major, then source rank
    std::vector<uint64_t> rcnt(V), roff(V), pbase(Q + 1, 0);
    uint64_t n1 = 0;
    for (uint32_t q = 0; q < Q; ++q) {
        pbase[q] = n1;
        for (int i = 0; i < P; ++i) {
            rcnt[q * P + i] = mat[(size_t)i * V + q * P + d.me];
            roff[q * P + i] = n1;
            n1 += rcnt[q * P + i];
        }
    }
    pbase[Q] = n1;
    // every buffer the pieces touch is sized before the first one leaves (a workspace slot that grows
    // synchronizes the device, which would wait for the exchange)
    K2 *xa = (K2 *)c.ws.get(Workspace::XA, std::max<uint64_t>(n1, 1) * sizeof(K2));
    K2 *xb = (K2 *)c.ws.get(Workspace::XB, std::max<uint64_t>(n1, 1) * sizeof(K2));
    uint32_t *xac = COUNTED ? (uint32_t *)c.ws.get(Workspace::XAC, std::max<uint64_t>(n1, 1) * 4) : nullptr;
    uint32_t *xbc = COUNTED ? (uint32_t *)c.ws.get(Workspace::XBC, std::max<uint64_t>(n1, 1) * 4) : nullptr;
    K2 *acc = (K2 *)c.ws.get(Workspace::CANON, std::max<uint64_t>(n1, 1) * sizeof(K2));
    uint32_t *accc = COUNTED ? (uint32_t *)c.ws.get(Workspace::CANONC, std::max<uint64_t>(n1, 1) * 4) : nullptr;
    uint32_t *dh1 = (uint32_t *)c.ws.get(Workspace::HIST1, nb1 * 4);
    if (!c.xstream) HIP_CHECK(hipStreamCreateWithFlags(&c.xstream, hipStreamNonBlocking));
    hipStream_t xs = c.xstream;
    // events: pass B done (build stream); exchange start + each piece's end (exchange stream); each sort's end
    std::vector<hipEvent_t> ev(2 * Q + 2);
    for (auto &e : ev) HIP_CHECK(hipEventCreate(&e));
    struct EvFree {
        std::vector<hipEvent_t> &v;
        ~EvFree() {
            for (auto e : v) (void)hipEventDestroy(e);
        }
    } ev_free{ev};
    hipEvent_t ev_b = ev[0], ev_x0 = ev[1];
    hipEvent_t *ev_x = ev.data() + 2, *ev_s = ev.data() + 2 + Q;
    HIP_CHECK(hipEventRecord(ev_b, c.stream));
    HIP_CHECK(hipStreamWaitEvent(xs, ev_b, 0));
    HIP_CHECK(hipEventRecord(ev_x0, xs));
    for (uint32_t q = 0; q < Q; ++q) {
        d.comm.alltoallv_async(ka, &scnt[q * P], &soff[q * P], xa, &rcnt[q * P], &roff[q * P], sizeof(K2), xs);
        if (COUNTED) d.comm.alltoallv_async(ca, &scnt[q * P], &soff[q * P], xac, &rcnt[q * P], &roff[q * P], 4, xs);
        HIP_CHECK(hipEventRecord(ev_x[q], xs));
        for (int j = 0; j < P; ++j)
            if (j != d.me) c.timings.n_sent += scnt[q * P + j];
    }
    tr("exchange 1 issued", n1);
    std::vector<std::vector<uint32_t>> hown(Q, std::vector<uint32_t>(nb1, 0));  // live until the end (async copies)
    uint64_t off = 0;
    double dup_raw = 0;  // the first piece's duplication estimate (before its spread), reused by the others
    for (uint32_t q = 0; q < Q; ++q) {
        HIP_CHECK(hipStreamWaitEvent(c.stream, ev_x[q], 0));
        const uint64_t rb0 = sub[d.me][q], rb1 = sub[d.me][q + 1];
        uint64_t nown = 0;
        for (uint32_t i = 0; i < NBH; ++i) {
            const uint32_t b = i >> (FUSED_HB - B1);
            if (b >= rb0 && b < rb1) {
                hown[q][b] += (uint32_t)H[i];
                nown += H[i];
            }
        }
        const uint64_t nq = pbase[q + 1] - pbase[q];
        if (nown != nq) throw std::runtime_error("received k-mers differ from the global histogram of the owned piece");
        uint64_t Ur = 0;
        K2 *pa = xa + pbase[q], *pb = xb + pbase[q];
        uint32_t *pac = COUNTED ? xac + pbase[q] : nullptr, *pbc = COUNTED ? xbc + pbase[q] : nullptr;
        if (nq) {
            HIP_CHECK(hipMemcpyAsync(dh1, hown[q].data(), nb1 * 4, hipMemcpyHostToDevice, c.stream));
            const double spread = (double)nb1 / (double)std::max<uint64_t>(1, rb1 - rb0);
            if (dup_raw == 0) dup_raw = estimate_dup<1>(c, pa, nq, 8.0);
            const double dup = dup_raw / spread;
            MsdPlan plan = msd_plan<1>(c, nq, 2 * K, dup);
            unsigned T = plan.levels ? plan.digit_end[plan.levels] : 0;
            T = std::min(2 * K, std::max(T, B1 + 1));
            MsdPlan fp{};
            fp.levels = 1 + (T - B1 + MSD_DBITS - 1) / MSD_DBITS;
            fp.digit_end[1] = B1;
            for (unsigned l = 2; l <= fp.levels; ++l) fp.digit_end[l] = B1 + (T - B1) * (l - 1) / (fp.levels - 1);
            c.track_partition = q == 0;
            // the sort's final gather writes the piece's distinct keys straight after the previous pieces' (no
            // append copy: 0.9 ms a rank-step at P = 2 with 4 pieces); CANON is neither its input nor its tmp
            c.sort_out = acc + off;
            c.sort_out_vals = COUNTED ? accc + off : nullptr;
            Ur = msd_sort_unique<1, COUNTED>(c, &pa, &pb, &pac, &pbc, nq, 2 * K, cmax, dup, dh1, false, nullptr, true,
                                             nullptr, &fp);
            c.sort_out = nullptr;
            c.sort_out_vals = nullptr;
            c.track_partition = false;
            if (Ur && pa != acc + off) {  // (a path without the final gather)
                HIP_CHECK(hipMemcpyAsync(acc + off, pa, Ur * sizeof(K2), hipMemcpyDeviceToDevice, c.stream));
                if (COUNTED) HIP_CHECK(hipMemcpyAsync(accc + off, pac, Ur * 4, hipMemcpyDeviceToDevice, c.stream));
            }
        }
        HIP_CHECK(hipEventRecord(ev_s[q], c.stream));
        off += Ur;
        tr("piece sorted", nq, Ur);
    }
    HIP_CHECK(hipStreamSynchronize(c.stream));
    HIP_CHECK(hipStreamSynchronize(xs));
    // exchange wall time and the part of it the build stream spent sorting: piece q's exposed wait is how
    // far it ended after the build stream became free (pass B for piece 0, the sort of piece q - 1 after)
    float span = 0;
    HIP_CHECK(hipEventElapsedTime(&span, ev_x0, ev_x[Q - 1]));
    double exposed = 0;
    for (uint32_t q = 0; q < Q; ++q) {
        float t = 0;
        HIP_CHECK(hipEventElapsedTime(&t, q ? ev_s[q - 1] : ev_b, ev_x[q]));
        exposed += std::max(0.0f, t);
    }
    *xspan_ms = span;
    *hidden_ms = std::max(0.0, (double)span - exposed);
    *out = acc;
    *outc = accc;
    return off;
}

// The routed collect's rounds with every exchange in flight under compute (configs[3]'s shares, 125 M
// reads a GPU, collect in rounds).  Round r's exchange 1 goes out on the exchange stream as soon as its
// pass B ends, so it runs under pass B of round r + 1 and under the owner sort of round r - 1; the send
// buffers (KA / KA2) and receive buffers (XA / XA2) alternate between even and odd rounds, and each is
// reused only once the exchange or sort that read it has ended (stream events).  Build-stream order:
// B0, B1, S0, B2, S1, ...; exchange-stream order: X0, X1, X2, ... (X_r after B_r and S_r-2).  Every
// round's send counts are known from pass A's histogram, so one all-gather sizes every receive.
// The merge semantics are the serial rounds' (sorted_multiset.cpp:54-84); the reference has no runtime
// exchange (cli/build.cpp:106-148).  *span_ms / *hidden_ms: exchange time, and the part of it the build
// stream spent computing.
template <bool COUNTED, class Layout, class PassB, class Sort, class Append>
static void routed_rounds_pipelined(Ctx &c, Dist &d, uint32_t R, Layout &round_layout, PassB &pass_b,
                                    Sort &owner_sort, Append &append, const std::vector<std::vector<uint64_t>> &sub,
                                    uint32_t nb1, Tracer &tr, double *span_ms, double *hidden_ms) {
    using K2 = Key<1>;
    const int P = d.P;
    std::vector<BucketSel> sel(R);
    std::vector<std::vector<unsigned long long>> cur(R);
    std::vector<uint64_t> nr(R);
    for (uint32_t r = 0; r < R; ++r) nr[r] = round_layout(r, sel[r], cur[r]);
    auto at = [&](uint32_t r, uint64_t b) -> uint64_t { return b >= nb1 ? nr[r] : cur[r][b]; };
    // this rank's slices (round-major, then owner) and every rank's counts
    const size_t V = (size_t)R * P;
    std::vector<uint64_t> scnt(V), soff(V);
    for (uint32_t r = 0; r < R; ++r)
        for (int o = 0; o < P; ++o) {
            soff[r * P + o] = at(r, sub[o][r]);
            scnt[r * P + o] = at(r, sub[o][r + 1]) - soff[r * P + o];
        }
    uint64_t *dm = (uint64_t *)c.ws.get(Workspace::XMAT, (V + V * P) * 8);
    HIP_CHECK(hipMemcpyAsync(dm, scnt.data(), V * 8, hipMemcpyHostToDevice, c.stream));
    const int e0 = d.tm->mark();
    d.comm.allgather_u64(dm, dm + V, V, c.stream);
    d.xev.push_back({e0, d.tm->mark()});
    std::vector<uint64_t> mat(V * P);
    HIP_CHECK(hipMemcpyAsync(mat.data(), dm + V, V * P * 8, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    std::vector<uint64_t> rcnt(V), roff(V), n1(R, 0);
    for (uint32_t r = 0; r < R; ++r)
        for (int i = 0; i < P; ++i) {
            rcnt[r * P + i] = mat[(size_t)i * V + r * P + d.me];
            roff[r * P + i] = n1[r];
            n1[r] += rcnt[r * P + i];
        }
    // the buffers of both parities, sized before the first exchange leaves (a slot that grows synchronizes
    // the device)
    uint64_t mk[2] = {1, 1}, mx[2] = {1, 1}, mb = 1;
    for (uint32_t r = 0; r < R; ++r) {
        mk[r & 1] = std::max(mk[r & 1], nr[r]);
        mx[r & 1] = std::max(mx[r & 1], n1[r]);
        mb = std::max(mb, n1[r]);
    }
    K2 *ka[2] = {(K2 *)c.ws.get(Workspace::KA, mk[0] * sizeof(K2)), (K2 *)c.ws.get(Workspace::KA2, mk[1] * sizeof(K2))};
    K2 *xr[2] = {(K2 *)c.ws.get(Workspace::XA, mx[0] * sizeof(K2)), (K2 *)c.ws.get(Workspace::XA2, mx[1] * sizeof(K2))};
    K2 *xb = (K2 *)c.ws.get(Workspace::XB, mb * sizeof(K2));
    uint32_t *ca[2] = {nullptr, nullptr}, *xrc[2] = {nullptr, nullptr}, *xbc = nullptr;
    if (COUNTED) {
        ca[0] = (uint32_t *)c.ws.get(Workspace::CA, mk[0] * 4);
        ca[1] = (uint32_t *)c.ws.get(Workspace::CA2, mk[1] * 4);
        xrc[0] = (uint32_t *)c.ws.get(Workspace::XAC, mx[0] * 4);
        xrc[1] = (uint32_t *)c.ws.get(Workspace::XAC2, mx[1] * 4);
        xbc = (uint32_t *)c.ws.get(Workspace::XBC, mb * 4);
    }
    if (!c.xstream) HIP_CHECK(hipStreamCreateWithFlags(&c.xstream, hipStreamNonBlocking));
    hipStream_t xs = c.xstream;
    // per round: pass B done, exchange start / end (exchange stream), build stream free before the sort's wait,
    // sort + append done
    std::vector<hipEvent_t> ev(5 * (size_t)R);
    for (auto &e : ev) HIP_CHECK(hipEventCreate(&e));
    struct EvFree {
        std::vector<hipEvent_t> &v;
        ~EvFree() {
            for (auto e : v) (void)hipEventDestroy(e);
        }
    } ev_free{ev};
    hipEvent_t *evB = ev.data(), *evXs = evB + R, *evX = evXs + R, *evC = evX + R, *evS = evC + R;
    std::vector<std::vector<uint32_t>> hown(R);  // the owner sorts' level-1 counts (copied asynchronously)
    auto issue = [&](uint32_t r) {  // pass B of round r, then its exchange
        const int p = r & 1;
        if (r >= 2) HIP_CHECK(hipStreamWaitEvent(c.stream, evX[r - 2], 0));  // ka[p] read by exchange r - 2
        pass_b(&sel[r], cur[r], ka[p], ca[p]);
        HIP_CHECK(hipEventRecord(evB[r], c.stream));
        tr("rounds: pass B", r, nr[r]);
        HIP_CHECK(hipStreamWaitEvent(xs, evB[r], 0));
        if (r >= 2) HIP_CHECK(hipStreamWaitEvent(xs, evS[r - 2], 0));  // xr[p] read by the sort of round r - 2
        HIP_CHECK(hipEventRecord(evXs[r], xs));
        d.comm.alltoallv_async(ka[p], &scnt[r * P], &soff[r * P], xr[p], &rcnt[r * P], &roff[r * P], sizeof(K2), xs);
        if (COUNTED)
            d.comm.alltoallv_async(ca[p], &scnt[r * P], &soff[r * P], xrc[p], &rcnt[r * P], &roff[r * P], 4, xs);
        HIP_CHECK(hipEventRecord(evX[r], xs));
        for (int j = 0; j < P; ++j)
            if (j != d.me) c.timings.n_sent += scnt[r * P + j];
    };
    issue(0);
    for (uint32_t r = 1; r <= R; ++r) {
        if (r < R) issue(r);
        const uint32_t q = r - 1;
        HIP_CHECK(hipEventRecord(evC[q], c.stream));
        HIP_CHECK(hipStreamWaitEvent(c.stream, evX[q], 0));
        K2 *pa = xr[q & 1], *pb = xb;
        uint32_t *pac = xrc[q & 1], *pbc = xbc;
        const uint64_t rb0 = sub[d.me][q], rb1 = sub[d.me][q + 1];
        const uint64_t Ur = owner_sort(&pa, &pb, &pac, &pbc, n1[q], rb0, rb1, hown[q], q == 0, false);
        append(pa, pac, Ur, rb0, rb1);
        HIP_CHECK(hipEventRecord(evS[q], c.stream));
        tr("rounds: exchange + owner sort", q, Ur);
    }
    HIP_CHECK(hipStreamSynchronize(c.stream));
    HIP_CHECK(hipStreamSynchronize(xs));
    double span = 0, exposed = 0;
    for (uint32_t r = 0; r < R; ++r) {
        float t = 0;
        HIP_CHECK(hipEventElapsedTime(&t, evXs[r], evX[r]));
        span += t;
        HIP_CHECK(hipEventElapsedTime(&t, evC[r], evX[r]));
        exposed += std::max(0.0f, t);
    }
    *span_ms = span;
    *hidden_ms = std::max(0.0, span - exposed);
}

template <bool COUNTED>
static bool dist_collect_routed(Ctx &c, Dist &d, unsigned K, bool canonical, uint32_t cmax, const BuildInput &in,
                                Key<1> **xa_out, uint32_t **xac_out, uint64_t *U_out, std::vector<uint64_t> *bounds,
                                Tracer &tr, EventTimer &tm, int *ev_extract, int *ev_sort) {
    using K2 = Key<1>;
    // the same on every rank (no input-size test: a rank may hold no reads)
    if (!routed_applies(c, K)) return false;
    constexpr unsigned OB = 8;   // owner-range prefix bits (4 node chars: whole chars for the lifted bounds)
    // canonical windows keep the strand whose key top hashes smaller (boss_kernels.hpp: take_rc): the
    // owners' canonical keys then follow the real edges, and one set of ranges balances both
    const int cmode = canonical ? (c.routed_min || d.P == 1 ? 1 : 2) : 0;
    // pass B's scatter digit: 10 bits across ranks (extract_partition_fast_kernel<512, 1024>), so that an
    // owner of 2 ranks' worth of keys at configs[1]'s density (19 planned bits) keeps a 2-level sort;
    // the counted pass B takes 9
    const unsigned B1 = c.fused_b1 ? std::max(c.fused_b1, OB) : (!COUNTED && c.wide_b1 && d.P >= 2) ? 10u : 9u;
    const uint64_t npos = in.seq_len >= K ? in.seq_len - K + 1 : 0;
    c.timings.n_positions = npos;
    constexpr int TILE = ExtractTraits<1>::TILE;
    const uint64_t tiles = ceil_div(npos, TILE);
    const int fbk = 512;
    const uint32_t rps = (uint32_t)(16 * fbk / TILE);
    // (stripe_cursor_kernel takes at most 1024 stripes: 2048 rows at rps = 2, 1024 at rps = 1)
    uint32_t nrows = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(tiles, c.hist_rows), 1024ull * rps);
    if (nrows >= rps) nrows -= nrows % rps;
    constexpr uint32_t NBH = 1u << FUSED_HB;
    // pass A: per-row histograms of the canonical keys' top 12 bits (and of the other strand's)
    uint32_t *rows = (uint32_t *)c.ws.get(Workspace::HIST_ROWS, std::max<uint64_t>((uint64_t)nrows * NBH, 1) * 4);
    uint32_t *rows_o = (uint32_t *)c.ws.get(Workspace::RC_COMB, std::max<uint64_t>((uint64_t)nrows * NBH, 1) * 4);
    uint64_t *hg = (uint64_t *)c.ws.get(Workspace::XHIST, 2 * NBH * 8);
    HIP_CHECK(hipMemsetAsync(hg, 0, 2 * NBH * 8, c.stream));
    const uint64_t tiles_b = ceil_div(npos, (uint64_t)16 * fbk);
    const uint32_t stripes = std::max<uint32_t>(1, nrows / rps);
    const uint64_t per_stripe = std::max<uint64_t>(1, ceil_div(tiles_b, stripes));
    const uint64_t per_row = stripes == 1 && nrows ? ceil_div(tiles_b * rps, nrows) : per_stripe;
    uint32_t *h12 = (uint32_t *)c.ws.get(Workspace::FUSED_HIST, 2 * NBH * 4);
    HIP_CHECK(hipMemsetAsync(h12, 0, 2 * NBH * 4, c.stream));
    if (nrows) {
        launch_hist_fast<true>(c, K, dim3(nrows), dim3(256), in.seq, in.seq_len, K, cmode, tiles, per_row, rows, rows_o,
                               1u);
        HIP_CHECK(hipGetLastError());
        hist_rows_reduce_kernel<<<dim3(std::min<uint32_t>(nrows, 256), (unsigned)ceil_div(NBH, 256)), dim3(256), 0,
                                  c.stream>>>(rows, nrows, NBH, h12);
        HIP_CHECK(hipGetLastError());
        hist_rows_reduce_kernel<<<dim3(std::min<uint32_t>(nrows, 256), (unsigned)ceil_div(NBH, 256)), dim3(256), 0,
                                  c.stream>>>(rows_o, nrows, NBH, h12 + NBH);
        HIP_CHECK(hipGetLastError());
    }
    std::vector<uint32_t> hl(2 * NBH);
    HIP_CHECK(hipMemcpyAsync(hl.data(), h12, 2 * NBH * 4, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));
    std::vector<uint64_t> hloc(2 * NBH);
    for (uint32_t i = 0; i < 2 * NBH; ++i) hloc[i] = hl[i];
    HIP_CHECK(hipMemcpyAsync(hg, hloc.data(), 2 * NBH * 8, hipMemcpyHostToDevice, c.stream));
    const int e0 = d.tm->mark();
    d.comm.allreduce_sum_u64(hg, 2 * NBH, c.stream);
    d.xev.push_back({e0, d.tm->mark()});
    std::vector<uint64_t> H(2 * NBH);
    HIP_CHECK(hipMemcpyAsync(H.data(), hg, 2 * NBH * 8, hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipStreamSynchronize(c.stream));  // hloc is a host local
    uint64_t N = 0, Nall = 0;
    for (uint32_t i = 0; i < NBH; ++i) {
        N += hl[i];
        Nall += H[i];
    }
    // owner ranges over the 256 4-char prefixes, balanced on the build's work: the collect and the rc
    // stage follow the canonical k-mers (2/3 of a step), the dummy and emit stages the real edges,
    // i.e. both strands (canonical mode; basic mode: the k-mers themselves)
    constexpr uint32_t NOB = 1u << OB;
    std::vector<uint64_t> wgt(NOB, 0);
    {
        uint64_t tc = 0, tr2 = 0;
        for (uint32_t i = 0; i < NBH; ++i) {
            tc += H[i];
            tr2 += H[i] + (canonical ? H[NBH + i] : H[i]);
        }
        for (uint32_t i = 0; i < NBH; ++i) {
            const double wc = tc ? (double)H[i] / (double)tc : 0.0;
            const double wr = tr2 ? (double)(H[i] + (canonical ? H[NBH + i] : H[i])) / (double)tr2 : 0.0;
            wgt[i >> (FUSED_HB - OB)] += (uint64_t)((2.0 * wc + wr) * 1e12);
        }
    }
    *bounds = balanced_bounds(wgt.data(), NOB, d.P);
    d.m = OB / 2;
    d.shift2 = 2 * K - OB;
    d.nb = NOB;
    tr("route plan", N, Nall);
    const uint32_t nb1 = 1u << B1;
    // rounds (configs[3]: 1.5e10 windows per rank): one pass when this rank's keys, the received runs
    // and their sort buffer fit; else every owner's level-1 buckets are cut into `rounds` sub-intervals
    // (balanced on the global histogram) and round r collects sub-interval r of every owner -- pass B
    // keeps only those buckets, exchange 1 and the owner sort run per round, and the owner appends the
    // rounds' distinct keys in BOSS order.  All ranks agree on the count (an all-gather of the most
    // any rank needs).  The key-range collect (collect_ranges_dist) re-scanned every read per range
    // and extracted both strands.
    uint32_t rounds = 1;
    bool pipe_ok = false;  // the rounds' exchanges pipelined (routed_rounds_pipelined)
    {
        uint64_t want = c.force_ranges;
        const double budget = dist_budget(c, d);
        const double per_key = 8.0 + (COUNTED ? 4.0 : 0.0);
        if (!want) {
            // one pass: the rank's keys, the received runs and their ping-pong buffer, plus ~3 N of later
            // stages (the owned canonical set, its rc keys, the real edges) at low duplication
            const double need = (double)N * per_key * 3.0;
            want = need * 2.0 <= budget ? 1 : (uint64_t)std::ceil(need / (0.45 * budget));
        }
        // every rank's wish, key count and budget: all ranks then take the same count and decide alike
        // whether two rounds' send and receive buffers fit (5 round-sized buffers instead of 3)
        const uint64_t mine[3] = {want, N, (uint64_t)budget};
        uint64_t *dv = (uint64_t *)c.ws.get(Workspace::XMAT, (3 + 3 * (uint64_t)d.P) * 8);
        HIP_CHECK(hipMemcpyAsync(dv, mine, 24, hipMemcpyHostToDevice, c.stream));
        d.comm.allgather_u64(dv, dv + 3, 3, c.stream);
        std::vector<uint64_t> all(3 * (size_t)d.P);
        HIP_CHECK(hipMemcpyAsync(all.data(), dv + 3, all.size() * 8, hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));  // `mine` is a host local
        uint64_t r = 1, nmax = 0;
        for (int i = 0; i < d.P; ++i) r = std::max(r, all[3 * i]), nmax = std::max(nmax, all[3 * i + 1]);
        rounds = (uint32_t)std::min<uint64_t>(r, 64);
        pipe_ok = c.dist_pieces > 1;
        for (int i = 0; i < d.P && pipe_ok && !c.force_ranges; ++i)
            pipe_ok = 5.0 * (double)nmax / rounds * per_key <= 0.6 * (double)all[3 * i + 2];
    }
    // global level-1 counts, and every owner's bucket interval cut into the rounds
    std::vector<uint64_t> gh1(nb1, 0);
    for (uint32_t i = 0; i < NBH; ++i) gh1[i >> (FUSED_HB - B1)] += H[i];
    std::vector<std::vector<uint64_t>> sub(d.P);
    for (int o = 0; o < d.P; ++o) {
        const uint64_t o0 = std::min<uint64_t>((*bounds)[o] << (B1 - OB), nb1);
        const uint64_t o1 = std::min<uint64_t>((*bounds)[o + 1] << (B1 - OB), nb1);
        sub[o] = balanced_bounds(gh1.data() + o0, o1 - o0, (int)rounds);
        for (auto &v : sub[o]) v += o0;
    }
    const uint64_t ob0 = std::min<uint64_t>((*bounds)[d.me] << (B1 - OB), nb1);
    const uint64_t ob1 = std::min<uint64_t>((*bounds)[d.me + 1] << (B1 - OB), nb1);
    c.timings.n_extracted = N;
    c.timings.n_batches = rounds;
    if (rounds > 1) {
        c.timings.collect_mode = 2;
        c.ws.release_stage_buffers();  // a previous build's would crowd out the rounds' buffers
        *ev_extract = tm.mark();
    }
    K2 *acc = nullptr;  // rounds: the owned distinct keys so far
    uint32_t *accc = nullptr;
    uint64_t off = 0, cap = 0;
    K2 *xa = nullptr;
    uint32_t *xac = nullptr;
    uint64_t U = 0;
    // the round's level-1 layout of this rank's k-mers: bucket starts (and ends at nb1 + i) of the buckets
    // its mask keeps (every bucket in a one-round build)
    auto round_layout = [&](uint32_t r, BucketSel &sel, std::vector<unsigned long long> &cur) -> uint64_t {
        for (int o = 0; o < d.P; ++o) sel.add(sub[o][r], sub[o][r + 1]);
        std::vector<uint32_t> h1(nb1, 0);
        for (uint32_t i = 0; i < NBH; ++i) {
            const uint32_t b = i >> (FUSED_HB - B1);
            if (rounds == 1 || sel.has(b)) h1[b] += hl[i];
        }
        cur.assign(2 * nb1, 0);
        unsigned long long nr = 0;
        for (uint32_t i = 0; i < nb1; ++i) {
            cur[i] = nr;
            nr += h1[i];
        }
        for (uint32_t i = 0; i < nb1; ++i) cur[nb1 + i] = cur[i] + h1[i];
        return nr;
    };
    // pass B: this rank's k-mers (of the round's buckets) scattered by their top B1 bits into ka (the single
    // build's fused pass)
    auto pass_b = [&](const BucketSel *rs, const std::vector<unsigned long long> &cur, K2 *ka, uint32_t *ca) {
        if (!nrows) return;
        uint32_t *dsel = nullptr;
        if (rs) {
            dsel = (uint32_t *)c.ws.get(Workspace::FUSED_SEL, sizeof(rs->m));
            HIP_CHECK(hipMemcpyAsync(dsel, rs->m, sizeof(rs->m), hipMemcpyHostToDevice, c.stream));
        }
        unsigned long long *dcur = (unsigned long long *)c.ws.get(Workspace::FUSED_CUR, cur.size() * 8);
        HIP_CHECK(hipMemcpyAsync(dcur, cur.data(), cur.size() * 8, hipMemcpyHostToDevice, c.stream));
        auto *scur = (unsigned long long *)c.ws.get(Workspace::STRIPE_CUR, (size_t)stripes * nb1 * 16);
        unsigned long long *send = scur + (size_t)stripes * nb1;
        stripe_cursor_kernel<<<dim3(nb1), dim3(256), 0, c.stream>>>(rows, nrows, FUSED_HB, B1, stripes, rps, dcur,
                                                                     scur, send, dsel);
        HIP_CHECK(hipGetLastError());
        if (!COUNTED && B1 > 9) {
            launch_part_fast<512, 1024>(c, K, dim3((unsigned)xcd_grid(ceil_div(npos, 16 * 512))), dim3(512), in.seq,
                                        in.seq_len, K, cmode, B1, per_stripe, scur, send, ka, &c.small->error,
                                        (const uint32_t *)dsel, (uint32_t *)nullptr);
        } else if (!COUNTED) {
            launch_part_fast<512, 512>(c, K, dim3((unsigned)xcd_grid(ceil_div(npos, 16 * 512))), dim3(512), in.seq,
                                       in.seq_len, K, cmode, B1, per_stripe, scur, send, ka, &c.small->error,
                                       (const uint32_t *)dsel, (uint32_t *)nullptr);
        } else {
            if (B1 > 9) throw std::runtime_error("the counted pass B takes at most 9 bits");
            const uint64_t ftiles = ceil_div(npos, FusedTraits<COUNTED, 512>::TILE);
            extract_partition_kernel<1, COUNTED, 512><<<dim3((unsigned)xcd_grid(ftiles)), dim3(512), 0, c.stream>>>(
                in.seq, in.seq_len, K, cmode, in.read_starts, in.read_counts, in.n_reads, in.rid_at, cmax,
                B1, per_stripe, scur, send, ka, ca, &c.small->error, dsel);
        }
        HIP_CHECK(hipGetLastError());
        cursor_check_kernel<<<dim3((unsigned)ceil_div((uint64_t)stripes * nb1, 256)), dim3(256), 0, c.stream>>>(
            scur, send, stripes * nb1, &c.small->error);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipStreamSynchronize(c.stream));  // cur / sel are host memory
    };
    // the owner's sort of one round's (or piece's) received keys: level 1 is the routing digit (its counts
    // from the global pass-A histogram over the owned buckets [rb0, rb1)), level 2 partitions the runs in any
    // order; returns the distinct keys, left in *pa
    auto owner_sort = [&](K2 **pa, K2 **pb, uint32_t **pac, uint32_t **pbc, uint64_t n1, uint64_t rb0, uint64_t rb1,
                          std::vector<uint32_t> &hown, bool track, bool gidx) -> uint64_t {
        hown.assign(nb1, 0);
        uint64_t nown = 0;
        for (uint32_t i = 0; i < NBH; ++i) {
            const uint32_t b = i >> (FUSED_HB - B1);
            if (b >= rb0 && b < rb1) {
                hown[b] += (uint32_t)H[i];
                nown += H[i];
            }
        }
        if (nown != n1) throw std::runtime_error("received k-mers differ from the global histogram of the owned range");
        if (!n1) return 0;
        uint32_t *dh1 = (uint32_t *)c.ws.get(Workspace::HIST1, nb1 * 4);
        HIP_CHECK(hipMemcpyAsync(dh1, hown.data(), nb1 * 4, hipMemcpyHostToDevice, c.stream));
        const double spread = (double)nb1 / (double)std::max<uint64_t>(1, rb1 - rb0);
        const double dup = estimate_dup<1>(c, *pa, n1, 8.0) / spread;
        MsdPlan plan = msd_plan<1>(c, n1, 2 * K, dup);
        unsigned T = plan.levels ? plan.digit_end[plan.levels] : 0;
        T = std::min(2 * K, std::max(T, B1 + 1));  // at least one partition pass after the routing digit
        MsdPlan fp{};
        fp.levels = 1 + (T - B1 + MSD_DBITS - 1) / MSD_DBITS;
        fp.digit_end[1] = B1;
        for (unsigned l = 2; l <= fp.levels; ++l) fp.digit_end[l] = B1 + (T - B1) * (l - 1) / (fp.levels - 1);
        c.track_partition = track;
        c.want_gidx = gidx;
        const uint64_t u = msd_sort_unique<1, COUNTED>(c, pa, pb, pac, pbc, n1, 2 * K, cmax, dup, dh1, false, nullptr,
                                                       true, nullptr, &fp);
        c.want_gidx = false;
        c.track_partition = false;
        return u;
    };
    // the rounds' distinct keys appended to the owned canonical set (sized from the first filled round's
    // share of the owner's range, +25 %)
    auto append = [&](const K2 *src, const uint32_t *srcc, uint64_t Ur, uint64_t rb0, uint64_t rb1) {
        if (off + Ur > cap) {
            uint64_t gr = 0, go = 0;
            for (uint64_t b = rb0; b < rb1; ++b) gr += gh1[b];
            for (uint64_t b = ob0; b < ob1; ++b) go += gh1[b];
            const uint64_t want = off == 0 && gr ? (uint64_t)((double)Ur / (double)gr * (double)go * 1.25) + Ur
                                                 : (off + Ur) + (off + Ur) / 4;
            cap = std::max(want, off + Ur);
            acc = (K2 *)c.ws.get(Workspace::CANON, cap * sizeof(K2), off * sizeof(K2), c.stream);
            if (COUNTED) accc = (uint32_t *)c.ws.get(Workspace::CANONC, cap * 4, off * 4, c.stream);
        }
        if (Ur) {
            HIP_CHECK(hipMemcpyAsync(acc + off, src, Ur * sizeof(K2), hipMemcpyDeviceToDevice, c.stream));
            if (COUNTED) HIP_CHECK(hipMemcpyAsync(accc + off, srcc, Ur * 4, hipMemcpyDeviceToDevice, c.stream));
        }
        off += Ur;
    };
    const bool pipe_rounds = rounds > 1 && d.P > 1 && pipe_ok;
    if (pipe_rounds) {
        double span = 0, hidden = 0;
        routed_rounds_pipelined<COUNTED>(c, d, rounds, round_layout, pass_b, owner_sort, append, sub, nb1, tr, &span,
                                         &hidden);
        c.timings.exchange_ms += span;
        c.timings.exchange_hidden_ms += hidden;
    }
    for (uint32_t r = 0; r < (pipe_rounds ? 0u : rounds); ++r) {
        BucketSel sel;
        std::vector<unsigned long long> cur;
        const uint64_t nr = round_layout(r, sel, cur);
        const BucketSel *rs = rounds > 1 ? &sel : nullptr;
        K2 *ka = (K2 *)c.ws.get(Workspace::KA, std::max<uint64_t>(nr, 1) * 8);
        uint32_t *ca = COUNTED ? (uint32_t *)c.ws.get(Workspace::CA, std::max<uint64_t>(nr, 1) * 4) : nullptr;
        pass_b(rs, cur, ka, ca);
        if (rounds == 1) *ev_extract = tm.mark();
        tr("extract + scatter", nr);
        // exchange 1 in pieces under the owner sort (routed_pieces): pieces of at least 2^28 keys an owner
        // (each piece's sort pays ~0.7 ms of its own launches and host reads, more than a smaller piece's
        // sort can hide), exactly MTG_DIST_PIECES when given; the same count on every rank (global totals)
        const uint32_t Q = c.dist_pieces_set ? c.dist_pieces
                                             : (uint32_t)std::min<uint64_t>(c.dist_pieces,
                                                                            std::max<uint64_t>(1, Nall / d.P >> 28));
        if (rounds == 1 && d.P > 1 && Q > 1) {
            double span = 0, hidden = 0;
            U = routed_pieces<COUNTED>(c, d, K, cmax, ka, ca, cur, nr, nb1, B1, OB, *bounds, gh1, H, Q, &xa, &xac,
                                       &span, &hidden, tr);
            c.timings.exchange_ms += span;
            c.timings.exchange_hidden_ms += hidden;
            // (the piece buffers stay in their slots for the next build of the same shape: given back, they
            // went to the rc stage's requests and the next build allocated and freed them again, +3.7 ms a
            // rank at P = 8)
            break;
        }
        // exchange 1: owner o gets the rank's buckets of its prefixes [bounds[o], bounds[o + 1]) (of
        // this round: the other buckets are empty)
        std::vector<std::vector<uint64_t>> soff(1, std::vector<uint64_t>(d.P + 1));
        for (int j = 0; j <= d.P; ++j) {
            const uint64_t b = (*bounds)[j] << (B1 - OB);  // first level-1 bucket of the prefix
            soff[0][j] = b >= nb1 ? nr : cur[b];
        }
        xa = ka;
        xac = ca;
        uint64_t n1 = nr;
        if (d.P == 1) {  // one rank: its keys stay where they are (the buffers change slots instead of a copy)
            c.ws.swap(Workspace::KA, Workspace::XA);
            if (COUNTED) c.ws.swap(Workspace::CA, Workspace::XAC);
        } else {
            const K2 *arrs[1] = {ka};
            const uint32_t *cnts[1] = {ca};
            n1 = exchange_runs<K2>(c, d, 1, arrs, COUNTED ? cnts : nullptr, soff, Workspace::XA, Workspace::XAC, &xa,
                                   &xac);
        }
        tr("exchange 1", n1);
        // the owner's level-1 counts: the global pass-A histogram over its buckets (of this round)
        const uint64_t rb0 = rs ? sub[d.me][r] : ob0, rb1 = rs ? sub[d.me][r + 1] : ob1;
        std::vector<uint32_t> hown;
        uint64_t Ur = 0;
        if (n1) {
            K2 *xb = (K2 *)c.ws.get(Workspace::XB, n1 * sizeof(K2));
            uint32_t *xbc = COUNTED ? (uint32_t *)c.ws.get(Workspace::XBC, n1 * 4) : nullptr;
            Ur = owner_sort(&xa, &xb, &xac, &xbc, n1, rb0, rb1, hown, r == 0, canonical && rounds == 1);
        } else {
            owner_sort(&xa, &xa, &xac, &xac, 0, rb0, rb1, hown, false, false);  // (checks the count)
        }
        tr("owner sort", Ur);
        if (rounds == 1) {
            U = Ur;
            break;
        }
        append(xa, xac, Ur, rb0, rb1);
    }
    if (rounds > 1) {
        if (!acc) {
            acc = (K2 *)c.ws.get(Workspace::CANON, sizeof(K2));
            if (COUNTED) accc = (uint32_t *)c.ws.get(Workspace::CANONC, 4);
        }
        xa = acc;
        xac = accc;
        U = off;
        // the round buffers go before the rc exchange and the dummy stage grow theirs
        for (auto sl : {Workspace::XA, Workspace::XB, Workspace::XAC, Workspace::XBC, Workspace::SPEC_A,
                        Workspace::SPEC_B})
            c.ws.release(sl);
    }
    *ev_sort = tm.mark();
    *xa_out = xa;
    *xac_out = xac;
    *U_out = U;
    return true;
}

// ------------------------------------------------ multi-GPU: exchange 0, super-k-mers (superkmer.hpp)
//
// Every rank's windows go to their collect owner (a hash of the window's canonical minimizer) as
// 2-bit packed runs; *out becomes the owner's input: the received runs unpacked into a read buffer
// (each run one read, carrying its read's count).  The owner's collect then extracts, sorts and
// dedupes each k-mer exactly once in the whole job, and its distinct keys are disjoint from every
// other owner's.  Returns false where the path does not apply (the caller collects its own reads).
static bool dist_superkmers(Ctx &c, Dist &d, unsigned K, bool canonical, const BuildInput &in, BuildInput *out,
                            Tracer &tr) {
    if (c.dist_collect != 0 || d.P < 2 || d.P > SK_MAX_OWNERS || K < 20 || K + 16 > (unsigned)SK_KMAX) return false;
    const unsigned M = std::min(11u, K - 12);
    const uint32_t P = (uint32_t)d.P;
    const uint64_t npos = in.seq_len >= K ? in.seq_len - K + 1 : 0;
    const uint64_t ntiles = ceil_div(npos, SK_TILE);
    const bool per_read = in.read_counts != nullptr;
    std::vector<std::vector<uint64_t>> soff_r(1, std::vector<uint64_t>(P + 1, 0)), soff_w(1, std::vector<uint64_t>(P + 1, 0));
    uint64_t *words = nullptr;
    uint32_t *nwords = nullptr, *cnt = nullptr;
    if (npos) {
        uint8_t *own = (uint8_t *)c.ws.get(Workspace::SK_OWN, npos + 16);
        uint32_t *tcnt = (uint32_t *)c.ws.get(Workspace::SK_TCNT, (2 * P * ntiles + 1) * 4);
        uint64_t *toff = (uint64_t *)c.ws.get(Workspace::SK_TOFF, (2 * P * ntiles + 2) * 8);
        uint64_t *toffw = toff + P * ntiles + 1;
        sk_owner_kernel<<<dim3((unsigned)ntiles), dim3(SK_BLOCK), 0, c.stream>>>(in.seq, in.seq_len, K, M,
                                                                               canonical ? 1 : 0, P, own);
        HIP_CHECK(hipGetLastError());
        sk_runs_kernel<true><<<dim3((unsigned)ntiles), dim3(SK_BLOCK), 0, c.stream>>>(
            own, npos, in.seq, K, P, ntiles, tcnt, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
            nullptr);
        HIP_CHECK(hipGetLastError());
        for (int half = 0; half < 2; ++half) {
            uint32_t ep;
            const uint64_t st = ceil_div(P * ntiles, 4096);
            uint64_t *desc = acquire_desc(c, st, &ep);
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(
                tcnt + half * P * ntiles, P * ntiles, half ? toffw : toff, desc, ep, &c.small->counter, &c.small->error);
            HIP_CHECK(hipGetLastError());
        }
        uint64_t *g = (uint64_t *)c.ws.get(Workspace::XGATHER, 2 * (P + 1) * 8);
        gather_strided_kernel<<<1, 256, 0, c.stream>>>(toff, ntiles, P + 1, g);
        gather_strided_kernel<<<1, 256, 0, c.stream>>>(toffw, ntiles, P + 1, g + P + 1);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(soff_r[0].data(), g, (P + 1) * 8, hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipMemcpyAsync(soff_w[0].data(), g + P + 1, (P + 1) * 8, hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));
        const uint64_t nruns = soff_r[0][P], nwtot = soff_w[0][P];
        words = (uint64_t *)c.ws.get(Workspace::SK_WORDS, std::max<uint64_t>(nwtot, 1) * 8);
        if (per_read) {
            nwords = (uint32_t *)c.ws.get(Workspace::SK_LENS, std::max<uint64_t>(nruns, 1) * 4);
            cnt = (uint32_t *)c.ws.get(Workspace::SK_CNT, std::max<uint64_t>(nruns, 1) * 4);
        }
        sk_runs_kernel<false><<<dim3((unsigned)ntiles), dim3(SK_BLOCK), 0, c.stream>>>(
            own, npos, in.seq, K, P, ntiles, nullptr, toff, toffw, in.read_starts, in.read_counts, in.n_reads,
            in.rid_at, words, nwords, cnt);
        HIP_CHECK(hipGetLastError());
    }
    tr("super-k-mers", soff_r[0][P], soff_w[0][P]);
    uint64_t *rwords = nullptr;
    uint32_t *rnw = nullptr, *rcnt = nullptr, *unused = nullptr;
    const uint64_t *wa[1] = {words};
    const uint64_t nw = exchange_runs<uint64_t>(c, d, 1, wa, nullptr, soff_w, Workspace::SK_RWORDS, Workspace::SK_RCNT,
                                                &rwords, &unused);
    uint64_t nr = 0;
    if (per_read) {
        const uint32_t *la[1] = {nwords};
        const uint32_t *ca[1] = {cnt};
        nr = exchange_runs<uint32_t>(c, d, 1, la, ca, soff_r, Workspace::SK_RLENS, Workspace::SK_RCNT, &rnw, &rcnt);
    }
    tr("exchange 0", nr, nw);
    // the received words -> a read buffer of 28 bytes per word (every run ends in a separator)
    *out = BuildInput{};
    uint8_t *seq = (uint8_t *)c.ws.get(Workspace::SK_SEQ, std::max<uint64_t>(SK_WCH * nw, 4));
    if (nw) {
        sk_unpack_kernel<<<dim3((unsigned)std::min<uint64_t>(ceil_div(nw, 256), 65536)), dim3(256), 0, c.stream>>>(
            rwords, nw, (uint32_t *)seq);
        HIP_CHECK(hipGetLastError());
    }
    out->seq = seq;
    out->seq_len = SK_WCH * nw;
    if (per_read && nr) {
        uint64_t *wstart = (uint64_t *)c.ws.get(Workspace::SK_WOFF, (nr + 1) * 8);
        uint64_t *starts = (uint64_t *)c.ws.get(Workspace::SK_STARTS, nr * 8);
        uint32_t ep;
        const uint64_t st = ceil_div(nr, 4096);
        uint64_t *desc = acquire_desc(c, st, &ep);
        HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
        scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(rnw, nr, wstart, desc, ep, &c.small->counter,
                                                                          &c.small->error);
        HIP_CHECK(hipGetLastError());
        if (read_u64(c, (const unsigned long long *)(wstart + nr)) != nw)
            throw std::runtime_error("received super-k-mer words differ from their runs' word counts");
        const unsigned g = (unsigned)std::min<uint64_t>(ceil_div(nr, 256), 16384);
        sk_starts_kernel<<<dim3(g), dim3(256), 0, c.stream>>>(wstart, nr, starts);
        HIP_CHECK(hipGetLastError());
        out->read_starts = starts;
        out->read_counts = rcnt;
        out->n_reads = nr;
        if (nr > 1) {
            const uint64_t nq = (out->seq_len >> RID_SHIFT) + 2;
            uint64_t *rid = (uint64_t *)c.ws.get(Workspace::SK_RID, nq * 8);
            read_index_kernel<<<dim3((unsigned)std::min<uint64_t>(ceil_div(nr, 256), 65536)), dim3(256), 0, c.stream>>>(
                starts, nr, nq, rid);
            HIP_CHECK(hipGetLastError());
            out->rid_at = rid;
        }
    }
    return true;
}

template <int L2, int L3, bool COUNTED>
static void run_pipeline_dist(Ctx &c, Comm &comm, unsigned k, bool canonical, unsigned bits,
                              const BuildInput &in, BuildOutput *out) {
    using K2 = Key<L2>;
    using K3 = Key<L3>;
    const unsigned K = k + 1;
    const unsigned cbits = bits <= 8 ? 8 : bits <= 16 ? 16 : 32;
    const uint32_t cmax = cbits == 8 ? 0xFFu : cbits == 16 ? 0xFFFFu : 0xFFFFFFFFu;
    mtg_boss_timings &T = c.timings;
    T = mtg_boss_timings{};
    note_bucket_index(c, nullptr, 0, nullptr, 0);
    HIP_CHECK(hipMemsetAsync(c.small, 0, sizeof(Small), c.stream));
    EventTimer tm(c.stream);
    const int ev_start = tm.mark();
    Dist d{comm, comm.size(), comm.rank(), 0, 0, 1, &tm, {}};
    const uint64_t sent0 = comm.sent_bytes;
    if (d.P > MAX_RANKS) throw std::runtime_error("more ranks than the routing kernels support");
    d.coresident = dist_coresident(c, d);
    T.coresident = d.coresident;
    T.world = (uint64_t)d.P;
    T.n_batches = 1;
    // ranges on the top m node chars, m <= k - 1 keeps every emission group inside one rank
    d.m = std::min(8u, k >= 2 ? k - 1 : 0u);
    d.shift2 = 2 * K - 2 * d.m;
    d.nb = 1ull << (2 * d.m);

    Tracer tr{c, d.me};
    c.radix_ms = 0;
    c.radix_bytes = 0;
    c.radix_launches = 0;
    int ev_extract, ev_sort, ev_unique;
    K2 *E = nullptr;
    uint32_t *Ec = nullptr;
    uint64_t R = 0;
    std::vector<uint64_t> bounds;
    // the routed collect plans its own rounds (canonical k-mers of the fused K1); the other collects
    // batch in key ranges that re-scan the reads
    bool routed_try = L2 == 1 && c.dist_collect != 2 && !c.disk && routed_applies(c, K);
    if (routed_try) routed_try = !dist_window_input(c, d, K, in);
    const uint32_t rounds = routed_try ? 1 : plan_rounds_dist<L2, COUNTED>(c, d, K, canonical, in);
    if (rounds > 1) {
        T.collect_mode = 1;
        // ---- K1-K4 in rounds of key batches (both strands in canonical mode): the owned real edges
        d.m = RB_CHARS;
        d.shift2 = 2 * K - 2 * d.m;
        d.nb = RB_BINS;
        ev_extract = tm.mark();
        R = collect_ranges_dist<L2, COUNTED>(c, d, K, canonical, cmax, in, rounds, &E, &Ec, &bounds, tr);
        ev_sort = ev_unique = tm.mark();
        T.n_unique = R;
    } else {
        K2 *xa = nullptr;
        uint32_t *xac = nullptr;
        std::vector<uint64_t> b1;
        bool routed = false;
        // exchange 0: the windows to their collect owners as super-k-mers (the collect below then runs
        // on the received runs); else the routed collect, else every rank collects its own reads
        BuildInput sk_in{};
        const bool sk = dist_superkmers(c, d, K, canonical, in, &sk_in, tr);
        if constexpr (L2 == 1)  // the fused extraction routes every k-mer to its owner
            if (!sk && routed_try)
                routed = dist_collect_routed<COUNTED>(c, d, K, canonical, cmax, in, &xa, &xac, &T.n_unique, &b1, tr, tm,
                                                      &ev_extract, &ev_sort);
        if (!routed) {
        const BuildInput &cin = sk ? sk_in : in;
        // ---- K1-K3 on this rank's reads
        K2 *ka, *kb;
        uint32_t *ca, *cb;
        uint64_t N = 0;
        double dup = 0;
        const uint32_t *hist1 = nullptr;
        MsdPlan fplan{};
        // a super-k-mer owner keeps the representative whose top bits hash smaller (cmode 2): its keys
        // spread evenly over the key space instead of piling up at small prefixes (min(fwd, rc)), so the
        // local sort's buckets do not overflow, and the range owners' shares stay even
        struct ModeScope {
            Ctx &c;
            int old;
            ~ModeScope() { c.canon_mode = old; }
        } mode_scope{c, c.canon_mode};
        if (sk && d.P > 1) c.canon_mode = 2;
        if (stage_extract_windows<L2, COUNTED>(c, K, canonical, cmax, cin, &ka, &kb, &ca, &cb, &N))
            dup = 1.0;
        else if (!stage_extract_fused<L2, COUNTED>(c, K, canonical, cmax, cin, &ka, &kb, &ca, &cb, &N, &dup, &hist1,
                                                    &fplan))
            N = stage_extract<L2, COUNTED>(c, K, canonical, cmax, cin, &ka, &kb, &ca, &cb);
        c.canon_mode = mode_scope.old;
        if (sk) {  // the windows of this rank's reads, not of the received runs
            T.n_positions = in.seq_len >= K ? in.seq_len - K + 1 : 0;
        }
        ev_extract = tm.mark();
        tr("extract", N);
        const uint64_t Ul = stage_collect<L2, COUNTED>(c, K, cmax, &ka, &kb, &ca, &cb, N, dup, true, hist1, &fplan);
        ev_sort = tm.mark();
        tr("local collect", Ul);

        // ---- exchange 1: the distinct k-mers by range of their own prefix, merged at the owner
        std::vector<std::vector<uint64_t>> soff;
        {
            // canonical mode: the ranges balance both strands (the canonical keys and their rc keys)
            // and are final, so exchange 2 moves only the rc keys
            const K2 *arrs[1] = {ka};
            const uint64_t ns[1] = {Ul};
            b1 = dist_ranges<L2>(c, d, 1, arrs, ns, &soff, canonical ? K : 0);
        }
        tr("ranges 1");
        {
            const K2 *arrs[1] = {ka};
            const uint32_t *cnts[1] = {ca};
            std::vector<uint64_t> runs;
            const uint64_t n1 = exchange_runs<K2>(c, d, 1, arrs, COUNTED ? cnts : nullptr, soff, Workspace::XA,
                                                  Workspace::XAC, &xa, &xac, &runs);
            tr("exchange 1", n1);
            if (d.P == 1) {  // one rank: its own sorted distinct k-mers came back unchanged
                T.n_unique = n1;
            } else {
                K2 *xb = (K2 *)c.ws.get(Workspace::XB, n1 * sizeof(K2));
                uint32_t *xbc = COUNTED ? (uint32_t *)c.ws.get(Workspace::XBC, n1 * 4) : nullptr;
                // the P runs are sorted and distinct within a run; duplicates across runs collapse and
                // their counts add with saturation (sorted_multiset.cpp:54-84).  The keys cover ~1/P of
                // the prefix space: P times denser buckets than their count says
                const double dup1 = estimate_dup<L2>(c, xa, n1, 1.0) / d.P;
                c.want_gidx = canonical;
                T.n_unique = msd_sort_unique<L2, COUNTED>(c, &xa, &xb, &xac, &xbc, n1, 2 * K, cmax, dup1, nullptr,
                                                          false, &runs);
                c.want_gidx = false;
            }
        }
        }
        const uint64_t U = T.n_unique;
        tr("owner dedupe", U);
        debug_check_sorted(c, "owned k-mers", xa, U);
        ev_unique = tm.mark();

        // ---- canonical: rc of the owned canonical set, routed to the owners of the rc keys
        E = xa;
        Ec = xac;
        R = U;
        bounds = b1;  // final in both modes
        if (canonical) {
            // rc keys of the owned canonical set, unsorted (even K: palindromes stay out with their
            // counts doubled, boss_chunk_construct.cpp:188-200)
            K2 *rbuf = (K2 *)c.ws.get(Workspace::KA, std::max<uint64_t>(U, 1) * sizeof(K2));
            uint32_t *rbufc = COUNTED ? (uint32_t *)c.ws.get(Workspace::CA, std::max<uint64_t>(U, 1) * 4) : nullptr;
            K2 *rk = rbuf;
            uint32_t *rkc = rbufc;
            uint64_t Urc = 0;
            if (U) Urc = stage_rc<L2, COUNTED>(c, K, cbits, cmax, xa, xac, U, rbuf, rbufc, &rk, &rkc, nullptr, false);
            tr("rc", Urc);
            K2 *rsend = (K2 *)c.ws.get(Workspace::QSEND, std::max<uint64_t>(Urc, 1) * sizeof(K2));
            uint32_t *rsendc = COUNTED ? (uint32_t *)c.ws.get(Workspace::RC_SENDC, std::max<uint64_t>(Urc, 1) * 4) : nullptr;
            std::vector<std::vector<uint64_t>> roff(1);
            roff[0] = route<L2, 1>(c, d, rk, Urc, K, d.shift2, 2 * d.m, bounds, rsend, COUNTED ? rkc : nullptr, rsendc);
            tr("route rc", Urc);
            // exchange 2: the rc keys only.  Every owned canonical key has exactly one owner, so the
            // received rc keys are distinct, and distinct from the canonical keys (a palindrome has no
            // rc key)
            K2 *rkeys;
            uint32_t *rcc = nullptr;
            const K2 *arrs[1] = {rsend};
            const uint32_t *cnts[1] = {rsendc};
            const uint64_t nrc = exchange_runs<K2>(c, d, 1, arrs, COUNTED ? cnts : nullptr, roff, Workspace::REAL,
                                                   Workspace::REALC, &rkeys, &rcc);
            tr("exchange 2", nrc);
            // the single build's rc sort, its local pass fused with the merge into the owned canonical
            // keys (local_merge_kernel); the keys cover ~1/P of the prefix space, so the plan is told
            // they are as dense as P * (nrc + U) / 2 rc keys of a single build
            K2 *out = (K2 *)c.ws.get(Workspace::KA, std::max<uint64_t>(U + nrc, 1) * sizeof(K2));
            uint32_t *outc = COUNTED ? (uint32_t *)c.ws.get(Workspace::CA, std::max<uint64_t>(U + nrc, 1) * 4) : nullptr;
            K2 *ralt = (K2 *)c.ws.get(Workspace::KB, std::max<uint64_t>(nrc, 1) * sizeof(K2));
            uint32_t *rcalt = COUNTED ? (uint32_t *)c.ws.get(Workspace::CB, std::max<uint64_t>(nrc, 1) * 4) : nullptr;
            RcMerge<L2> rm{xa, xac, U, out, outc};
            // the dummy stage's and the split emit's bucket index of the owned edges comes out of the
            // fused merge (as in the single build), sized for R = U + nrc
            rm.ib = bucket_bits<L2>(U + nrc, 2 * K);
            rm.istart = (uint64_t *)c.ws.get(Workspace::BUCKETS, ((1ull << rm.ib) + 2) * 8);
            const double dupm = nrc ? 2.0 * (double)nrc / ((double)d.P * (double)(nrc + U)) : 1.0;
            if (nrc && U && !COUNTED) {
                // the fused merge's speculative final level reads the owned canonical keys through their
                // bucket index over that level's bits: the owner sort's own index when its final bits are
                // the rc sort's, else one index pass here (the exchange pieces sort in several groups)
                const MsdPlan rp = msd_plan<L2>(c, nrc, 2 * K, dupm);
                const unsigned fb = rp.levels ? rp.digit_end[rp.levels] : 0;
                if (fb && fb <= 26 &&
                    !(c.gidx.keys == (const void *)xa && c.gidx.n == U && c.gidx.bits == fb && c.gidx.nbits == 2 * K)) {
                    const uint64_t nbk = 1ull << fb;
                    uint64_t *gi = (uint64_t *)c.ws.get(Workspace::CANON_IDX, (nbk + 2) * 8);
                    bucket_index<L2>(c, xa, U, 2 * K - fb, nbk, gi);
                    HIP_CHECK(hipMemcpyAsync(gi + nbk + 1, gi + nbk, 8, hipMemcpyDeviceToDevice, c.stream));
                    c.gidx = Ctx::GroupIndex{xa, U, fb, 2 * K, gi};
                }
            }
            uint64_t nr = 0;
            if (nrc)
                nr = msd_sort_unique<L2, COUNTED>(c, &rkeys, &ralt, &rcc, &rcalt, nrc, 2 * K, cmax, dupm, nullptr, true,
                                                  nullptr, false, U ? &rm : nullptr);
            if (!rm.done) merge_sorted<L2, L2, false, COUNTED, true>(c, xa, xac, U, rkeys, rcc, nr, K, out, outc, 0);
            R = U + nr;
            E = out;
            Ec = outc;
        }
    }
    T.n_real = R;
    tr("owner merge", R);
    debug_check_sorted(c, "real k-mers (owned)", E, R);
    const int ev_rc = tm.mark();

    // ---- K5/K6: sink / in-edge queries to the target node's owner, sources to theirs
    const unsigned k_b = K - 1;
    uint64_t D = 0;
    K3 *dk = nullptr;
    if (d.P == 1) {  // one rank owns every target node: the single build's local join
        D = stage_dummies_local<L2, L3>(c, K, E, R, &dk);
        tr("dummies (local)", D);
    } else if (c.dist_pull && d.m + 1 <= k_b) {
        // the pulled sink join (dist_kernels.hpp: pull_bounds_kernel): every rank sends each owner the
        // slices of its edges whose nodes the owner's edges target, the owner runs the single build's
        // join (dummy_sink_kernel) of its edges against them and returns an in-edge byte per received
        // edge; sinks and sources are then written like the single build's and routed to their owners
        uint8_t *flags = (uint8_t *)c.ws.get(Workspace::FLAGS, R + 1);
        std::vector<std::vector<uint64_t>> qoff(4, std::vector<uint64_t>(d.P + 1, 0));
        std::vector<uint64_t> cstart(5, R);
        cstart[0] = 0;
        if (R) {
            uint64_t *db = (uint64_t *)c.ws.get(Workspace::BOUNDS, (d.P + 1) * 8);
            uint64_t *g = (uint64_t *)c.ws.get(Workspace::XGATHER, 4 * (d.P + 1) * 8);
            HIP_CHECK(hipMemcpyAsync(db, bounds.data(), (d.P + 1) * 8, hipMemcpyHostToDevice, c.stream));
            pull_bounds_kernel<L2><<<dim3((unsigned)ceil_div(4 * (d.P + 1), 256)), dim3(256), 0, c.stream>>>(
                E, R, db, (uint32_t)d.P, K, d.m, g);
            HIP_CHECK(hipGetLastError());
            std::vector<uint64_t> pos(4 * (d.P + 1));
            HIP_CHECK(hipMemcpyAsync(pos.data(), g, pos.size() * 8, hipMemcpyDeviceToHost, c.stream));
            HIP_CHECK(hipStreamSynchronize(c.stream));  // bounds / pos are host locals
            for (int cl = 0; cl < 4; ++cl) {
                cstart[cl] = pos[cl * (d.P + 1)];
                for (int j = 0; j <= d.P; ++j) qoff[cl][j] = pos[cl * (d.P + 1) + j] - cstart[cl];
            }
            if (cstart[0] != 0 || pos[3 * (d.P + 1) + d.P] != R)
                throw std::logic_error("pulled join: the class slices do not cover the edges");
        }
        tr("pull bounds", R);
        K2 *qr;
        uint32_t *unused_c = nullptr;
        const K2 *qarr[4] = {E + cstart[0], E + cstart[1], E + cstart[2], E + cstart[3]};
        std::vector<uint64_t> qruns;
        const uint64_t nq = exchange_runs<K2>(c, d, 4, qarr, nullptr, qoff, Workspace::QRECV, Workspace::XAC, &qr,
                                              &unused_c, &qruns);
        tr("exchange pulled edges", nq);
        // the received edges are sorted (array-major = by top char, then by source rank = key order)
        const unsigned QB = bucket_bits<L2>(nq, 2 * K);
        const unsigned qshift = 2 * K - QB;
        uint64_t *qstart = (uint64_t *)c.ws.get(Workspace::QINDEX, ((1ull << QB) + 2) * 8);
        bucket_index<L2>(c, qr, nq, qshift, 1ull << QB, qstart);
        uint8_t *qin = (uint8_t *)c.ws.get(Workspace::QFLAG, nq + 1);
        if (nq) HIP_CHECK(hipMemsetAsync(qin, 0, nq, c.stream));
        if (R) {
            dummy_sink_kernel<L2><<<dim3((unsigned)ceil_div(R, DummyTraits<L2>::TILE)), dim3(256), 0, c.stream>>>(
                E, R, K, qstart, qshift, flags, qin, qr, nq);
            HIP_CHECK(hipGetLastError());
        }
        tr("pulled join", nq);
        // exchange back: the in-edge byte of every received edge to its sender, where the 4 x P pieces
        // land aligned with the sender's edge array (its classes in order, each by owner)
        std::vector<std::vector<uint64_t>> boff(4, std::vector<uint64_t>(d.P + 1, 0));
        const uint8_t *barr[4];
        for (int cl = 0; cl < 4; ++cl) {
            const uint64_t b0 = qruns[cl * d.P];
            barr[cl] = qin + b0;
            for (int i = 0; i < d.P; ++i) boff[cl][i] = qruns[cl * d.P + i] - b0;
            boff[cl][d.P] = qruns[(cl + 1) * d.P] - b0;  // the next class's first run (or the total)
        }
        uint8_t *in_flag;
        uint32_t *unused_b = nullptr;
        const uint64_t nback = exchange_runs<uint8_t>(c, d, 4, barr, nullptr, boff, Workspace::INFLAG, Workspace::XAC,
                                                      &in_flag, &unused_b);
        if (nback != R) throw std::logic_error("pulled join: in-edge bytes do not match the edges");
        tr("exchange in-edge bytes", nback);
        // the bucket index of the owned edges, for the split emit's dummy ranks (unless the fused rc
        // merge wrote it)
        if (!bidx_valid(c, E, R)) {
            const unsigned B = bucket_bits<L2>(R, 2 * K);
            const unsigned bshift = 2 * K - B;
            uint64_t *bstart = (uint64_t *)c.ws.get(Workspace::BUCKETS, ((1ull << B) + 2) * 8);
            bucket_index<L2>(c, E, R, bshift, 1ull << B, bstart);
            note_bucket_index(c, E, R, bstart, bshift);
        }
        // sinks (lift(to_next(x, 0)) with label $) and sources of every level, as the single build writes
        // them, routed to the owners of their lifted prefixes
        const uint64_t wtiles = ceil_div(R, DummyTraits<L2>::WTILE);
        uint32_t *tcnt = (uint32_t *)c.ws.get(Workspace::DTCNT, (wtiles + 1) * 4);
        uint64_t *toff = (uint64_t *)c.ws.get(Workspace::DTOFF, (wtiles + 1) * 8);
        uint64_t nraw = 0;
        if (R) {
            dummy_count_kernel<<<dim3((unsigned)wtiles), dim3(256), 0, c.stream>>>(flags, in_flag, R, k_b, tcnt);
            HIP_CHECK(hipGetLastError());
            uint32_t ep;
            const uint64_t st = ceil_div(wtiles, 4096);
            uint64_t *desc = acquire_desc(c, st, &ep);
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(tcnt, wtiles, toff, desc, ep,
                                                                              &c.small->counter, &c.small->error);
            HIP_CHECK(hipGetLastError());
            nraw = read_u64(c, (const unsigned long long *)(toff + wtiles));
        }
        K3 *src = (K3 *)c.ws.get(Workspace::DSRC, std::max<uint64_t>(nraw, 1) * sizeof(K3));
        if (nraw) {
            dummy_write_kernel<L2, L3><<<dim3((unsigned)wtiles), dim3(256), 0, c.stream>>>(E, flags, in_flag, R, K,
                                                                                            toff, src);
            HIP_CHECK(hipGetLastError());
        }
        tr("sinks + sources", nraw);
        K3 *ssend = (K3 *)c.ws.get(Workspace::DSEND, std::max<uint64_t>(nraw, 1) * sizeof(K3));
        std::vector<std::vector<uint64_t>> doff(1);
        doff[0] = route<L3, 1>(c, d, src, nraw, K, 3 * K - 3 * d.m, 3 * d.m, lifted_bounds(bounds, d.m), ssend);
        K3 *drecv;
        const K3 *darr[1] = {ssend};
        const uint64_t Draw = exchange_runs<K3>(c, d, 1, darr, nullptr, doff, Workspace::DRECV, Workspace::XAC, &drecv,
                                                &unused_c);
        tr("route + exchange dummies", Draw);
        if (Draw) {
            K3 *da = (K3 *)c.ws.get(Workspace::DA, Draw * sizeof(K3));
            K3 *db = (K3 *)c.ws.get(Workspace::DB, Draw * sizeof(K3));
            HIP_CHECK(hipMemcpyAsync(da, drecv, Draw * sizeof(K3), hipMemcpyDeviceToDevice, c.stream));
            D = sort_unique_dummies<L3>(c, K, da, db, Draw, &dk);
            tr("dummy sort", D);
        }
    } else {
        const unsigned B = bucket_bits<L2>(R, 2 * K);
        const unsigned bshift = 2 * K - B;
        const uint64_t nbk = 1ull << B;
        uint64_t *bstart = (uint64_t *)c.ws.get(Workspace::BUCKETS, (nbk + 2) * 8);
        bucket_index<L2>(c, E, R, bshift, nbk, bstart);
        note_bucket_index(c, E, R, bstart, bshift);
        uint8_t *flags = (uint8_t *)c.ws.get(Workspace::FLAGS, R + 1);
        uint8_t *in_flag = (uint8_t *)c.ws.get(Workspace::INFLAG, R + 1);
        if (R) {
            HIP_CHECK(hipMemsetAsync(in_flag, 0, R, c.stream));
            first_flag_kernel<L2><<<dim3((unsigned)std::min<uint64_t>(ceil_div(R, 256), 16384)), dim3(256), 0,
                                    c.stream>>>(E, R, flags);
            HIP_CHECK(hipGetLastError());
        }
        // queries t = to_next(x, 0) of every owned edge, as 4 sorted arrays (one per label of the
        // querying edge, dist_kernels.hpp: target_split_kernel); every owner's share is a slice of each
        K2 *qs = (K2 *)c.ws.get(Workspace::QSEND, std::max<uint64_t>(R, 1) * sizeof(K2));
        std::vector<std::vector<uint64_t>> qoff(4, std::vector<uint64_t>(d.P + 1, 0));
        std::vector<uint64_t> cstart(5, 0);
        if (R) {
            const uint64_t stiles = ceil_div(R, SplitTraits<L2>::TILE);
            uint32_t *tcnt = (uint32_t *)c.ws.get(Workspace::RTCNT, (4 * stiles + 1) * 4);
            uint64_t *toff = (uint64_t *)c.ws.get(Workspace::RTOFF, (4 * stiles + 1) * 8);
            target_split_kernel<L2, true><<<dim3((unsigned)stiles), dim3(256), 0, c.stream>>>(E, R, K, stiles, tcnt,
                                                                                               nullptr, nullptr);
            HIP_CHECK(hipGetLastError());
            uint32_t ep;
            const uint64_t st = ceil_div(4 * stiles, 4096);
            uint64_t *desc = acquire_desc(c, st, &ep);
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(tcnt, 4 * stiles, toff, desc, ep,
                                                                              &c.small->counter, &c.small->error);
            HIP_CHECK(hipGetLastError());
            target_split_kernel<L2, false><<<dim3((unsigned)stiles), dim3(256), 0, c.stream>>>(E, R, K, stiles, nullptr,
                                                                                                toff, qs);
            HIP_CHECK(hipGetLastError());
            uint64_t *g = (uint64_t *)c.ws.get(Workspace::XGATHER, (5 + 4 * (d.P + 1)) * 8);
            gather_strided_kernel<<<1, 256, 0, c.stream>>>(toff, stiles, 5, g);
            HIP_CHECK(hipGetLastError());
            uint64_t *db = (uint64_t *)c.ws.get(Workspace::BOUNDS, (d.P + 1) * 8);
            HIP_CHECK(hipMemcpyAsync(db, bounds.data(), (d.P + 1) * 8, hipMemcpyHostToDevice, c.stream));
            class_bounds_kernel<L2><<<dim3((unsigned)ceil_div(4 * (d.P + 1), 256)), dim3(256), 0, c.stream>>>(
                qs, g, db, (uint32_t)d.P, d.shift2, g + 5);
            HIP_CHECK(hipGetLastError());
            std::vector<uint64_t> pos(4 * (d.P + 1));
            HIP_CHECK(hipMemcpyAsync(cstart.data(), g, 5 * 8, hipMemcpyDeviceToHost, c.stream));
            HIP_CHECK(hipMemcpyAsync(pos.data(), g + 5, pos.size() * 8, hipMemcpyDeviceToHost, c.stream));
            HIP_CHECK(hipStreamSynchronize(c.stream));  // bounds / pos are host locals
            for (int cl = 0; cl < 4; ++cl)
                for (int j = 0; j <= d.P; ++j) qoff[cl][j] = pos[cl * (d.P + 1) + j] - cstart[cl];
            // the last owner ends at its class end
            for (int cl = 0; cl < 4; ++cl) qoff[cl][d.P] = cstart[cl + 1] - cstart[cl];
        }
        tr("first flags + split q", R);
        K2 *qr;
        uint32_t *unused_c = nullptr;
        const K2 *qarr[4] = {qs + cstart[0], qs + cstart[1], qs + cstart[2], qs + cstart[3]};
        const uint64_t nq = exchange_runs<K2>(c, d, 4, qarr, nullptr, qoff, Workspace::QRECV, Workspace::XAC,
                                         &qr, &unused_c);
        tr("exchange q", nq);
        uint8_t *qflag = (uint8_t *)c.ws.get(Workspace::QFLAG, nq + 1);
        if (nq) {
            query_join_kernel<L2><<<dim3((unsigned)ceil_div(nq, JoinTraits<L2>::TILE)), dim3(256), 0, c.stream>>>(
                E, R, bstart, bshift, qr, nq, in_flag, qflag);
            HIP_CHECK(hipGetLastError());
        }
        tr("answer q", nq);
        // sinks of the missed queries: count + scan now, written once the buffer is sized
        const uint64_t qtiles = ceil_div(nq, RT_TILE);
        uint32_t *qtcnt = (uint32_t *)c.ws.get(Workspace::QTCNT, (qtiles + 1) * 4);
        uint64_t *qtoff = (uint64_t *)c.ws.get(Workspace::QTOFF, (qtiles + 1) * 8);
        uint64_t nsink = 0;
        if (nq) {
            sink_count_kernel<<<dim3((unsigned)qtiles), dim3(RT_BLOCK), 0, c.stream>>>(qflag, nq, qtcnt);
            HIP_CHECK(hipGetLastError());
            uint32_t ep;
            const uint64_t st = ceil_div(qtiles, 4096);
            uint64_t *desc = acquire_desc(c, st, &ep);
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(qtcnt, qtiles, qtoff, desc, ep,
                                                                              &c.small->counter, &c.small->error);
            HIP_CHECK(hipGetLastError());
            nsink = read_u64(c, (const unsigned long long *)(qtoff + qtiles));
        }
        tr("sink count", nsink);
        // sources of the owned edges (in_flag is complete: every rank's queries are answered)
        const uint64_t wtiles = ceil_div(R, DummyTraits<L2>::WTILE);
        uint32_t *tcnt = (uint32_t *)c.ws.get(Workspace::DTCNT, (wtiles + 1) * 4);
        uint64_t *toff = (uint64_t *)c.ws.get(Workspace::DTOFF, (wtiles + 1) * 8);
        uint64_t nsrc = 0;
        if (R) {
            dummy_count_kernel<<<dim3((unsigned)wtiles), dim3(256), 0, c.stream>>>(flags, in_flag, R, k_b, tcnt);
            HIP_CHECK(hipGetLastError());
            uint32_t ep;
            const uint64_t st = ceil_div(wtiles, 4096);
            uint64_t *desc = acquire_desc(c, st, &ep);
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(tcnt, wtiles, toff, desc, ep,
                                                                              &c.small->counter, &c.small->error);
            HIP_CHECK(hipGetLastError());
            nsrc = read_u64(c, (const unsigned long long *)(toff + wtiles));
        }
        K3 *src = (K3 *)c.ws.get(Workspace::DSRC, std::max<uint64_t>(nsrc, 1) * sizeof(K3));
        if (nsrc) {
            dummy_write_kernel<L2, L3><<<dim3((unsigned)wtiles), dim3(256), 0, c.stream>>>(E, flags, in_flag, R, K,
                                                                                            toff, src);
            HIP_CHECK(hipGetLastError());
        }
        tr("sources", nsrc);
        K3 *ssend = (K3 *)c.ws.get(Workspace::DSEND, std::max<uint64_t>(nsrc, 1) * sizeof(K3));
        std::vector<std::vector<uint64_t>> doff(1);
        doff[0] = route<L3, 1>(c, d, src, nsrc, K, 3 * K - 3 * d.m, 3 * d.m, lifted_bounds(bounds, d.m), ssend);
        K3 *drecv;
        const K3 *darr[1] = {ssend};
        const uint64_t nsrc_in = exchange_runs<K3>(c, d, 1, darr, nullptr, doff, Workspace::DRECV, Workspace::XAC,
                                              &drecv, &unused_c);
        const uint64_t Draw = nsink + nsrc_in;
        tr("route + exchange src", nsrc_in);
        if (Draw) {
            K3 *da = (K3 *)c.ws.get(Workspace::DA, Draw * sizeof(K3));
            K3 *db = (K3 *)c.ws.get(Workspace::DB, Draw * sizeof(K3));
            if (nsink) {
                sink_write_kernel<L2, L3><<<dim3((unsigned)qtiles), dim3(RT_BLOCK), 0, c.stream>>>(qr, qflag, nq, K,
                                                                                                  qtoff, da);
                HIP_CHECK(hipGetLastError());
            }
            if (nsrc_in)
                HIP_CHECK(hipMemcpyAsync(da + nsink, drecv, nsrc_in * sizeof(K3), hipMemcpyDeviceToDevice,
                                         c.stream));
            tr("sink write", Draw);
            D = sort_unique_dummies<L3>(c, K, da, db, Draw, &dk);
            tr("dummy sort", D);
        }
    }
    T.n_dummy = D + (d.me == 0 ? 1 : 0);
    debug_check_sorted(c, "dummy k-mers (owned)", dk, D);
    const int ev_dummy = tm.mark();

    // ---- K7 + K8 on the owned range; rank 0 carries the main dummy row
    int ev_merge;
    stage_merge_emit<L2, L3, COUNTED>(c, tm, &ev_merge, k, bits, E, Ec, R, dk, D, d.me == 0, out);
    const int ev_emit = tm.mark();
    tr("merge + emit", out->n);
    check_error_word(c);
    HIP_CHECK(hipStreamSynchronize(c.stream));

    T.n_rows = out->n;
    T.extract_ms = tm.ms(ev_start, ev_extract);
    T.sort_ms = tm.ms(ev_extract, ev_sort);
    T.unique_ms = tm.ms(ev_sort, ev_unique);
    T.rc_ms = tm.ms(ev_unique, ev_rc);
    T.dummy_ms = tm.ms(ev_rc, ev_dummy);
    T.merge_ms = tm.ms(ev_dummy, ev_merge);
    T.emit_ms = tm.ms(ev_merge, ev_emit);
    T.total_ms = tm.ms(ev_start, ev_emit);
    for (auto &p : d.xev) T.exchange_ms += tm.ms(p.first, p.second);
    T.sent_bytes = comm.sent_bytes - sent0;
    T.radix_launches = c.radix_launches;
    T.radix_pass_ms = c.radix_launches ? c.radix_ms / c.radix_launches : 0;
    T.radix_bytes = c.radix_launches ? c.radix_bytes / c.radix_launches : 0;
    T.peak_bytes = c.ws.held();
}

// ------------------------------------------------------------- spilled build (out of HBM, f3)
//
// The disk container's role (SortedSetDisk + construct_boss_chunk_disk, boss_chunk_construct.cpp:
// 664-933; sorted_set_disk_base.cpp:36-278) when even the real edges do not fit the budget: the
// distributed algorithm with the key ranges as its "ranks", run one range at a time, every exchange
// going through host memory (or files under swap_dir) instead of a peer GPU.  HBM holds one range's
// edges and buffers at a time:
//   1. per range: collect its real edges (collect_ranges' extraction, both strands in canonical
//      mode) -> host; split their sink queries by label into 4 sorted arrays -> host;
//   2. per range r: its edges and every range's queries that target r -> sinks of r (misses) and
//      in-edge marks -> the dummy sources of r's nodes, routed by their lifted prefix -> host;
//   3. per range: its edges, sinks and the sources routed to it -> sort + unique -> split emit ->
//      the chunk rows appended on the host (BOSS::Chunk::extend, boss_chunk.cpp:230-270).
class SpillStore {
  public:
    SpillStore(std::string dir, uint64_t disk_cap) : dir_(std::move(dir)), cap_(disk_cap) {}
    ~SpillStore() {
        for (auto &b : blocks_)
            if (!b.path.empty()) std::remove(b.path.c_str());
    }
    // bytes of device memory d -> a new block (stream-ordered, synchronous)
    uint32_t put(const void *d, uint64_t bytes, hipStream_t s) {
        Block b;
        b.bytes = bytes;
        std::vector<uint8_t> h(bytes);
        if (bytes) {
            HIP_CHECK(hipMemcpyAsync(h.data(), d, bytes, hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
        }
        if (!dir_.empty() && on_disk_ + bytes <= cap_ && bytes) {
            b.path = dir_ + "/mtg_spill_" + std::to_string((unsigned long)getpid()) + "_" +
                     std::to_string((unsigned long)(uintptr_t)this) + "_" + std::to_string(blocks_.size()) + ".bin";
            FILE *f = fopen(b.path.c_str(), "wb");
            const bool ok = f && fwrite(h.data(), 1, bytes, f) == bytes;
            if (f) fclose(f);
            if (ok) {
                on_disk_ += bytes;
            } else {  // swap_dir unusable: keep the block in RAM
                std::remove(b.path.c_str());
                b.path.clear();
                b.ram = std::move(h);
            }
        } else {
            b.ram = std::move(h);
        }
        total_ += bytes;
        blocks_.push_back(std::move(b));
        return (uint32_t)blocks_.size() - 1;
    }
    // bytes [off, off + n) of block id -> device memory d
    void get(uint32_t id, uint64_t off, uint64_t n, void *d, hipStream_t s) {
        if (!n) return;
        const Block &b = blocks_[id];
        if (off + n > b.bytes) throw std::runtime_error("spill block read past its end");
        if (b.path.empty()) {
            HIP_CHECK(hipMemcpyAsync(d, b.ram.data() + off, n, hipMemcpyHostToDevice, s));
            HIP_CHECK(hipStreamSynchronize(s));
            return;
        }
        std::vector<uint8_t> h(n);
        FILE *f = fopen(b.path.c_str(), "rb");
        const bool ok = f && fseeko(f, (off_t)off, SEEK_SET) == 0 && fread(h.data(), 1, n, f) == n;
        if (f) fclose(f);
        if (!ok) throw std::runtime_error("cannot read spill file " + b.path);
        HIP_CHECK(hipMemcpyAsync(d, h.data(), n, hipMemcpyHostToDevice, s));
        HIP_CHECK(hipStreamSynchronize(s));
    }
    uint64_t bytes(uint32_t id) const { return blocks_[id].bytes; }
    uint64_t total() const { return total_; }
    uint64_t on_disk() const { return on_disk_; }

  private:
    struct Block {
        uint64_t bytes = 0;
        std::vector<uint8_t> ram;
        std::string path;
    };
    std::string dir_;
    uint64_t cap_;
    uint64_t total_ = 0, on_disk_ = 0;
    std::vector<Block> blocks_;
};

// the exchange layer of a spilled build has no peers: the routing helpers only read P from it
class NoComm : public Comm {
  public:
    explicit NoComm(int P) : Comm(0, P) {}
    void allreduce_sum_u64(uint64_t *, size_t, hipStream_t) override { fail(); }
    void allgather_u64(const uint64_t *, uint64_t *, size_t, hipStream_t) override { fail(); }
    void alltoallv_impl(const void *, const uint64_t *, const uint64_t *, void *, const uint64_t *, const uint64_t *,
                        size_t, hipStream_t) override {
        fail();
    }

  private:
    static void fail() { throw std::runtime_error("a spilled build has no exchange"); }
};

// spill when the build runs in key ranges, its arrays go to the host, and the real edges (at most
// the windows of both strands) may not fit the budget -- or always with MTG_SPILL=1
template <int L2, bool COUNTED>
static bool want_spill(Ctx &c, unsigned K, bool canonical, const BuildInput &in, uint32_t P) {
    if (P < 2 || !c.host_output || K < RB_CHARS + 2) return false;
    if (c.force_spill) return true;
    if (!c.disk) return false;
    const uint64_t npos = in.seq_len >= K ? in.seq_len - K + 1 : 0;
    double budget = c.mem_budget;
    if (budget <= 0) {
        size_t fr = 0, tot = 0;
        HIP_CHECK(hipMemGetInfo(&fr, &tot));
        budget = 0.9 * ((double)fr + (double)c.ws.held());
    }
    const double per_key = (double)sizeof(Key<L2>) + (COUNTED ? 4.0 : 0.0);
    // the in-HBM tail holds the real edges, their flags, the dummies and the output rows
    return (double)npos * (canonical ? 2.0 : 1.0) * (per_key + 4.0) > budget;
}

template <int L2, int L3, bool COUNTED>
static void run_pipeline_spill(Ctx &c, unsigned k, bool canonical, unsigned bits, const BuildInput &in, uint32_t P,
                               BuildOutput *out) {
    using K2 = Key<L2>;
    using K3 = Key<L3>;
    const unsigned K = k + 1;
    const unsigned cbits = bits <= 8 ? 8 : bits <= 16 ? 16 : 32;
    const uint32_t cmax = cbits == 8 ? 0xFFu : cbits == 16 ? 0xFFFFu : 0xFFFFFFFFu;
    mtg_boss_timings &T = c.timings;
    EventTimer tm(c.stream);
    const int ev_start = tm.mark();
    const uint64_t npos = in.seq_len >= K ? in.seq_len - K + 1 : 0;
    T.n_positions = npos;
    const int both = canonical ? 1 : 0;
    constexpr int TILE = RangeTraits<L2>::TILE;
    const uint64_t tiles = ceil_div(npos, TILE);
    // the ranges: count pass, bins balanced (collect_ranges)
    std::vector<uint64_t> hist(RB_BINS, 0);
    uint16_t *tbins = (uint16_t *)c.ws.get(Workspace::RANGE_BINS, std::max<uint64_t>(tiles, 1) * RB_BINS * 2);
    if (tiles) {
        auto *dh = (unsigned long long *)c.ws.get(Workspace::XHIST, RB_BINS * 8);
        HIP_CHECK(hipMemsetAsync(dh, 0, RB_BINS * 8, c.stream));
        range_count_kernel<L2><<<dim3((unsigned)tiles), dim3(256), 0, c.stream>>>(in.seq, in.seq_len, K, both, tbins);
        HIP_CHECK(hipGetLastError());
        range_bins_reduce_kernel<<<dim3((unsigned)std::min<uint64_t>(tiles, 2048)), dim3(RB_BINS), 0, c.stream>>>(
            tbins, tiles, dh);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(hist.data(), dh, RB_BINS * 8, hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));
    }
    uint64_t total = 0;
    for (uint64_t v : hist) total += v;
    P = std::min<uint32_t>(P, RB_BINS);
    const std::vector<uint64_t> bounds = balanced_bounds(hist.data(), RB_BINS, (int)P);
    NoComm nocomm((int)P);
    Dist d{nocomm, (int)P, 0, RB_CHARS, 2 * K - 2 * RB_CHARS, RB_BINS, &tm, {}};
    SpillStore st(c.disk ? c.swap_dir : std::string(), c.disk_cap);
    uint32_t *tcnt = (uint32_t *)c.ws.get(Workspace::DTCNT, (tiles + 1) * 4);
    uint64_t *toff = (uint64_t *)c.ws.get(Workspace::DTOFF, (tiles + 1) * 8);
    std::vector<uint32_t> eid(P), ecid(P), qid(P);
    std::vector<uint64_t> rn(P, 0);
    std::vector<std::vector<uint64_t>> qpos(P), qcs(P);  // per range: query slices [4][P + 1], class starts [5]
    // ---- 1. the real edges of every range, and their sink queries split by label
    for (uint32_t j = 0; j < P; ++j) {
        const uint32_t lo = (uint32_t)bounds[j], hi = (uint32_t)bounds[j + 1];
        uint64_t nj = 0;
        for (uint32_t b = lo; b < hi; ++b) nj += hist[b];
        K2 *ka = (K2 *)c.ws.get(Workspace::KA, std::max<uint64_t>(nj, 1) * sizeof(K2));
        K2 *kb = (K2 *)c.ws.get(Workspace::KB, std::max<uint64_t>(nj, 1) * sizeof(K2));
        uint32_t *ca = COUNTED ? (uint32_t *)c.ws.get(Workspace::CA, std::max<uint64_t>(nj, 1) * 4) : nullptr;
        uint32_t *cb = COUNTED ? (uint32_t *)c.ws.get(Workspace::CB, std::max<uint64_t>(nj, 1) * 4) : nullptr;
        uint64_t U = 0;
        if (nj) {
            BinSet sel{};
            sel.add(lo, hi);
            range_tile_counts_kernel<<<dim3((unsigned)ceil_div(tiles, 4)), dim3(256), 0, c.stream>>>(tbins, tiles, sel,
                                                                                                     tcnt);
            HIP_CHECK(hipGetLastError());
            uint32_t ep;
            const uint64_t sct = ceil_div(tiles, 4096);
            uint64_t *desc = acquire_desc(c, sct, &ep);
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            scan_counts_kernel<<<dim3((unsigned)sct), dim3(512), 0, c.stream>>>(tcnt, tiles, toff, desc, ep,
                                                                               &c.small->counter, &c.small->error);
            HIP_CHECK(hipGetLastError());
            range_write_kernel<L2, COUNTED><<<dim3((unsigned)tiles), dim3(256), 0, c.stream>>>(
                in.seq, in.seq_len, K, both, in.read_starts, in.read_counts, in.n_reads, in.rid_at, cmax, sel, toff, ka,
                ca);
            HIP_CHECK(hipGetLastError());
            if (read_u64(c, (const unsigned long long *)(toff + tiles)) != nj)
                throw std::runtime_error("range extraction count differs from its histogram");
            const double spread = (double)RB_BINS / (double)(hi - lo);
            const double dup = estimate_dup<L2>(c, ka, nj, 8.0) / spread;
            U = msd_sort_unique<L2, COUNTED>(c, &ka, &kb, &ca, &cb, nj, 2 * K, cmax, dup);
        }
        rn[j] = U;
        eid[j] = st.put(ka, U * sizeof(K2), c.stream);
        if (COUNTED) ecid[j] = st.put(ca, U * 4, c.stream);
        // the queries of the range's edges, 4 sorted arrays, sliced by target range
        qcs[j].assign(5, 0);
        qpos[j].assign(4 * (P + 1), 0);
        K2 *qs = (K2 *)c.ws.get(Workspace::QSEND, std::max<uint64_t>(U, 1) * sizeof(K2));
        if (U) {
            const uint64_t stiles = ceil_div(U, SplitTraits<L2>::TILE);
            uint32_t *qtc = (uint32_t *)c.ws.get(Workspace::RTCNT, (4 * stiles + 1) * 4);
            uint64_t *qto = (uint64_t *)c.ws.get(Workspace::RTOFF, (4 * stiles + 1) * 8);
            target_split_kernel<L2, true><<<dim3((unsigned)stiles), dim3(256), 0, c.stream>>>(ka, U, K, stiles, qtc,
                                                                                               nullptr, nullptr);
            HIP_CHECK(hipGetLastError());
            uint32_t ep;
            const uint64_t sct = ceil_div(4 * stiles, 4096);
            uint64_t *desc = acquire_desc(c, sct, &ep);
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            scan_counts_kernel<<<dim3((unsigned)sct), dim3(512), 0, c.stream>>>(qtc, 4 * stiles, qto, desc, ep,
                                                                               &c.small->counter, &c.small->error);
            HIP_CHECK(hipGetLastError());
            target_split_kernel<L2, false><<<dim3((unsigned)stiles), dim3(256), 0, c.stream>>>(ka, U, K, stiles, nullptr,
                                                                                                qto, qs);
            HIP_CHECK(hipGetLastError());
            uint64_t *g = (uint64_t *)c.ws.get(Workspace::XGATHER, (5 + 4 * (P + 1)) * 8);
            gather_strided_kernel<<<1, 256, 0, c.stream>>>(qto, stiles, 5, g);
            HIP_CHECK(hipGetLastError());
            uint64_t *db = (uint64_t *)c.ws.get(Workspace::BOUNDS, (P + 1) * 8);
            HIP_CHECK(hipMemcpyAsync(db, bounds.data(), (P + 1) * 8, hipMemcpyHostToDevice, c.stream));
            class_bounds_kernel<L2><<<dim3((unsigned)ceil_div(4 * (P + 1), 256)), dim3(256), 0, c.stream>>>(
                qs, g, db, P, d.shift2, g + 5);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipMemcpyAsync(qcs[j].data(), g, 5 * 8, hipMemcpyDeviceToHost, c.stream));
            HIP_CHECK(hipMemcpyAsync(qpos[j].data(), g + 5, qpos[j].size() * 8, hipMemcpyDeviceToHost, c.stream));
            HIP_CHECK(hipStreamSynchronize(c.stream));
            for (int cl = 0; cl < 4; ++cl) qpos[j][cl * (P + 1) + P] = qcs[j][cl + 1];
        }
        qid[j] = st.put(qs, U * sizeof(K2), c.stream);
    }
    T.n_extracted = total / (canonical ? 2 : 1);
    uint64_t R = 0;
    for (uint64_t v : rn) R += v;
    T.n_unique = T.n_real = R;
    const int ev_collect = tm.mark();
    // ---- 2. sinks and in-edge marks at every range, then the sources of its nodes, routed
    std::vector<uint32_t> skid(P), srcid(P);
    std::vector<uint64_t> nsk(P, 0);
    std::vector<std::vector<uint64_t>> soffs(P);
    const std::vector<uint64_t> b3 = lifted_bounds(bounds, RB_CHARS);
    for (uint32_t r = 0; r < P; ++r) {
        const uint64_t Rr = rn[r];
        K2 *E = (K2 *)c.ws.get(Workspace::REAL, std::max<uint64_t>(Rr, 1) * sizeof(K2));
        st.get(eid[r], 0, Rr * sizeof(K2), E, c.stream);
        const unsigned B = bucket_bits<L2>(Rr, 2 * K);
        const unsigned bshift = 2 * K - B;
        uint64_t *bstart = (uint64_t *)c.ws.get(Workspace::BUCKETS, ((1ull << B) + 2) * 8);
        bucket_index<L2>(c, E, Rr, bshift, 1ull << B, bstart);
        // every range's queries that target r: 4 sorted runs per range, in class order
        uint64_t nq = 0;
        for (uint32_t j = 0; j < P; ++j)
            for (int cl = 0; cl < 4; ++cl) nq += qpos[j][cl * (P + 1) + r + 1] - qpos[j][cl * (P + 1) + r];
        K2 *qr = (K2 *)c.ws.get(Workspace::QRECV, std::max<uint64_t>(nq, 1) * sizeof(K2));
        uint64_t o = 0;
        for (uint32_t j = 0; j < P; ++j)
            for (int cl = 0; cl < 4; ++cl) {
                const uint64_t a = qpos[j][cl * (P + 1) + r], b = qpos[j][cl * (P + 1) + r + 1];
                st.get(qid[j], a * sizeof(K2), (b - a) * sizeof(K2), qr + o, c.stream);
                o += b - a;
            }
        uint8_t *flags = (uint8_t *)c.ws.get(Workspace::FLAGS, Rr + 1);
        uint8_t *in_flag = (uint8_t *)c.ws.get(Workspace::INFLAG, Rr + 1);
        uint8_t *qflag = (uint8_t *)c.ws.get(Workspace::QFLAG, nq + 1);
        if (Rr) {
            HIP_CHECK(hipMemsetAsync(in_flag, 0, Rr, c.stream));
            first_flag_kernel<L2><<<dim3((unsigned)std::min<uint64_t>(ceil_div(Rr, 256), 16384)), dim3(256), 0,
                                    c.stream>>>(E, Rr, flags);
            HIP_CHECK(hipGetLastError());
        }
        if (nq) {
            query_join_kernel<L2><<<dim3((unsigned)ceil_div(nq, JoinTraits<L2>::TILE)), dim3(256), 0, c.stream>>>(
                E, Rr, bstart, bshift, qr, nq, in_flag, qflag);
            HIP_CHECK(hipGetLastError());
        }
        // the sinks of r: the queries that missed
        const uint64_t qtiles = ceil_div(nq, RT_TILE);
        uint32_t *qtcnt = (uint32_t *)c.ws.get(Workspace::QTCNT, (qtiles + 1) * 4);
        uint64_t *qtoff = (uint64_t *)c.ws.get(Workspace::QTOFF, (qtiles + 1) * 8);
        uint64_t nsink = 0;
        K3 *sk = nullptr;
        if (nq) {
            sink_count_kernel<<<dim3((unsigned)qtiles), dim3(RT_BLOCK), 0, c.stream>>>(qflag, nq, qtcnt);
            HIP_CHECK(hipGetLastError());
            uint32_t ep;
            const uint64_t sct = ceil_div(qtiles, 4096);
            uint64_t *desc = acquire_desc(c, sct, &ep);
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            scan_counts_kernel<<<dim3((unsigned)sct), dim3(512), 0, c.stream>>>(qtcnt, qtiles, qtoff, desc, ep,
                                                                               &c.small->counter, &c.small->error);
            HIP_CHECK(hipGetLastError());
            nsink = read_u64(c, (const unsigned long long *)(qtoff + qtiles));
            sk = (K3 *)c.ws.get(Workspace::DA, std::max<uint64_t>(nsink, 1) * sizeof(K3));
            if (nsink) {
                sink_write_kernel<L2, L3><<<dim3((unsigned)qtiles), dim3(RT_BLOCK), 0, c.stream>>>(qr, qflag, nq, K,
                                                                                                  qtoff, sk);
                HIP_CHECK(hipGetLastError());
            }
        }
        nsk[r] = nsink;
        skid[r] = st.put(sk, nsink * sizeof(K3), c.stream);
        // the sources of r's nodes (first edges no query hit), every level, routed by lifted prefix
        const uint64_t wtiles = ceil_div(Rr, DummyTraits<L2>::WTILE);
        uint32_t *wc = (uint32_t *)c.ws.get(Workspace::DTCNT, (std::max(wtiles, tiles) + 1) * 4);
        uint64_t *wo = (uint64_t *)c.ws.get(Workspace::DTOFF, (std::max(wtiles, tiles) + 1) * 8);
        uint64_t nsrc = 0;
        if (Rr) {
            dummy_count_kernel<<<dim3((unsigned)wtiles), dim3(256), 0, c.stream>>>(flags, in_flag, Rr, k, wc);
            HIP_CHECK(hipGetLastError());
            uint32_t ep;
            const uint64_t sct = ceil_div(wtiles, 4096);
            uint64_t *desc = acquire_desc(c, sct, &ep);
            HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
            scan_counts_kernel<<<dim3((unsigned)sct), dim3(512), 0, c.stream>>>(wc, wtiles, wo, desc, ep,
                                                                               &c.small->counter, &c.small->error);
            HIP_CHECK(hipGetLastError());
            nsrc = read_u64(c, (const unsigned long long *)(wo + wtiles));
        }
        K3 *src = (K3 *)c.ws.get(Workspace::DSRC, std::max<uint64_t>(nsrc, 1) * sizeof(K3));
        if (nsrc) {
            dummy_write_kernel<L2, L3><<<dim3((unsigned)wtiles), dim3(256), 0, c.stream>>>(E, flags, in_flag, Rr, K, wo,
                                                                                            src);
            HIP_CHECK(hipGetLastError());
        }
        K3 *ssend = (K3 *)c.ws.get(Workspace::DSEND, std::max<uint64_t>(nsrc, 1) * sizeof(K3));
        soffs[r] = route<L3, 1>(c, d, src, nsrc, K, 3 * K - 3 * RB_CHARS, 3 * RB_CHARS, b3, ssend);
        srcid[r] = st.put(ssend, nsrc * sizeof(K3), c.stream);
    }
    const int ev_dummy_route = tm.mark();
    // ---- 3. per range: dummies sorted, rows emitted, appended on the host
    c.spill_W.clear();
    c.spill_last.clear();
    c.spill_weights.clear();
    uint64_t F[5] = {0, 0, 0, 0, 0}, ndummy = 0;
    for (uint32_t r = 0; r < P; ++r) {
        const uint64_t Rr = rn[r];
        K2 *E = (K2 *)c.ws.get(Workspace::REAL, std::max<uint64_t>(Rr, 1) * sizeof(K2));
        uint32_t *Ec = COUNTED ? (uint32_t *)c.ws.get(Workspace::REALC, std::max<uint64_t>(Rr, 1) * 4) : nullptr;
        st.get(eid[r], 0, Rr * sizeof(K2), E, c.stream);
        if (COUNTED) st.get(ecid[r], 0, Rr * 4, Ec, c.stream);
        uint64_t Draw = nsk[r];
        for (uint32_t j = 0; j < P; ++j) Draw += soffs[j][r + 1] - soffs[j][r];
        K3 *da = (K3 *)c.ws.get(Workspace::DA, std::max<uint64_t>(Draw, 1) * sizeof(K3));
        K3 *db = (K3 *)c.ws.get(Workspace::DB, std::max<uint64_t>(Draw, 1) * sizeof(K3));
        st.get(skid[r], 0, nsk[r] * sizeof(K3), da, c.stream);
        uint64_t o = nsk[r];
        for (uint32_t j = 0; j < P; ++j) {
            const uint64_t a = soffs[j][r], b = soffs[j][r + 1];
            st.get(srcid[j], a * sizeof(K3), (b - a) * sizeof(K3), da + o, c.stream);
            o += b - a;
        }
        K3 *dk = nullptr;
        uint64_t D = 0;
        if (Draw) D = sort_unique_dummies<L3>(c, K, da, db, Draw, &dk);
        note_bucket_index(c, nullptr, 0, nullptr, 0);
        BuildOutput o2{};
        int ev_m;
        stage_merge_emit<L2, L3, COUNTED>(c, tm, &ev_m, k, bits, E, Ec, Rr, dk, D, r == 0, &o2);
        check_error_word(c);
        // extend: range 0 keeps its leading row 0, the others append the rows after it
        const uint64_t from = r == 0 ? 0 : 1, rows = o2.n - from;
        const uint64_t at = c.spill_W.size();
        c.spill_W.resize(at + rows);
        c.spill_last.resize(at + rows);
        HIP_CHECK(hipMemcpyAsync(c.spill_W.data() + at, o2.W + from, rows, hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipMemcpyAsync(c.spill_last.data() + at, o2.last + from, rows, hipMemcpyDeviceToHost, c.stream));
        if (COUNTED) {
            c.spill_weights.resize(at + rows);
            HIP_CHECK(hipMemcpyAsync(c.spill_weights.data() + at, o2.weights + from, rows * 4, hipMemcpyDeviceToHost,
                                     c.stream));
        }
        HIP_CHECK(hipStreamSynchronize(c.stream));
        for (int ch = 0; ch < 5; ++ch) F[ch] += o2.F[ch];
        ndummy += o2.n_dummy;
    }
    const int ev_emit = tm.mark();
    HIP_CHECK(hipStreamSynchronize(c.stream));
    out->host = true;
    out->W = c.spill_W.data();
    out->last = c.spill_last.data();
    out->weights = COUNTED ? c.spill_weights.data() : nullptr;
    out->n = c.spill_W.size();
    std::memcpy(out->F, F, sizeof(F));
    out->n_real = R;
    out->n_dummy = ndummy;
    c.spilled_bytes = st.total();
    T.spilled_bytes = st.total();
    T.n_dummy = ndummy;
    T.n_rows = out->n;
    T.n_batches = P;
    T.extract_ms = tm.ms(ev_start, ev_collect);
    T.dummy_ms = tm.ms(ev_collect, ev_dummy_route);
    T.emit_ms = tm.ms(ev_dummy_route, ev_emit);
    T.total_ms = tm.ms(ev_start, ev_emit);
    T.peak_bytes = c.ws.held();
}

// ------------------------------------------------------------------ suffix-filtered route
//
// IBOSSChunkConstructor with a non-empty filter suffix (boss_chunk_construct.cpp:946-1013): the
// (k+1)-mers of the `$`-padded read segments whose node ends with the suffix, both strands in
// BOTH mode (suffix_extract.hpp), sorted and deduplicated (counts added with saturation), then
// initialize_chunk over that set as it is -- the padding supplies the dummy edges, so there is
// no dummy reconstruction.  The chunk of the all-`$` suffix also holds the main dummy edge
// (:977-980).  The chunks of all suffixes concatenate (in suffix order) into the graph
// (cli/build.cpp:359-456; mtg_boss_concatenate prunes their redundant source dummies).
template <int L3, bool COUNTED>
static void run_suffix(Ctx &c, unsigned k, bool both, unsigned bits, const SuffixSpec &suf, bool all_sentinel,
                       const BuildInput &in, BuildOutput *out) {
    using K3 = Key<L3>;
    using T = SuffixTraits;
    const unsigned K = k + 1;
    const unsigned cbits = bits <= 8 ? 8 : bits <= 16 ? 16 : 32;
    const uint32_t cmax = cbits == 8 ? 0xFFu : cbits == 16 ? 0xFFFFu : 0xFFFFFFFFu;
    const uint32_t wmax = bits >= 32 ? 0xFFFFFFFFu : (uint32_t)((1ull << bits) - 1);
    mtg_boss_timings &Tm = c.timings;
    Tm = mtg_boss_timings{};
    Tm.world = 1;
    Tm.n_batches = 1;
    HIP_CHECK(hipMemsetAsync(c.small, 0, sizeof(Small), c.stream));
    EventTimer tm(c.stream);
    const int ev_start = tm.mark();

    // ---- K1: count -> scan -> write over identical tiles of buffer positions
    const uint64_t tiles = ceil_div(in.seq_len + 1, T::TILE);
    uint32_t *tcnt = (uint32_t *)c.ws.get(Workspace::DTCNT, (tiles + 1) * 4);
    uint64_t *toff = (uint64_t *)c.ws.get(Workspace::DTOFF, (tiles + 1) * 8);
    suffix_extract_kernel<L3, COUNTED, true><<<dim3((unsigned)tiles), dim3(T::BLOCK), 0, c.stream>>>(
        in.seq, in.seq_len, K, both ? 1 : 0, suf, in.read_starts, in.read_counts, in.n_reads, in.rid_at, cmax, tcnt,
        nullptr, nullptr, nullptr);
    HIP_CHECK(hipGetLastError());
    {
        uint32_t ep;
        const uint64_t st = ceil_div(tiles, 4096);
        uint64_t *desc = acquire_desc(c, st, &ep);
        HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
        scan_counts_kernel<<<dim3((unsigned)st), dim3(512), 0, c.stream>>>(tcnt, tiles, toff, desc, ep,
                                                                          &c.small->counter, &c.small->error);
        HIP_CHECK(hipGetLastError());
    }
    uint64_t N = read_u64(c, (const unsigned long long *)(toff + tiles));
    Tm.n_positions = in.seq_len;
    const uint64_t cap = N + (all_sentinel ? 1 : 0);
    K3 *ka = (K3 *)c.ws.get(Workspace::KA, std::max<uint64_t>(cap, 1) * sizeof(K3));
    K3 *kb = (K3 *)c.ws.get(Workspace::KB, std::max<uint64_t>(cap, 1) * sizeof(K3));
    uint32_t *ca = COUNTED ? (uint32_t *)c.ws.get(Workspace::CA, std::max<uint64_t>(cap, 1) * 4) : nullptr;
    uint32_t *cb = COUNTED ? (uint32_t *)c.ws.get(Workspace::CB, std::max<uint64_t>(cap, 1) * 4) : nullptr;
    if (N) {
        suffix_extract_kernel<L3, COUNTED, false><<<dim3((unsigned)tiles), dim3(T::BLOCK), 0, c.stream>>>(
            in.seq, in.seq_len, K, both ? 1 : 0, suf, in.read_starts, in.read_counts, in.n_reads, in.rid_at, cmax, nullptr,
            toff, ka, ca);
        HIP_CHECK(hipGetLastError());
    }
    if (all_sentinel) {  // add_kmer(k+1 sentinels): the main dummy edge, count 1
        HIP_CHECK(hipMemsetAsync(ka + N, 0, sizeof(K3), c.stream));
        if (COUNTED) {
            const uint32_t one = 1;
            HIP_CHECK(hipMemcpyAsync(ca + N, &one, 4, hipMemcpyHostToDevice, c.stream));
            HIP_CHECK(hipStreamSynchronize(c.stream));
        }
        ++N;
    }
    Tm.n_extracted = N;
    const int ev_extract = tm.mark();

    // ---- sort + unique / saturating count merge of the lifted keys (LSD over 3K bits)
    radix_sort<L3, COUNTED>(c, &ka, &kb, &ca, &cb, N, 3 * K, false);
    uint64_t U = 0;
    reset_small(c);
    if (N) {
        const uint64_t utiles = ceil_div(N, 2048);
        uint32_t desc_ep;
        uint64_t *desc = acquire_desc(c, utiles, &desc_ep);
        unsigned long long *sums = nullptr;
        if (COUNTED) {
            sums = (unsigned long long *)c.ws.get(Workspace::SUMS, N * 8);
            HIP_CHECK(hipMemsetAsync(sums, 0, N * 8, c.stream));
        }
        unique_kernel<L3, COUNTED><<<dim3((unsigned)utiles), dim3(256), 0, c.stream>>>(
            ka, ca, N, kb, sums, desc, desc_ep, &c.small->counter, &c.small->total, &c.small->error);
        HIP_CHECK(hipGetLastError());
        U = read_u64(c, &c.small->total);
        if (COUNTED && U) {
            count_clamp_kernel<<<dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(U, 256), 4096))),
                                 dim3(256), 0, c.stream>>>(sums, U, cmax, cb);
            HIP_CHECK(hipGetLastError());
        }
        std::swap(ka, kb);
        std::swap(ca, cb);
    }
    Tm.n_unique = U;
    debug_check_sorted(c, "suffix k-mers", ka, U);
    const int ev_sort = tm.mark();

    // ---- K8 over the set as it is
    emit_stream<L3, COUNTED>(c, k, wmax, ka, ca, U, U, out);
    const int ev_emit = tm.mark();
    check_error_word(c);
    HIP_CHECK(hipStreamSynchronize(c.stream));
    Tm.n_real = out->n ? out->n - 1 : 0;
    Tm.n_dummy = 0;
    Tm.n_rows = out->n;
    Tm.extract_ms = tm.ms(ev_start, ev_extract);
    Tm.sort_ms = tm.ms(ev_extract, ev_sort);
    Tm.emit_ms = tm.ms(ev_sort, ev_emit);
    Tm.total_ms = tm.ms(ev_start, ev_emit);
    Tm.peak_bytes = c.ws.held();
}

// word choice of the suffix route: lifted keys by (k+1)*3 (boss_chunk_construct.cpp:1080-1091)
static void run_suffix_dispatch(Ctx &c, unsigned k, bool both, unsigned bits, const SuffixSpec &suf,
                                bool all_sentinel, const BuildInput &in, BuildOutput *out) {
    const unsigned K = k + 1;
    if (3 * K <= 64) {
        if (bits) run_suffix<1, true>(c, k, both, bits, suf, all_sentinel, in, out);
        else run_suffix<1, false>(c, k, both, bits, suf, all_sentinel, in, out);
    } else if (3 * K <= 128) {
        if (bits) run_suffix<2, true>(c, k, both, bits, suf, all_sentinel, in, out);
        else run_suffix<2, false>(c, k, both, bits, suf, all_sentinel, in, out);
    } else {
        if (bits) run_suffix<4, true>(c, k, both, bits, suf, all_sentinel, in, out);
        else run_suffix<4, false>(c, k, both, bits, suf, all_sentinel, in, out);
    }
}

// the builder's KMC1 writer (kmc.hpp): every k-mer of the reads with count 1, mapped to KMC words,
// sorted + counted (saturating at 2^32 - 1), then written on the host; returns the records
static uint64_t kmc_count_write(Ctx &c, const BuildInput &in, unsigned K, bool canonical, unsigned counter_size,
                                unsigned lut_len, const std::string &base, unsigned threads) {
    if (K < 1 || K > 32) throw std::runtime_error("KMC writer: k must be in [1, 32]");
    HIP_CHECK(hipMemsetAsync(c.small, 0, sizeof(Small), c.stream));
    Key<1> *ka, *kb;
    uint32_t *ca, *cb;
    const uint64_t N = stage_extract<1, true>(c, K, false, 0xFFFFFFFFu, in, &ka, &kb, &ca, &cb);
    uint64_t U = 0;
    if (N) {
        kmc_key_kernel<<<dim3((unsigned)std::min<uint64_t>(ceil_div(N, 256), 65536)), dim3(256), 0, c.stream>>>(
            (uint64_t *)ka, N, K, canonical ? 1 : 0);
        HIP_CHECK(hipGetLastError());
        const double dup = estimate_dup<1>(c, ka, N, 8.0);
        U = msd_sort_unique<1, true>(c, &ka, &kb, &ca, &cb, N, 2 * K, 0xFFFFFFFFu, dup);
    }
    check_error_word(c);
    std::vector<uint64_t> keys(U);
    std::vector<uint32_t> counts(U);
    if (U) {
        HIP_CHECK(hipMemcpyAsync(keys.data(), ka, U * 8, hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipMemcpyAsync(counts.data(), ca, U * 4, hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));
    }
    kmc_write_files(base, keys.data(), counts.data(), U, K, lut_len, counter_size, canonical, threads);
    return U;
}

template <int L2, int L3>
static void run_counted(Ctx &c, Comm *comm, unsigned k, bool canonical, unsigned bits, const BuildInput &in,
                        BuildOutput *out) {
    if (comm) {
        if (bits) run_pipeline_dist<L2, L3, true>(c, *comm, k, canonical, bits, in, out);
        else run_pipeline_dist<L2, L3, false>(c, *comm, k, canonical, bits, in, out);
    } else {
        if (bits) run_pipeline<L2, L3, true>(c, k, canonical, bits, in, out);
        else run_pipeline<L2, L3, false>(c, k, canonical, bits, in, out);
    }
}

// word choice as boss_chunk_construct.cpp:1068-1079 (2-bit, by (k+1)*2) and :1030-1036
// (lifted, by (k+1)*3)
static void run_dispatch(Ctx &c, Comm *comm, unsigned k, bool canonical, unsigned bits, const BuildInput &in,
                         BuildOutput *out) {
    const unsigned K = k + 1;
    if (3 * K <= 64) run_counted<1, 1>(c, comm, k, canonical, bits, in, out);
    else if (2 * K <= 64) run_counted<1, 2>(c, comm, k, canonical, bits, in, out);
    else if (3 * K <= 128) run_counted<2, 2>(c, comm, k, canonical, bits, in, out);
    else if (2 * K <= 128) run_counted<2, 4>(c, comm, k, canonical, bits, in, out);
    else run_counted<4, 4>(c, comm, k, canonical, bits, in, out);
}
}  // namespace mtg

// ============================================================================ C ABI

struct mtg_boss_ctor {
    mtg_boss_params params{};
    std::string suffix;
    int device = 0;
    mtg::Ctx ctx;
    std::mutex mu;                   // one build at a time; adds run concurrently (HostStage)
    mtg::HostStage stage;            // staged reads in pinned memory, each followed by '$'
    std::mutex kmc_mu;
    std::vector<mtg::KmcInput> kmc;  // KMC databases, decoded on the device at build time
    std::atomic<uint64_t> stage_ns{0};  // host time spent staging since the last build
    std::mutex fa_mu;
    std::vector<mtg::FastaInput> fasta;  // FASTA / FASTQ files, split into reads on the device
    uint8_t *w4_host = nullptr;          // pinned landing buffer of the 4-bit W copy
    uint64_t w4_cap = 0;
    uint8_t *wn_host = nullptr;          // pinned landing buffer of the narrowed weights copy
    uint64_t wn_cap = 0;
    ~mtg_boss_ctor() {
        for (auto &f : fasta) mtg::free_fasta(f);
        if (w4_host) (void)hipHostFree(w4_host);
        if (wn_host) (void)hipHostFree(wn_host);
    }
};

// staged reads (host_stage.hpp) -> one byte per char: ACGT, or 'N' for every char that breaks a
// k-mer window (separators, alignment gaps, N and the rest); one 32-char word per thread
__global__ void unpack_reads_kernel(const uint64_t *__restrict__ codes, const uint32_t *__restrict__ valid,
                                    uint64_t nw, uint8_t *__restrict__ out) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nw) return;
    const uint64_t c = codes[w];
    const uint32_t v = valid[w];
    uint32_t o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        uint32_t word = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int j = 4 * q + b;
            const uint32_t ch = (v >> j) & 1u ? (0x54474341u >> (8 * ((c >> (2 * j)) & 3u))) & 0xFFu : (uint32_t)'N';
            word |= ch << (8 * b);
        }
        o[q] = word;
    }
    uint4 *dst = (uint4 *)(out + 32 * w);
    dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
    dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
}

// one packed `last` word per thread: bit j of word w = last[64 w + j] (sdsl bit_vector layout)
__global__ void pack_bits_kernel(const uint8_t *__restrict__ bytes, uint64_t n, uint64_t *__restrict__ words) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = w * 64;
    if (i0 >= n) return;
    uint64_t v = 0;
    if (i0 + 64 <= n && ((uintptr_t)(bytes + i0) & 7) == 0) {
        const uint64_t *p = reinterpret_cast<const uint64_t *>(bytes + i0);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint64_t x = p[q];  // 8 flag bytes (0/1) -> 8 bits
            v |= ((x * 0x0102040810204080ull) >> 56 & 0xFFull) << (8 * q);
        }
    } else {
        for (uint64_t j = 0; j < 64 && i0 + j < n; ++j) v |= (uint64_t)(bytes[i0 + j] & 1) << j;
    }
    words[w] = v;
}

using namespace mtg;

extern "C" {

int mtg_boss_abi_version(void) { return MTG_BOSS_ABI_VERSION; }

const char *mtg_last_error(void) { return g_last_error.c_str(); }

mtg_boss_ctor *mtg_boss_ctor_create(const mtg_boss_params *p) {
    if (!p) {
        set_error("null params");
        return nullptr;
    }
    if (p->k < 1 || p->k > 84) {
        set_error("For succinct graph, k must be between 2 and 85");
        return nullptr;
    }
    if (p->bits_per_count > 32) {
        set_error("Error: trying to allocate too many bits per k-mer count");
        return nullptr;
    }
    if (p->container_type != MTG_CONTAINER_VECTOR && p->container_type != MTG_CONTAINER_VECTOR_DISK) {
        set_error("an unknown container does not run on the GPU path");
        return nullptr;
    }
    const std::string suffix = p->filter_suffix ? p->filter_suffix : "";
    if (suffix.size() >= p->k + 1) {  // kmer_extractor.cpp:325: the suffix excludes the last char
        set_error("the filter suffix must be shorter than k + 1");
        return nullptr;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= p->device_id || p->device_id < 0) {
        set_error("no HIP device " + std::to_string(p->device_id) + " visible");
        return nullptr;
    }
    auto *c = new mtg_boss_ctor();
    c->params = *p;
    c->params.filter_suffix = nullptr;  // the caller's strings need not outlive the call
    c->params.swap_dir = nullptr;
    c->suffix = suffix;
    c->device = p->device_id;
    c->stage.enable_mirror(c->device);
    try {
        HIP_CHECK(hipSetDevice(c->device));
        HIP_CHECK(hipStreamCreateWithFlags(&c->ctx.stream, hipStreamNonBlocking));
        HIP_CHECK(hipMalloc(&c->ctx.small, sizeof(Small)));
        load_knobs(c->ctx);
        c->ctx.mem_budget = p->memory_preallocated;
        c->ctx.swap_dir = p->swap_dir ? p->swap_dir : "";
        c->ctx.disk_cap = p->disk_cap_bytes;
        // the disk container bounds memory: always collect in key ranges (boss_chunk_construct.cpp:664-933)
        if (p->container_type == MTG_CONTAINER_VECTOR_DISK && !c->ctx.force_ranges) c->ctx.disk = true;
    } catch (const std::exception &e) {
        set_error(e.what());
        delete c;
        return nullptr;
    }
    return c;
}

void mtg_boss_ctor_destroy(mtg_boss_ctor *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->ctx.stream) (void)hipStreamSynchronize(c->ctx.stream);
    if (c->ctx.small) (void)hipFree(c->ctx.small);
    if (c->ctx.stream) (void)hipStreamDestroy(c->ctx.stream);
    if (c->ctx.xstream) {
        (void)hipStreamSynchronize(c->ctx.xstream);
        (void)hipStreamDestroy(c->ctx.xstream);
    }
    delete c;
}

uint64_t mtg_boss_ctor_get_k(const mtg_boss_ctor *c) { return c ? c->params.k : 0; }

int mtg_boss_ctor_trim(mtg_boss_ctor *c) {
    if (!c) {
        set_error("bad arguments");
        return MTG_ERR_ARGUMENT;
    }
    std::lock_guard<std::mutex> lock(c->mu);
    try {
        HIP_CHECK(hipSetDevice(c->device));
        // the last build's stage buffers too (its device chunk arrays stay valid): a configs[2] build
        // holds ~200 GB in them, and a second constructor in the same process had 110 MiB left
        c->ctx.ws.release_stage_buffers(true);
        note_bucket_index(c->ctx, nullptr, 0, nullptr, 0);
        c->ctx.gap.valid = false;
        c->ctx.gidx = Ctx::GroupIndex{};
        c->ctx.ws.drop_cache();
        c->ctx.timings.cached_bytes = 0;
        return MTG_OK;
    } catch (const std::exception &e) {
        set_error(e.what());
        return MTG_ERR_DEVICE;
    }
}

struct StageTimer {
    std::atomic<uint64_t> &acc;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~StageTimer() {
        acc += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0)
                   .count();
    }
};

static unsigned stage_threads(const mtg_boss_ctor *c) {
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(c->params.num_threads, 64));
}

int mtg_boss_ctor_add_sequences(mtg_boss_ctor *c, const char *const *seqs, const uint64_t *lens,
                                const uint64_t *counts, size_t n) {
    if (!c || (n && (!seqs || !lens))) {
        set_error("bad arguments");
        return MTG_ERR_ARGUMENT;
    }
    try {
        StageTimer t{c->stage_ns};
        c->stage.add(seqs, lens, counts, n, stage_threads(c));
        return MTG_OK;
    } catch (const std::exception &e) {
        set_error(e.what());
        return MTG_ERR_ARGUMENT;
    }
}

int mtg_boss_ctor_add_sequence(mtg_boss_ctor *c, const char *seq, uint64_t len, uint64_t count) {
    if (!c || (len && !seq)) {
        set_error("bad arguments");
        return MTG_ERR_ARGUMENT;
    }
    const char *p = seq ? seq : "";
    return mtg_boss_ctor_add_sequences(c, &p, &len, &count, 1);
}

int mtg_boss_ctor_add_packed(mtg_boss_ctor *c, const char *data, const uint64_t *offsets,
                             const uint64_t *counts, size_t n) {
    if (!c || (n && (!data || !offsets))) {
        set_error("bad arguments");
        return MTG_ERR_ARGUMENT;
    }
    for (size_t i = 0; i < n; ++i) {
        if (offsets[i + 1] < offsets[i]) {
            set_error("offsets must be nondecreasing");
            return MTG_ERR_ARGUMENT;
        }
    }
    try {
        StageTimer t{c->stage_ns};
        c->stage.add_packed(data, offsets, counts, n, stage_threads(c));
        return MTG_OK;
    } catch (const std::exception &e) {
        set_error(e.what());
        return MTG_ERR_ARGUMENT;
    }
}

int mtg_boss_ctor_add_kmc(mtg_boss_ctor *c, const char *kmc_path, uint64_t min_count, uint64_t max_count,
                          int call_both_from_canonical) {
    if (!c || !kmc_path) {
        set_error("bad arguments");
        return MTG_ERR_ARGUMENT;
    }
    try {
        // the first database of a batch is copied to the device while its files are read (the
        // workspace's KMC slots; a later database is copied by build_chunk, the slots being taken)
        std::unique_lock<std::mutex> lock(c->kmc_mu, std::defer_lock);
        if (c->ctx.kmc_mirror) lock.lock();
        const bool mirror = c->ctx.kmc_mirror && c->kmc.empty();
        DeviceGuard g(c->device);
        DeviceMirror mpre, msuf;
        mpre.stream = msuf.stream = c->ctx.stream;
        mpre.device = msuf.device = c->device;
        mpre.alloc = [&](uint64_t b) { return (uint8_t *)c->ctx.ws.get(Workspace::KMC_LUT, b); };
        msuf.alloc = [&](uint64_t b) { return (uint8_t *)c->ctx.ws.get(Workspace::KMC_REC, b); };
        KmcInput in = kmc_open(kmc_path, min_count, max_count, call_both_from_canonical != 0, stage_threads(c),
                               mirror ? &mpre : nullptr, mirror ? &msuf : nullptr);
        if (!lock.owns_lock()) lock.lock();
        if (in.total) c->kmc.push_back(std::move(in));
        return MTG_OK;
    } catch (const std::exception &e) {
        set_error(e.what());
        return MTG_ERR_ARGUMENT;
    }
}

int mtg_boss_ctor_add_fasta(mtg_boss_ctor *c, const char *path) {
    if (!c || !path) {
        set_error("bad arguments");
        return MTG_ERR_ARGUMENT;
    }
    try {
        StageTimer t{c->stage_ns};
        FastaInput in = load_fasta_file(path);  // read + inflate in the caller's thread
        std::lock_guard<std::mutex> lock(c->fa_mu);
        if (in.size) c->fasta.push_back(in);
        else free_fasta(in);
        return MTG_OK;
    } catch (const std::exception &e) {
        set_error(e.what());
        return MTG_ERR_ARGUMENT;
    }
}

// the staged FASTA / FASTQ files -> reads appended to dseq at *seq_base (fasta.hpp); with
// per-read counts (rstarts != nullptr) also their starts (count 1) from read index *read_base.
// count_only: only sizes (*seq_base / *read_base advance by what the files will write).
static void split_fasta_files(mtg_boss_ctor *c, uint8_t *dseq, uint64_t *seq_base, uint64_t *rstarts,
                              uint32_t *rcounts, uint64_t *read_base, bool count_only) {
    Ctx &x = c->ctx;
    hipStream_t s = x.stream;
    for (const FastaInput &f : c->fasta) {
        const uint64_t n = f.size;
        const uint64_t nt = ceil_div(n, FA_TILE);
        uint8_t *raw = (uint8_t *)x.ws.get(Workspace::FA_RAW, n + 64);
        int64_t *tlast = (int64_t *)x.ws.get(Workspace::FA_TLAST, (nt + 1) * 8);
        int64_t *prev = (int64_t *)x.ws.get(Workspace::FA_PREV, (nt + 1) * 8);
        uint32_t *ta = (uint32_t *)x.ws.get(Workspace::FA_TA, (nt + 1) * 4);
        uint32_t *tb = (uint32_t *)x.ws.get(Workspace::FA_TB, (nt + 1) * 4);
        uint64_t *oa = (uint64_t *)x.ws.get(Workspace::FA_OA, (nt + 1) * 8);
        uint64_t *ob = (uint64_t *)x.ws.get(Workspace::FA_OB, (nt + 1) * 8);
        HIP_CHECK(hipMemcpyAsync(raw, f.data, n, hipMemcpyHostToDevice, s));
        fasta_stats_kernel<<<dim3((unsigned)nt), dim3(FA_BLOCK), 0, s>>>(raw, n, tlast, ta);
        HIP_CHECK(hipGetLastError());
        fasta_prefix_kernel<<<1, 1024, 0, s>>>(tlast, ta, nullptr, nt, prev, oa, nullptr);  // prev nl, lines
        HIP_CHECK(hipGetLastError());
        const uint64_t fh = f.first_header;
        HIP_CHECK(hipMemsetAsync(&x.small->fasta_bad, 0, 4, s));
        fasta_split_kernel<false><<<dim3((unsigned)nt), dim3(FA_BLOCK), 0, s>>>(
            raw, n, f.fastq ? 1 : 0, fh, prev, oa, ta, tb, nullptr, nullptr, nullptr, 0, nullptr, nullptr, 0,
            f.lines_before, &x.small->fasta_bad);
        HIP_CHECK(hipGetLastError());
        uint64_t *koff = (uint64_t *)x.ws.get(Workspace::FA_KOFF, (nt + 1) * 8);
        fasta_prefix_kernel<<<1, 1024, 0, s>>>(nullptr, ta, tb, nt, nullptr, koff, ob);
        HIP_CHECK(hipGetLastError());
        uint64_t tot[2];
        uint32_t bad = 0;
        HIP_CHECK(hipMemcpyAsync(&tot[0], koff + nt, 8, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipMemcpyAsync(&tot[1], ob + nt, 8, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipMemcpyAsync(&bad, &x.small->fasta_bad, 4, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        if (bad)
            throw std::runtime_error("ERROR: " + f.path + ": a FASTA sequence line starts with '+' (FASTQ quality in a "
                                     "FASTA record) -- not supported");
        if (!count_only) {
            // the line-number prefix `oa` is still valid: the second prefix wrote koff / ob
            fasta_split_kernel<true><<<dim3((unsigned)nt), dim3(FA_BLOCK), 0, s>>>(
                raw, n, f.fastq ? 1 : 0, fh, prev, oa, nullptr, nullptr, koff, ob, dseq, *seq_base, rstarts,
                rcounts, *read_base, f.lines_before, nullptr);
            HIP_CHECK(hipGetLastError());
            const uint8_t sep = '$';  // the last record's separator
            HIP_CHECK(hipMemcpyAsync(dseq + *seq_base + tot[0], &sep, 1, hipMemcpyHostToDevice, s));
            HIP_CHECK(hipStreamSynchronize(s));  // the slots are reused by the next file
        }
        *seq_base += tot[0] + 1;
        *read_base += tot[1];
    }
}

// encode_filter_suffix_boss (boss_chunk_construct.cpp:935-945): '$' -> 0, else the BOSS code
// of the char (kmer/alphabets.hpp:68-77: A C G T/U -> 1..4, anything else 5, which never matches)
static mtg::SuffixSpec encode_suffix(const std::string &suffix, bool *all_sentinel) {
    mtg::SuffixSpec spec{};
    spec.n = (uint32_t)suffix.size();
    *all_sentinel = !suffix.empty();
    for (size_t i = 0; i < suffix.size(); ++i) {
        const char ch = suffix[i];
        uint8_t code = 5;
        if (ch == '$') code = 0;
        else if (ch == 'A' || ch == 'a') code = 1;
        else if (ch == 'C' || ch == 'c') code = 2;
        else if (ch == 'G' || ch == 'g') code = 3;
        else if (ch == 'T' || ch == 't' || ch == 'U' || ch == 'u') code = 4;
        spec.c[i] = code;
        if (ch != '$') *all_sentinel = false;
    }
    return spec;
}

static const char *kSuffixDist =
    "the suffix-filtered route builds one chunk per suffix on one GPU; it has no multi-GPU form";

// the build on the device buffers: the suffix route or the full construction
static void dispatch_build(mtg_boss_ctor *c, mtg::Comm *comm, const BuildInput &in_, BuildOutput *out) {
    BuildInput in = in_;
    if (in.read_counts && in.n_reads > 1) {  // bracket the per-read count searches (device_common.hpp)
        const uint64_t nq = (in.seq_len >> mtg::RID_SHIFT) + 2;
        uint64_t *rid = (uint64_t *)c->ctx.ws.get(mtg::Workspace::RID_AT, nq * 8);
        read_index_kernel<<<dim3((unsigned)std::min<uint64_t>(ceil_div(in.n_reads, 256), 65536)), dim3(256), 0,
                            c->ctx.stream>>>(in.read_starts, in.n_reads, nq, rid);
        HIP_CHECK(hipGetLastError());
        in.rid_at = rid;
    }
    if (!c->suffix.empty()) {
        bool all_sentinel = false;
        const mtg::SuffixSpec spec = encode_suffix(c->suffix, &all_sentinel);
        mtg::run_suffix_dispatch(c->ctx, (unsigned)c->params.k, c->params.both_strands != 0,
                                 c->params.bits_per_count, spec, all_sentinel, in, out);
    } else {
        run_dispatch(c->ctx, comm, (unsigned)c->params.k, c->params.both_strands != 0, c->params.bits_per_count,
                     in, out);
    }
    c->ctx.ws.end_build();  // idle kept blocks go back to the device
    c->ctx.timings.cached_bytes = c->ctx.ws.cached();
}

static int run_build(mtg_boss_ctor *c, mtg::Comm *comm, const BuildInput &in, BuildOutput *out) {
    if (comm && !c->suffix.empty()) {
        set_error(kSuffixDist);
        return MTG_ERR_UNSUPPORTED;
    }
    try {
        HIP_CHECK(hipSetDevice(c->device));
        // the build's device work, bracketed for the exchange layer (LocalComm's serial mode)
        struct Scope {
            mtg::Comm *comm;
            hipStream_t s;
            ~Scope() {
                if (comm) comm->end_build(s);
            }
        } scope{comm, c->ctx.stream};
        if (comm) comm->begin_build(c->ctx.stream);
        dispatch_build(c, comm, in, out);
        return MTG_OK;
    } catch (const std::exception &e) {
        set_error(e.what());
        return MTG_ERR_DEVICE;
    }
}

static int build_device_impl(mtg_boss_ctor *c, mtg::Comm *comm, const uint8_t *d_seq, uint64_t seq_len,
                             const uint64_t *d_read_starts, const uint32_t *d_counts, uint64_t n_reads,
                             void *stream, mtg_boss_device_chunk *out) {
    if (!c || !out || (seq_len && !d_seq) || (!d_read_starts != !d_counts)) {
        set_error("bad arguments");
        return MTG_ERR_ARGUMENT;
    }
    std::lock_guard<std::mutex> lock(c->mu);
    hipStream_t saved = c->ctx.stream;
    if (stream) c->ctx.stream = (hipStream_t)stream;
    BuildInput in{d_seq, seq_len, d_read_starts, d_counts, d_counts ? n_reads : 0};
    BuildOutput o{};
    int rc = run_build(c, comm, in, &o);
    c->ctx.stream = saved;
    if (rc != MTG_OK) return rc;
    out->k = c->params.k;
    out->n = o.n;
    out->W = o.W;
    out->last = o.last;
    out->weights = o.weights;
    std::memcpy(out->F, o.F, sizeof(o.F));
    out->n_real = o.n_real;
    out->n_dummy = o.n_dummy;
    return MTG_OK;
}

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// W (values 0..9) crosses PCIe as 4-bit codes: packed on the device, copied in pieces, and
// unpacked by the host threads as the pieces land (half the bytes of the largest D2H)
__global__ void pack_w4_kernel(const uint8_t *__restrict__ w, uint64_t n, uint8_t *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // 16 output bytes each
    const uint64_t b0 = i * 32;
    if (b0 >= n) return;
    uint32_t o[4] = {0, 0, 0, 0};
    if (b0 + 32 <= n) {
        const uint4 a = *(const uint4 *)(w + b0), b = *(const uint4 *)(w + b0 + 16);
        const uint32_t in[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int q = 0; q < 8; ++q) {  // 4 W bytes -> 2 packed bytes
            const uint32_t v = in[q];
            const uint32_t p = (v & 0xF) | ((v >> 4) & 0xF0) | (((v >> 16) & 0xF) << 8) | (((v >> 24) & 0xF) << 12);
            o[q / 2] |= p << (16 * (q & 1));
        }
    } else {
        for (uint64_t j = b0; j < n; ++j) {
            const uint32_t k = (uint32_t)(j - b0);
            o[k / 8] |= (uint32_t)(w[j] & 0xF) << (4 * (k % 8));
        }
    }
    const uint64_t nb = (n + 1) / 2, ob = b0 / 2;
    if (ob + 16 <= nb) {
        *(uint4 *)(out + ob) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
        for (uint64_t j = ob; j < nb; ++j) out[j] = (uint8_t)(o[(j - ob) / 4] >> (8 * ((j - ob) % 4)));
    }
}

__attribute__((target("avx2"))) static void unpack_w4_avx2(const uint8_t *in, uint64_t nbytes, uint8_t *out) {
    uint64_t i = 0;
    const __m256i m = _mm256_set1_epi8(0x0F);
    for (; i + 32 <= nbytes; i += 32) {
        const __m256i v = _mm256_loadu_si256((const __m256i *)(in + i));
        const __m256i lo = _mm256_and_si256(v, m), hi = _mm256_and_si256(_mm256_srli_epi16(v, 4), m);
        const __m256i a = _mm256_unpacklo_epi8(lo, hi), b = _mm256_unpackhi_epi8(lo, hi);
        _mm256_storeu_si256((__m256i *)(out + 2 * i), _mm256_permute2x128_si256(a, b, 0x20));
        _mm256_storeu_si256((__m256i *)(out + 2 * i + 32), _mm256_permute2x128_si256(a, b, 0x31));
    }
    for (; i < nbytes; ++i) {
        out[2 * i] = in[i] & 0xF;
        out[2 * i + 1] = in[i] >> 4;
    }
}

static void unpack_w4(const uint8_t *in, uint64_t nbytes, uint8_t *out) {
    if (__builtin_cpu_supports("avx2")) return unpack_w4_avx2(in, nbytes, out);
    for (uint64_t i = 0; i < nbytes; ++i) {
        out[2 * i] = in[i] & 0xF;
        out[2 * i + 1] = in[i] >> 4;
    }
}

static unsigned stage_threads(const mtg_boss_ctor *c);

// W[0..n) on the device -> host W (out, n bytes): 4-bit pieces of 16 MiB, unpacked as they land
static void copy_w_to_host(mtg_boss_ctor *c, const uint8_t *dW, uint64_t n, uint8_t *out) {
    if (!n) return;
    hipStream_t s = c->ctx.stream;
    if (n < (128ull << 20)) {  // small W: one plain copy (the pieces' sync and thread costs do not pay)
        HIP_CHECK(hipMemcpyAsync(out, dW, n, hipMemcpyDeviceToHost, s));
        return;
    }
    const uint64_t nb = (n + 1) / 2;
    uint8_t *d4 = (uint8_t *)c->ctx.ws.get(Workspace::W4, nb + 16);
    pack_w4_kernel<<<dim3((unsigned)ceil_div(ceil_div(n, 32), 256)), dim3(256), 0, s>>>(dW, n, d4);
    HIP_CHECK(hipGetLastError());
    if (c->w4_cap < nb + 16) {  // the ctor's pinned landing buffer, grown on demand
        if (c->w4_host) (void)hipHostFree(c->w4_host);
        c->w4_host = nullptr;
        c->w4_cap = 0;
        HIP_CHECK(hipHostMalloc((void **)&c->w4_host, nb + nb / 4 + 16, hipHostMallocDefault));
        c->w4_cap = nb + nb / 4 + 16;
    }
    uint8_t *h4 = c->w4_host;
    constexpr uint64_t PIECE = 16ull << 20;  // packed bytes per piece
    const uint64_t np = ceil_div(nb, PIECE);
    std::vector<hipEvent_t> ev(np);
    for (uint64_t p = 0; p < np; ++p) {
        const uint64_t b0 = p * PIECE, len = std::min(PIECE, nb - b0);
        HIP_CHECK(hipEventCreateWithFlags(&ev[p], hipEventDisableTiming));
        HIP_CHECK(hipMemcpyAsync(h4 + b0, d4 + b0, len, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipEventRecord(ev[p], s));
    }
    const unsigned T = std::max(1u, std::min<unsigned>(stage_threads(c), (unsigned)np));
    std::atomic<bool> failed{false};
    parallel_ranges(T, T, 1, [&](uint64_t t0, uint64_t t1) {
        DeviceGuard g(c->device);
        for (uint64_t t = t0; t < t1; ++t)
            for (uint64_t p = t; p < np; p += T) {
                if (hipEventSynchronize(ev[p]) != hipSuccess) {
                    failed = true;
                    return;
                }
                const uint64_t b0 = p * PIECE, len = std::min(PIECE, nb - b0);
                // the last packed byte of an odd n holds one W value
                const uint64_t full = (b0 + len == nb && (n & 1)) ? len - 1 : len;
                unpack_w4(h4 + b0, full, out + 2 * b0);
                if (full < len) out[2 * (b0 + full)] = h4[b0 + full] & 0xF;
            }
    });
    for (auto e : ev) (void)hipEventDestroy(e);
    if (failed) throw std::runtime_error("W copy to the host failed");
}

// u32 weights (already clamped to the count width) -> `bytes` (1 or 2) per weight, 16 weights a thread
__global__ void narrow_weights_kernel(const uint32_t *__restrict__ w, uint64_t n, unsigned bytes,
                                      uint8_t *__restrict__ out) {
    const uint64_t i0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16;
    if (i0 >= n) return;
    if (i0 + 16 <= n) {
        const uint4 *src = (const uint4 *)(w + i0);
        uint32_t v[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 a = src[q];
            v[4 * q] = a.x, v[4 * q + 1] = a.y, v[4 * q + 2] = a.z, v[4 * q + 3] = a.w;
        }
        if (bytes == 1) {
            uint32_t o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                o[q] = (v[4 * q] & 0xFF) | (v[4 * q + 1] & 0xFF) << 8 | (v[4 * q + 2] & 0xFF) << 16 | v[4 * q + 3] << 24;
            *(uint4 *)(out + i0) = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
            uint32_t o[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) o[q] = (v[2 * q] & 0xFFFF) | v[2 * q + 1] << 16;
            *(uint4 *)(out + 2 * i0) = make_uint4(o[0], o[1], o[2], o[3]);
            *(uint4 *)(out + 2 * i0 + 16) = make_uint4(o[4], o[5], o[6], o[7]);
        }
        return;
    }
    for (uint64_t i = i0; i < n; ++i) {
        out[bytes * i] = (uint8_t)w[i];
        if (bytes == 2) out[2 * i + 1] = (uint8_t)(w[i] >> 8);
    }
}

// weights[0..n) (u32) on the device -> the host's u32 array: for count widths <= 16 bits they cross
// PCIe as 1 or 2 bytes a weight (configs[4]'s 8-bit weights: 1.5 GB -> 0.39 GB), in 16 MiB pieces
// that the host threads widen as they land
static void copy_weights_to_host(mtg_boss_ctor *c, const uint32_t *dwt, uint64_t n, unsigned bits, uint32_t *out) {
    if (!n) return;
    hipStream_t s = c->ctx.stream;
    const unsigned bytes = bits <= 8 ? 1 : bits <= 16 ? 2 : 4;
    if (bytes == 4 || n < (16ull << 20)) {
        HIP_CHECK(hipMemcpyAsync(out, dwt, n * 4, hipMemcpyDeviceToHost, s));
        return;
    }
    const uint64_t nb = n * bytes;
    uint8_t *dn = (uint8_t *)c->ctx.ws.get(Workspace::WN, nb + 64);
    narrow_weights_kernel<<<dim3((unsigned)ceil_div(ceil_div(n, 16), 256)), dim3(256), 0, s>>>(dwt, n, bytes, dn);
    HIP_CHECK(hipGetLastError());
    if (c->wn_cap < nb + 64) {  // the ctor's pinned landing buffer, grown on demand
        if (c->wn_host) (void)hipHostFree(c->wn_host);
        c->wn_host = nullptr;
        c->wn_cap = 0;
        HIP_CHECK(hipHostMalloc((void **)&c->wn_host, nb + nb / 4 + 64, hipHostMallocDefault));
        c->wn_cap = nb + nb / 4 + 64;
    }
    uint8_t *hn = c->wn_host;
    constexpr uint64_t PIECE = 16ull << 20;  // narrowed bytes per piece (a multiple of 2)
    const uint64_t np = ceil_div(nb, PIECE);
    std::vector<hipEvent_t> ev(np);
    for (uint64_t p = 0; p < np; ++p) {
        const uint64_t b0 = p * PIECE, len = std::min(PIECE, nb - b0);
        HIP_CHECK(hipEventCreateWithFlags(&ev[p], hipEventDisableTiming));
        HIP_CHECK(hipMemcpyAsync(hn + b0, dn + b0, len, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipEventRecord(ev[p], s));
    }
    const unsigned T = std::max(1u, std::min<unsigned>(stage_threads(c), (unsigned)np));
    std::atomic<bool> failed{false};
    parallel_ranges(T, T, 1, [&](uint64_t t0, uint64_t t1) {
        DeviceGuard g(c->device);
        for (uint64_t t = t0; t < t1; ++t)
            for (uint64_t p = t; p < np; p += T) {
                if (hipEventSynchronize(ev[p]) != hipSuccess) {
                    failed = true;
                    return;
                }
                const uint64_t b0 = p * PIECE, len = std::min(PIECE, nb - b0);
                const uint64_t w0 = b0 / bytes, wn = len / bytes;
                if (bytes == 1)
                    for (uint64_t i = 0; i < wn; ++i) out[w0 + i] = hn[b0 + i];
                else
                    for (uint64_t i = 0; i < wn; ++i) out[w0 + i] = (uint32_t)hn[b0 + 2 * i] | (uint32_t)hn[b0 + 2 * i + 1] << 8;
            }
    });
    for (auto e : ev) (void)hipEventDestroy(e);
    if (failed) throw std::runtime_error("weights copy to the host failed");
}

// build_chunk on the staged reads: one H2D copy of the pinned read buffer (+ KMC records), the
// device path, then W / packed last / weights D2H into pinned blocks the chunk owns
static int build_chunk_impl(mtg_boss_ctor *c, mtg::Comm *comm, mtg_boss_chunk *out) {
    if (!c || !out) {
        set_error("bad arguments");
        return MTG_ERR_ARGUMENT;
    }
    if (comm && !c->suffix.empty()) {
        set_error(kSuffixDist);
        return MTG_ERR_UNSUPPORTED;
    }
    const auto t_start = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> lock(c->mu);
    std::unique_lock<std::shared_mutex> stage_lock(c->stage.lock());  // no add runs during the build
    std::lock_guard<std::mutex> kmc_lock(c->kmc_mu);
    std::lock_guard<std::mutex> fa_lock(c->fa_mu);
    std::memset(out, 0, sizeof(*out));
    try {
        HIP_CHECK(hipSetDevice(c->device));
        hipStream_t s = c->ctx.stream;
        HostStage &st = c->stage;
        const uint64_t len = st.size();
        const uint64_t nr = st.n_reads();
        uint64_t kmc_bytes = 0, kmc_reads = 0;
        for (const auto &m : c->kmc) {
            kmc_bytes += m.total * (m.k + 1) * (m.both ? 2 : 1);
            kmc_reads += m.total * (m.both ? 2 : 1);
        }
        uint64_t fa_bytes = 0, fa_reads = 0;
        for (const auto &f : c->fasta) fa_bytes += f.size + 1;  // split output <= raw bytes + a separator
        const bool per_read_inputs = st.any_count_not_one() || kmc_reads;
        if (c->params.bits_per_count && per_read_inputs && !c->fasta.empty()) {
            uint64_t sb = 0;  // record counts first: the read-start arrays are sized by them
            split_fasta_files(c, nullptr, &sb, nullptr, nullptr, &fa_reads, true);
        }
        const uint64_t total_len = len + kmc_bytes + fa_bytes, total_reads = nr + kmc_reads + fa_reads;
        const auto t_h2d = std::chrono::steady_clock::now();
        uint8_t *dseq = (uint8_t *)c->ctx.ws.get(Workspace::SEQ, total_len + 1);
        if (len) {
            // the staged 2-bit codes + valid mask: on the device already (the stage's mirror, copied
            // while the reads were staged), else copied now; unpacked to one byte per char
            const uint64_t nw = len / 32;
            const uint64_t *dcodes = nullptr;
            const uint32_t *dvalid = nullptr;
            if (!st.mirror_wait(&dcodes, &dvalid)) {
                uint64_t *pk = (uint64_t *)c->ctx.ws.get(Workspace::PACKED, nw * 12);
                HIP_CHECK(hipMemcpyAsync(pk, st.codes(), nw * 8, hipMemcpyHostToDevice, s));
                HIP_CHECK(hipMemcpyAsync(pk + nw, st.valid(), nw * 4, hipMemcpyHostToDevice, s));
                dcodes = pk;
                dvalid = (const uint32_t *)(pk + nw);
            }
            unpack_reads_kernel<<<dim3((unsigned)ceil_div(nw, 256)), dim3(256), 0, s>>>(dcodes, dvalid, nw, dseq);
            HIP_CHECK(hipGetLastError());
        }
        uint64_t *dstarts = nullptr;
        uint32_t *dcounts = nullptr;
        const bool per_read = c->params.bits_per_count && per_read_inputs && total_reads;
        if (per_read) {
            dstarts = (uint64_t *)c->ctx.ws.get(Workspace::STARTS, total_reads * 8);
            dcounts = (uint32_t *)c->ctx.ws.get(Workspace::RCOUNTS, total_reads * 4);
            if (nr) {
                HIP_CHECK(hipMemcpyAsync(dstarts, st.starts().data(), nr * 8, hipMemcpyHostToDevice, s));
                HIP_CHECK(hipMemcpyAsync(dcounts, st.counts().data(), nr * 4, hipMemcpyHostToDevice, s));
            }
        }
        HIP_CHECK(hipStreamSynchronize(s));
        const double h2d_ms = ms_since(t_h2d);
        // KMC records -> reads, on the device (kmc.hpp)
        const auto t_input = std::chrono::steady_clock::now();
        uint64_t seq_base = len, read_base = nr;
        for (const auto &m : c->kmc) {
            const uint64_t *dlut;
            const uint8_t *drec;
            if (m.dpre) {  // copied while add_kmc read the files (same stream)
                dlut = (const uint64_t *)(m.dpre + 8);
                drec = m.dsuf + 8;
            } else {
                uint64_t *l = (uint64_t *)c->ctx.ws.get(Workspace::KMC_LUT, m.nlut * 8);
                uint8_t *r = (uint8_t *)c->ctx.ws.get(Workspace::KMC_REC, m.record_bytes() + 1);
                HIP_CHECK(hipMemcpyAsync(l, m.lut_bytes(), m.nlut * 8, hipMemcpyHostToDevice, s));
                HIP_CHECK(hipMemcpyAsync(r, m.records(), m.record_bytes(), hipMemcpyHostToDevice, s));
                dlut = l;
                drec = r;
            }
            kmc_decode_kernel<<<dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(m.total, 256), 65536))),
                                dim3(256), 0, s>>>(drec, dlut, m.nlut, m.total, m.k, m.lut_len,
                                                   m.counter_size, m.min_count, m.max_count, m.both ? 1 : 0,
                                                   dseq, seq_base, dstarts, dcounts, read_base);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipStreamSynchronize(s));  // the slots are reused by the next database
            seq_base += m.total * (m.k + 1) * (m.both ? 2 : 1);
            read_base += m.total * (m.both ? 2 : 1);
        }
        split_fasta_files(c, dseq, &seq_base, per_read ? dstarts : nullptr, per_read ? dcounts : nullptr, &read_base,
                          false);
        HIP_CHECK(hipStreamSynchronize(s));
        const double input_ms = ms_since(t_input);
        BuildInput in{dseq, seq_base, dstarts, dcounts, per_read ? total_reads : 0};
        BuildOutput o{};
        c->ctx.host_output = comm == nullptr;  // a single build with host arrays may spill
        dispatch_build(c, comm, in, &o);
        c->ctx.host_output = false;
        const auto t_d2h = std::chrono::steady_clock::now();
        if (o.host) {  // the spilled build: its rows are already on the host
            PinnedPool &pool = PinnedPool::get();
            const uint64_t nwords = ceil_div(o.n, 64);
            out->k = c->params.k;
            out->alph_size = 5;
            out->n = o.n;
            out->bits_per_count = c->params.bits_per_count;
            out->n_real = o.n_real;
            out->n_dummy = o.n_dummy;
            std::memcpy(out->F, o.F, sizeof(o.F));
            out->W = (uint8_t *)pool.take(std::max<uint64_t>(o.n, 1));
            std::memcpy(out->W, o.W, o.n);
            out->last = (uint64_t *)pool.take(std::max<uint64_t>(nwords, 1) * 8);
            std::memset(out->last, 0, std::max<uint64_t>(nwords, 1) * 8);
            for (uint64_t i = 0; i < o.n; ++i) out->last[i >> 6] |= (uint64_t)(o.last[i] & 1) << (i & 63);
            if (o.weights) {
                out->weights = (uint32_t *)pool.take(std::max<uint64_t>(o.n, 1) * 4);
                std::memcpy(out->weights, o.weights, o.n * 4);
            }
            c->ctx.spill_W = std::vector<uint8_t>();
            c->ctx.spill_last = std::vector<uint8_t>();
            c->ctx.spill_weights = std::vector<uint32_t>();
            mtg_boss_timings &T = c->ctx.timings;
            T.d2h_ms = ms_since(t_d2h);
            T.h2d_ms = h2d_ms;
            T.input_ms = input_ms;
            T.stage_ms = (double)c->stage_ns.exchange(0) * 1e-6;
            c->stage.clear_locked();
            stage_lock.unlock();
            c->kmc.clear();
            for (auto &f : c->fasta) free_fasta(f);
            c->fasta.clear();
            T.host_total_ms = ms_since(t_start);
            return MTG_OK;
        }
        const uint64_t nwords = ceil_div(o.n, 64);
        uint64_t *dbits = (uint64_t *)c->ctx.ws.get(Workspace::LAST_BITS, std::max<uint64_t>(nwords, 1) * 8);
        if (nwords) {
            pack_bits_kernel<<<dim3((unsigned)ceil_div(nwords, 256)), dim3(256), 0, s>>>(o.last, o.n, dbits);
            HIP_CHECK(hipGetLastError());
        }
        out->k = c->params.k;
        out->alph_size = 5;
        out->n = o.n;
        out->bits_per_count = c->params.bits_per_count;
        out->n_real = o.n_real;
        out->n_dummy = o.n_dummy;
        std::memcpy(out->F, o.F, sizeof(o.F));
        PinnedPool &pool = PinnedPool::get();
        out->W = (uint8_t *)pool.take(o.n);
        out->last = (uint64_t *)pool.take(std::max<uint64_t>(nwords, 1) * 8);
        HIP_CHECK(hipMemcpyAsync(out->last, dbits, nwords * 8, hipMemcpyDeviceToHost, s));
        copy_w_to_host(c, o.W, o.n, out->W);
        if (o.weights) {
            out->weights = (uint32_t *)pool.take(o.n * 4);
            copy_weights_to_host(c, o.weights, o.n, c->params.bits_per_count, out->weights);
        }
        HIP_CHECK(hipStreamSynchronize(s));
        mtg_boss_timings &T = c->ctx.timings;
        T.d2h_ms = ms_since(t_d2h);
        T.h2d_ms = h2d_ms;
        T.input_ms = input_ms;
        T.stage_ms = (double)c->stage_ns.exchange(0) * 1e-6;
        c->stage.clear_locked();  // under the build's exclusive lock: a waiting add lands in the next batch
        stage_lock.unlock();
        c->kmc.clear();
        for (auto &f : c->fasta) free_fasta(f);
        c->fasta.clear();
        T.host_total_ms = ms_since(t_start);
        return MTG_OK;
    } catch (const std::exception &e) {
        set_error(e.what());
        mtg_boss_chunk_free(out);
        return MTG_ERR_DEVICE;
    }
}

int mtg_kmc_write_device(mtg_boss_ctor *c, const uint8_t *d_seq, uint64_t seq_len, unsigned k, int canonical,
                         unsigned counter_size, unsigned lut_len, const char *outbase, uint64_t *n_written) {
    if (!c || !outbase || (seq_len && !d_seq)) {
        set_error("bad arguments");
        return MTG_ERR_ARGUMENT;
    }
    std::lock_guard<std::mutex> lock(c->mu);
    try {
        HIP_CHECK(hipSetDevice(c->device));
        BuildInput in{d_seq, seq_len, nullptr, nullptr, 0};
        const uint64_t n = mtg::kmc_count_write(c->ctx, in, k, canonical != 0, counter_size, lut_len, outbase,
                                                stage_threads(c));
        if (n_written) *n_written = n;
        return MTG_OK;
    } catch (const std::exception &e) {
        set_error(e.what());
        return MTG_ERR_DEVICE;
    }
}

int mtg_kmc_load_device(const char *kmc_path, uint64_t min_count, uint64_t max_count, int call_both_from_canonical,
                        int device_id, mtg_device_reads *out) {
    if (!kmc_path || !out) {
        set_error("bad arguments");
        return MTG_ERR_ARGUMENT;
    }
    std::memset(out, 0, sizeof(*out));
    out->device_id = device_id;
    uint64_t *dlut = nullptr;
    uint8_t *drec = nullptr;
    try {
        KmcInput m = kmc_open(kmc_path, min_count, max_count, call_both_from_canonical != 0);
        HIP_CHECK(hipSetDevice(device_id));
        const uint64_t per = m.both ? 2 : 1;
        out->seq_len = m.total * (m.k + 1) * per;
        out->n_reads = m.total * per;
        HIP_CHECK(hipMalloc(&out->seq, out->seq_len + 1));
        HIP_CHECK(hipMalloc(&out->read_starts, std::max<uint64_t>(out->n_reads, 1) * 8));
        HIP_CHECK(hipMalloc(&out->counts, std::max<uint64_t>(out->n_reads, 1) * 4));
        if (m.total) {
            HIP_CHECK(hipMalloc(&dlut, m.nlut * 8));
            HIP_CHECK(hipMalloc(&drec, m.record_bytes() + 1));
            HIP_CHECK(hipMemcpy(dlut, m.lut_bytes(), m.nlut * 8, hipMemcpyHostToDevice));
            HIP_CHECK(hipMemcpy(drec, m.records(), m.record_bytes(), hipMemcpyHostToDevice));
            kmc_decode_kernel<<<dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(m.total, 256), 65536))),
                                dim3(256)>>>(drec, dlut, m.nlut, m.total, m.k, m.lut_len, m.counter_size,
                                             m.min_count, m.max_count, m.both ? 1 : 0, out->seq, 0, out->read_starts,
                                             out->counts, 0);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipDeviceSynchronize());
            (void)hipFree(dlut);
            (void)hipFree(drec);
        }
        return MTG_OK;
    } catch (const std::exception &e) {
        set_error(e.what());
        if (dlut) (void)hipFree(dlut);
        if (drec) (void)hipFree(drec);
        mtg_device_reads_free(out);
        return MTG_ERR_DEVICE;
    }
}

void mtg_device_reads_free(mtg_device_reads *r) {
    if (!r) return;
    (void)hipSetDevice(r->device_id);
    if (r->seq) (void)hipFree(r->seq);
    if (r->read_starts) (void)hipFree(r->read_starts);
    if (r->counts) (void)hipFree(r->counts);
    r->seq = nullptr;
    r->read_starts = nullptr;
    r->counts = nullptr;
    r->seq_len = r->n_reads = 0;
}

int mtg_boss_build_device(mtg_boss_ctor *c, const uint8_t *d_seq, uint64_t seq_len,
                          const uint64_t *d_read_starts, const uint32_t *d_counts,
                          uint64_t n_reads, void *stream, mtg_boss_device_chunk *out) {
    return build_device_impl(c, nullptr, d_seq, seq_len, d_read_starts, d_counts, n_reads, stream, out);
}

int mtg_boss_ctor_build_chunk(mtg_boss_ctor *c, mtg_boss_chunk *out) { return build_chunk_impl(c, nullptr, out); }

// ---- multi-GPU build

struct mtg_comm {
    std::unique_ptr<mtg::Comm> comm;
};

int mtg_comm_get_unique_id(uint8_t *id) {
    if (!id) return MTG_ERR_ARGUMENT;
    try {
        ncclUniqueId u;
        RCCL_CHECK(RcclApi::get().GetUniqueId(&u));
        std::memcpy(id, u.internal, MTG_COMM_ID_BYTES);
        return MTG_OK;
    } catch (const std::exception &e) {
        set_error(e.what());
        return MTG_ERR_DEVICE;
    }
}

mtg_comm *mtg_comm_create_rccl(const uint8_t *id, int world, int rank, int device_id) {
    if (!id || world < 1 || rank < 0 || rank >= world || world > mtg::MAX_RANKS) {
        set_error("bad arguments");
        return nullptr;
    }
    try {
        ncclUniqueId u;
        std::memcpy(u.internal, id, MTG_COMM_ID_BYTES);
        auto *c = new mtg_comm();
        c->comm.reset(new mtg::RcclComm(u, world, rank, device_id));
        return c;
    } catch (const std::exception &e) {
        set_error(e.what());
        return nullptr;
    }
}

int mtg_comm_create_local(int world, mtg_comm **comms) {
    if (world < 1 || world > mtg::MAX_RANKS || !comms) {
        set_error("bad arguments");
        return MTG_ERR_ARGUMENT;
    }
    auto group = std::make_shared<mtg::LocalGroup>(world);
    const char *ser = getenv("MTG_LOCAL_SERIAL");
    group->serial = ser && ser[0] == '1';
    for (int r = 0; r < world; ++r) {
        comms[r] = new mtg_comm();
        comms[r]->comm.reset(new mtg::LocalComm(group, r));
    }
    return MTG_OK;
}

mtg_comm *mtg_comm_create_callbacks(const mtg_comm_callbacks *cb) {
    if (!cb || cb->world < 1 || cb->rank < 0 || cb->rank >= cb->world || cb->world > mtg::MAX_RANKS ||
        !cb->allreduce_sum_u64 || !cb->allgather_u64 || !cb->alltoallv) {
        set_error("bad arguments");
        return nullptr;
    }
    mtg::CommCallbacks f;
    f.user = cb->user;
    f.allreduce_sum_u64 = cb->allreduce_sum_u64;
    f.allgather_u64 = cb->allgather_u64;
    f.alltoallv = cb->alltoallv;
    auto *c = new mtg_comm();
    c->comm.reset(new mtg::CallbackComm(f, cb->rank, cb->world));
    return c;
}

void mtg_comm_destroy(mtg_comm *comm) { delete comm; }

double mtg_comm_local_held_ms(mtg_comm *comm, int reset) {
    auto *lc = comm ? dynamic_cast<mtg::LocalComm *>(comm->comm.get()) : nullptr;
    return lc ? lc->held_ms(reset != 0) : -1.0;
}

int mtg_comm_rank(const mtg_comm *comm) { return comm ? comm->comm->rank() : -1; }

int mtg_comm_size(const mtg_comm *comm) { return comm ? comm->comm->size() : -1; }

int mtg_boss_build_device_dist(mtg_boss_ctor *c, mtg_comm *comm, const uint8_t *d_seq, uint64_t seq_len,
                               const uint64_t *d_read_starts, const uint32_t *d_counts, uint64_t n_reads,
                               void *stream, mtg_boss_device_chunk *out) {
    if (!comm) {
        set_error("bad arguments");
        return MTG_ERR_ARGUMENT;
    }
    return build_device_impl(c, comm->comm.get(), d_seq, seq_len, d_read_starts, d_counts, n_reads, stream,
                             out);
}

int mtg_boss_ctor_build_chunk_dist(mtg_boss_ctor *c, mtg_comm *comm, mtg_boss_chunk *out) {
    if (!comm) {
        set_error("bad arguments");
        return MTG_ERR_ARGUMENT;
    }
    return build_chunk_impl(c, comm->comm.get(), out);
}

uint64_t mtg_device_identity(const char *host, const char *pci_bus_id) {
    return device_identity(host ? host : "", pci_bus_id ? pci_bus_id : "");
}

uint32_t mtg_dist_coresident(const uint64_t *ids, int world, int rank) {
    if (!ids || world < 1 || rank < 0 || rank >= world) return 0;
    return coresident_count(ids, world, ids[rank]);
}

int mtg_dist_bounds(const uint64_t *hist, uint64_t n_prefixes, int world, uint64_t *bounds) {
    if (!hist || !bounds || world < 1) return MTG_ERR_ARGUMENT;
    const std::vector<uint64_t> b = balanced_bounds(hist, n_prefixes, world);
    std::memcpy(bounds, b.data(), b.size() * 8);
    return MTG_OK;
}

void mtg_boss_chunk_free(mtg_boss_chunk *chunk) {
    if (!chunk) return;
    PinnedPool &pool = PinnedPool::get();
    for (void *p : {(void *)chunk->W, (void *)chunk->last, (void *)chunk->weights})
        if (!pool.give(p)) std::free(p);
    chunk->W = nullptr;
    chunk->last = nullptr;
    chunk->weights = nullptr;
    chunk->n = 0;
}

int mtg_boss_write_dbg(const mtg_boss_chunk *chunk, const char *outbase, int graph_mode, int mask_dummy,
                       int64_t suffix_length, uint64_t *n_valid) {
    if (!chunk || !outbase || !chunk->W || !chunk->last || chunk->n < 1 || graph_mode < 0 || graph_mode > 1) {
        set_error("write_dbg: bad arguments");
        return MTG_ERR_ARGUMENT;
    }
    try {
        const uint64_t v = dbgio::write_dbg(outbase, chunk->W, chunk->last, chunk->n, chunk->F, chunk->k,
                                            (uint64_t)graph_mode, mask_dummy, suffix_length, chunk->weights,
                                            chunk->bits_per_count);
        if (n_valid) *n_valid = v;
        return MTG_OK;
    } catch (const std::exception &e) {
        set_error(e.what());
        return MTG_ERR_ARGUMENT;
    }
}

int mtg_sdsl_write(const char *path, int kind, const void *data, uint64_t nbits) {
    if (!path || (!data && nbits) || kind < 0 || kind > 4) {
        set_error("sdsl_write: bad arguments");
        return MTG_ERR_ARGUMENT;
    }
    try {
        std::ofstream o(path, std::ios::binary);
        if (!o.good()) throw std::runtime_error(std::string("Can't write to file ") + path);
        const uint64_t *w = (const uint64_t *)data;
        std::vector<uint64_t> zero(1, 0);
        if (!nbits) w = zero.data();
        if (kind == 0) sdslio::put_bit_vector_stat(o, w, nbits);
        else if (kind == 1) sdslio::put_bit_vector_small(o, w, nbits);
        else if (kind == 2) sdslio::put_wt_huff(o, (const uint8_t *)data, nbits);
        else if (kind == 3) {
            std::vector<uint64_t> pos;
            for (uint64_t i = 0; i < nbits; ++i)
                if (sdslio::bit(w, i)) pos.push_back(i);
            sdslio::put_sd_vector(o, pos, nbits);
        } else {
            sdslio::put_rrr_vector(o, w, nbits);
        }
        if (!o.good()) throw std::runtime_error(std::string("Can't write to file ") + path);
        return MTG_OK;
    } catch (const std::exception &e) {
        set_error(e.what());
        return MTG_ERR_ARGUMENT;
    }
}

int mtg_boss_read_dbg(const char *outbase, mtg_dbg_file *out) {
    if (!outbase || !out) return MTG_ERR_ARGUMENT;
    std::memset(out, 0, sizeof(*out));
    try {
        dbgio::DbgFile f = dbgio::read_dbg(outbase);
        out->k = f.k;
        out->n = f.n;
        for (int c = 0; c < 5; ++c) out->F[c] = f.F[c];
        out->state = f.state;
        out->mode = f.mode;
        out->suffix_length = f.suffix_length;
        out->n_ranges = f.ranges.size();
        out->W = (uint8_t *)std::malloc(std::max<size_t>(f.W.size(), 1));
        std::memcpy(out->W, f.W.data(), f.W.size());
        out->last = (uint64_t *)std::malloc(std::max<size_t>(f.last.size() * 8, 8));
        std::memcpy(out->last, f.last.data(), f.last.size() * 8);
        out->ranges = (uint64_t *)std::malloc(std::max<size_t>(f.ranges.size() * 16, 16));
        for (size_t i = 0; i < f.ranges.size(); ++i) {
            out->ranges[2 * i] = f.ranges[i].first;
            out->ranges[2 * i + 1] = f.ranges[i].second;
        }
        if (f.has_mask) {
            out->valid = (uint64_t *)std::malloc(std::max<size_t>(f.valid.size() * 8, 8));
            std::memcpy(out->valid, f.valid.data(), f.valid.size() * 8);
            for (uint64_t x : f.valid) out->n_valid += __builtin_popcountll(x);
        }
        return MTG_OK;
    } catch (const std::exception &e) {
        set_error(e.what());
        mtg_dbg_file_free(out);
        return MTG_ERR_ARGUMENT;
    }
}

void mtg_dbg_file_free(mtg_dbg_file *f) {
    if (!f) return;
    std::free(f->W);
    std::free(f->last);
    std::free(f->ranges);
    std::free(f->valid);
    f->W = nullptr;
    f->last = nullptr;
    f->ranges = nullptr;
    f->valid = nullptr;
}

uint64_t mtg_host_pool_bytes(void) { return PinnedPool::get().spare_bytes(); }

void mtg_host_pool_trim(void) { PinnedPool::get().trim(); }

void mtg_dna_encode_table(uint8_t *out) {
    for (uint32_t c = 0; c < 256; ++c) out[c] = (uint8_t)encode_dna(c);
}

int mtg_boss_last_timings(const mtg_boss_ctor *c, mtg_boss_timings *out) {
    if (!c || !out) return MTG_ERR_ARGUMENT;
    *out = c->ctx.timings;
    return MTG_OK;
}

void *mtg_device_alloc(int device_id, uint64_t bytes) {
    void *p = nullptr;
    if (hipSetDevice(device_id) != hipSuccess) return nullptr;
    if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) {
        set_error("hipMalloc failed");
        return nullptr;
    }
    return p;
}

int mtg_device_free(void *ptr) { return hipFree(ptr) == hipSuccess ? MTG_OK : MTG_ERR_DEVICE; }

int mtg_memcpy_h2d(void *dst, const void *src, uint64_t bytes) {
    return hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess ? MTG_OK : MTG_ERR_DEVICE;
}

int mtg_memcpy_d2h(void *dst, const void *src, uint64_t bytes) {
    return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) == hipSuccess ? MTG_OK : MTG_ERR_DEVICE;
}

// The bench's achievable-bandwidth copy: one 16-byte nontemporal vector load and store per thread
// (global_load_dwordx4 / global_store_dwordx4 nt), a workgroup per 4 KiB.  tools/copy_bench.hip on
// MI355X, 4 GiB (profiles/r6_copy_bench.txt): 6.44 TB/s -- above the guide's 6.29 float4 copy -- against
// 6.21 for plain 16-byte accesses, 5.85 for round 5's 4 x (2 x 8-byte nt) per thread (the kernel this
// replaces: its 8-byte nt halves), 4.6-4.95 for grid-stride loops, 4.96 for hipMemcpyAsync D2D.
typedef unsigned int mtg_u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void copy16_kernel(const mtg_u32x4 *__restrict__ src, mtg_u32x4 *__restrict__ dst,
                                                     uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

int mtg_device_copy(void *dst, const void *src, uint64_t bytes, void *stream) {
    if (!dst || !src || (bytes & 15) || ((uintptr_t)dst & 15) || ((uintptr_t)src & 15)) return MTG_ERR_ARGUMENT;
    const uint64_t n = bytes / 16;
    if (!n) return MTG_OK;
    if (ceil_div(n, 256) > 0x7fffffffull) return MTG_ERR_ARGUMENT;
    const unsigned grid = (unsigned)ceil_div(n, 256);
    copy16_kernel<<<dim3(grid), dim3(256), 0, (hipStream_t)stream>>>((const mtg_u32x4 *)src, (mtg_u32x4 *)dst, n);
    return hipGetLastError() == hipSuccess ? MTG_OK : MTG_ERR_DEVICE;
}

int mtg_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int mtg_device_synchronize(int device_id) {
    if (hipSetDevice(device_id) != hipSuccess) return MTG_ERR_DEVICE;
    return hipDeviceSynchronize() == hipSuccess ? MTG_OK : MTG_ERR_DEVICE;
}

}  // extern "C"
