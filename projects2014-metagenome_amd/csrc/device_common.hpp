// device_common.hpp -- wave64 / workgroup primitives and the decoupled look-back protocol
// shared by the sort, scan and compaction kernels.
//
// Inter-workgroup hand-off: every tile publishes 64-bit granules
//     {epoch:16 | status:2 | value:46}
// with one agent-scope relaxed atomic store; readers poll them with agent-scope relaxed atomic
// loads.  The data IS the flag (8-byte granule, R2 of the CDNA4 guide), so no fences are needed.
// The epoch is the launch's id: a granule from an older launch reads as "not ready", so the
// descriptor array needs zeroing only when it is (re)allocated or the 16-bit epoch wraps.
//
// Why windows: on MI355X a tile's predecessors run on other XCDs, so every poll is a fabric
// round trip (~0.5-2 us).  Walking back one tile per round trip serialises the chain; both
// look-backs below inspect many predecessors per round trip (64 lanes of a wave for a single
// column, LB_WINDOW loads in flight per lane for the per-digit columns of the radix sort).
// Spins are bounded: a timeout sets an error word the host checks.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mtg {

constexpr int kWave = 64;

constexpr int kEpochShift = 48;
constexpr int kStatusShift = 46;
constexpr uint64_t kValueMask = (1ull << kStatusShift) - 1;
constexpr uint64_t kAgg = 1;
constexpr uint64_t kIncl = 2;
constexpr uint32_t kSpinLimit = 1u << 22;
constexpr int LB_WINDOW = 4;

__device__ __forceinline__ uint64_t granule(uint32_t epoch, uint64_t status, uint64_t value) {
    return ((uint64_t)epoch << kEpochShift) | (status << kStatusShift) | value;
}

// status of a granule for this launch: 0 = not ready (or stale epoch), 1 = aggregate,
// 2 = inclusive prefix
__device__ __forceinline__ uint32_t granule_status(uint64_t v, uint32_t epoch) {
    return (uint32_t)(v >> kEpochShift) == epoch ? (uint32_t)((v >> kStatusShift) & 3) : 0u;
}

__device__ __forceinline__ void publish(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t poll(const uint64_t *p) {
    return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

/*
 * Single-column look-back by ONE whole wave: returns the exclusive prefix of `agg` over all
 * tiles < tile (same value in every lane) and publishes this tile's inclusive prefix.
 * Lane i inspects tile (base - i), so each round trip covers 64 predecessors.
 */
__device__ __forceinline__ uint64_t wave_lookback(uint64_t *desc, uint32_t tile, uint64_t agg,
                                                  uint32_t epoch, uint32_t *error) {
    const uint32_t lane = __lane_id();
    if (tile == 0) {
        if (lane == 0) publish(desc, granule(epoch, kIncl, agg));
        return 0;
    }
    if (lane == 0) publish(desc + tile, granule(epoch, kAgg, agg));
    uint64_t excl = 0;
    int64_t base = (int64_t)tile - 1;
    uint32_t spins = 0;
    while (true) {
        const int64_t t = base - (int64_t)lane;
        const uint64_t v = t >= 0 ? poll(desc + t) : granule(epoch, kIncl, 0);
        const uint32_t st = granule_status(v, epoch);
        const uint64_t incl = __ballot(st == 2);
        const uint64_t notready = __ballot(st == 0);
        const uint32_t first = incl ? (uint32_t)(__ffsll((unsigned long long)incl) - 1) : 64u;
        const uint64_t upto = first < 63 ? ((2ull << first) - 1) : ~0ull;
        if (notready & upto) {
            if (++spins > kSpinLimit) {
                if (lane == 0) atomicOr(error, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        excl += wave_sum_u64(lane <= first ? (v & kValueMask) : 0);
        if (first < 64) break;
        base -= 64;
    }
    if (lane == 0) publish(desc + tile, granule(epoch, kIncl, excl + agg));
    return excl;
}

/*
 * Per-column look-back (one lane per column, e.g. per radix digit): desc[tile * stride].
 * Each lane keeps LB_WINDOW predecessor loads in flight per round trip.
 */
__device__ __forceinline__ uint64_t column_lookback(uint64_t *desc, uint32_t tile, uint32_t stride,
                                                    uint64_t agg, uint32_t epoch,
                                                    uint32_t *error) {
    if (tile == 0) {
        publish(desc, granule(epoch, kIncl, agg));
        return 0;
    }
    publish(desc + (size_t)tile * stride, granule(epoch, kAgg, agg));
    uint64_t excl = 0;
    int64_t t = (int64_t)tile - 1;
    uint32_t spins = 0;
    bool done = false;
    while (!done) {
        uint64_t v[LB_WINDOW];
#pragma unroll
        for (int i = 0; i < LB_WINDOW; ++i)
            v[i] = t - i >= 0 ? poll(desc + (size_t)(t - i) * stride) : granule(epoch, kIncl, 0);
        bool stalled = false;
#pragma unroll
        for (int i = 0; i < LB_WINDOW; ++i) {
            if (done || stalled) continue;
            const uint32_t st = granule_status(v[i], epoch);
            if (st == 0) {
                stalled = true;
                continue;
            }
            excl += v[i] & kValueMask;
            --t;
            if (st == 2) done = true;
        }
        if (stalled && !done) {
            if (++spins > kSpinLimit) {
                atomicOr(error, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    publish(desc + (size_t)tile * stride, granule(epoch, kIncl, excl + agg));
    return excl;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    uint32_t lane = __lane_id();
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// popcount of the bits of m below this lane: v_mbcnt_lo + v_mbcnt_hi, two VALU (popcll(m & lanemask_lt())
// built the mask with a runtime 64-bit shift and selects every time: ~8 VALU per call, per key in the
// local passes' list positions)
__device__ __forceinline__ uint32_t popc_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// inclusive wave scan (sum) of 32-bit values
__device__ __forceinline__ uint32_t wave_inclusive_sum(uint32_t v) {
    const uint32_t lane = __lane_id();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t o = __shfl_up(v, off, 64);
        if (lane >= (uint32_t)off) v += o;
    }
    return v;
}

// Exclusive block scan of one 32-bit value per thread; returns exclusive prefix and total.
// `scratch` must hold BLOCK / 64 + 1 words.  Contains __syncthreads().
template <int BLOCK>
__device__ __forceinline__ uint32_t block_exclusive_sum(uint32_t v, uint32_t *scratch,
                                                        uint32_t *total) {
    constexpr int NW = BLOCK / 64;
    const uint32_t lane = __lane_id();
    const uint32_t wid = threadIdx.x / 64;
    uint32_t inc = wave_inclusive_sum(v);
    if (lane == 63) scratch[wid] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int w = 0; w < NW; ++w) {
            uint32_t t = scratch[w];
            scratch[w] = s;
            s += t;
        }
        scratch[NW] = s;
    }
    __syncthreads();
    uint32_t res = scratch[wid] + inc - v;
    *total = scratch[NW];
    __syncthreads();
    return res;
}

// The same over 64-bit values (`scratch`: BLOCK / 64 + 1 u64 words): the bucket-count scans, whose
// tile of 4096 counts can total more than 2^32 keys (a level-1 histogram of > 4.3e9 keys)
__device__ __forceinline__ uint64_t wave_inclusive_sum_u64(uint64_t v) {
    const uint32_t lane = __lane_id();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint64_t o = __shfl_up(v, off, 64);
        if (lane >= (uint32_t)off) v += o;
    }
    return v;
}

template <int BLOCK>
__device__ __forceinline__ uint64_t block_exclusive_sum_u64(uint64_t v, uint64_t *scratch, uint64_t *total) {
    constexpr int NW = BLOCK / 64;
    const uint32_t lane = __lane_id();
    const uint32_t wid = threadIdx.x / 64;
    const uint64_t inc = wave_inclusive_sum_u64(v);
    if (lane == 63) scratch[wid] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t s = 0;
        for (int w = 0; w < NW; ++w) {
            const uint64_t t = scratch[w];
            scratch[w] = s;
            s += t;
        }
        scratch[NW] = s;
    }
    __syncthreads();
    const uint64_t res = scratch[wid] + inc - v;
    *total = scratch[NW];
    __syncthreads();
    return res;
}

// XCD-contiguous tiles for the scatter passes.  The dispatcher hands workgroups to the 8 XCDs
// round-robin (workgroup b on XCD b % 8), and every XCD has its own L2.  Workgroup b takes tile
// (b % 8) * per + b / 8, so each XCD walks its own contiguous eighth of the tiles: the tiles it
// runs at once are neighbours, whose runs of one bucket are neighbours in the output, and the
// partial lines at their edges meet in one L2 instead of going to HBM from two XCDs (the level-2
// partition pass: 4.59 -> 4.05 ms, tools/part_bench.hip).  The grid is xcd_grid(ntiles); the
// surplus workgroups (tile >= ntiles) return at once.
constexpr int kXcds = 8;
__device__ __forceinline__ uint64_t xcd_tile(uint64_t ntiles) {
    const uint64_t per = (ntiles + kXcds - 1) / kXcds;
    return (uint64_t)(blockIdx.x % kXcds) * per + blockIdx.x / kXcds;
}
static inline uint64_t xcd_grid(uint64_t ntiles) { return (ntiles + kXcds - 1) / kXcds * kXcds; }

// Tile prologue shared by the single-column compaction kernels: dynamic tile id (so every
// predecessor is already resident) and, after the block's count is known, the wave-0
// look-back.  `s_tile` / `s_base` are LDS words.
__device__ __forceinline__ uint32_t take_tile(uint32_t *tile_counter, uint32_t *s_tile) {
    if (threadIdx.x == 0) *s_tile = atomicAdd(tile_counter, 1u);
    __syncthreads();
    return *s_tile;
}

__device__ __forceinline__ void tile_base_lookback(uint64_t *desc, uint32_t tile, uint64_t count,
                                                   uint32_t epoch, uint32_t *error,
                                                   uint64_t *s_base) {
    if (threadIdx.x < 64) {
        const uint64_t b = wave_lookback(desc, tile, count, epoch, error);
        if (threadIdx.x == 0) *s_base = b;
    }
    __syncthreads();
}

// ---------------------------------------------------------------- per-read counts lookup
//
// The read holding buffer position p (the last r with read_starts[r] <= p), for per-read counts.
// rid_at (optional, read_index_kernel) brackets the search: rid_at[q] = that read for position
// q << RID_SHIFT, so a window searches the one or two reads of its 32-position block instead of
// all of them.  (4 K-position blocks left a 7-step search of global memory per window for KMC input
// -- one 32-byte read per record, 1.9e8 reads at configs[4] -- 42.8 ms of extraction per step.)
constexpr unsigned RID_SHIFT = 5;

__device__ __forceinline__ uint64_t read_of(const uint64_t *__restrict__ read_starts, uint64_t n_reads,
                                            const uint64_t *__restrict__ rid_at, uint64_t p) {
    uint64_t lo = 0, hi = n_reads;
    if (rid_at) {
        const uint64_t q = p >> RID_SHIFT;
        lo = rid_at[q];
        hi = min(n_reads, rid_at[q + 1] + 1);
    }
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) / 2;
        if (read_starts[mid] <= p) lo = mid; else hi = mid;
    }
    return lo;
}

// rid_at[0..nq) from the sorted read starts, one thread per read: read r owns the blocks whose first
// position lies in [start_r, start_{r+1}) (read 0 also every block before it), O(reads + blocks)
__global__ void read_index_kernel(const uint64_t *__restrict__ read_starts, uint64_t n_reads, uint64_t nq,
                                  uint64_t *__restrict__ rid_at) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    constexpr uint64_t B = 1ull << RID_SHIFT;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_reads; r += gs) {
        const uint64_t q0 = r == 0 ? 0 : (read_starts[r] + B - 1) >> RID_SHIFT;
        const uint64_t q1 = r + 1 < n_reads ? min(nq, (read_starts[r + 1] + B - 1) >> RID_SHIFT) : nq;
        for (uint64_t q = q0; q < q1; ++q) rid_at[q] = r;
    }
}

}  // namespace mtg
