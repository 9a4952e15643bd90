// device_common.hpp -- wave64 / workgroup primitives and the decoupled look-back protocol
// shared by the sort, scan and compaction kernels.
//
// Inter-workgroup hand-off: every tile publishes 64-bit granules {status:2 | value:62} with a
// single agent-scope relaxed atomic store; readers poll them with agent-scope relaxed atomic
// loads.  The data IS the flag (8-byte granule, R2 of the CDNA4 guide), so no fences are
// needed; the descriptor arrays are zeroed by hipMemsetAsync before every launch and spins are
// bounded (a timeout sets an error word the host checks).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mtg {

constexpr int kWave = 64;

constexpr uint64_t kStatusShift = 62;
constexpr uint64_t kStatusAgg = 1ull << kStatusShift;
constexpr uint64_t kStatusIncl = 2ull << kStatusShift;
constexpr uint64_t kValueMask = (1ull << kStatusShift) - 1;
constexpr uint32_t kSpinLimit = 1u << 26;

__device__ __forceinline__ void publish(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t poll(const uint64_t *p) {
    return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive prefix of `agg` over all tiles < tile, via decoupled look-back on desc[tile*stride].
// Called by ONE lane per (tile, column).  Publishes the inclusive prefix for its successors.
__device__ __forceinline__ uint64_t lookback(uint64_t *desc, uint32_t tile, uint32_t stride,
                                             uint64_t agg, uint32_t *error) {
    if (tile == 0) {
        publish(desc, kStatusIncl | agg);
        return 0;
    }
    publish(desc + (size_t)tile * stride, kStatusAgg | agg);
    uint64_t excl = 0;
    int64_t t = (int64_t)tile - 1;
    uint32_t spins = 0;
    while (t >= 0) {
        uint64_t v = poll(desc + (size_t)t * stride);
        uint64_t st = v >> kStatusShift;
        if (st == 0) {
            if (++spins > kSpinLimit) {
                atomicOr(error, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        excl += v & kValueMask;
        if (st == 2) break;
        --t;
    }
    publish(desc + (size_t)tile * stride, kStatusIncl | (excl + agg));
    return excl;
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t lanemask_lt() {
    uint32_t lane = __lane_id();
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
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
// `scratch` must hold blockDim.x / 64 + 1 words.  Contains __syncthreads().
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

}  // namespace mtg
