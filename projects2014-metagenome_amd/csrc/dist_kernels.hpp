// dist_kernels.hpp -- device kernels of the multi-GPU build (one rank per GPU, RCCL exchange).
//
// A global BOSS table is a range partition of BOSS order: rank j owns the edges whose top m
// node characters (the most significant chars of the key, kmer_boss.hpp:58-72) fall in
// [bounds[j], bounds[j+1]) of the 4^m prefixes.  With m <= k - 1, every group the row emission
// looks at (one node for `last` and the redundant-sink skip, one chars-2..k suffix for the W
// "minus" flag, boss_chunk.cpp:78-101) lies inside one rank, so the per-rank chunks concatenate
// with BOSS::Chunk::extend (boss_chunk.cpp:230-270).  The kernels here route the keys whose
// owner differs from their producer:
//   * sink / in-edge queries t = to_next(x, 0) of every real edge x (the dummy-sink probe of
//     add_dummy_sink_kmers, boss_chunk_construct.cpp:54-98) go to owner(t); the owner answers
//     them against its edges (marking in-edges for the source test, :123-168) and emits the
//     dummy sinks of the misses;
//   * dummy sources (all levels, :286-306) go to the owner of their lifted prefix.
// Routing is count -> scan -> write over identical 4096-item tiles; the order inside a tile's
// run is free because every routed set is sorted (or only probed) at its owner.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "boss_kernels.hpp"
#include "device_common.hpp"
#include "keys.hpp"

namespace mtg {

constexpr int MAX_RANKS = 64;
constexpr int RT_BLOCK = 256;
constexpr int RT_TILE = 4096;
constexpr int RT_PER = RT_TILE / RT_BLOCK;

// rank of a prefix: #{j in 1..P-1 : bounds[j] <= v}
__device__ __forceinline__ uint32_t owner_of(uint64_t v, const uint64_t *s_bounds, uint32_t P) {
    uint32_t o = 0;
    for (uint32_t j = 1; j < P; ++j) o += s_bounds[j] <= v ? 1u : 0u;
    return o;
}

// MODE 0: the routed key is t = to_next(x, K, 0) of a 2-bit edge x (node a_2..a_K, label $);
// MODE 1: the key itself (lifted dummies)
template <int L, int MODE>
__device__ __forceinline__ Key<L> routed_key(const Key<L> &x, unsigned K) {
    if constexpr (MODE == 0)
        return (shr(x, 2) | shl(Key<L>::from(x.w[0] & 3), 2 * (K - 1))) & ~Key<L>::from(3);
    else
        return x;
}

// Per (owner, tile) counts: tcnt[o * ntiles + tile].  Items of a tile are strided by the block
// size (coalesced loads); the owner prefix is bits [pshift, pshift + pbits) of the routed key.
template <int L, int MODE>
__global__ __launch_bounds__(RT_BLOCK) void route_count_kernel(
    const Key<L> *__restrict__ in, uint64_t n, unsigned K, unsigned pshift, unsigned pbits,
    const uint64_t *__restrict__ bounds, uint32_t P, uint32_t *__restrict__ tcnt, uint64_t ntiles) {
    __shared__ uint64_t s_b[MAX_RANKS + 1];
    __shared__ uint32_t s_c[MAX_RANKS];
    const uint32_t tid = threadIdx.x;
    for (uint32_t j = tid; j <= P; j += RT_BLOCK) s_b[j] = bounds[j];
    for (uint32_t j = tid; j < P; j += RT_BLOCK) s_c[j] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * RT_TILE;
#pragma unroll 4
    for (int q = 0; q < RT_PER; ++q) {
        const uint64_t i = t0 + (uint64_t)q * RT_BLOCK + tid;
        const bool valid = i < n;
        uint32_t o = ~0u;
        if (valid) o = owner_of(bits_at(shr(routed_key<L, MODE>(in[i], K), pshift), 0, pbits), s_b, P);
        // wave-aggregated: one LDS atomic per distinct owner in the wave
        uint64_t active = __ballot(valid);
        while (active) {
            const uint32_t leader = (uint32_t)(__ffsll((unsigned long long)active) - 1);
            const uint32_t lo = __shfl(o, leader, 64);
            const uint64_t same = __ballot(valid && o == lo);
            if (__lane_id() == leader) atomicAdd(&s_c[lo], (uint32_t)__popcll(same));
            active &= ~same;
        }
    }
    __syncthreads();
    for (uint32_t j = tid; j < P; j += RT_BLOCK) tcnt[(uint64_t)j * ntiles + blockIdx.x] = s_c[j];
}

// Scatter of the routed keys to out[toff[o * ntiles + tile] + rank inside the tile's run]
template <int L, int MODE>
__global__ __launch_bounds__(RT_BLOCK) void route_write_kernel(
    const Key<L> *__restrict__ in, uint64_t n, unsigned K, unsigned pshift, unsigned pbits,
    const uint64_t *__restrict__ bounds, uint32_t P, const uint64_t *__restrict__ toff,
    uint64_t ntiles, Key<L> *__restrict__ out, const uint32_t *__restrict__ in_v = nullptr,
    uint32_t *__restrict__ out_v = nullptr) {
    // in_v / out_v (optional): a count per key, moved with it
    __shared__ uint64_t s_b[MAX_RANKS + 1];
    __shared__ uint64_t s_base[MAX_RANKS];
    __shared__ uint32_t s_c[MAX_RANKS];
    const uint32_t tid = threadIdx.x;
    for (uint32_t j = tid; j <= P; j += RT_BLOCK) s_b[j] = bounds[j];
    for (uint32_t j = tid; j < P; j += RT_BLOCK) {
        s_c[j] = 0;
        s_base[j] = toff[(uint64_t)j * ntiles + blockIdx.x];
    }
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * RT_TILE;
#pragma unroll 4
    for (int q = 0; q < RT_PER; ++q) {
        const uint64_t i = t0 + (uint64_t)q * RT_BLOCK + tid;
        const bool valid = i < n;
        uint32_t o = ~0u;
        Key<L> y = Key<L>::zero();
        if (valid) {
            y = routed_key<L, MODE>(in[i], K);
            o = owner_of(bits_at(shr(y, pshift), 0, pbits), s_b, P);
        }
        uint64_t active = __ballot(valid);
        uint32_t pos = 0;
        while (active) {
            const uint32_t leader = (uint32_t)(__ffsll((unsigned long long)active) - 1);
            const uint32_t lo = __shfl(o, leader, 64);
            const uint64_t same = __ballot(valid && o == lo);
            uint32_t b = 0;
            if (__lane_id() == leader) b = atomicAdd(&s_c[lo], (uint32_t)__popcll(same));
            b = __shfl(b, leader, 64);
            if (valid && o == lo) pos = b + (uint32_t)__popcll(same & lanemask_lt());
            active &= ~same;
        }
        if (valid) {
            out[s_base[o] + pos] = y;
            if (in_v) out_v[s_base[o] + pos] = in_v[i];
        }
    }
}

// Balancing samples of the reverse-complement set: every stride-th canonical key x adds stride
// to hist[prefix of rc(x)] (the rc keys of the owned canonical set go to those prefixes' owners,
// so the ranges are balanced on both strands before the first exchange)
template <int L>
__global__ void rc_prefix_sample_kernel(const Key<L> *__restrict__ keys, uint64_t n, unsigned K,
                                        unsigned pshift, unsigned pbits, uint64_t stride,
                                        unsigned long long *__restrict__ hist) {
    const uint64_t ns = (n + stride - 1) / stride;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < ns; j += gs) {
        const Key<L> r = revcomp2(keys[j * stride], K);
        atomicAdd(&hist[bits_at(shr(r, pshift), 0, pbits)], (unsigned long long)stride);
    }
}

// per-bucket counts of a sorted array from its bucket index: hist[b] (+)= start[b+1] - start[b]
__global__ void hist_from_starts_kernel(const uint64_t *__restrict__ start, uint64_t nb,
                                        uint64_t *__restrict__ hist, int accumulate) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const uint64_t v = start[b + 1] - start[b];
    hist[b] = accumulate ? hist[b] + v : v;
}

// flags[i] = (x_i is the first edge of its node) << 1; no sink bit (sinks come from queries)
template <int L>
__global__ void first_flag_kernel(const Key<L> *__restrict__ keys, uint64_t n,
                                  uint8_t *__restrict__ flags) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const bool first = i == 0 || shr(keys[i - 1], 2) != shr(keys[i], 2);
        flags[i] = (uint8_t)(first ? 2u : 0u);
    }
}

/*
 * Owner side of the sink join: query p = node (a_2..a_K) with label $ of some edge x anywhere.
 * The first edge of node p (lower bound of p among the owner's sorted edges) gets its in-edge
 * mark -- x targets that node, so it needs no dummy source (:148-166); a miss means x's target
 * node has no out-edge and needs a dummy sink (:80-95): qflag = 1.
 */
template <int L>
__global__ void query_answer_kernel(const Key<L> *__restrict__ keys, uint64_t n,
                                    const uint64_t *__restrict__ start, unsigned bshift,
                                    const Key<L> *__restrict__ q, uint64_t nq,
                                    uint8_t *__restrict__ in_flag, uint8_t *__restrict__ qflag) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += stride) {
        const Key<L> p = q[i];
        bool hit = false;
        if (n) {
            const uint64_t b = bits_at(shr(p, bshift), 0, 32);
            uint64_t lo = start[b], hi = start[b + 1];
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1;
                if (keys[mid] < p) lo = mid + 1; else hi = mid;
            }
            if (lo < n && shr(keys[lo], 2) == shr(p, 2)) {
                hit = true;
                in_flag[lo] = 1;
            }
        }
        qflag[i] = hit ? 0 : 1;
    }
}

// sink compaction over the answered queries: per-tile miss counts ...
__global__ __launch_bounds__(RT_BLOCK) void sink_count_kernel(const uint8_t *__restrict__ qflag,
                                                             uint64_t nq, uint32_t *__restrict__ tcnt) {
    __shared__ uint32_t s_scan[RT_BLOCK / 64 + 1];
    const uint64_t t0 = (uint64_t)blockIdx.x * RT_TILE;
    uint32_t cnt = 0;
#pragma unroll
    for (int q = 0; q < RT_PER; ++q) {
        const uint64_t i = t0 + (uint64_t)q * RT_BLOCK + threadIdx.x;
        if (i < nq) cnt += qflag[i];
    }
    uint32_t total;
    block_exclusive_sum<RT_BLOCK>(cnt, s_scan, &total);
    if (threadIdx.x == 0) tcnt[blockIdx.x] = total;
}

// ... and the writes: lift(p) with the label char cleared to $ (boss_chunk_construct.cpp:94)
template <int L2, int L3>
__global__ __launch_bounds__(RT_BLOCK) void sink_write_kernel(const Key<L2> *__restrict__ q,
                                                             const uint8_t *__restrict__ qflag,
                                                             uint64_t nq, unsigned K,
                                                             const uint64_t *__restrict__ toff,
                                                             Key<L3> *__restrict__ out) {
    __shared__ uint32_t s_c;
    if (threadIdx.x == 0) s_c = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * RT_TILE;
    const uint64_t base = toff[blockIdx.x];
    for (int qq = 0; qq < RT_PER; ++qq) {
        const uint64_t i = t0 + (uint64_t)qq * RT_BLOCK + threadIdx.x;
        const bool miss = i < nq && qflag[i];
        const uint64_t m = __ballot(miss);
        uint32_t b = 0;
        if (m && __lane_id() == (uint32_t)(__ffsll((unsigned long long)m) - 1))
            b = atomicAdd(&s_c, (uint32_t)__popcll(m));
        b = __shfl(b, (uint32_t)(__ffsll((unsigned long long)(m ? m : 1)) - 1), 64);
        if (miss) {
            const uint32_t pos = b + (uint32_t)__popcll(m & lanemask_lt());
            out[base + pos] = lift_fast<L3>(q[i], K) & ~Key<L3>::from(7);
        }
    }
}

}  // namespace mtg
