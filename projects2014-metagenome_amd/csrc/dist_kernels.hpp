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
// destinations of one routing launch: ranks, or the key ranges of a spilled build (<= RB_BINS)
constexpr int MAX_ROUTE = 256;
constexpr int RT_BLOCK = 256;
constexpr int RT_TILE = 4096;
constexpr int RT_PER = RT_TILE / RT_BLOCK;

// rank of a prefix: #{j in 1..P-1 : bounds[j] <= v} (bounds ascending)
__device__ __forceinline__ uint32_t owner_of(uint64_t v, const uint64_t *s_bounds, uint32_t P) {
    uint32_t a = 1, b = P;
    while (a < b) {
        const uint32_t mid = (a + b) >> 1;
        if (s_bounds[mid] <= v) a = mid + 1; else b = mid;
    }
    return a - 1;
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
    __shared__ uint64_t s_b[MAX_ROUTE + 1];
    __shared__ uint32_t s_c[MAX_ROUTE];
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
    __shared__ uint64_t s_b[MAX_ROUTE + 1];
    __shared__ uint64_t s_base[MAX_ROUTE];
    __shared__ uint32_t s_c[MAX_ROUTE];
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
            if (valid && o == lo) pos = b + popc_below(same);
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
            const uint32_t pos = b + popc_below(m);
            out[base + pos] = lift_fast<L3>(q[i], K) & ~Key<L3>::from(7);
        }
    }
}

/*
 * The sink / in-edge queries as 4 sorted arrays (one per label c of the querying edge).  The query of
 * edge x is t = to_next(x, 0) (node a_2..a_K, label $), whose top char is x's label, and on the edges
 * of one label to_next is monotone -- so the queries of label c, in edge order, are sorted, and the 4
 * label classes occupy disjoint key ranges.  A stable split of the owned edges by label therefore
 * yields the queries sorted, every owner's share is a contiguous slice of each class (found by
 * binary search), and the owner receives 4 P sorted runs: its answering probes (query_join_kernel)
 * join tiles of sorted queries against the edge range they span.
 * One tile = SplitTraits::TILE edges.  The count pass reads the labels coalesced; the write pass
 * loads the tile coalesced, ranks every edge inside its class (PER consecutive edges per thread, one
 * block scan), permutes the queries in LDS and writes each class's run of the tile contiguously to
 * toff[c * ntiles + tile] (class-major: the 4 sorted arrays back to back).  Per-thread scattered
 * 8-byte stores instead (round 3, first cut): 16.6 ms for the write pass at configs[1]/2.
 */
template <int L>
struct SplitTraits {
    static constexpr int PER = L == 1 ? 16 : L == 2 ? 8 : 4;
    static constexpr int TILE = 256 * PER;
};

template <int L, bool COUNT_ONLY>
__global__ __launch_bounds__(256) void target_split_kernel(const Key<L> *__restrict__ E, uint64_t n, unsigned K,
                                                          uint64_t ntiles, uint32_t *__restrict__ tcnt,
                                                          const uint64_t *__restrict__ toff, Key<L> *__restrict__ out) {
    constexpr int PER = SplitTraits<L>::PER, TILE = SplitTraits<L>::TILE;
    const uint32_t tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * TILE;
    const uint32_t tn = (uint32_t)min((uint64_t)TILE, n - base);
    if constexpr (COUNT_ONLY) {
        __shared__ uint32_t s_t[4];
        if (tid < 4) s_t[tid] = 0;
        uint32_t cnt01 = 0, cnt23 = 0;  // 16-bit fields
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const uint32_t i = j * 256 + tid;
            if (i < tn) {
                const uint32_t c = (uint32_t)(E[base + i].w[0] & 3);
                if (c < 2) cnt01 += 1u << (16 * c); else cnt23 += 1u << (16 * (c - 2));
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            cnt01 += __shfl_xor(cnt01, off, 64);
            cnt23 += __shfl_xor(cnt23, off, 64);
        }
        __syncthreads();
        if (__lane_id() == 0) {
            atomicAdd(&s_t[0], cnt01 & 0xFFFFu);
            atomicAdd(&s_t[1], cnt01 >> 16);
            atomicAdd(&s_t[2], cnt23 & 0xFFFFu);
            atomicAdd(&s_t[3], cnt23 >> 16);
        }
        __syncthreads();
        if (tid < 4) tcnt[(uint64_t)tid * ntiles + blockIdx.x] = s_t[tid];
        return;
    } else {
        __shared__ Key<L> s_k[TILE];
        __shared__ uint16_t s_dst[TILE];
        __shared__ uint8_t s_lab[TILE];
        __shared__ uint32_t s_scan[256 / 64 + 1];
        Key<L> x[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const uint32_t i = j * 256 + tid;
            if (i < tn) {
                x[j] = E[base + i];
                s_lab[i] = (uint8_t)(x[j].w[0] & 3);
            }
        }
        __syncthreads();
        // thread tid ranks edges tid * PER .. + PER inside their classes
        uint32_t lab = 0, cnt01 = 0, cnt23 = 0;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint32_t i = tid * PER + q;
            const uint32_t c = i < tn ? s_lab[i] : 4u;
            lab |= (c & 3u) << (2 * q);
            if (c < 2) cnt01 += 1u << (16 * c); else if (c < 4) cnt23 += 1u << (16 * (c - 2));
        }
        uint32_t t01, t23;
        const uint32_t o01 = block_exclusive_sum<256>(cnt01, s_scan, &t01);
        const uint32_t o23 = block_exclusive_sum<256>(cnt23, s_scan, &t23);
        // class starts inside the tile
        const uint32_t cs1 = t01 & 0xFFFFu, cs2 = cs1 + (t01 >> 16), cs3 = cs2 + (t23 & 0xFFFFu);
        uint32_t pos[4] = {o01 & 0xFFFFu, cs1 + (o01 >> 16), cs2 + (o23 & 0xFFFFu), cs3 + (o23 >> 16)};
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint32_t i = tid * PER + q;
            if (i < tn) {
                const uint32_t c = (lab >> (2 * q)) & 3u;
                const uint32_t p = c == 0 ? pos[0]++ : c == 1 ? pos[1]++ : c == 2 ? pos[2]++ : pos[3]++;
                s_dst[i] = (uint16_t)p;
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const uint32_t i = j * 256 + tid;
            if (i < tn) s_k[s_dst[i]] = routed_key<L, 0>(x[j], K);
        }
        __syncthreads();
        const uint64_t g0 = toff[blockIdx.x], g1 = toff[ntiles + blockIdx.x] - cs1,
                       g2 = toff[2 * ntiles + blockIdx.x] - cs2, g3 = toff[3 * ntiles + blockIdx.x] - cs3;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const uint32_t sl = j * 256 + tid;
            if (sl < tn) {
                const uint64_t g = sl >= cs3 ? g3 : sl >= cs2 ? g2 : sl >= cs1 ? g1 : g0;
                out[g + sl] = s_k[sl];
            }
        }
    }
}

/*
 * Owner side of the sink join over sorted query runs: query p = node (a_2..a_K) with label $ of
 * some edge x anywhere.  The first edge of node p (lower bound of p among the owner's sorted
 * edges) gets its in-edge mark -- x targets that node, so it needs no dummy source (:148-166); a
 * miss means x's target node has no out-edge and needs a dummy sink (:80-95): qflag = 1.
 * A workgroup takes JoinTraits::TILE consecutive queries.  Inside one sorted run they span a short
 * key range [min, max]; the edges of its buckets are staged in LDS (coalesced) and every probe
 * binary-searches them there.  A tile whose range does not fit (it straddles two runs, or the
 * edges are dense there) binary-searches the bucketed global array instead.
 */
template <int L>
struct JoinTraits {
    static constexpr int PER = L == 1 ? 4 : 2;
    static constexpr int TILE = 256 * PER;
    static constexpr int CAP = TILE * 5 / 4;
};

template <int L>
__device__ __forceinline__ Key<L> wave_min_key(Key<L> v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        Key<L> o;
#pragma unroll
        for (int w = 0; w < L; ++w) o.w[w] = __shfl_xor(v.w[w], off, 64);
        if (o < v) v = o;
    }
    return v;
}

template <int L>
__device__ __forceinline__ Key<L> wave_max_key(Key<L> v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        Key<L> o;
#pragma unroll
        for (int w = 0; w < L; ++w) o.w[w] = __shfl_xor(v.w[w], off, 64);
        if (v < o) v = o;
    }
    return v;
}

template <int L>
__global__ __launch_bounds__(256) void query_join_kernel(const Key<L> *__restrict__ keys, uint64_t n,
                                                         const uint64_t *__restrict__ start, unsigned bshift,
                                                         const Key<L> *__restrict__ q, uint64_t nq,
                                                         uint8_t *__restrict__ in_flag, uint8_t *__restrict__ qflag) {
    using T = JoinTraits<L>;
    constexpr int PER = T::PER;
    __shared__ Key<L> s_r[T::CAP];
    __shared__ Key<L> s_mm[8];
    __shared__ uint64_t s_a;
    __shared__ uint32_t s_cnt;
    const uint32_t tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * T::TILE;
    const uint32_t tn = (uint32_t)min((uint64_t)T::TILE, nq - base);
    const uint32_t j0 = tid * PER;
    Key<L> x[PER];
    Key<L> mn = ~Key<L>::zero(), mx = Key<L>::zero();
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        x[k] = Key<L>::zero();
        if (j0 + k < tn) {
            x[k] = q[base + j0 + k];
            if (x[k] < mn) mn = x[k];
            if (mx < x[k]) mx = x[k];
        }
    }
    mn = wave_min_key<L>(mn);
    mx = wave_max_key<L>(mx);
    if (__lane_id() == 0) {
        s_mm[tid / 64] = mn;
        s_mm[4 + tid / 64] = mx;
    }
    __syncthreads();
    if (tid == 0) {
        Key<L> a = s_mm[0], b = s_mm[4];
        for (int w = 1; w < 4; ++w) {
            if (s_mm[w] < a) a = s_mm[w];
            if (b < s_mm[4 + w]) b = s_mm[4 + w];
        }
        uint32_t cnt = ~0u;
        uint64_t lo = 0;
        if (n) {
            const uint64_t blo = bits_at(shr(a, bshift), 0, 32), bhi = bits_at(shr(b | Key<L>::from(3), bshift), 0, 32);
            lo = start[blo];
            const uint64_t hi = start[bhi + 1];
            if (hi - lo <= (uint64_t)T::CAP) cnt = (uint32_t)(hi - lo);
        }
        s_a = lo;
        s_cnt = cnt;
    }
    __syncthreads();
    const uint32_t cnt = s_cnt;
    const uint64_t a = s_a;
    if (cnt != ~0u) {
        for (uint32_t j = tid; j < cnt; j += 256) s_r[j] = keys[a + j];
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        if (j0 + k >= tn) continue;
        const Key<L> p = x[k];
        uint64_t hit = ~0ull;
        if (!n) {
        } else if (cnt != ~0u) {
            uint32_t lo = 0, hi = cnt;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_r[mid] < p) lo = mid + 1; else hi = mid;
            }
            if (lo < cnt && shr(s_r[lo], 2) == shr(p, 2)) hit = a + lo;
        } else {
            const uint64_t i = lower_bound_bucketed(keys, start, bshift, p);
            if (i < n && shr(keys[i], 2) == shr(p, 2)) hit = i;
        }
        if (hit != ~0ull) in_flag[hit] = 1;
        qflag[base + j0 + k] = hit == ~0ull ? 1 : 0;
    }
}

/*
 * The pulled sink join (run_pipeline_dist): instead of sending every edge's query to the owner of its
 * target node, every rank sends each owner j the edges y whose NODE some edge of j targets: x = (a_1
 * .. a_k; label c) targets node (a_2 .. a_k, c), whose edges y have top char c and then a_k, a_(k-1),
 * .. -- so y goes to the owner of the m-char prefix below y's top char, i.e. of y's (m+1)-char prefix
 * minus c 4^m.  Within one top char c that prefix is monotone along the sorted edges, so every
 * (class c, owner j) share is a contiguous slice: out[c * (P + 1) + j] = the first edge with top char
 * c whose (m+1)-char prefix is >= c 4^m + bounds[j] (bounds[0] = 0, bounds[P] = 4^m).  Each edge is
 * sent once, unchanged (no split pass, no to_next transform); the owner receives its 4 classes' slices
 * from every rank sorted (array-major, then by source rank), probes them with its own edges
 * (dummy_sink_kernel with q), and returns one in-edge byte per received edge, which arrives aligned
 * with the sender's edge array.
 */
template <int L>
__global__ void pull_bounds_kernel(const Key<L> *__restrict__ e, uint64_t n, const uint64_t *__restrict__ bounds,
                                   uint32_t P, unsigned K, unsigned m, uint64_t *__restrict__ out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 4 * (P + 1)) return;
    const uint32_t c = t / (P + 1), j = t % (P + 1);
    const uint64_t v = ((uint64_t)c << (2 * m)) + bounds[j];
    const unsigned sh = 2 * K - 2 * (m + 1);  // (m+1)-char prefix = key >> sh
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (bits_at(shr(e[mid], sh), 0, 2 * (m + 1)) < v) lo = mid + 1; else hi = mid;
    }
    out[t] = lo;
}

// first query index of every owner in every class: out[c * (P + 1) + j] = lower bound of the prefix
// bounds[j] in the sorted class array [cstart[c], cstart[c + 1])
template <int L>
__global__ void class_bounds_kernel(const Key<L> *__restrict__ q, const uint64_t *__restrict__ cstart,
                                    const uint64_t *__restrict__ bounds, uint32_t P, unsigned pshift,
                                    uint64_t *__restrict__ out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 4 * (P + 1)) return;
    const uint32_t c = t / (P + 1), j = t % (P + 1);
    uint64_t lo = cstart[c], hi = cstart[c + 1];
    const uint64_t b = bounds[j];
    while (lo < hi) {  // first query whose owner prefix is >= b
        const uint64_t mid = (lo + hi) >> 1;
        if (bits_at(shr(q[mid], pshift), 0, 32) < b) lo = mid + 1; else hi = mid;
    }
    out[t] = lo;
}

}  // namespace mtg
