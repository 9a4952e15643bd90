// radix_sort.hpp -- LSD radix sort of Key<L> words (optional u32 payload) for gfx950.
//
// Replaces ips4o::parallel::sort at sorted_set.cpp:43-44, sorted_multiset.cpp:59-64 and
// boss_chunk_construct.cpp:221, :280-306.  One histogram pass computes the digit histograms of
// every pass at once; then one "onesweep" kernel per 8-bit digit:
//   * a workgroup takes the next tile id from an atomic counter (so predecessors are always
//     resident), loads its tile wave-striped (each wave owns 64*ITEMS consecutive keys, lanes
//     coalesced), ranks every key inside its wave with 8 ballots (wave64 match-any), keeps
//     per-wave digit counters in LDS,
//   * publishes per-digit tile counts and resolves the per-digit global offset with a
//     decoupled look-back (device_common.hpp),
//   * reorders the tile in LDS by digit and writes each digit run contiguously.
// Passes whose digit is constant over all keys are skipped (keys are 2K- or 3K-bit, so the
// upper bytes of a word are usually constant).
#pragma once

#include "device_common.hpp"
#include "keys.hpp"

namespace mtg {

template <int L>
struct SortTraits {
    static constexpr int ITEMS = L == 1 ? 16 : L == 2 ? 8 : 4;
    static constexpr int BLOCK = 512;
    static constexpr int TILE = ITEMS * BLOCK;
};

template <int L>
__global__ __launch_bounds__(256) void radix_histogram_kernel(const Key<L> *__restrict__ keys,
                                                              uint64_t n, int passes,
                                                              unsigned long long *__restrict__ hist) {
    __shared__ uint32_t s_hist[32 * 256];
    for (int i = threadIdx.x; i < passes * 256; i += blockDim.x) s_hist[i] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        Key<L> k = keys[i];
        for (int p = 0; p < passes; ++p) atomicAdd(&s_hist[p * 256 + bits_at(k, 8 * p, 8)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < passes * 256; i += blockDim.x)
        if (s_hist[i]) atomicAdd(&hist[i], (unsigned long long)s_hist[i]);
}

// ABL (timing ablations for tools/sort_bench only; 0 in the product): bit 0 = replace the
// look-back by an atomic per-digit cursor, bit 1 = write the tile back in place (no
// scatter), bit 2 = skip the wave ranking
template <int L, bool HAS_VAL, int ABL = 0>
__global__ __launch_bounds__(512) void onesweep_kernel(
    const Key<L> *__restrict__ kin, Key<L> *__restrict__ kout, const uint32_t *__restrict__ vin,
    uint32_t *__restrict__ vout, uint64_t n, unsigned shift,
    const uint64_t *__restrict__ digit_start, uint64_t *desc, uint32_t epoch,
    uint32_t *tile_counter, uint32_t *error) {
    constexpr int ITEMS = SortTraits<L>::ITEMS;
    constexpr int BLOCK = SortTraits<L>::BLOCK;
    constexpr int NW = BLOCK / 64;
    constexpr int TILE = ITEMS * BLOCK;
    constexpr int WT = ITEMS * 64;

    __shared__ Key<L> s_keys[TILE];
    __shared__ uint32_t s_vals[HAS_VAL ? TILE : 1];
    __shared__ uint32_t s_whist[NW * 256];
    __shared__ uint32_t s_loff[256];
    __shared__ uint64_t s_gbase[256];
    __shared__ uint32_t s_scan[NW + 1];
    __shared__ uint32_t s_tile;

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = __lane_id();
    const uint32_t wid = tid / 64;

    if (tid == 0) s_tile = atomicAdd(tile_counter, 1u);
    for (int i = tid; i < NW * 256; i += BLOCK) s_whist[i] = 0;
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t base = (uint64_t)tile * TILE;
    const uint64_t wbase = base + (uint64_t)wid * WT;

    Key<L> k[ITEMS];
    uint32_t v[ITEMS];
    uint32_t rank[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        uint64_t idx = wbase + (uint64_t)j * 64 + lane;
        if (idx < n) {
            k[j] = kin[idx];
            if (HAS_VAL) v[j] = vin[idx];
        } else {
            k[j] = Key<L>::zero();
            v[j] = 0;
        }
    }


#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const bool valid = wbase + (uint64_t)j * 64 + lane < n;
        const uint32_t d = bits_at(k[j], shift, 8);
        if (ABL & 4) {
            rank[j] = j * 64 + lane;
            continue;
        }
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1;
            const uint64_t bal = __ballot(bit);
            peers &= bit ? bal : ~bal;
        }
        const uint32_t leader = valid ? (uint32_t)(__ffsll((unsigned long long)peers) - 1) : lane;
        uint32_t old = 0;
        if (valid && lane == leader) {
            old = s_whist[wid * 256 + d];
            s_whist[wid * 256 + d] = old + (uint32_t)__popcll(peers);
        }
        old = __shfl(old, (int)leader, 64);
        rank[j] = old + popc_below(peers);
    }
    __syncthreads();

    // per digit (threads 0..255): exclusive prefix over waves, tile total, tile-local digit
    // offsets, and the per-digit look-back for the global offset
    uint32_t total = 0;
    if (tid < 256) {
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            uint32_t c = s_whist[w * 256 + tid];
            s_whist[w * 256 + tid] = s;
            s += c;
        }
        total = s;
    }
    uint32_t tile_total;
    const uint32_t loff = block_exclusive_sum<BLOCK>(total, s_scan, &tile_total);
    if (tid < 256) {
        s_loff[tid] = loff;
        const uint64_t excl = (ABL & 1) ? atomicAdd((unsigned long long *)desc + tid,
                                                    (unsigned long long)total)
                                        : column_lookback(desc + tid, tile, 256, total, epoch, error);
        s_gbase[tid] = digit_start[tid] + excl;
    }
    __syncthreads();

#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        if (wbase + (uint64_t)j * 64 + lane < n) {
            const uint32_t d = bits_at(k[j], shift, 8);
            uint32_t pos = s_loff[d] + s_whist[wid * 256 + d] + rank[j];
            if (ABL & 4) pos = wid * WT + j * 64 + lane;
            s_keys[pos] = k[j];
            if (HAS_VAL) s_vals[pos] = v[j];
        }
    }
    __syncthreads();

    const uint32_t tile_n = (uint32_t)min((uint64_t)TILE, n - base);
    for (uint32_t p = tid; p < tile_n; p += BLOCK) {
        const Key<L> key = s_keys[p];
        const uint32_t d = bits_at(key, shift, 8);
        uint64_t o = s_gbase[d] + (p - s_loff[d]);
        if (ABL & 2) o = base + p;
        if (ABL & 5) o = o % n;
        kout[o] = key;
        if (HAS_VAL) vout[o] = s_vals[p];
    }
}

}  // namespace mtg
