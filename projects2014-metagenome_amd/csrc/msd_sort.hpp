// msd_sort.hpp -- sort + unique (+ saturating count merge) of k-mer words by MSD partitioning
// and per-group LDS hashing.  Replaces ips4o::parallel::sort + std::unique
// (sorted_set.cpp:41-48) and the sort + saturating merge of sorted_multiset.cpp:54-84.
//
// Why not LSD: every LSD pass re-reads and re-writes all N keys (8 passes for 62-bit keys)
// before duplicates can be removed.  Here:
//   level l = 1..L : partition by the top 8l significant bits, given that keys are already
//                    grouped by the top 8(l-1) bits (msd_hist_kernel + scan + msd_partition).
//                    Order inside a bucket does not matter, so a tile reserves its bucket runs
//                    with one atomic per (tile, bucket): no look-back chain.
//   local          : consecutive buckets form groups of <= G keys; one workgroup per group
//                    hashes its keys into LDS (duplicates collapse, counts add), sorts the
//                    distinct keys with a bitonic network and writes them; a scan + gather
//                    packs the groups.  A group with more distinct keys than the table holds
//                    is flagged and finished by the LSD fallback (radix_sort.hpp).
// The final array is globally sorted because groups are contiguous key ranges in order.
#pragma once

#include "device_common.hpp"
#include "keys.hpp"

namespace mtg {


constexpr int MSD_BLOCK = 512;
constexpr int MSD_WIN = 2;    // previous-level segments a tile keeps in its LDS window
constexpr int MSD_DBITS = 9;  // widest digit of one partition level

template <int L>
struct MsdTraits {
    static constexpr int ITEMS = L == 1 ? 16 : L == 2 ? 8 : 4;
    static constexpr int TILE = ITEMS * MSD_BLOCK;
};

// top `bits` of the nbits-bit significant range of a key, as an integer (bits <= 32)
template <int L>
__device__ __forceinline__ uint32_t key_prefix(const Key<L> &k, unsigned nbits, unsigned bits) {
    return bits ? bits_at(k, nbits - bits, bits) : 0u;
}

/*
 * Histogram of bucket = top `b` bits over all keys (keys grouped by their top `bp` bits).
 * Counts go to an LDS window of MSD_WIN previous-level segments starting at the tile's first
 * key; keys beyond the window add to global memory directly.
 */
template <int L>
__global__ __launch_bounds__(MSD_BLOCK) void msd_hist_kernel(const Key<L> *__restrict__ keys,
                                                             uint64_t n, unsigned nbits,
                                                             unsigned b, unsigned bp,
                                                             uint32_t *__restrict__ counts,
                                                             uint32_t tstride = 1, uint32_t slice = 1,
                                                             uint32_t gtiles = 1,
                                                             const uint32_t *__restrict__ tvalid = nullptr) {
    // tvalid (the speculative level-1 layout, extract_partition.hpp: spec_l1_caps_kernel): tile t holds
    // keys only in its first tvalid[t] positions
    // tstride > 1: a sample -- workgroup i counts tile i * tstride (msd_sort_unique's speculative
    // final level sizes its buckets from it); slice > 1: a finer sample -- workgroup i counts 1/slice
    // of tiles i * gtiles .. + gtiles - 1, one line of every 8 * slice keys (previous-level buckets only
    // a few tiles long, or a fraction of one, are still sampled evenly).  gtiles tiles share one LDS
    // window flush: a sample of 1/8 of every tile flushing per tile cost as much as the full histogram
    // (a 3-level round of configs[3]'s share: 9.7 vs 10.4 ms, its global atomics)
    constexpr int TILE = MsdTraits<L>::TILE;
    constexpr int WMAX = MSD_WIN << 8;
    __shared__ uint32_t s_cnt[WMAX];
    const uint64_t tile0 = (uint64_t)blockIdx.x * tstride * (slice > 1 ? gtiles : 1u);
    const uint64_t base = tile0 * TILE;
    if (base >= n) return;
    auto tile_end = [&](uint64_t t) {  // end of tile t's keys
        return min(n, t * TILE + (tvalid ? (uint64_t)tvalid[t] : (uint64_t)TILE));
    };
    // the LDS window starts at the first key of the workgroup's first non-empty tile
    uint64_t wkey = base;
    if (tvalid) {
        const uint32_t ng = slice > 1 ? gtiles : 1u;
        uint32_t t = 0;
        while (t < ng && (tile0 + t) * TILE < n && tvalid[tile0 + t] == 0) ++t;
        if (t == ng || (tile0 + t) * TILE >= n) return;
        wkey = (tile0 + t) * TILE;
    }
    const unsigned sub = b - bp;
    const uint32_t wsize = min((uint32_t)WMAX, (uint32_t)MSD_WIN << sub);  // 9-bit digits: one segment
    for (int i = threadIdx.x; i < (int)wsize; i += MSD_BLOCK) s_cnt[i] = 0;
    const uint32_t wbase = key_prefix(keys[wkey], nbits, bp) << sub;
    __syncthreads();
    const uint64_t end = min(tile_end(tile0), base + TILE / slice);
    auto add = [&](const Key<L> &key) {
        const uint32_t bucket = key_prefix(key, nbits, b);
        const uint32_t lb = bucket - wbase;
        if (lb < wsize) atomicAdd(&s_cnt[lb], 1u);
        else atomicAdd(&counts[bucket], 1u);
    };
    if constexpr (L == 1) {
      if (slice > 1) {
        // the finer sample spread over the whole tile: the first 128-byte line (16 keys) of every
        // 16 * slice keys, eight lanes per line (a contiguous 1/slice prefix would miss previous-level
        // buckets that start late in the tile; 64-byte lines fetched twice the bytes they counted)
        const uint32_t lines = TILE / (16 * slice);
        for (uint32_t t = 0; t < gtiles; ++t) {
            const uint64_t tb = base + (uint64_t)t * TILE;
            if (tb >= n) break;
            const uint64_t tend = tile_end(tile0 + t);
            for (uint32_t j = threadIdx.x; j < 8 * lines; j += MSD_BLOCK) {
                const uint64_t i = tb + (uint64_t)(j >> 3) * (16 * slice) + 2 * (j & 7);
                if (i + 1 < tend) {
                    const ulonglong2 v = *(const ulonglong2 *)(keys + i);
                    add(Key<L>::from(v.x));
                    add(Key<L>::from(v.y));
                } else if (i < tend) {
                    add(keys[i]);
                }
            }
        }
      } else {  // 16-byte loads: two keys per lane
        for (uint64_t i = base + 2 * threadIdx.x; i < end; i += 2 * MSD_BLOCK) {
            if (i + 1 < end) {
                const ulonglong2 v = *(const ulonglong2 *)(keys + i);
                add(Key<L>::from(v.x));
                add(Key<L>::from(v.y));
            } else {
                add(keys[i]);
            }
        }
      }
    } else {
        for (uint64_t i = base + threadIdx.x; i < end; i += MSD_BLOCK) add(keys[i]);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < (int)wsize; i += MSD_BLOCK)
        if (s_cnt[i]) atomicAdd(&counts[wbase + i], s_cnt[i]);
}

/*
 * First-level histogram (bp = 0, at most 512 buckets): every workgroup counts a grid-stride
 * share of the keys in LDS and stores its row rows[block][bucket]; hist_rows_reduce_kernel adds
 * the rows.  No global atomics on the few bucket words (thousands of workgroups adding to the
 * same 256 words serialise at the memory-side atomic unit).
 */
template <int L>
__global__ __launch_bounds__(512) void msd_hist_rows_kernel(const Key<L> *__restrict__ keys,
                                                            uint64_t n, unsigned nbits, unsigned b,
                                                            uint32_t *__restrict__ rows) {
    __shared__ uint32_t s_h[512];
    const uint32_t nb = 1u << b;
    for (uint32_t i = threadIdx.x; i < nb; i += 512) s_h[i] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * 512;
    if constexpr (L == 1) {  // 16-byte loads: two keys per lane
        for (uint64_t p = (uint64_t)blockIdx.x * 512 + threadIdx.x; 2 * p < n; p += stride) {
            const uint64_t i = 2 * p;
            if (i + 1 < n) {
                const ulonglong2 v = *(const ulonglong2 *)(keys + i);
                atomicAdd(&s_h[key_prefix(Key<L>::from(v.x), nbits, b)], 1u);
                atomicAdd(&s_h[key_prefix(Key<L>::from(v.y), nbits, b)], 1u);
            } else {
                atomicAdd(&s_h[key_prefix(keys[i], nbits, b)], 1u);
            }
        }
    } else {
        for (uint64_t i = (uint64_t)blockIdx.x * 512 + threadIdx.x; i < n; i += stride)
            atomicAdd(&s_h[key_prefix(keys[i], nbits, b)], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += 512) rows[(uint64_t)blockIdx.x * nb + i] = s_h[i];
}

// out[bin] += sum of rows[r][bin] over this block's slice of rows (out zeroed by the caller)
__global__ __launch_bounds__(256) void hist_rows_reduce_kernel(const uint32_t *__restrict__ rows,
                                                               uint32_t nrows, uint32_t nb,
                                                               uint32_t *__restrict__ out) {
    const uint32_t bin = blockIdx.y * 256 + threadIdx.x;
    if (bin >= nb) return;
    uint32_t sum = 0;
    for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) sum += rows[(uint64_t)r * nb + bin];
    if (sum) atomicAdd(&out[bin], sum);
}

/*
 * Exclusive scan of u32 counts into u64 starts (starts[n] = total), chained by a wave
 * look-back over tiles of 4096 entries.
 */
__global__ __launch_bounds__(512) void scan_counts_kernel(const uint32_t *__restrict__ counts,
                                                          uint64_t n, uint64_t *__restrict__ starts,
                                                          uint64_t *desc, uint32_t epoch,
                                                          uint32_t *tile_counter, uint32_t *error) {
    constexpr int ITEMS = 8, TILE = 512 * ITEMS;
    __shared__ uint64_t s_scan[512 / 64 + 1];
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_base;
    const uint32_t tile = take_tile(tile_counter, &s_tile);
    const uint64_t i0 = (uint64_t)tile * TILE + (uint64_t)threadIdx.x * ITEMS;
    uint32_t v[ITEMS];
    uint64_t sum = 0;  // 64-bit: a tile of bucket counts may hold more than 2^32 keys
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        v[j] = i0 + j < n ? counts[i0 + j] : 0;
        sum += v[j];
    }
    uint64_t tile_total;
    const uint64_t off = block_exclusive_sum_u64<512>(sum, s_scan, &tile_total);
    tile_base_lookback(desc, tile, tile_total, epoch, error, &s_base);
    uint64_t s = s_base + off;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        if (i0 + j < n) starts[i0 + j] = s;
        s += v[j];
    }
    const uint64_t ntiles = (n + TILE - 1) / TILE;
    if (tile + 1 == ntiles && threadIdx.x == 511) starts[n] = s_base + tile_total;
}

/*
 * Partition by bucket = top `b` bits.  cursor[bucket] starts at the bucket's first slot and
 * is advanced by one atomic per (tile, bucket) run; the tile is reordered by bucket in LDS
 * and each run is written contiguously.  Keys outside the tile's LDS window (tiles spanning
 * more than MSD_WIN tiny segments) take one atomic each.
 */
template <int L>
__device__ __forceinline__ Key<L> load_key(const Key<L> *p, bool nt) {
    if (!nt) return *p;
    Key<L> k;
#pragma unroll
    for (int i = 0; i < L; ++i) k.w[i] = __builtin_nontemporal_load(&p->w[i]);
    return k;
}

template <int L>
__device__ __forceinline__ void store_key(Key<L> *p, const Key<L> &k, bool nt) {
    if (nt) {
#pragma unroll
        for (int i = 0; i < L; ++i) __builtin_nontemporal_store(k.w[i], &p->w[i]);
    } else {
        *p = k;
    }
}

template <int L, bool HAS_VAL, int BLOCK = MSD_BLOCK, bool NT = false>
__global__ __launch_bounds__(BLOCK) void msd_partition_kernel(
    const Key<L> *__restrict__ kin, Key<L> *__restrict__ kout, const uint32_t *__restrict__ vin,
    uint32_t *__restrict__ vout, uint64_t n, unsigned nbits, unsigned b, unsigned bp,
    unsigned long long *__restrict__ cursor, unsigned cstride = 1,
    const unsigned long long *__restrict__ bend = nullptr, uint32_t *__restrict__ povf = nullptr,
    const uint32_t *__restrict__ tvalid = nullptr) {
    // tvalid (the speculative level-1 layout): tile t holds keys only in its first tvalid[t] positions
    // NT: nontemporal loads and stores (the streaming wide-digit pass: nothing it touches is
    // re-read from L2; measured 4.65 vs 4.67 ms on the cfg2 pass)
    // bend (speculative buckets, sized from a sample): a reservation past its bucket's end writes
    // nothing and raises *povf -- the caller then partitions again from the exact histogram
    constexpr int ITEMS = MsdTraits<L>::ITEMS;
    constexpr int TILE = ITEMS * BLOCK;
    constexpr int WMAX = MSD_WIN << 8;
    __shared__ Key<L> s_keys[TILE];
    __shared__ uint32_t s_vals[HAS_VAL ? TILE : 1];
    __shared__ uint32_t s_cnt[WMAX];
    __shared__ uint32_t s_loff[WMAX];
    __shared__ unsigned long long s_gbase[WMAX];
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];

    const uint32_t tid = threadIdx.x;
    const uint64_t tile = xcd_tile((n + TILE - 1) / TILE);  // grid = xcd_grid(tiles)
    if (tile * TILE >= n) return;
    const uint32_t tv = tvalid ? tvalid[tile] : (uint32_t)TILE;
    if (tv == 0) return;
    const uint64_t base = tile * TILE;
    const unsigned sub = b - bp;
    const uint32_t wsize = min((uint32_t)WMAX, (uint32_t)MSD_WIN << sub);  // 9-bit digits: one segment
    for (int i = tid; i < (int)wsize; i += BLOCK) s_cnt[i] = 0;
    const uint32_t wbase = key_prefix(kin[base], nbits, bp) << sub;
    __syncthreads();

    Key<L> k[ITEMS];
    uint32_t v[ITEMS];
    uint32_t r[ITEMS];
    bool have[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint64_t i = base + (uint64_t)j * BLOCK + tid;
        have[j] = i < n && (uint32_t)j * BLOCK + tid < tv;
        if (have[j]) {
            k[j] = load_key(kin + i, NT);
            if (HAS_VAL) v[j] = vin[i];
        }
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        r[j] = 0xFFFFFFFFu;
        if (have[j]) {
            const uint32_t lb = key_prefix(k[j], nbits, b) - wbase;
            if (lb < wsize) {
                r[j] = atomicAdd(&s_cnt[lb], 1u);
            } else {  // outside the window: reserve and write directly
                const unsigned long long o = atomicAdd(&cursor[(size_t)(lb + wbase) * cstride], 1ull);
                if (bend && o >= bend[lb + wbase]) {
                    *povf = 1u;
                } else {
                    kout[o] = k[j];
                    if (HAS_VAL) vout[o] = v[j];
                }
            }
        }
    }
    __syncthreads();
    // exclusive scan of the window counts (wsize <= 1024: two per thread)
    constexpr int PER = WMAX / BLOCK > 0 ? WMAX / BLOCK : 1;
    uint32_t c[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid * PER + q;
        c[q] = i < wsize ? s_cnt[i] : 0;
        sum += c[q];
    }
    uint32_t total;
    uint32_t off = block_exclusive_sum<BLOCK>(sum, s_scan, &total);
    // (round 5) the run reservations are issued here and consumed after the LDS scatter below, so their
    // round trip to the cursors overlaps the scatter
    unsigned long long gq[PER], be[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid * PER + q;
        gq[q] = 0, be[q] = 0;
        if (i < wsize) {
            s_loff[i] = off;
            if (c[q]) {
                gq[q] = atomicAdd(&cursor[(size_t)(wbase + i) * cstride], (unsigned long long)c[q]);
                if (bend) be[q] = bend[wbase + i];
            }
        }
        off += c[q];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        if (r[j] != 0xFFFFFFFFu) {
            const uint32_t lb = key_prefix(k[j], nbits, b) - wbase;
            const uint32_t pos = s_loff[lb] + r[j];
            s_keys[pos] = k[j];
            if (HAS_VAL) s_vals[pos] = v[j];
        }
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid * PER + q;
        if (i < wsize) {
            unsigned long long gb = gq[q];
            if (bend && c[q] && gb + c[q] > be[q]) {
                *povf = 1u;
                gb = ~0ull;  // this run is not written
            }
            s_gbase[i] = gb;
        }
    }
    __syncthreads();
    for (uint32_t p = tid; p < total; p += BLOCK) {
        const Key<L> key = s_keys[p];
        const uint32_t lb = key_prefix(key, nbits, b) - wbase;
        if (bend && s_gbase[lb] == ~0ull) continue;
        const uint64_t o = s_gbase[lb] + (p - s_loff[lb]);
        store_key(kout + o, key, NT);
        if (HAS_VAL) vout[o] = s_vals[p];
    }
}

// Group boundaries over buckets (buckets never split): bucket b opens a group when it crosses
// a multiple of G or when it or its predecessor holds more than G keys, so every big bucket is
// a group of its own (and can be processed in key-range slices).  flags[b] = 1 for openers.
__global__ void group_flags_kernel(const uint64_t *__restrict__ bstart, uint64_t nbuckets,
                                   uint64_t G, uint32_t *__restrict__ flags) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nbuckets) return;
    const uint64_t s0 = bstart[b], s1 = bstart[b + 1];
    uint32_t f = 0;
    if (s1 > s0) {  // empty buckets never open a group
        if (b == 0 || s0 == 0) {
            f = 1;
        } else {
            // previous non-empty bucket ends at s0; its start is the previous distinct start
            uint64_t p = b;
            uint64_t ps = s0;
            while (p > 0 && bstart[p - 1] == s0) --p;  // skip empty predecessors
            if (p > 0) ps = bstart[p - 1];
            f = (s0 / G != ps / G) || (s1 - s0 > G) || (s0 - ps > G);
        }
    }
    flags[b] = f;
}

// c[i] = a[i] + b[i] (bucket starts of two key sets -> starts of their union)
__global__ void add_starts_kernel(const uint64_t *__restrict__ a, const uint64_t *__restrict__ b, uint64_t n,
                                  uint64_t *__restrict__ c) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) c[i] = a[i] + b[i];
}

__global__ void group_scatter_kernel(const uint64_t *__restrict__ bstart,
                                     const uint32_t *__restrict__ flags,
                                     const uint64_t *__restrict__ pos, uint64_t nbuckets,
                                     uint64_t n, uint64_t *__restrict__ gstart,
                                     uint64_t *__restrict__ gbucket = nullptr) {
    // gbucket (optional): each group's first bucket; group 0 from bucket 0, the end = nbuckets
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nbuckets && flags[b]) {
        gstart[pos[b]] = bstart[b];
        if (gbucket) gbucket[pos[b]] = pos[b] == 0 ? 0 : b;
    }
    if (b == nbuckets) {
        gstart[pos[nbuckets]] = n;
        if (gbucket) gbucket[pos[nbuckets]] = nbuckets;
    }
}

/*
 * Sorted runs instead of partition passes: when the input is P sorted runs (the P slices a
 * rank receives in the multi-GPU exchange), the bucket layout of the top T bits follows from
 * one bucket index per run -- no histogram or partition pass.  runs_delta_kernel turns the
 * per-run indexes idx[j][b] (keys of run j below bucket b) into the global bucket starts and,
 * per (run, bucket), the shift from a key's run position to its bucket-major position (runs
 * in order inside a bucket); runs_gather_kernel then moves every key once, streaming.
 */
__global__ void runs_delta_kernel(const uint64_t *__restrict__ idx, uint32_t P, uint64_t nb,
                                  uint64_t *__restrict__ bstart, int64_t *__restrict__ delta) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b <= nb; b += stride) {
        uint64_t s = 0;
        for (uint32_t j = 0; j < P; ++j) s += idx[(uint64_t)j * (nb + 1) + b];
        bstart[b] = s;
        if (b == nb) continue;
        uint64_t o = s;
        for (uint32_t j = 0; j < P; ++j) {
            const uint64_t lo = idx[(uint64_t)j * (nb + 1) + b], hi = idx[(uint64_t)j * (nb + 1) + b + 1];
            delta[(uint64_t)j * nb + b] = (int64_t)o - (int64_t)lo;
            o += hi - lo;
        }
    }
}

template <int L, bool HAS_VAL>
__global__ __launch_bounds__(256) void runs_gather_kernel(const Key<L> *__restrict__ kin,
                                                          const uint32_t *__restrict__ vin, uint64_t n,
                                                          const uint64_t *__restrict__ roff, uint32_t P,
                                                          const int64_t *__restrict__ delta, uint64_t nb,
                                                          unsigned nbits, unsigned T, Key<L> *__restrict__ kout,
                                                          uint32_t *__restrict__ vout) {
    __shared__ uint64_t s_off[129];  // up to 128 runs (two arrays from 64 ranks)
    for (uint32_t j = threadIdx.x; j <= P; j += blockDim.x) s_off[j] = roff[j];
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint32_t j = 0;
        while (j + 1 < P && s_off[j + 1] <= i) ++j;
        const Key<L> k = kin[i];
        const uint32_t b = key_prefix(k, nbits, T);
        const uint64_t o = (uint64_t)((int64_t)(i - s_off[j]) + delta[(uint64_t)j * nb + b]);
        kout[o] = k;
        if (HAS_VAL) vout[o] = vin[i];
    }
}

template <int L>
struct LocalTraits {
    // hash slots per group: keys (+ state) (+ u32 counts) within the LDS budget
    static constexpr int SLOTS = L == 1 ? 8192 : L == 2 ? 4096 : 2048;
    static constexpr uint32_t LIMIT = SLOTS / 2;  // distinct keys per group (load <= 1/2)
};

template <int L>
__device__ __forceinline__ uint32_t key_hash(const Key<L> &k) {
    uint64_t h = k.w[0] * 0x9E3779B97F4A7C15ull;
#pragma unroll
    for (int i = 1; i < L; ++i) h ^= (k.w[i] + (h << 6) + (h >> 2)) * 0xC2B2AE3D27D4EB4Full;
    return (uint32_t)(h >> 32);
}

// a 32-bit hash onto [0, N): a mask for a power of two, else the high half of hash * N.  (A 3072-slot
// table with 384-thread workgroups -- 5 groups per CU instead of 4 -- measured slower for the configs[1]
// sort: 11.5 vs 10.4 ms sort stage; so was a persistent kernel loading the next group's keys while
// the current group sorts: 12.3-14.2 ms for 2-4 workgroups per CU.)
template <int N>
__device__ __forceinline__ uint32_t slot_of(uint32_t h) {
    if constexpr ((N & (N - 1)) == 0) return h & (N - 1);
    else return (uint32_t)(((uint64_t)h * (uint64_t)N) >> 32);
}

// atomicMax of a block-uniform LDS word from every lane, reduced over the wave first so that one lane
// issues the atomic: a uniform-address atomic from all lanes becomes the atomic optimizer's lane-by-
// lane loop (~5 scalar instructions per active lane; 0.8 ms of local_unique_kernel and 0.5 ms of
// local_merge_kernel at configs[1]).  Every lane of the wave must call it.
__device__ __forceinline__ void wave_atomic_max(int *p, int v) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    if (__lane_id() == 0 && v >= 0) atomicMax(p, v);
}

// index of the highest set bit of a key (-1 for zero)
template <int L>
__device__ __forceinline__ int key_msb(const Key<L> &k) {
    int r = -1;
#pragma unroll
    for (int i = 0; i < L; ++i)
        if (k.w[i]) r = 64 * i + 63 - __clzll((long long)k.w[i]);
    return r;
}

/*
 * One workgroup per group [gstart[g], gstart[g+1]):
 *   1. LDS open-addressing hash of the group's keys.  KEYCAS: the key word itself is CASed
 *      against an EMPTY sentinel no key can take (top bit of a 64-bit word whose significant
 *      range is narrower); otherwise a per-slot state word is claimed (0 -> 1), the key stored
 *      and the state published (-> 2).  Counts add with saturation (sorted_multiset.cpp:66-83).
 *   2. The D distinct keys are compacted; min/max give the highest bit in which they differ;
 *      a counting sort on the 8 bits below it splits them into 256 ordered sub-buckets; each
 *      key's final slot is its sub-bucket start + the number of smaller keys in its sub-bucket.
 *   3. Keys (and counts) go to tmp[gstart[g] + slot]; ucount[g] = D.
 * More than LIMIT distinct keys -> overflow[g] = 1 (the host finishes the group otherwise).
 */
// waves per SIMD the uncounted local_unique_kernel is compiled for (its VGPR budget: 512 / MTG_LU_WPE)
#ifndef MTG_LU_WPE
#define MTG_LU_WPE 8
#endif
// SLICED: the launch may pass sbits > 0 (the sliced reruns); false compiles the key-range slice test
// out of the per-key loop (the first launch and the speculative level's)
template <int L, bool COUNTED, bool KEYCAS, int LB = 512, int SL = LocalTraits<L>::SLOTS,
          bool NODUP = false, int WPE = (L == 1 && KEYCAS && !NODUP && !COUNTED) ? MTG_LU_WPE : 1, bool FAST = false,
          bool SLICED = true>
__global__ __launch_bounds__(LB) __attribute__((amdgpu_waves_per_eu(WPE))) void local_unique_kernel(
    const Key<L> *__restrict__ keys, const uint32_t *__restrict__ vals,
    const uint64_t *__restrict__ gstart, const uint32_t *__restrict__ glist, unsigned nbits,
    unsigned b, unsigned sbits_, Key<L> *__restrict__ tmp, uint32_t *__restrict__ tcnt,
    uint32_t *__restrict__ ucount, uint32_t *__restrict__ overflow, uint32_t *__restrict__ novf,
    uint32_t cmax, const unsigned long long *__restrict__ gend = nullptr, uint64_t g_base = 0) {
    // gend (speculative buckets): group g is [gstart[g], gend[g]), with gaps between groups; g_base: the
    // first group of this launch (a grid holds < 2^32 work-items, so 2^23+ buckets launch in pieces)
    constexpr int SLOTS = SL;
    constexpr uint32_t LIMIT = SL / 2;
    constexpr uint64_t EMPTY = ~0ull;
    // LIST: every new key records its slot (insertion order), so compaction gathers D slots
    // instead of scanning all SLOTS (and needs no block scan)
    constexpr bool LIST = KEYCAS && !NODUP;
    __shared__ Key<L> s_key[SLOTS];
    __shared__ uint16_t s_slot[LIST ? LIMIT : 1];
    // FAST (LIST only): a batch's loads without per-key bounds when the whole batch lies in the
    // group, and the batch's new keys take their list positions from the wave's ballots (no LDS) with
    // one LDS atomic per wave and batch, instead of an LDS atomic + an LDS broadcast (ds_bpermute) per
    // key slot.  The kernel's LDS pipe is its busiest (SQ_ACTIVE_INST_LDS ~ one wave per CU at all
    // times at configs[1]), so LDS instructions are what this variant removes.
    static_assert(!FAST || (LIST && (SL & (SL - 1)) == 0), "FAST is the LIST path, power-of-two tables");
    __shared__ uint32_t s_state[KEYCAS ? 1 : SLOTS];
    __shared__ uint32_t s_sum[COUNTED ? SLOTS : 1];
    __shared__ uint32_t s_hist[256];
    __shared__ uint32_t s_fill[256];
    __shared__ uint32_t s_distinct;
    __shared__ uint32_t s_scan[LB / 64 + 1];
    __shared__ int s_hb;

    const uint64_t g = glist ? glist[blockIdx.x] : g_base + blockIdx.x;
    const uint64_t g0 = gstart[g], g1 = gend ? (uint64_t)gend[g] : gstart[g + 1];
    const uint32_t tid = threadIdx.x;
    if (g0 >= g1) {
        if (tid == 0) ucount[g] = 0;
        return;
    }
    // slices: keys split by the sbits bits right below the b-bit bucket prefix; only valid for
    // a group made of one bucket (several buckets would interleave)
    const unsigned sbits = SLICED ? sbits_ : 0u;
    const unsigned sshift = nbits - b - sbits;
    if (sbits && key_prefix(keys[g0], nbits, b) != key_prefix(keys[g1 - 1], nbits, b)) {
        if (tid == 0) {
            overflow[g] = 1;
            atomicAdd(novf, 1u);
        }
        return;
    }
    uint64_t out_off = 0;
    for (uint32_t slice = 0; slice < (1u << sbits); ++slice) {
        if (!NODUP) {
            for (int i = tid; i < SLOTS; i += LB) {
                if (KEYCAS) s_key[i].w[0] = EMPTY;
                else s_state[i] = 0;
                if (COUNTED) s_sum[i] = 0;
            }
        }
        if (tid < 256) {
            s_hist[tid] = 0;
            s_fill[tid] = 0;
        }
        if (tid == 0) {
            s_distinct = 0;
            s_hb = -1;
        }
        __syncthreads();

        bool ovf = false;
        uint32_t mynew = 0;  // distinct keys this thread inserted (summed once per thread)
        // keys are loaded BATCH at a time per thread so the global loads overlap; 8-byte keys
        // as 16-byte pairs from the even index at or below g0
        constexpr int PAIR = L == 1 ? 2 : 1;
        // keys per thread and load batch: 4 at 64 VGPRs (6: 4.47 -> 4.19 ms in round 3; 4: sort stage
        // 8.56 -> 8.29-8.38 ms in round 4, the 6-key batch spilled 16-20 bytes per lane to scratch);
        // MTG_LU_BATCH overrides it at build time for A/B runs
#ifdef MTG_LU_BATCH
        constexpr int BATCH = (KEYCAS && !COUNTED && !NODUP ? MTG_LU_BATCH : (LB >= 1024 ? 12 : WPE >= 6 ? 4 : 8)) / PAIR;
#else
        constexpr int BATCH = (LB >= 1024 ? 12 : WPE >= 6 ? 4 : 8) / PAIR;
#endif
        const uint64_t a0 = PAIR == 2 ? (g0 & ~1ull) : g0;
        for (uint64_t ib = a0 + (uint64_t)tid * PAIR; ib < g1 && !ovf; ib += (uint64_t)LB * BATCH * PAIR) {
            Key<L> kb[BATCH * PAIR];
            uint32_t vb[BATCH * PAIR];
            bool hv[BATCH * PAIR];
            if (FAST && ib >= g0 && ib + (uint64_t)(BATCH - 1) * LB * PAIR + PAIR <= g1) {
#pragma unroll
                for (int q = 0; q < BATCH; ++q) {
                    const uint64_t i = ib + (uint64_t)q * LB * PAIR;
                    if constexpr (PAIR == 2) {
                        const ulonglong2 kv = *(const ulonglong2 *)(keys + i);
                        kb[2 * q] = Key<L>::from(kv.x);
                        kb[2 * q + 1] = Key<L>::from(kv.y);
                        hv[2 * q] = hv[2 * q + 1] = true;
                        if (COUNTED) {
                            const uint2 vv = *(const uint2 *)(vals + i);
                            vb[2 * q] = vv.x;
                            vb[2 * q + 1] = vv.y;
                        }
                    } else {
                        kb[q] = keys[i];
                        hv[q] = true;
                        if (COUNTED) vb[q] = vals[i];
                    }
                }
            } else
#pragma unroll
            for (int q = 0; q < BATCH; ++q) {
                const uint64_t i = ib + (uint64_t)q * LB * PAIR;
                if constexpr (PAIR == 2) {
                    hv[2 * q] = i >= g0 && i < g1;
                    hv[2 * q + 1] = i + 1 < g1;
                    if (i + 1 < g1) {
                        const ulonglong2 kv = *(const ulonglong2 *)(keys + i);
                        kb[2 * q] = Key<L>::from(kv.x);
                        kb[2 * q + 1] = Key<L>::from(kv.y);
                        if (COUNTED) {
                            const uint2 vv = *(const uint2 *)(vals + i);
                            vb[2 * q] = vv.x;
                            vb[2 * q + 1] = vv.y;
                        }
                    } else if (i < g1 && i >= g0) {
                        kb[2 * q] = keys[i];
                        if (COUNTED) vb[2 * q] = vals[i];
                    }
                } else {
                    hv[q] = i < g1;
                    if (i < g1) {
                        kb[q] = keys[i];
                        if (COUNTED) vb[q] = vals[i];
                    }
                }
            }
            if constexpr (NODUP) {
                // distinct input (the rc set): append the slice's keys, positions by wave ballot
                const uint32_t lane = __lane_id();
#pragma unroll
                for (int q = 0; q < BATCH * PAIR; ++q) {
                    const bool act = hv[q] && (!SLICED || !sbits || bits_at(kb[q], sshift, sbits) == slice);
                    const uint64_t m = __ballot(act);
                    if (!m) continue;
                    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1;
                    uint32_t wb = 0;
                    if (lane == leader) wb = atomicAdd(&s_distinct, (uint32_t)__popcll(m));
                    wb = __shfl(wb, leader, 64);
                    const uint32_t pos = wb + popc_below(m);
                    if (act) {
                        if (pos < LIMIT) {
                            s_key[pos] = kb[q];
                            if (COUNTED) s_sum[pos] = vb[q];
                        } else {
                            ovf = true;
                        }
                    }
                }
                continue;
            }
            // (issuing the first-probe CASes of all the thread's keys back to back, one LDS round trip per
            // batch instead of a chain per key, measured slower: 11.4 vs 10.5 ms sort stage, the
            // in-flight results spill at 64 VGPRs; 10.6 ms with 4-key batches)
            constexpr int NQ = BATCH * PAIR;
            uint32_t dpos[FAST ? NQ : 1];  // FAST: (position in the batch << 16 | slot), ~0 = not new
            uint32_t wnew = 0;             // FAST: new keys of the wave in this batch so far (uniform)
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                // LIST: the new keys of a wave take their list positions by ballot after the probe
                // loop, one LDS atomic per wave (an atomicAdd on s_distinct from the inserting lanes
                // is the atomic optimizer's lane-by-lane loop: ~5 SALU per new key)
                int32_t ins = -1;
                if (hv[q] && !ovf && (!SLICED || !sbits || bits_at(kb[q], sshift, sbits) == slice)) {
                const Key<L> key = kb[q];
                uint32_t h = slot_of<SLOTS>(key_hash(key));
                for (uint32_t probes = 0;;) {
                    if (KEYCAS) {
                        // (a plain LDS read of the slot before the CAS -- most keys are repeats that
                        // find themselves in their first slot -- measured 0.2-0.3 ms slower per step)
                        const uint64_t old = atomicCAS((unsigned long long *)&s_key[h].w[0],
                                                       (unsigned long long)EMPTY,
                                                       (unsigned long long)key.w[0]);
                        if (old == EMPTY) {
                            if (LIST) ins = (int32_t)h;
                            else ++mynew;
                            break;
                        }
                        if (old == key.w[0]) break;
                    } else {
                        const uint32_t st = atomicCAS(&s_state[h], 0u, 1u);
                        if (st == 0) {
                            s_key[h] = key;
                            __atomic_store_n(&s_state[h], 2u, __ATOMIC_RELEASE);
                            ++mynew;
                            break;
                        }
                        if (st != 2 && __atomic_load_n(&s_state[h], __ATOMIC_ACQUIRE) != 2) continue;
                        if (s_key[h] == key) break;
                    }
                    h = h + 1 == SLOTS ? 0 : h + 1;
                    if (++probes >= SLOTS) {
                        ovf = true;
                        break;
                    }
                }
                if (COUNTED && !ovf) {
                    const uint32_t add = vb[q];
                    if (cmax <= 0xFFFFu) {
                        // 8/16-bit containers: a plain add, clamped on output; a sum past 2^30 is
                        // pulled back to cmax at once, so it never wraps (every add is <= cmax)
                        const uint32_t o = atomicAdd(&s_sum[h], add);
                        if (o + add > 0x40000000u) atomicMin(&s_sum[h], cmax);
                    } else {
                        uint32_t old = s_sum[h], assumed;
                        do {
                            assumed = old;
                            const uint32_t nv = assumed > cmax - add ? cmax : assumed + add;
                            old = atomicCAS(&s_sum[h], assumed, nv);
                        } while (old != assumed);
                    }
                }
                }
                if constexpr (FAST) {
                    // deferred list positions: this key's rank among the batch's new keys of the wave
                    // (ballots and popcounts, no LDS); one LDS atomic per wave and batch below
                    const uint64_t m = __ballot(ins >= 0);
                    dpos[q] = ins >= 0 ? ((wnew + popc_below(m)) << 16 | (uint32_t)ins) : ~0u;
                    wnew += (uint32_t)__popcll(m);
                } else if constexpr (LIST) {
                    const uint64_t m = __ballot(ins >= 0);
                    if (m) {
                        const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1;
                        uint32_t wb = 0;
                        if (__lane_id() == leader) wb = atomicAdd(&s_distinct, (uint32_t)__popcll(m));
                        wb = __shfl(wb, leader, 64);
                        const uint32_t pos = wb + popc_below(m);
                        if (ins >= 0) {
                            if (pos < LIMIT) s_slot[pos] = (uint16_t)ins;
                            else ovf = true;
                        }
                    }
                }
            }
            if constexpr (FAST) {
                if (wnew) {  // the batch's new keys of the wave: one LDS atomic, positions known
                    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)__ballot(1)) - 1;
                    uint32_t wb = 0;
                    if (__lane_id() == leader) wb = atomicAdd(&s_distinct, wnew);
                    wb = (uint32_t)__builtin_amdgcn_readlane((int)wb, (int)leader);
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        if (dpos[q] != ~0u) {
                            const uint32_t pos = wb + (dpos[q] >> 16);
                            if (pos < LIMIT) s_slot[pos] = (uint16_t)(dpos[q] & 0xFFFFu);
                            else ovf = true;
                        }
                    }
                }
            }
        }
        {  // one atomic per wave (see wave_atomic_max)
            uint32_t t = mynew;
#pragma unroll
            for (int o = 32; o; o >>= 1) t += __shfl_xor(t, o, 64);
            if (__lane_id() == 0 && t) atomicAdd(&s_distinct, t);
        }
        if (__syncthreads_or(ovf) || s_distinct > LIMIT) {
            if (tid == 0) {
                overflow[g] = 1;
                ucount[g] = 0;
                atomicAdd(novf, 1u);
            }
            return;
        }
        const uint32_t D = s_distinct;

        if constexpr (LIST) {
            // gather the D recorded slots, then write them compacted to s_key[0..D)
            constexpr int PERL = (LIMIT + LB - 1) / LB;
            Key<L> kk[PERL];
            uint32_t ss[PERL];
#pragma unroll
            for (int q = 0; q < PERL; ++q) {
                const uint32_t i = tid + q * LB;
                if (i < D) {
                    const uint32_t sl = s_slot[i];
                    kk[q] = s_key[sl];
                    if (COUNTED) ss[q] = s_sum[sl];
                }
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < PERL; ++q) {
                const uint32_t i = tid + q * LB;
                if (i < D) {
                    s_key[i] = kk[q];
                    if (COUNTED) s_sum[i] = ss[q];
                }
            }
            __syncthreads();
            if (D) {
                const Key<L> ref = s_key[0];
                int hb_local = -1;
#pragma unroll
                for (int q = 0; q < PERL; ++q) {
                    if (tid + q * LB < D) {
                        Key<L> dx;
#pragma unroll
                        for (int w = 0; w < L; ++w) dx.w[w] = kk[q].w[w] ^ ref.w[w];
                        hb_local = max(hb_local, key_msb(dx));
                    }
                }
                wave_atomic_max(&s_hb, hb_local);
            }
            __syncthreads();
        } else if constexpr (NODUP) {
            // already compact: highest differing bit over s_key[0..D)
            if (D) {
                const Key<L> ref = s_key[0];
                int hb_local = -1;
                for (uint32_t i = tid; i < D; i += LB) {
                    Key<L> dx;
#pragma unroll
                    for (int w = 0; w < L; ++w) dx.w[w] = s_key[i].w[w] ^ ref.w[w];
                    hb_local = max(hb_local, key_msb(dx));
                }
                wave_atomic_max(&s_hb, hb_local);
            }
            __syncthreads();
        } else {
        // compact occupied slots to s_key[0..D) / s_sum[0..D)
        constexpr int PER = SLOTS / LB;
        Key<L> kk[PER];
        uint32_t ss[PER];
        uint32_t mine = 0, occ = 0;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int slot = tid * PER + q;
            kk[q] = s_key[slot];
            if (COUNTED) ss[q] = s_sum[slot];
            const bool o = KEYCAS ? kk[q].w[0] != EMPTY : s_state[slot] == 2;
            occ |= (uint32_t)o << q;
            mine += o;
        }
        uint32_t tot;
        uint32_t o = block_exclusive_sum<LB>(mine, s_scan, &tot);
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            if (occ & (1u << q)) {
                s_key[o] = kk[q];
                if (COUNTED) s_sum[o] = ss[q];
                ++o;
            }
        }
        __syncthreads();
        // highest bit in which the slice's keys differ = max over keys of msb(key ^ s_key[0])
        if (D) {
            const Key<L> ref = s_key[0];
            int hb_local = -1;
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                if (occ & (1u << q)) {
                    Key<L> dx;
#pragma unroll
                    for (int i = 0; i < L; ++i) dx.w[i] = kk[q].w[i] ^ ref.w[i];
                    hb_local = max(hb_local, key_msb(dx));
                }
            }
            wave_atomic_max(&s_hb, hb_local);
        }
        __syncthreads();
        }
        const int hb = s_hb;
        const unsigned dshift = hb >= 7 ? (unsigned)(hb - 7) : 0u;
        Key<L> *scratch = s_key + LIMIT;  // free half of the table
        uint32_t *sscr = COUNTED ? s_sum + LIMIT : nullptr;
        for (uint32_t i = tid; i < D; i += LB) atomicAdd(&s_hist[bits_at(s_key[i], dshift, 8)], 1u);
        __syncthreads();
        if (tid < 64) {  // exclusive scan of the 256 counts by one wave (4 per lane)
            const uint32_t c0 = s_hist[4 * tid], c1 = s_hist[4 * tid + 1], c2 = s_hist[4 * tid + 2],
                           c3 = s_hist[4 * tid + 3];
            const uint32_t sum4 = c0 + c1 + c2 + c3;
            const uint32_t bb = wave_inclusive_sum(sum4) - sum4;
            s_hist[4 * tid] = bb;
            s_hist[4 * tid + 1] = bb + c0;
            s_hist[4 * tid + 2] = bb + c0 + c1;
            s_hist[4 * tid + 3] = bb + c0 + c1 + c2;
        }
        __syncthreads();
        for (uint32_t i = tid; i < D; i += LB) {
            const uint32_t d = bits_at(s_key[i], dshift, 8);
            const uint32_t p = s_hist[d] + atomicAdd(&s_fill[d], 1u);
            scratch[p] = s_key[i];
            if (COUNTED) sscr[p] = s_sum[i];
        }
        __syncthreads();
        // (a 9-bit counting sort -- half the sub-bucket scans, its fill counters in the gathered slot list's
        // words -- measured even, 7.90-7.94 vs 7.94-7.96 ms sort stage in round 6; 10 bits cost occupancy:
        // 8.57 ms)
        // (staging the sorted run in LDS for one coalesced store halves the HBM write bytes -- PMC
        // WRITE_SIZE 2.89 GB for 1.5 GB of keys stored one by one at their ranks -- but the extra
        // barrier cost more: sort stage 10.5 -> 11.0 ms)
        for (uint32_t p = tid; p < D; p += LB) {
            const Key<L> key = scratch[p];
            const uint32_t d = bits_at(key, dshift, 8);
            const uint32_t b0 = s_hist[d], b1 = b0 + s_fill[d];
            uint32_t rank = 0;
            for (uint32_t j = b0; j < b1; ++j) rank += scratch[j] < key;
            tmp[g0 + out_off + b0 + rank] = key;
            if (COUNTED) tcnt[g0 + out_off + b0 + rank] = min(sscr[p], cmax);
        }
        out_off += D;
        __syncthreads();  // the next slice reuses the table
    }
    if (tid == 0) {
        ucount[g] = (uint32_t)out_off;
        overflow[g] = 0;
    }
}

/*
 * The reverse-complement sort's local pass fused with the merge into the real edges
 * (add_reverse_complements, boss_chunk_construct.cpp:179-222): one workgroup per group of the rc
 * partition sorts the group's rc keys in LDS (distinct input: the counting sort + rank of
 * local_unique_kernel<NODUP>), merges them with the canonical keys of the same bucket range
 * (cstart: bucket index of the sorted canonical set over the same top b bits), and writes the
 * merged run at its final place: the canonical keys before the range + the rc keys before the
 * group.  A group or range over CAP keys sets *ovf and the caller takes the unfused path.
 */
template <int L>
struct MergeLocalTraits {
    // keys per LDS array (3 arrays): a u64 group of the configs[1] rc sort holds ~710 rc + ~710
    // canonical keys (up to ~1420 where either strand is twice as dense), so 1536-key arrays (36 KB,
    // 4 workgroups per CU) instead of 2048 (48 KB, 3 per CU): rc stage 5.9 -> 5.5 ms; the few larger
    // groups rerun with twice the arrays (1280: 6.4 ms, too many reruns)
    static constexpr int CAP = L == 1 ? 1536 : L == 2 ? 1024 : 512;
};

// CAP: keys per LDS array; glist (optional): the groups to run (the big-CAP rerun of the groups
// the first launch listed); *ovf counts groups left over, and gflag (optional) receives their ids at
// gflag[0 .. *ovf) in any order -- the rerun's glist, no flag array to scan on the host
template <int L, bool COUNTED, int CAP, int LB = 512>
__global__ __launch_bounds__(LB) void local_merge_kernel(
    const Key<L> *__restrict__ keys, const uint32_t *__restrict__ vals, const uint64_t *__restrict__ gstart,
    const uint64_t *__restrict__ gbucket, const uint32_t *__restrict__ glist, const Key<L> *__restrict__ ck,
    const uint32_t *__restrict__ cv, const uint64_t *__restrict__ cstart, Key<L> *__restrict__ out,
    uint32_t *__restrict__ outc, uint32_t *__restrict__ gflag, uint32_t *__restrict__ ovf,
    unsigned b, unsigned nbits, unsigned ib, uint64_t *__restrict__ istart,
    const unsigned long long *__restrict__ gend = nullptr, const uint64_t *__restrict__ gbase = nullptr,
    const uint64_t *__restrict__ cgap = nullptr, uint64_t g_base = 0, uint32_t it_min = 1) {
    // cgap (optional, one bucket per group): the canonical keys of bucket g are read at ck[cgap[g] ..)
    // (a set left in its speculative buckets) instead of ck[cstart[g] ..); cstart stays their compact
    // index
    // istart (optional): the bucket index over the top ib >= b bits of the merged output that the
    // dummy stage uses (bucket_index_kernel's layout); the group fills the entries of its range.
    // gend (speculative buckets, one per group, gbucket == nullptr): the group's rc keys are
    // [gstart[g], gend[g]) with gaps between groups, and gbase[g] counts the rc keys before it
    __shared__ Key<L> s_r[CAP];  // rc keys, then sorted
    __shared__ Key<L> s_s[CAP];  // rc keys by sub-bucket
    __shared__ Key<L> s_c[CAP];  // canonical keys of the range
    __shared__ uint32_t s_rv[COUNTED ? CAP : 1], s_sv[COUNTED ? CAP : 1], s_cv[COUNTED ? CAP : 1];
    __shared__ uint32_t s_hist[256], s_fill[256];
    // index gaps longer than IGAP entries between two consecutive outputs, filled by the whole workgroup
    // after the merge (a thread filling them alone serialized groups that span many sparse buckets: an
    // 8-rank super-k-mer build's rc merge took 0.1-0.8 s per launch)
    constexpr uint32_t IGAP = 64, NGAP = 64;
    __shared__ uint32_t s_glo[NGAP], s_ghi[NGAP], s_go[NGAP];
    __shared__ uint32_t s_gn;
    const uint32_t tid = threadIdx.x;
    const uint64_t g = glist ? glist[blockIdx.x] : g_base + blockIdx.x;
    const uint64_t g0 = gstart[g], g1 = gend ? (uint64_t)gend[g] : gstart[g + 1];
    const uint64_t gb0 = gbucket ? gbucket[g] : g, gb1 = gbucket ? gbucket[g + 1] : g + 1;
    const uint64_t c0 = cstart[gb0], c1 = cstart[gb1];
    if (g1 - g0 > (uint64_t)CAP || c1 - c0 > (uint64_t)CAP) {
        if (tid == 0) {  // appended to the overflow list (one entry a group at most: room for every group)
            const uint32_t p = atomicAdd(ovf, 1u);
            if (gflag) gflag[p] = (uint32_t)g;
        }
        return;
    }
    const uint32_t nr = (uint32_t)(g1 - g0), nc = (uint32_t)(c1 - c0);
    if (nr == 0 && nc == 0) {
        // an empty bucket range (most of them on a rank of a multi-GPU build, whose keys fill 1/P of the
        // buckets): its index entries only, no table setup and no barriers
        if (istart) {
            const uint64_t base = c0 + (gbase ? gbase[g] : g0);
            const uint64_t ifirst = gb0 << (ib - b), iend = gb1 << (ib - b);
            for (uint64_t x = ifirst + tid; x < iend; x += LB) istart[x] = base;
        }
        return;
    }
    // (round 5) the group's rc keys stay in registers until their counting sort scatters them (no raw copy
    // in LDS, one barrier fewer); the wave maxima of their highest differing bit go to per-wave words
    constexpr int PR = (CAP + LB - 1) / LB;
    constexpr int NWV = LB / 64;
    __shared__ int s_wmax[NWV];
    Key<L> rk[PR];
    uint32_t rv[PR];
#pragma unroll
    for (int q = 0; q < PR; ++q) {
        const uint32_t i = tid + q * LB;
        rk[q] = Key<L>::zero();  // (defined on every lane: a partly written key array went to scratch)
        if (i < nr) {
            rk[q] = keys[g0 + i];
            if (COUNTED) rv[q] = vals[g0 + i];
        }
    }
    const uint64_t cr = cgap ? cgap[gb0] : c0;
    if constexpr (L <= 2) {
        // the canonical keys' loads all in flight with the rc keys' before the LDS stores (a rolled loop
        // waited for each load before issuing the next; u64 and u128 keys -- PR = 2 for u128 -- the wider
        // ones' registers spill)
        Key<L> ckr[PR];
        uint32_t cvr[PR];
#pragma unroll
        for (int q = 0; q < PR; ++q) {
            const uint32_t i = tid + q * LB;
            ckr[q] = Key<L>::zero();
            if (i < nc) {
                ckr[q] = ck[cr + i];
                if (COUNTED) cvr[q] = cv[cr + i];
            }
        }
#pragma unroll
        for (int q = 0; q < PR; ++q) {
            const uint32_t i = tid + q * LB;
            if (i < nc) {
                s_c[i] = ckr[q];
                if (COUNTED) s_cv[i] = cvr[q];
            }
        }
    } else {
        for (uint32_t i = tid; i < nc; i += LB) {
            s_c[i] = ck[cr + i];
            if (COUNTED) s_cv[i] = cv[cr + i];
        }
    }
    if (tid < 256) {
        s_hist[tid] = 0;
        s_fill[tid] = 0;
    }
    if (tid == 0) s_gn = 0;
    {
        int hb_local = -1;
        if (nr) {
            const Key<L> ref = keys[g0];  // the same key for every lane
#pragma unroll
            for (int q = 0; q < PR; ++q) {
                if (tid + q * LB < nr) {
                    Key<L> dx;
#pragma unroll
                    for (int w = 0; w < L; ++w) dx.w[w] = rk[q].w[w] ^ ref.w[w];
                    hb_local = max(hb_local, key_msb(dx));
                }
            }
        }
#pragma unroll
        for (int o = 32; o; o >>= 1) hb_local = max(hb_local, __shfl_xor(hb_local, o, 64));
        if (__lane_id() == 0) s_wmax[tid >> 6] = hb_local;
    }
    __syncthreads();
    int hb = -1;
#pragma unroll
    for (int w = 0; w < NWV; ++w) hb = max(hb, s_wmax[w]);
    const unsigned dshift = hb >= 7 ? (unsigned)(hb - 7) : 0u;
#pragma unroll
    for (int q = 0; q < PR; ++q)
        if (tid + q * LB < nr) atomicAdd(&s_hist[bits_at(rk[q], dshift, 8)], 1u);
    __syncthreads();
    if (tid < 64) {
        const uint32_t a0 = s_hist[4 * tid], a1 = s_hist[4 * tid + 1], a2 = s_hist[4 * tid + 2], a3 = s_hist[4 * tid + 3];
        const uint32_t sum4 = a0 + a1 + a2 + a3;
        const uint32_t bb = wave_inclusive_sum(sum4) - sum4;
        s_hist[4 * tid] = bb;
        s_hist[4 * tid + 1] = bb + a0;
        s_hist[4 * tid + 2] = bb + a0 + a1;
        s_hist[4 * tid + 3] = bb + a0 + a1 + a2;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PR; ++q) {
        if (tid + q * LB < nr) {
            const uint32_t d = bits_at(rk[q], dshift, 8);
            const uint32_t p = s_hist[d] + atomicAdd(&s_fill[d], 1u);
            s_s[p] = rk[q];
            if (COUNTED) s_sv[p] = rv[q];
        }
    }
    __syncthreads();
    for (uint32_t p = tid; p < nr; p += LB) {
        const Key<L> key = s_s[p];
        const uint32_t d = bits_at(key, dshift, 8);
        const uint32_t b0 = s_hist[d], b1 = b0 + s_fill[d];
        uint32_t rank = 0;
        for (uint32_t j = b0; j < b1; ++j) rank += s_s[j] < key;
        s_r[b0 + rank] = key;
        if (COUNTED) s_rv[b0 + rank] = s_sv[p];
    }
    __syncthreads();
    // merge path over (s_r[0..nr), s_c[0..nc)): thread t writes outputs [t * IT, (t + 1) * IT).  it_min:
    // at least that many outputs a thread (fewer diagonal searches of ~11 LDS steps, longer serial runs)
    const uint32_t n = nr + nc;
    const uint32_t IT = max((n + LB - 1) / LB, it_min);
    const uint32_t o0 = min(tid * IT, n), o1 = min(o0 + IT, n);
    uint32_t lo = o0 > nc ? o0 - nc : 0, hi = min(o0, nr);
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_r[mid] < s_c[o0 - mid - 1]) lo = mid + 1; else hi = mid;
    }
    uint32_t i = lo, j = o0 - lo;
    const uint64_t base = c0 + (gbase ? gbase[g] : g0);
    const unsigned ishift = nbits - ib;
    // index bucket of the output before o0 (or the first bucket of the group's range - 1)
    const uint64_t ifirst = gb0 << (ib - b), iend = gb1 << (ib - b);
    uint64_t prevb = ifirst - 1;
    if (istart && o0 > 0 && o0 < o1) {
        const uint32_t pi = lo, pj = o0 - lo;  // the merged element o0 - 1
        const bool pr = pi > 0 && (pj == 0 || s_c[pj - 1] < s_r[pi - 1]);
        prevb = bits_at(shr(pr ? s_r[pi - 1] : s_c[pj - 1], ishift), 0, 32);
    }
    // (round 5) the two run heads stay in registers: one LDS read a step (the consumed side's next key,
    // from a selected address) and no branches around the comparison -- the step read both heads and
    // then the taken one again, under two nested exec masks
    Key<L> ha = s_r[min(i, (uint32_t)CAP - 1)], hc = s_c[min(j, (uint32_t)CAP - 1)];
    for (uint32_t o = o0; o < o1; ++o) {
        const bool take_r = (i < nr) & ((j >= nc) | (ha < hc));  // (no short-circuit: no exec mask)
        // (limb by limb: a select of whole u128 keys went through scratch memory -- the two heads stored,
        // the taken one reloaded by address, every output key)
        Key<L> key;
#pragma unroll
        for (int w = 0; w < L; ++w) key.w[w] = take_r ? ha.w[w] : hc.w[w];
        out[base + o] = key;
        if (COUNTED) outc[base + o] = *(take_r ? s_rv + i : s_cv + j);
        i += take_r ? 1u : 0u;
        j += take_r ? 0u : 1u;
        const Key<L> nx = *(take_r ? s_r + min(i, (uint32_t)CAP - 1) : s_c + min(j, (uint32_t)CAP - 1));
#pragma unroll
        for (int w = 0; w < L; ++w) {
            ha.w[w] = take_r ? nx.w[w] : ha.w[w];
            hc.w[w] = take_r ? hc.w[w] : nx.w[w];
        }
        if (istart) {
            const uint64_t kb = bits_at(shr(key, ishift), 0, 32);
            uint32_t q = NGAP;
            if (kb > prevb + IGAP && kb - ifirst < 0xFFFFFFFFull) q = atomicAdd(&s_gn, 1u);
            if (q < NGAP) {
                s_glo[q] = (uint32_t)(prevb + 1 - ifirst);
                s_ghi[q] = (uint32_t)(kb - ifirst);
                s_go[q] = o;
            } else {
                for (uint64_t x = prevb + 1; x <= kb; ++x) istart[x] = base + o;
            }
            prevb = kb;
        }
    }
    if (istart) {  // the long gaps, by the whole workgroup
        __syncthreads();
        const uint32_t ng = min(s_gn, NGAP);
        for (uint32_t q = 0; q < ng; ++q)
            for (uint64_t x = ifirst + s_glo[q] + tid; x <= ifirst + s_ghi[q]; x += LB) istart[x] = base + s_go[q];
    }
    if (istart) {  // after the group's last key, up to the end of its range
        uint64_t lastb = ifirst - 1;
        if (n) {
            const Key<L> lk = nr && (nc == 0 || s_c[nc - 1] < s_r[nr - 1]) ? s_r[nr - 1] : s_c[nc - 1];
            lastb = bits_at(shr(lk, ishift), 0, 32);
        }
        for (uint64_t x = lastb + 1 + tid; x < iend; x += LB) istart[x] = base + n;
    }
}

// copy every group's distinct keys from tmp[gstart[g]..] to out[ustart[g]..].  istart (optional):
// the bucket index of out over the top bits of the keys above ishift (bucket_index_kernel's layout),
// each group filling the entries of its buckets [gbucket[g], gbucket[g + 1]) as it copies -- the
// fused rc merge then needs no bucket_index pass over the canonical keys
template <int L, bool COUNTED>
__global__ __launch_bounds__(256) void group_gather_kernel(
    const Key<L> *__restrict__ tmp, const uint32_t *__restrict__ tcnt,
    const uint64_t *__restrict__ gstart, const uint64_t *__restrict__ ustart,
    Key<L> *__restrict__ out, uint32_t *__restrict__ ocnt, const uint64_t *__restrict__ gbucket = nullptr,
    unsigned ishift = 0, uint64_t *__restrict__ istart = nullptr, uint32_t *__restrict__ ibad = nullptr,
    uint64_t g_base = 0, unsigned gshift = 0, uint64_t ioff = 0, uint64_t ilo = 0, uint64_t ihi = ~0ull) {
    // a run of more than IRUN empty buckets between two keys would be one thread's serial loop:
    // the index is abandoned (*ibad) and the caller builds it with bucket_index_kernel
    // gshift: a group covers 2^gshift index buckets; ioff: added to every index entry (the output's place
    // in a bigger array); only index entries in [ilo, ihi) are written (a batched collect's round owns those)
    constexpr uint64_t IRUN = 4096;
    const uint64_t g = g_base + blockIdx.x;
    const uint64_t src = gstart[g], dst = ustart[g], m = ustart[g + 1] - dst;
    // gbucket == nullptr: one bucket per group (the speculative final level)
    const uint64_t gb0 = istart ? (gbucket ? gbucket[g] : g) << gshift : 0;
    const uint64_t gb1 = istart ? (gbucket ? gbucket[g + 1] : g + 1) << gshift : 0;
    bool bad = false;
    // one bucket a group (gbucket == nullptr, the speculative final level): its 2^gshift index buckets
    // start at the group's first key at or above each -- a binary search per bucket, no per-key work
    // (the per-key walk below re-reads every key's predecessor: ~2 ms a configs[3] round)
    const bool per_key = istart && gbucket;
    for (uint64_t i = threadIdx.x; i < m; i += 256) {
        const Key<L> key = tmp[src + i];
        out[dst + i] = key;
        if (COUNTED) ocnt[dst + i] = tcnt[src + i];
        if (per_key) {  // buckets (previous key's, this key's] start here
            const uint64_t kb = bits_at(shr(key, ishift), 0, 32);
            const uint64_t pb = i == 0 ? gb0 - 1 : bits_at(shr(tmp[src + i - 1], ishift), 0, 32);
            if (kb - pb > IRUN) bad = true;
            else
                for (uint64_t x = pb + 1; x <= kb; ++x)
                    if (x >= ilo && x < ihi) istart[x] = ioff + dst + i;
        }
    }
    if (istart && !gbucket) {
        for (uint64_t t = threadIdx.x; t < gb1 - gb0; t += 256) {
            const uint64_t x = gb0 + t;
            uint64_t lo = 0, hi = t ? m : 0;
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1;
                if (bits_at(shr(tmp[src + mid], ishift), 0, 32) < x) lo = mid + 1;
                else hi = mid;
            }
            if (x >= ilo && x < ihi) istart[x] = ioff + dst + lo;
        }
    } else if (istart) {  // the group's buckets after its last key start at its end
        const uint64_t lb = m ? bits_at(shr(tmp[src + m - 1], ishift), 0, 32) : gb0 - 1;
        if (gb1 - (lb + 1) > 256 * IRUN) bad = true;
        else
            for (uint64_t x = lb + 1 + threadIdx.x; x < gb1; x += 256)
                if (x >= ilo && x < ihi) istart[x] = ioff + dst + m;
        if (bad) atomicOr(ibad, 1u);
    }
}

}  // namespace mtg
