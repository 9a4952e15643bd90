// boss_kernels.hpp -- the device kernels of the BOSS construction path (K1, K3-K8 of
// SURVEY.md §2.2; K2 is radix_sort.hpp).  Each kernel names the reference loop it replaces.
//
// Layout in HBM: keys are arrays of Key<L> (8/16/32 B, little-endian limbs), counts are u32
// arrays parallel to the keys, the output BOSS arrays are byte arrays (W, last) and a u32
// weight array, one entry per row, with the reference's leading row 0.
#pragma once

#include "device_common.hpp"
#include "keys.hpp"

namespace mtg {

// kmer/alphabets.hpp:127-143 -- A/a 0, C/c 1, G/g 2, T/t/U/u 3, anything else invalid (4);
// negative chars map like '\0' (kmer_extractor.cpp:31-34), i.e. invalid.
__device__ __forceinline__ uint32_t encode_dna(uint32_t c) {
    switch (c) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': case 'U': case 'u': return 3;
        default: return 4;
    }
}

template <int L>
struct ExtractTraits {
    static constexpr int PPT = L == 4 ? 8 : 16;  // positions per thread
    static constexpr int BLOCK = 256;
    static constexpr int TILE = PPT * BLOCK;
    static constexpr int MAXK = 96;
};

// BOSS word from the plain (co-lex) packing P = sum a_i << 2(i-1): rotate the last char to
// the bottom (KMerBOSS keeps a_K in the LSBs, kmer_boss.hpp:58-72).
template <int L>
__device__ __forceinline__ Key<L> plain_to_boss(const Key<L> &P, unsigned K, const Key<L> &low) {
    return shl(P & low, 2) | shr(P, 2 * (K - 1));
}

/*
 * K1: extract_pack_canon.  Replaces KmerExtractorT<2>::sequence_to_kmers
 * (kmer/kmer_extractor.cpp:472-507; slides :86-108 / :165-196; skip rule from
 * utils::drag_and_mark_segments, common/algorithms.hpp:50-67) and the per-read count clamp of
 * count_kmers (kmer_collector.cpp:92).
 *
 * The input is ONE byte buffer holding all reads, each followed by at least one invalid byte
 * (so no window spans two reads).  Workgroup = TILE consecutive window starts; its bytes are
 * staged in LDS as 2-bit codes (4 = invalid); each thread slides PPT windows keeping the
 * forward and reverse-complement plain words and the position of the last invalid char.
 * Valid k-mers are compacted in position order: block scan + decoupled look-back for the tile
 * base, staged in LDS, written coalesced.
 */
template <int L, bool COUNTED>
__global__ __launch_bounds__(256) void extract_kernel(
    const uint8_t *__restrict__ seq, uint64_t seq_len, unsigned K, int canonical,
    const uint64_t *__restrict__ read_starts, const uint32_t *__restrict__ read_counts,
    uint64_t n_reads, uint32_t cmax, Key<L> *__restrict__ out_keys,
    uint32_t *__restrict__ out_counts, uint64_t *desc, uint32_t epoch, uint32_t *tile_counter,
    unsigned long long *total_out, uint32_t *error) {
    using T = ExtractTraits<L>;
    constexpr int BLOCK = T::BLOCK, PPT = T::PPT, TILE = T::TILE;
    __shared__ uint8_t s_code[TILE + T::MAXK];
    __shared__ Key<L> s_out[TILE];
    __shared__ uint32_t s_cnt[COUNTED ? TILE : 1];
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_base;

    const uint32_t tid = threadIdx.x;
    if (tid == 0) s_tile = atomicAdd(tile_counter, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t npos = seq_len >= K ? seq_len - K + 1 : 0;
    const uint64_t base = (uint64_t)tile * TILE;
    const uint64_t span_end = min(seq_len, base + TILE + K - 1);
    for (uint64_t i = base + tid; i < span_end; i += BLOCK) s_code[i - base] = encode_dna(seq[i]);
    __syncthreads();

    const Key<L> low = Key<L>::lowmask(2 * (K - 1));
    const Key<L> full = Key<L>::lowmask(2 * K);
    const uint64_t p0 = base + (uint64_t)tid * PPT;
    Key<L> kk[PPT];
    uint32_t cc[PPT];
    uint32_t nvalid = 0;
    uint32_t valid_mask = 0;
    if (p0 < npos) {
        const uint32_t r0 = tid * PPT;
        Key<L> P = Key<L>::zero(), R = Key<L>::zero();
        int64_t last_bad = -1;
        for (unsigned i = 0; i < K; ++i) {
            uint32_t c = s_code[r0 + i];
            if (c == 4) { last_bad = i; c = 0; }
            P = P | shl(Key<L>::from(c), 2 * i);
            R = R | shl(Key<L>::from(3 - c), 2 * (K - 1 - i));
        }
        uint64_t rid = 0;
        if (COUNTED && read_counts) {
            uint64_t lo = 0, hi = n_reads;  // last read with start <= p0
            while (hi - lo > 1) {
                uint64_t mid = (lo + hi) / 2;
                if (read_starts[mid] <= p0) lo = mid; else hi = mid;
            }
            rid = lo;
        }
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const uint64_t p = p0 + j;
            if (p < npos) {
                if (last_bad < (int64_t)j) {
                    Key<L> f = plain_to_boss(P, K, low);
                    if (canonical) {
                        Key<L> r = plain_to_boss(R, K, low);
                        if (r < f) f = r;
                    }
                    kk[j] = f;
                    if (COUNTED) {
                        uint32_t c = 1;
                        if (read_counts) {
                            while (rid + 1 < n_reads && read_starts[rid + 1] <= p) ++rid;
                            c = read_counts[rid];
                        }
                        cc[j] = c < cmax ? c : cmax;
                    }
                    valid_mask |= 1u << j;
                    ++nvalid;
                }
                if (j + 1 < PPT && p + 1 < npos) {
                    uint32_t c = s_code[r0 + j + K];
                    if (c == 4) { last_bad = j + K; c = 0; }
                    P = shr(P, 2) | shl(Key<L>::from(c), 2 * (K - 1));
                    R = (shl(R, 2) & full) | Key<L>::from(3 - c);
                }
            }
        }
    }
    uint32_t tile_total;
    const uint32_t off = block_exclusive_sum<BLOCK>(nvalid, s_scan, &tile_total);
    tile_base_lookback(desc, tile, tile_total, epoch, error, &s_base);
    if (tid == 0) {
        const uint64_t ntiles = (npos + TILE - 1) / TILE;
        if (tile + 1 == ntiles) *total_out = s_base + tile_total;
    }
    {
        uint32_t o = off;
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            if (valid_mask & (1u << j)) {
                s_out[o] = kk[j];
                if (COUNTED) s_cnt[o] = cc[j];
                ++o;
            }
        }
    }
    __syncthreads();
    const uint64_t gb = s_base;
    for (uint32_t i = tid; i < tile_total; i += BLOCK) {
        out_keys[gb + i] = s_out[i];
        if (COUNTED) out_counts[gb + i] = s_cnt[i];
    }
}

/*
 * K3: unique_compact / count_reduce_sat.  Replaces std::unique (sorted_set.cpp:46) and the
 * saturating merge of sorted_multiset.cpp:66-83 over a sorted array.  Heads (key != previous)
 * are compacted in order (block scan + look-back).  With counts, every thread adds the partial
 * sums of the runs it touches into a 64-bit accumulator per head (one atomic per run piece);
 * count_clamp_kernel then saturates at the container maximum (saturating addition of values
 * <= max is min(sum, max) in any order).
 */
template <int L, bool COUNTED>
__global__ __launch_bounds__(256) void unique_kernel(const Key<L> *__restrict__ in,
                                                     const uint32_t *__restrict__ in_counts,
                                                     uint64_t n, Key<L> *__restrict__ out,
                                                     unsigned long long *__restrict__ sums,
                                                     uint64_t *desc, uint32_t epoch, uint32_t *tile_counter,
                                                     unsigned long long *total_out,
                                                     uint32_t *error) {
    constexpr int BLOCK = 256, ITEMS = 8, TILE = BLOCK * ITEMS;
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_base;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) s_tile = atomicAdd(tile_counter, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t i0 = (uint64_t)tile * TILE + (uint64_t)tid * ITEMS;
    Key<L> k[ITEMS];
    uint32_t heads = 0, nheads = 0;
    Key<L> prev = i0 > 0 && i0 <= n ? in[i0 - 1] : Key<L>::zero();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint64_t i = i0 + j;
        if (i < n) {
            k[j] = in[i];
            if (i == 0 || k[j] != prev) {
                heads |= 1u << j;
                ++nheads;
            }
            prev = k[j];
        }
    }
    uint32_t tile_total;
    const uint32_t off = block_exclusive_sum<BLOCK>(nheads, s_scan, &tile_total);
    tile_base_lookback(desc, tile, tile_total, epoch, error, &s_base);
    if (tid == 0) {
        const uint64_t ntiles = (n + TILE - 1) / TILE;
        if (tile + 1 == ntiles) *total_out = s_base + tile_total;
    }
    __syncthreads();
    // index of the head of element i0 (inclusive head count - 1)
    uint64_t h = s_base + off;  // number of heads before i0
    unsigned long long acc = 0;
    bool have = false;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint64_t i = i0 + j;
        if (i < n) {
            if (heads & (1u << j)) {
                if (COUNTED && have) atomicAdd(&sums[h - 1], acc);
                out[h] = k[j];
                ++h;
                acc = 0;
            }
            if (COUNTED) {
                acc += in_counts[i];
                have = true;
            }
        }
    }
    if (COUNTED && have) atomicAdd(&sums[h - 1], acc);
}

__global__ void count_clamp_kernel(const unsigned long long *__restrict__ sums, uint64_t n,
                                   uint32_t cmax, uint32_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        unsigned long long s = sums[i];
        out[i] = s < cmax ? (uint32_t)s : cmax;
    }
}

/*
 * K4: rc_augment.  Replaces add_reverse_complements (boss_chunk_construct.cpp:179-222):
 * appends rc(x) for every non-palindromic x behind the array (compacted in order) and doubles
 * a palindrome's count with saturation (c >> (bits-1) ? max : 2c).  The caller re-sorts.
 */
template <int L, bool COUNTED>
__global__ __launch_bounds__(256) void rc_augment_kernel(Key<L> *keys, uint32_t *counts,
                                                         uint64_t n, unsigned K, unsigned cbits,
                                                         uint32_t cmax, uint64_t *desc, uint32_t epoch,
                                                         uint32_t *tile_counter,
                                                         unsigned long long *total_out,
                                                         uint32_t *error) {
    constexpr int BLOCK = 256, ITEMS = 4, TILE = BLOCK * ITEMS;
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_base;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) s_tile = atomicAdd(tile_counter, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t i0 = (uint64_t)tile * TILE + (uint64_t)tid * ITEMS;
    Key<L> r[ITEMS];
    uint32_t c[ITEMS];
    uint32_t mask = 0, cnt = 0;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint64_t i = i0 + j;
        if (i < n) {
            const Key<L> x = keys[i];
            r[j] = revcomp2(x, K);
            if (r[j] != x) {
                mask |= 1u << j;
                ++cnt;
                if (COUNTED) c[j] = counts[i];
            } else if (COUNTED) {
                uint32_t v = counts[i];
                counts[i] = (v >> (cbits - 1)) ? cmax : 2 * v;
            }
        }
    }
    uint32_t tile_total;
    const uint32_t off = block_exclusive_sum<BLOCK>(cnt, s_scan, &tile_total);
    tile_base_lookback(desc, tile, tile_total, epoch, error, &s_base);
    if (tid == 0) {
        const uint64_t ntiles = (n + TILE - 1) / TILE;
        if (tile + 1 == ntiles) *total_out = s_base + tile_total;
    }
    __syncthreads();
    uint64_t o = n + s_base + off;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        if (mask & (1u << j)) {
            keys[o] = r[j];
            if (COUNTED) counts[o] = c[j];
            ++o;
        }
    }
}

/*
 * Bucket index over the top B bits of a sorted 2K-bit key array: start[b] = lower_bound of the
 * first key whose top bits are >= b.  Turns every membership probe below into a short binary
 * search inside one bucket (the probes of a wave land in a few neighbouring buckets).
 */
template <int L>
__global__ void bucket_index_kernel(const Key<L> *__restrict__ keys, uint64_t n, unsigned shift,
                                    uint64_t nbuckets, uint64_t *__restrict__ start) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += stride) {
        uint64_t b = i < n ? bits_at(shr(keys[i], shift), 0, 32) : nbuckets;
        uint64_t bp = i > 0 ? bits_at(shr(keys[i - 1], shift), 0, 32) + 1 : 0;
        for (uint64_t x = bp; x <= b && x <= nbuckets; ++x) start[x] = i;
    }
}

template <int L>
__device__ __forceinline__ uint64_t lower_bound_bucketed(const Key<L> *__restrict__ keys,
                                                         const uint64_t *__restrict__ start,
                                                         unsigned shift, const Key<L> &x) {
    const uint64_t b = bits_at(shr(x, shift), 0, 32);
    uint64_t lo = start[b], hi = start[b + 1];
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (keys[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

/*
 * K5 + K6 (flag pass): for each real edge x (sorted, 2-bit):
 *   sink   -- add_dummy_sink_kmers (boss_chunk_construct.cpp:54-98): the target node
 *             a_2..a_K has no real out-edge  <=>  no key y with y >> 2 == to_next(x, 0) >> 2;
 *   source -- add_dummy_source_kmers (:123-168): x is the first edge of its node and no real
 *             y has chars 2..k equal to x's chars 1..k-1 with label a_k (y >> 4 == prev >> 4
 *             and y & 3 == prev & 3, prev = to_prev(x, 0)).
 * flags[i] = sink | source << 1.  Duplicated sinks (several x with one target) are removed by
 * the final unique over all dummies, as are repeated higher-level sources.
 */
template <int L>
__global__ __launch_bounds__(256) void dummy_flag_kernel(const Key<L> *__restrict__ keys,
                                                         uint64_t n, unsigned K,
                                                         const uint64_t *__restrict__ start,
                                                         unsigned bshift, uint8_t *__restrict__ flags,
                                                         unsigned long long *totals) {
    __shared__ unsigned long long s_tot[2];
    if (threadIdx.x < 2) s_tot[threadIdx.x] = 0;
    __syncthreads();
    unsigned long long ns = 0, nsrc = 0;
    const Key<L> full = Key<L>::lowmask(2 * K);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const Key<L> x = keys[i];
        uint8_t f = 0;
        // to_next(x, K, 0): node a_2..a_K, label 0
        const Key<L> t = (shr(x, 2) | shl(Key<L>::from(x.w[0] & 3), 2 * (K - 1))) &
                         ~Key<L>::from(3);
        {
            const uint64_t j = lower_bound_bucketed(keys, start, bshift, t);
            if (j >= n || shr(keys[j], 2) != shr(t, 2)) f |= 1;
        }
        if (i == 0 || shr(keys[i - 1], 2) != shr(x, 2)) {
            // to_prev(x, K, 0): node 0 a_1..a_{k-1}, label a_k
            const Key<L> prev = (shl(x & ~Key<L>::from(3), 2) & full) | shr(x, 2 * (K - 1));
            const Key<L> lo = prev & ~Key<L>::from(15);
            uint64_t j = lower_bound_bucketed(keys, start, bshift, lo);
            bool redundant = false;
            const uint32_t label = (uint32_t)(prev.w[0] & 3);
            while (j < n && shr(keys[j], 4) == shr(prev, 4)) {
                if ((uint32_t)(keys[j].w[0] & 3) == label) {
                    redundant = true;
                    break;
                }
                ++j;
            }
            if (!redundant) f |= 2;
        }
        flags[i] = f;
        ns += f & 1;
        nsrc += f >> 1;
    }
    atomicAdd(&s_tot[0], ns);
    atomicAdd(&s_tot[1], nsrc);
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(&totals[0], s_tot[0]);
        atomicAdd(&totals[1], s_tot[1]);
    }
}

// byte of four 2-bit chars -> four 3-bit chars, each + 1 ($ACGT lift, kmer_transform.hpp:102-165)
__device__ __forceinline__ uint64_t lift_byte(uint32_t b) {
    return ((b & 3u) | ((b & 0xCu) << 1) | ((b & 0x30u) << 2) | ((b & 0xC0u) << 3)) + 0x249u;
}

template <int LO, int LI>
__device__ __forceinline__ Key<LO> lift_fast(const Key<LI> &x, unsigned K) {
    Key<LO> r = Key<LO>::zero();
    const unsigned nbytes = (2 * K + 7) / 8;
    for (unsigned b = 0; b < nbytes; ++b)
        r = r | shl(Key<LO>::from(lift_byte(bits_at(x, 8 * b, 8))), 12 * b);
    return r & Key<LO>::lowmask(3 * K);
}

/*
 * K5/K6 (write pass): emit the lifted dummy k-mers in edge order (block scan + look-back):
 * a sink as lift(to_next(x,0)) with its label char cleared to $ (:94), a source as
 * lift(to_prev(x,0)) with char 1 cleared to $ (:165) followed by its k-1 higher levels
 * to_prev(., $) (:286-303).
 */
template <int L2, int L3>
__global__ __launch_bounds__(256) void dummy_write_kernel(
    const Key<L2> *__restrict__ keys, const uint8_t *__restrict__ flags, uint64_t n, unsigned K,
    Key<L3> *__restrict__ out, uint64_t *desc, uint32_t epoch, uint32_t *tile_counter, uint32_t *error) {
    constexpr int BLOCK = 256, ITEMS = 4, TILE = BLOCK * ITEMS;
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_base;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) s_tile = atomicAdd(tile_counter, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t i0 = (uint64_t)tile * TILE + (uint64_t)tid * ITEMS;
    const unsigned k = K - 1;
    uint32_t cnt = 0;
    uint8_t f[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        f[j] = i0 + j < n ? flags[i0 + j] : 0;
        cnt += (f[j] & 1) + (f[j] >> 1) * k;
    }
    uint32_t tile_total;
    const uint32_t off = block_exclusive_sum<BLOCK>(cnt, s_scan, &tile_total);
    tile_base_lookback(desc, tile, tile_total, epoch, error, &s_base);
    uint64_t o = s_base + off;
    const Key<L2> full = Key<L2>::lowmask(2 * K);
    const Key<L3> full3 = Key<L3>::lowmask(3 * K);
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        if (!f[j]) continue;
        const Key<L2> x = keys[i0 + j];
        if (f[j] & 1) {
            const Key<L2> t = (shr(x, 2) | shl(Key<L2>::from(x.w[0] & 3), 2 * (K - 1))) &
                              ~Key<L2>::from(3);
            out[o++] = lift_fast<L3>(t, K) & ~Key<L3>::from(7);
        }
        if (f[j] & 2) {
            const Key<L2> prev = (shl(x & ~Key<L2>::from(3), 2) & full) | shr(x, 2 * (K - 1));
            Key<L3> d = lift_fast<L3>(prev, K) & ~Key<L3>::from(7 << 3);
            out[o++] = d;
            for (unsigned lev = 2; lev <= k; ++lev) {
                // KMerBOSS<., 3>::to_prev(K, $) -- kmer_boss.hpp:171-186
                const Key<L3> last_char = shr(d, 3 * (K - 1));
                d = (shl(d & ~Key<L3>::from(7), 3) & full3) | last_char;
                out[o++] = d;
            }
        }
    }
}

/*
 * K7: lift + merge (boss_chunk_construct.cpp:308-348).  Output row 0 is the main dummy
 * KMER(0); rows 1.. merge lift(real) (+ its count) with the sorted dummies (count 0).
 * Merge path: every thread finds its diagonal split by binary search and merges ITEMS outputs.
 */
template <int L2, int L3, bool COUNTED>
__global__ __launch_bounds__(256) void merge_kernel(const Key<L2> *__restrict__ a,
                                                    const uint32_t *__restrict__ ac, uint64_t na,
                                                    const Key<L3> *__restrict__ b, uint64_t nb,
                                                    unsigned K, Key<L3> *__restrict__ out,
                                                    uint32_t *__restrict__ oc) {
    constexpr int ITEMS = 8;
    const uint64_t total = na + nb;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t d0 = t * ITEMS;
    if (d0 == 0 && t == 0) {
        out[0] = Key<L3>::zero();
        if (COUNTED) oc[0] = 0;
    }
    if (d0 >= total) return;
    // split: smallest i in [max(0,d0-nb), min(d0,na)] with a[i] > b[d0-i-1] (a first on ties,
    // ties cannot occur: real and dummy k-mers differ)
    uint64_t lo = d0 > nb ? d0 - nb : 0, hi = d0 < na ? d0 : na;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        // take a[mid] before b[d0-mid-1]?
        if (lift_fast<L3>(a[mid], K) < b[d0 - mid - 1]) lo = mid + 1; else hi = mid;
    }
    uint64_t i = lo, j = d0 - lo;
    const uint64_t end = min(total, d0 + ITEMS);
    Key<L3> la = i < na ? lift_fast<L3>(a[i], K) : Key<L3>::zero();
    for (uint64_t o = d0; o < end; ++o) {
        const bool take_a = i < na && (j >= nb || la < b[j]);
        if (take_a) {
            out[1 + o] = la;
            if (COUNTED) oc[1 + o] = ac[i];
            ++i;
            if (i < na) la = lift_fast<L3>(a[i], K);
        } else {
            out[1 + o] = b[j];
            if (COUNTED) oc[1 + o] = 0;
            ++j;
        }
    }
}

/*
 * K8: emit_W_last_F (initialize_chunk, boss_chunk.cpp:32-133) over the merged stream s[0..m):
 *   last  = the next row has a different node (chars 1..k);
 *   skip  = redundant dummy sink: label $, last node char != $, next row same node;
 *   W     = label, + 5 if an earlier row of the same chars-2..k group has the same label
 *           (groups hold at most 25 rows: look back);
 *   F[c]  = #emitted rows whose last node char < c (histogram of top chars);
 *   weight= min(count, 2^bits - 1) if count && W && char 1 != $ else 0.
 * Rows are compacted past skipped ones (block scan + look-back); output row r goes to
 * index 1 + r, behind the leading row 0 the caller zeroes.
 */
template <int L3, bool COUNTED>
__global__ __launch_bounds__(256) void emit_kernel(
    const Key<L3> *__restrict__ s, const uint32_t *__restrict__ sc, uint64_t m, unsigned k,
    uint32_t wmax, uint8_t *__restrict__ W, uint8_t *__restrict__ last,
    uint32_t *__restrict__ weights, unsigned long long *__restrict__ fhist, uint64_t *desc,
    uint32_t epoch,
    uint32_t *tile_counter, unsigned long long *total_out, uint32_t *error) {
    constexpr int BLOCK = 256, ITEMS = 4, TILE = BLOCK * ITEMS;
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_base;
    __shared__ uint32_t s_f[8];
    const uint32_t tid = threadIdx.x;
    if (tid == 0) s_tile = atomicAdd(tile_counter, 1u);
    if (tid < 8) s_f[tid] = 0;
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t i0 = (uint64_t)tile * TILE + (uint64_t)tid * ITEMS;
    uint8_t w[ITEMS], la[ITEMS];
    uint32_t wt[ITEMS];
    uint32_t keep = 0, nkeep = 0;
    uint32_t fcount[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint64_t i = i0 + j;
        if (i >= m) continue;
        const Key<L3> key = s[i];
        const uint32_t c = (uint32_t)(key.w[0] & 7);
        const uint32_t top = char_at(key, k, 3);
        const Key<L3> node = shr(key, 3);
        const bool same_next = i + 1 < m && shr(s[i + 1], 3) == node;
        if (same_next && c == 0 && top > 0) continue;
        keep |= 1u << j;
        ++nkeep;
        la[j] = same_next ? 0 : 1;
        uint32_t ww = c;
        if (c) {
            const Key<L3> grp = shr(key, 6);
            for (uint64_t p = i; p > 0; --p) {
                const Key<L3> q = s[p - 1];
                if (shr(q, 6) != grp) break;
                if ((uint32_t)(q.w[0] & 7) == c) {
                    ww = c + 5;
                    break;
                }
            }
        }
        w[j] = (uint8_t)ww;
        if (COUNTED) {
            const uint32_t cnt = sc[i];
            wt[j] = (cnt && ww && char_at(key, 1, 3)) ? (cnt < wmax ? cnt : wmax) : 0;
        }
        fcount[top < 5 ? top : 4]++;
    }
#pragma unroll
    for (int c = 0; c < 5; ++c)
        if (fcount[c]) atomicAdd(&s_f[c], fcount[c]);
    uint32_t tile_total;
    const uint32_t off = block_exclusive_sum<BLOCK>(nkeep, s_scan, &tile_total);
    tile_base_lookback(desc, tile, tile_total, epoch, error, &s_base);
    if (tid == 0) {
        const uint64_t ntiles = (m + TILE - 1) / TILE;
        if (tile + 1 == ntiles) *total_out = s_base + tile_total;
    }
    __syncthreads();
    if (tid < 5 && s_f[tid]) atomicAdd(&fhist[tid], (unsigned long long)s_f[tid]);
    uint64_t o = 1 + s_base + off;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        if (keep & (1u << j)) {
            W[o] = w[j];
            last[o] = la[j];
            if (COUNTED) weights[o] = wt[j];
            ++o;
        }
    }
}

}  // namespace mtg
