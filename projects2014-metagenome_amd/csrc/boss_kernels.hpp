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
 * writes rc(x) for every non-palindromic x to rc_out (compacted in order) and doubles a
 * palindrome's count with saturation (c >> (bits-1) ? max : 2c).  The caller sorts rc_out
 * and merges it with the (sorted) canonical array instead of re-sorting both.
 */
template <int L, bool COUNTED>
__global__ __launch_bounds__(256) void rc_augment_kernel(Key<L> *keys, uint32_t *counts,
                                                         Key<L> *__restrict__ rc_out,
                                                         uint32_t *__restrict__ rc_counts,
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
    uint64_t o = s_base + off;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        if (mask & (1u << j)) {
            rc_out[o] = r[j];
            if (COUNTED) rc_counts[o] = c[j];
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

// first index with keys[i] > hi (hi within the 2K-bit key range, or all-ones)
template <int L>
__device__ __forceinline__ uint64_t upper_bucketed(const Key<L> *__restrict__ keys, uint64_t n,
                                                   const uint64_t *__restrict__ start,
                                                   unsigned shift, uint64_t nbuckets,
                                                   const Key<L> &hi, unsigned K) {
    if (hi == Key<L>::lowmask(2 * K)) return n;
    const Key<L> h1 = hi + Key<L>::from(1);
    if (bits_at(shr(h1, shift), 0, 32) >= nbuckets) return n;
    return lower_bound_bucketed(keys, start, shift, h1);
}

template <int L>
struct DummyTraits {
    static constexpr int TILE = L == 1 ? 2048 : L == 2 ? 1024 : 512;
    static constexpr int CAP = 2 * TILE;
    static constexpr int PER = TILE / 256;
};

/*
 * K5 + K6 flag pass, tiled (same predicates as dummy_flag_kernel below).  A workgroup takes
 * TILE consecutive real edges.  Per probe class -- sink probes of label c = 0..3 and the source
 * probes -- the probes of the tile are monotone, so every real edge they can hit lies in one
 * contiguous key range: two bucketed searches find it, it is staged in LDS and the probes are
 * resolved there.  A range larger than CAP (or source probes of a tile that straddles a change
 * of the last node char) falls back to per-probe bucketed searches.
 */
template <int L>
__global__ __launch_bounds__(256) void dummy_flag_tiled_kernel(
    const Key<L> *__restrict__ keys, uint64_t n, unsigned K, const uint64_t *__restrict__ start,
    unsigned bshift, uint64_t nbuckets, uint8_t *__restrict__ flags,
    unsigned long long *totals) {
    using T = DummyTraits<L>;
    __shared__ Key<L> s_x[T::TILE];
    __shared__ Key<L> s_r[T::CAP];
    __shared__ uint64_t s_a, s_cnt;
    __shared__ unsigned long long s_tot[2];
    const uint32_t tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * T::TILE;
    const uint32_t tn = (uint32_t)min((uint64_t)T::TILE, n - base);
    if (tid < 2) s_tot[tid] = 0;
    for (uint32_t j = tid; j < tn; j += 256) s_x[j] = keys[base + j];
    __syncthreads();
    const Key<L> full = Key<L>::lowmask(2 * K);
    const Key<L> x_first = s_x[0], x_last = s_x[tn - 1];
    const unsigned k = K - 1;
    uint8_t f[T::PER];
    Key<L> probe[T::PER];
#pragma unroll
    for (int q = 0; q < T::PER; ++q) f[q] = 0;

    // classes 0..3: sink probes of label c over the whole tile; classes 4..7: source probes of
    // one quarter of the tile each (their key range is ~4x wider than the edges' range)
    constexpr uint32_t QT = T::TILE / 4;
    for (int cls = 0; cls < 8; ++cls) {
        const uint32_t sub = cls < 4 ? 0 : cls - 4;
        const uint32_t q0 = sub * QT, q1 = min(tn, q0 + QT);
        if (cls >= 4 && q0 >= tn) break;
        // this class's probes and the key range they can hit
        bool mine[T::PER];
#pragma unroll
        for (int q = 0; q < T::PER; ++q) {
            const uint32_t j = tid + 256 * q;
            mine[q] = false;
            if (j >= tn) continue;
            if (cls >= 4 && (j < q0 || j >= q1)) continue;
            const Key<L> x = s_x[j];
            if (cls < 4) {
                if ((uint32_t)(x.w[0] & 3) != (uint32_t)cls) continue;
                // to_next(x, K, 0): node a_2..a_K, label 0 (kmer_boss.hpp:147-169)
                probe[q] = (shr(x, 2) | shl(Key<L>::from(x.w[0] & 3), 2 * (K - 1))) & ~Key<L>::from(3);
                mine[q] = true;
            } else {
                const bool first = base + j == 0 ||
                                   shr(j ? s_x[j - 1] : keys[base - 1], 2) != shr(x, 2);
                if (!first) continue;
                // to_prev(x, K, 0): node 0 a_1..a_{k-1}, label a_k (kmer_boss.hpp:171-186)
                probe[q] = (shl(x & ~Key<L>::from(3), 2) & full) | shr(x, 2 * (K - 1));
                mine[q] = true;
            }
        }
        if (tid == 0) {
            Key<L> lo, hi;
            bool ok = true;
            if (cls < 4) {
                const Key<L> c = shl(Key<L>::from(cls), 2 * (K - 1));
                lo = (shr(x_first, 2) | c) & ~Key<L>::from(3);
                hi = shr(x_last, 2) | c | Key<L>::from(3);
            } else {
                const Key<L> xf = s_x[q0], xl = s_x[q1 - 1];
                ok = char_at(xf, k, 2) == char_at(xl, k, 2);
                const Key<L> pf = (shl(xf & ~Key<L>::from(3), 2) & full) | shr(xf, 2 * (K - 1));
                const Key<L> pl = (shl(xl & ~Key<L>::from(3), 2) & full) | shr(xl, 2 * (K - 1));
                lo = pf & ~Key<L>::from(15);
                hi = pl | Key<L>::from(15);
            }
            uint64_t a = 0, b = 0;
            if (ok) {
                a = lower_bound_bucketed(keys, start, bshift, lo);
                b = upper_bucketed(keys, n, start, bshift, nbuckets, hi, K);
            }
            s_a = a;
            s_cnt = ok && b - a <= (uint64_t)T::CAP ? b - a : ~0ull;
        }
        __syncthreads();
        const uint64_t a = s_a, cnt = s_cnt;
        if (cnt != ~0ull)
            for (uint32_t j = tid; j < cnt; j += 256) s_r[j] = keys[a + j];
        __syncthreads();
#pragma unroll
        for (int q = 0; q < T::PER; ++q) {
            if (!mine[q]) continue;
            const Key<L> p = probe[q];
            if (cls < 4) {
                bool found;
                if (cnt != ~0ull) {
                    uint32_t lo = 0, hi = (uint32_t)cnt;
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (s_r[mid] < p) lo = mid + 1; else hi = mid;
                    }
                    found = lo < cnt && shr(s_r[lo], 2) == shr(p, 2);
                } else {
                    const uint64_t j = lower_bound_bucketed(keys, start, bshift, p);
                    found = j < n && shr(keys[j], 2) == shr(p, 2);
                }
                if (!found) f[q] |= 1;
            } else {
                const Key<L> lo4 = p & ~Key<L>::from(15);
                const uint32_t label = (uint32_t)(p.w[0] & 3);
                bool redundant = false;
                if (cnt != ~0ull) {
                    uint32_t lo = 0, hi = (uint32_t)cnt;
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (s_r[mid] < lo4) lo = mid + 1; else hi = mid;
                    }
                    for (uint32_t j = lo; j < cnt && shr(s_r[j], 4) == shr(p, 4); ++j)
                        if ((uint32_t)(s_r[j].w[0] & 3) == label) { redundant = true; break; }
                } else {
                    for (uint64_t j = lower_bound_bucketed(keys, start, bshift, lo4);
                         j < n && shr(keys[j], 4) == shr(p, 4); ++j)
                        if ((uint32_t)(keys[j].w[0] & 3) == label) { redundant = true; break; }
                }
                if (!redundant) f[q] |= 2;
            }
        }
        __syncthreads();
    }
    unsigned long long ns = 0, nsrc = 0;
#pragma unroll
    for (int q = 0; q < T::PER; ++q) {
        const uint32_t j = tid + 256 * q;
        if (j < tn) {
            flags[base + j] = f[q];
            ns += f[q] & 1;
            nsrc += f[q] >> 1;
        }
    }
    atomicAdd(&s_tot[0], ns);
    atomicAdd(&s_tot[1], nsrc);
    __syncthreads();
    if (tid == 0) {
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
 * Merge path over two sorted arrays, tiled: A (LA-limb keys, lifted to LO limbs on the fly when
 * LIFT -- kmer_transform.hpp:75-100 + get_sentinel_delta) and B (LO-limb keys); equal keys do
 * not occur (real vs dummy k-mers, canonical vs non-canonical).  Output index off + i.
 * Used for K7 (boss_chunk_construct.cpp:308-348: lift(real) merged with the sorted dummies
 * behind the main dummy row, dummies carrying count 0) and for the reverse-complement merge.
 * A workgroup owns TILE consecutive outputs: one diagonal search per tile boundary, the two
 * input runs staged in LDS (A lifted once), per-thread merge of ITEMS outputs out of LDS, and a
 * coalesced store from an LDS output image.
 */
template <int LO, int LA, bool LIFT>
__device__ __forceinline__ Key<LO> merge_key(const Key<LA> &a, unsigned K) {
    if constexpr (LIFT) {
        return lift_fast<LO>(a, K);
    } else {
        Key<LO> r;
#pragma unroll
        for (int i = 0; i < LO; ++i) r.w[i] = i < LA ? a.w[i] : 0;
        return r;
    }
}

template <int LO, int LA, bool LIFT>
__device__ __forceinline__ uint64_t merge_split(const Key<LA> *__restrict__ a, uint64_t na,
                                                const Key<LO> *__restrict__ b, uint64_t nb,
                                                uint64_t diag, unsigned K) {
    uint64_t lo = diag > nb ? diag - nb : 0, hi = diag < na ? diag : na;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (merge_key<LO, LA, LIFT>(a[mid], K) < b[diag - mid - 1]) lo = mid + 1; else hi = mid;
    }
    return lo;
}

constexpr int MERGE_TILE = 2048;

// diagonal split of every tile boundary (one thread each, all in flight together)
template <int LO, int LA, bool LIFT>
__global__ void merge_partition_kernel(const Key<LA> *__restrict__ a, uint64_t na,
                                       const Key<LO> *__restrict__ b, uint64_t nb, unsigned K,
                                       uint64_t ntiles, uint64_t *__restrict__ splits) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntiles) return;
    const uint64_t diag = min(na + nb, t * MERGE_TILE);
    splits[t] = merge_split<LO, LA, LIFT>(a, na, b, nb, diag, K);
}

template <int LO, int LA, bool LIFT, bool COUNTED, bool BCOUNTS>
__global__ __launch_bounds__(256) void merge_kernel(const Key<LA> *__restrict__ a,
                                                    const uint32_t *__restrict__ ac, uint64_t na,
                                                    const Key<LO> *__restrict__ b,
                                                    const uint32_t *__restrict__ bc, uint64_t nb,
                                                    unsigned K, const uint64_t *__restrict__ splits,
                                                    Key<LO> *__restrict__ out,
                                                    uint32_t *__restrict__ oc, uint64_t off) {
    constexpr int ITEMS = MERGE_TILE / 256, TILE = MERGE_TILE;
    __shared__ Key<LO> s_in[TILE];
    __shared__ Key<LO> s_out[TILE];
    __shared__ uint32_t s_cin[COUNTED ? TILE : 1];
    __shared__ uint32_t s_cout[COUNTED ? TILE : 1];
    __shared__ uint64_t s_split[2];
    const uint64_t total = na + nb;
    const uint64_t d0 = (uint64_t)blockIdx.x * TILE;
    const uint64_t d1 = min(total, d0 + TILE);
    if (threadIdx.x < 2) s_split[threadIdx.x] = splits[blockIdx.x + threadIdx.x];
    __syncthreads();
    const uint64_t a0 = s_split[0], a1 = s_split[1];
    const uint64_t b0 = d0 - a0, b1 = d1 - a1;
    const uint32_t la = (uint32_t)(a1 - a0), lb = (uint32_t)(b1 - b0);
    for (uint32_t i = threadIdx.x; i < la; i += 256) {
        s_in[i] = merge_key<LO, LA, LIFT>(a[a0 + i], K);
        if (COUNTED) s_cin[i] = ac[a0 + i];
    }
    for (uint32_t i = threadIdx.x; i < lb; i += 256) {
        s_in[la + i] = b[b0 + i];
        if (COUNTED) s_cin[la + i] = BCOUNTS ? bc[b0 + i] : 0;
    }
    __syncthreads();
    // thread's sub-diagonal inside the tile: A run = s_in[0..la), B run = s_in[la..la+lb)
    const uint32_t t0 = min((uint32_t)threadIdx.x * ITEMS, la + lb);
    const uint32_t t1 = min(t0 + ITEMS, la + lb);
    uint32_t lo = t0 > lb ? t0 - lb : 0, hi = min(t0, la);
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_in[mid] < s_in[la + t0 - mid - 1]) lo = mid + 1; else hi = mid;
    }
    uint32_t i = lo, j = t0 - lo;
    for (uint32_t o = t0; o < t1; ++o) {
        const bool take_a = i < la && (j >= lb || s_in[i] < s_in[la + j]);
        const uint32_t src = take_a ? i : la + j;
        s_out[o] = s_in[src];
        if (COUNTED) s_cout[o] = s_cin[src];
        if (take_a) ++i; else ++j;
    }
    __syncthreads();
    for (uint32_t o = threadIdx.x; o < la + lb; o += 256) {
        out[off + d0 + o] = s_out[o];
        if (COUNTED) oc[off + d0 + o] = s_cout[o];
    }
}

__global__ void set_root_row_kernel(uint64_t *key_words, int limbs, uint32_t *count) {
    for (int i = 0; i < limbs; ++i) key_words[i] = 0;  // the main dummy KMER(0)
    if (count) *count = 0;
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
