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
// Branchless: OR-ing 0x20 folds upper onto lower case (its preimages are exactly {x, x ^ 0x20}),
// then a 3-bit-per-entry table indexed by (c | 0x20) - 'a' for 'a' .. 'u' (21 entries); anything
// outside that range is invalid.  Exhaustively equal to the switch over all 256 byte values.
__host__ __device__ __forceinline__ uint32_t encode_dna(uint32_t c) {
    constexpr uint64_t TAB = 0x37249249248a4860ull;  // a 0, c 1, g 2, t 3, u 3, others 4
    const uint32_t idx = (c | 0x20u) - 0x61u;
    return idx > 20u ? 4u : (uint32_t)(TAB >> (3u * idx)) & 7u;
}

// Which strand a canonical window keeps.  canonical == 1: the smaller key (kmer_extractor.cpp:165-196).
// canonical == 2 (the routed multi-GPU collect, boss_pipeline.hip: dist_collect_routed): the strand
// whose top 12 key bits hash smaller, the smaller key when the tops tie.  Every {x, rc(x)} pair still
// has one representative and the chunk is the same (the real edges are both strands, counts follow
// the pair), but the representatives spread over the key space like the real edges instead of
// piling into the low prefixes, so one range partition balances the collect and the later stages.
// A tie keeps the top either way, so the 12-bit histograms of pass A need only the tops.
__host__ __device__ __forceinline__ uint32_t top_hash12(uint32_t t) {
    t = (t + 0x9e3779b9u) * 0x85ebca6bu;
    t ^= t >> 13;
    t *= 0xc2b2ae35u;
    return t ^ (t >> 16);
}
__host__ __device__ __forceinline__ bool take_rc_top(int canonical, uint32_t ftop, uint32_t rtop) {
    if (canonical == 2) return ftop != rtop && top_hash12(rtop) < top_hash12(ftop);
    return canonical && rtop < ftop;
}
template <int L>
__device__ __forceinline__ bool take_rc(int canonical, const Key<L> &f, const Key<L> &r, unsigned K) {
    if (canonical == 2) {
        const uint32_t tf = (uint32_t)bits_at(shr(f, 2 * K - 12), 0, 12), tr = (uint32_t)bits_at(shr(r, 2 * K - 12), 0, 12);
        if (tf != tr) return top_hash12(tr) < top_hash12(tf);
    }
    return canonical && r < f;
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
 * One thread's PPT consecutive windows starting at p0 (tile-relative code offset r0 in s_code):
 * slides the forward and reverse-complement plain words, skips windows with an invalid char
 * (drag_and_mark_segments, common/algorithms.hpp:50-67), canonicalises (fwd <= rc in BOSS
 * integer order, kmer_extractor.cpp:165-196) and clamps per-read counts (kmer_collector.cpp:92).
 * Returns the valid mask; with KEYS = false only the mask (the counting passes).
 */
template <int L, bool COUNTED, int PPT, bool KEYS>
__device__ __forceinline__ uint32_t slide_windows(const uint8_t *s_code, uint32_t r0, uint64_t p0, uint64_t npos,
                                                  unsigned K, int canonical,
                                                  const uint64_t *__restrict__ read_starts,
                                                  const uint32_t *__restrict__ read_counts, uint64_t n_reads,
                                                  const uint64_t *__restrict__ rid_at,
                                                  uint32_t cmax, Key<L> (&kk)[PPT], uint32_t (&cc)[PPT]) {
    uint32_t valid_mask = 0;
    if (p0 >= npos) return 0;
    const Key<L> low = Key<L>::lowmask(2 * (K - 1));
    const Key<L> full = Key<L>::lowmask(2 * K);
    Key<L> P = Key<L>::zero(), R = Key<L>::zero();
    int64_t last_bad = -1;
    for (unsigned i = 0; i < K; ++i) {
        uint32_t c = s_code[r0 + i];
        if (c == 4) { last_bad = i; c = 0; }
        P = P | shl(Key<L>::from(c), 2 * i);
        R = R | shl(Key<L>::from(3 - c), 2 * (K - 1 - i));
    }
    uint64_t rid = ~0ull;  // the read of the thread's first valid window, searched when it comes
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        const uint64_t p = p0 + j;
        if (p < npos) {
            if (last_bad < (int64_t)j) {
                if (KEYS) {
                    Key<L> f = plain_to_boss(P, K, low);
                    if (canonical) {
                        Key<L> r = plain_to_boss(R, K, low);
                        if (take_rc(canonical, f, r, K)) f = r;
                    }
                    kk[j] = f;
                    if (COUNTED) {
                        uint32_t c = 1;
                        if (read_counts) {
                            if (rid == ~0ull) rid = read_of(read_starts, n_reads, rid_at, p);  // last start <= p
                            while (rid + 1 < n_reads && read_starts[rid + 1] <= p) ++rid;
                            c = read_counts[rid];
                        }
                        cc[j] = c < cmax ? c : cmax;
                    }
                }
                valid_mask |= 1u << j;
            }
            if (j + 1 < PPT && p + 1 < npos) {
                uint32_t c = s_code[r0 + j + K];
                if (c == 4) { last_bad = j + K; c = 0; }
                if (KEYS) {
                    P = shr(P, 2) | shl(Key<L>::from(c), 2 * (K - 1));
                    R = (shl(R, 2) & full) | Key<L>::from(3 - c);
                }
            }
        }
    }
    return valid_mask;
}

/*
 * K1 for an input whose every read is exactly one window: K chars + one separator, read r at
 * r * (K + 1) -- a KMC database decoded into reads (kmc.hpp: one record per read, seq_io/
 * kmc_parser.cpp:27-62), 1.9e8 reads of 32 bytes at configs[4].  The window extractor would visit
 * all K + 1 positions of every read to keep one; here one thread takes one read (lanes on adjacent
 * reads, so a wave reads 64 * (K + 1) contiguous bytes), builds its key as slide_windows does
 * (canonical by take_rc) and its clamped count, and the valid ones go out in any order through one
 * cursor atomic per workgroup: the sort that follows fixes the order, and saturating sums do not
 * depend on it.  A read start or separator that breaks the layout raises *bad (the caller then
 * takes the window extractor).
 */
template <int L, bool COUNTED>
__global__ __launch_bounds__(256) void window_reads_kernel(
    const uint8_t *__restrict__ seq, uint64_t seq_len, unsigned K, int canonical,
    const uint64_t *__restrict__ read_starts, const uint32_t *__restrict__ read_counts, uint64_t n_reads,
    uint32_t cmax, Key<L> *__restrict__ out, uint32_t *__restrict__ outc, unsigned long long *__restrict__ cursor,
    uint32_t *__restrict__ bad) {
    constexpr int PER = 8;  // reads per thread, 256 apart
    __shared__ uint32_t s_scan[256 / 64 + 1];
    __shared__ unsigned long long s_base;
    const uint32_t tid = threadIdx.x;
    const uint64_t stride = K + 1;
    const Key<L> low = Key<L>::lowmask(2 * (K - 1));
    Key<L> kk[PER];
    uint32_t cc[PER];
    uint32_t valid = 0;
    bool err = false;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint64_t r = (uint64_t)blockIdx.x * (256 * PER) + (uint64_t)q * 256 + tid;
        if (r >= n_reads) continue;
        const uint64_t s0 = r * stride;
        err |= read_starts[r] != s0 || (s0 + K < seq_len && encode_dna(seq[s0 + K]) != 4u) || s0 + K > seq_len;
        if (s0 + K > seq_len) continue;
        Key<L> P = Key<L>::zero(), R = Key<L>::zero();
        bool ok = true;
        // the K chars through aligned 4-byte loads (a word never reaches past the one holding the
        // read's last char, so never into another page)
        const uint64_t a0 = s0 & ~3ull;
        unsigned i = 0;
        for (uint64_t a = a0; i < K; a += 4) {
            const uint32_t w = *(const uint32_t *)(seq + a);
            for (unsigned b = a == a0 ? (unsigned)(s0 - a0) : 0u; b < 4 && i < K; ++b, ++i) {
                uint32_t c = encode_dna((w >> (8 * b)) & 0xFFu);
                if (c == 4u) {
                    ok = false;
                    c = 0;
                }
                P = P | shl(Key<L>::from(c), 2 * i);
                R = R | shl(Key<L>::from(3u - c), 2 * (K - 1 - i));
            }
        }
        if (!ok) continue;
        Key<L> f = plain_to_boss(P, K, low);
        if (canonical) {
            const Key<L> rr = plain_to_boss(R, K, low);
            if (take_rc(canonical, f, rr, K)) f = rr;
        }
        kk[q] = f;
        if (COUNTED) {
            const uint32_t c = read_counts ? read_counts[r] : 1u;
            cc[q] = c < cmax ? c : cmax;
        }
        valid |= 1u << q;
    }
    if (err) atomicOr(bad, 1u);
    uint32_t total;
    uint32_t o = block_exclusive_sum<256>((uint32_t)__popc(valid), s_scan, &total);
    if (tid == 0) s_base = total ? atomicAdd(cursor, (unsigned long long)total) : 0ull;
    __syncthreads();
    const uint64_t base = s_base + o;
    uint32_t j = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        if (!((valid >> q) & 1u)) continue;
        out[base + j] = kk[q];
        if (COUNTED) outc[base + j] = cc[q];
        ++j;
    }
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
 * Valid k-mers are compacted in position order in two launches over the same tiling: the
 * COUNT_ONLY launch writes each tile's number of valid windows, the caller scans them, and the
 * full launch writes its tile's k-mers at that offset (block scan, staged in LDS, written
 * coalesced).  No inter-workgroup hand-off, so tiles need no dequeue counter.
 */
template <int L, bool COUNTED, bool COUNT_ONLY>
__global__ __launch_bounds__(256) void extract_kernel(
    const uint8_t *__restrict__ seq, uint64_t seq_len, unsigned K, int canonical,
    const uint64_t *__restrict__ read_starts, const uint32_t *__restrict__ read_counts,
    uint64_t n_reads, const uint64_t *__restrict__ rid_at, uint32_t cmax, Key<L> *__restrict__ out_keys,
    uint32_t *__restrict__ out_counts, uint32_t *__restrict__ tcnt,
    const uint64_t *__restrict__ toff, uint32_t *__restrict__ hist, unsigned hist_bits) {
    // hist: when hist_bits > 0, counts of the top hist_bits (<= 9) bits of the 2K-bit keys
    // written (the first MSD level's histogram, so the sort skips its own histogram pass)
    using T = ExtractTraits<L>;
    constexpr int BLOCK = T::BLOCK, PPT = T::PPT, TILE = T::TILE;
    __shared__ uint8_t s_code[TILE + T::MAXK];
    __shared__ Key<L> s_out[COUNT_ONLY ? 1 : TILE];
    __shared__ uint32_t s_cnt[COUNTED && !COUNT_ONLY ? TILE : 1];
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    __shared__ uint32_t s_hist[COUNT_ONLY ? 1 : 512];

    const uint32_t tid = threadIdx.x;
    const uint32_t tile = blockIdx.x;
    if (!COUNT_ONLY && hist_bits)
        for (uint32_t i = tid; i < (1u << hist_bits); i += BLOCK) s_hist[i] = 0;
    const uint64_t npos = seq_len >= K ? seq_len - K + 1 : 0;
    const uint64_t base = (uint64_t)tile * TILE;
    const uint64_t span_end = min(seq_len, base + TILE + K - 1);
    for (uint64_t i = base + tid; i < span_end; i += BLOCK) s_code[i - base] = encode_dna(seq[i]);
    __syncthreads();

    const uint64_t p0 = base + (uint64_t)tid * PPT;
    Key<L> kk[PPT];
    uint32_t cc[PPT];
    const uint32_t valid_mask = slide_windows<L, COUNTED, PPT, !COUNT_ONLY>(
        s_code, tid * PPT, p0, npos, K, canonical, read_starts, read_counts, n_reads, rid_at, cmax, kk, cc);
    const uint32_t nvalid = __popc(valid_mask);
    uint32_t tile_total;
    const uint32_t off = block_exclusive_sum<BLOCK>(nvalid, s_scan, &tile_total);
    if constexpr (COUNT_ONLY) {
        if (tid == 0) tcnt[tile] = tile_total;
        return;
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
    const uint64_t gb = toff[tile];
    for (uint32_t i = tid; i < tile_total; i += BLOCK) {
        const Key<L> key = s_out[i];
        out_keys[gb + i] = key;
        if (COUNTED) out_counts[gb + i] = s_cnt[i];
        if (hist_bits) atomicAdd(&s_hist[bits_at(key, 2 * K - hist_bits, hist_bits)], 1u);
    }
    if (hist_bits) {
        __syncthreads();
        for (uint32_t i = tid; i < (1u << hist_bits); i += BLOCK)
            if (s_hist[i]) atomicAdd(&hist[i], s_hist[i]);
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

// K4 for odd K (no palindromes): rc_out[i] = rc(keys[i]), counts carried along; with hist_bits,
// also the histogram of the top hist_bits bits of the rc keys (the rc sort's first MSD level)
template <int L, bool COUNTED>
__global__ __launch_bounds__(256) void rc_map_kernel(const Key<L> *__restrict__ keys,
                                                     const uint32_t *__restrict__ counts,
                                                     Key<L> *__restrict__ rc_out,
                                                     uint32_t *__restrict__ rc_counts, uint64_t n,
                                                     unsigned K, uint32_t *__restrict__ hist,
                                                     unsigned hist_bits) {
    __shared__ uint32_t s_hist[512];
    if (hist_bits)
        for (uint32_t i = threadIdx.x; i < (1u << hist_bits); i += 256) s_hist[i] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const Key<L> r = revcomp2(keys[i], K);
        rc_out[i] = r;
        if (COUNTED) rc_counts[i] = counts[i];
        if (hist_bits) atomicAdd(&s_hist[bits_at(r, 2 * K - hist_bits, hist_bits)], 1u);
    }
    if (hist_bits) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < (1u << hist_bits); i += 256)
            if (s_hist[i]) atomicAdd(&hist[i], s_hist[i]);
    }
}

// rc_map_kernel over a canonical set left in its speculative buckets (Ctx::gap in boss_pipeline.hip):
// bucket g's keys keys[bstart[g] ..) map to rc_out[ustart[g] .. ustart[g + 1]), one wave per bucket,
// 4 loads in flight per lane
template <int L>
__global__ __launch_bounds__(256) void rc_map_gapped_kernel(const Key<L> *__restrict__ keys,
                                                            const uint64_t *__restrict__ bstart,
                                                            const uint64_t *__restrict__ ustart, uint64_t nb,
                                                            Key<L> *__restrict__ rc_out, unsigned K,
                                                            uint32_t *__restrict__ hist, unsigned hist_bits) {
    __shared__ uint32_t s_hist[512];
    if (hist_bits)
        for (uint32_t i = threadIdx.x; i < (1u << hist_bits); i += 256) s_hist[i] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint64_t g = (uint64_t)blockIdx.x * 4 + wid; g < nb; g += (uint64_t)gridDim.x * 4) {
        const uint64_t src = bstart[g], dst = ustart[g], m = ustart[g + 1] - dst;
        for (uint64_t i0 = lane; i0 < m; i0 += 256) {
            Key<L> x[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (i0 + 64 * q < m) x[q] = keys[src + i0 + 64 * q];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (i0 + 64 * q >= m) break;
                const Key<L> r = revcomp2(x[q], K);
                if (rc_out) rc_out[dst + i0 + 64 * q] = r;  // (nullptr: the histogram only)
                if (hist_bits) atomicAdd(&s_hist[bits_at(r, 2 * K - hist_bits, hist_bits)], 1u);
            }
        }
    }
    if (hist_bits) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < (1u << hist_bits); i += 256)
            if (s_hist[i]) atomicAdd(&hist[i], s_hist[i]);
    }
}

/*
 * K4 fused with the rc sort's first MSD level (odd K, the canonical set in its speculative buckets,
 * Ctx::gap): the rc keys go straight into their level-1 buckets -- one cursor reservation per (tile,
 * bucket), the tile ranked by bucket in LDS and written as runs, as msd_partition_kernel does -- instead
 * of being written in canonical order by rc_map_gapped_kernel and partitioned by a second pass (its
 * histogram pass, rc_map_gapped_kernel with no output, gives the bucket starts).  A tile is TILE
 * consecutive compact positions p of the canonical set; p lies in canonical bucket g with ustart[g] <= p <
 * ustart[g + 1] and is read at keys[bstart[g] + p - ustart[g]]: the tile's slice of (ustart, bstart) is
 * staged in LDS and a position -> bucket map is built there by a max-scan (a binary search per position
 * measured 1.15 ms per cfg2 rc set vs 0.71 for the separate partition pass; the map, 0.95).  The
 * histogram pass is rc_map_gapped_kernel without output (0.39 ms; this kernel's own tiles counting
 * only: 0.55).
 */
template <int L>
struct RcPartTraits {
#ifndef MTG_RCP_ITEMS
#define MTG_RCP_ITEMS 16
#endif
    static constexpr int BLOCK = 512, ITEMS = L == 1 ? MTG_RCP_ITEMS : 8, TILE = BLOCK * ITEMS;
    static constexpr int NBM = 512;  // level-1 buckets at most (9 bits, rc_map_gapped_kernel's histogram)
    static constexpr int GS = 256;   // canonical buckets of the staged slice
};

// tile_g[t] = the canonical bucket holding compact position t * TILE (one thread per bucket: the tiles
// starting inside it), in place of a per-tile binary search over ustart (~20 dependent loads)
__global__ __launch_bounds__(256) void rc_tile_bucket_kernel(const uint64_t *__restrict__ ustart, uint64_t nb,
                                                             uint32_t tile, uint64_t *__restrict__ tile_g) {
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= nb) return;
    const uint64_t a = ustart[g], e = ustart[g + 1];
    for (uint64_t t = (a + tile - 1) / tile; t * tile < e; ++t) tile_g[t] = g;
}

template <int L>
__global__ __launch_bounds__(512) void rc_partition_gapped_kernel(
    const Key<L> *__restrict__ keys, const uint64_t *__restrict__ bstart, const uint64_t *__restrict__ ustart,
    const uint64_t *__restrict__ tile_g, uint64_t nb, uint64_t U, unsigned K, unsigned hb,
    unsigned long long *__restrict__ cursor, Key<L> *__restrict__ out) {
    using T = RcPartTraits<L>;
    constexpr int BLOCK = T::BLOCK, ITEMS = T::ITEMS, TILE = T::TILE, GS = T::GS, PER = T::NBM / BLOCK > 0 ? T::NBM / BLOCK : 1;
    __shared__ Key<L> s_keys[TILE];
    __shared__ uint32_t s_cnt[T::NBM], s_loff[T::NBM];
    __shared__ unsigned long long s_gbase[T::NBM];
    __shared__ uint64_t s_us[GS + 1], s_bs[GS];
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    const uint32_t tid = threadIdx.x;
    const uint64_t tile = xcd_tile((U + TILE - 1) / TILE);  // grid = xcd_grid(tiles)
    const uint64_t p0 = tile * TILE;
    if (p0 >= U) return;
    const uint64_t p1 = min(U, p0 + TILE);
    const uint32_t nbk = 1u << hb;
    for (uint32_t i = tid; i < nbk; i += BLOCK) s_cnt[i] = 0;
    const uint64_t g0 = tile_g[tile];  // the canonical bucket holding p0: the last g with ustart[g] <= p0
    for (uint32_t j = tid; j <= (uint32_t)GS; j += BLOCK) {
        const uint64_t gi = g0 + j;
        s_us[j] = gi <= nb ? ustart[gi] : ~0ull;
        if (j < (uint32_t)GS) s_bs[j] = gi < nb ? bstart[gi] : 0;
    }
    __syncthreads();
    const uint64_t send = s_us[GS];  // positions below this are inside the staged slice
    // the staged bucket of every tile position, as a map in the (not yet used) key tile: each non-empty
    // bucket starting inside the tile marks its first position, a block max-scan fills the rest
    uint16_t *s_map = reinterpret_cast<uint16_t *>(s_keys);
    static_assert(TILE % (8 * BLOCK) == 0 && TILE * 2 <= (int)sizeof(s_keys), "map layout");
    for (uint32_t i = tid; i < TILE / 8; i += BLOCK) reinterpret_cast<uint4 *>(s_map)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    for (uint32_t i = tid + 1; i < (uint32_t)GS; i += BLOCK)
        if (s_us[i] < s_us[i + 1] && s_us[i] < p1) s_map[s_us[i] - p0] = (uint16_t)i;  // s_us[i] > p0 (g0)
    __syncthreads();
    {
        constexpr int PT = TILE / BLOCK;  // positions per thread, contiguous
        uint16_t v[PT];
#pragma unroll
        for (int q = 0; q < PT / 8; ++q) {
            const uint4 w = reinterpret_cast<const uint4 *>(s_map)[tid * (PT / 8) + q];
            const uint32_t x[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int h = 0; h < 4; ++h) v[8 * q + 2 * h] = (uint16_t)x[h], v[8 * q + 2 * h + 1] = (uint16_t)(x[h] >> 16);
        }
        uint32_t m = 0;
#pragma unroll
        for (int q = 0; q < PT; ++q) m = max(m, (uint32_t)v[q]);
        const uint32_t lane = tid & 63, wid = tid >> 6;
        uint32_t inc = m;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t o = __shfl_up(inc, off, 64);
            if (lane >= (uint32_t)off) inc = max(inc, o);
        }
        uint32_t run = __shfl_up(inc, 1, 64);
        if (lane == 0) run = 0;
        if (lane == 63) s_scan[wid] = inc;
        __syncthreads();
        for (uint32_t w = 0; w < wid; ++w) run = max(run, s_scan[w]);
#pragma unroll
        for (int q = 0; q < PT; ++q) run = max(run, (uint32_t)v[q]), v[q] = (uint16_t)run;
#pragma unroll
        for (int q = 0; q < PT / 8; ++q) {
            uint32_t x[4];
#pragma unroll
            for (int h = 0; h < 4; ++h) x[h] = (uint32_t)v[8 * q + 2 * h] | ((uint32_t)v[8 * q + 2 * h + 1] << 16);
            reinterpret_cast<uint4 *>(s_map)[tid * (PT / 8) + q] = make_uint4(x[0], x[1], x[2], x[3]);
        }
    }
    __syncthreads();
    // sources first, then all ITEMS loads in flight, then the rc keys ranked by bucket
    uint64_t src[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint64_t p = p0 + (uint64_t)j * BLOCK + tid;
        src[j] = ~0ull;
        if (p >= p1) continue;
        if (p < send) {
            const uint32_t i = s_map[j * BLOCK + tid];
            src[j] = s_bs[i] + (p - s_us[i]);
        } else {  // a tile spanning more than GS canonical buckets (sparse ones): search them all
            uint64_t glo = g0 + GS - 1, ghi = nb;
            while (glo < ghi) {
                const uint64_t mid = (glo + ghi + 1) >> 1;
                if (ustart[mid] <= p) glo = mid; else ghi = mid - 1;
            }
            src[j] = bstart[glo] + (p - ustart[glo]);
        }
    }
    Key<L> k[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
        if (src[j] != ~0ull) k[j] = keys[src[j]];
    uint32_t r[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        r[j] = 0xFFFFFFFFu;
        if (src[j] == ~0ull) continue;
        k[j] = revcomp2(k[j], K);
        r[j] = atomicAdd(&s_cnt[bits_at(k[j], 2 * K - hb, hb)], 1u);
    }
    __syncthreads();
    uint32_t c[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid * PER + q;
        c[q] = i < nbk ? s_cnt[i] : 0;
        sum += c[q];
    }
    uint32_t total;
    uint32_t off = block_exclusive_sum<BLOCK>(sum, s_scan, &total);
    // (the run reservations stay in flight across the LDS scatter, as in the partition passes)
    unsigned long long gq[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid * PER + q;
        gq[q] = 0;
        if (i < nbk) {
            s_loff[i] = off;
            if (c[q]) gq[q] = atomicAdd(&cursor[i], (unsigned long long)c[q]);
        }
        off += c[q];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
        if (r[j] != 0xFFFFFFFFu) s_keys[s_loff[bits_at(k[j], 2 * K - hb, hb)] + r[j]] = k[j];
#pragma unroll
    for (int q = 0; q < PER; ++q)
        if (tid * PER + q < nbk) s_gbase[tid * PER + q] = gq[q];
    __syncthreads();
    for (uint32_t q = tid; q < total; q += BLOCK) {
        const Key<L> key = s_keys[q];
        const uint32_t b = bits_at(key, 2 * K - hb, hb);
        out[s_gbase[b] + (q - s_loff[b])] = key;
    }
}

/*
 * Bucket index over the top B bits of a sorted 2K-bit key array: start[b] = lower_bound of the
 * first key whose top bits are >= b.  Turns every membership probe below into a short binary
 * search inside one bucket (the probes of a wave land in a few neighbouring buckets).
 * Key i fills start[bucket(i-1)+1 .. bucket(i)] = i.  A long run of empty buckets -- keys clustered
 * in part of the prefix space: one rank's range, one key range of a batched build, which leaves
 * gaps of 7/8 of the index before and after the keys at 8 ranks -- goes to a global list that
 * bucket_fill_kernel spreads over the whole grid (filled by the one workgroup that found it
 * instead: 1.28 ms for a rank's index at 8 ranks, 0.9 ms for the single build's whole one).
 * A full list falls back to the workgroup fill.
 */
template <int L>
__global__ __launch_bounds__(256) void bucket_index_kernel(const Key<L> *__restrict__ keys, uint64_t n,
                                                           unsigned shift, uint64_t nbuckets,
                                                           uint64_t *__restrict__ start,
                                                           uint64_t *__restrict__ runs = nullptr,
                                                           uint32_t *__restrict__ nruns = nullptr,
                                                           uint32_t cap = 0) {
    constexpr int SHORT = 16;
    __shared__ uint64_t s_lo[256], s_hi[256], s_v[256];
    __shared__ uint32_t s_n;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 <= n; i0 += stride) {
        const uint64_t i = i0 + threadIdx.x;
        if (i <= n) {
            const uint64_t b = i < n ? bits_at(shr(keys[i], shift), 0, 32) : nbuckets;
            const uint64_t bp = i > 0 ? bits_at(shr(keys[i - 1], shift), 0, 32) + 1 : 0;
            const uint64_t hi = min(b, nbuckets);
            if (bp <= hi) {
                uint32_t g = ~0u;
                if (hi - bp < SHORT) {
                    for (uint64_t x = bp; x <= hi; ++x) start[x] = i;
                } else if (runs && (g = atomicAdd(nruns, 1u)) < cap) {
                    runs[3 * (uint64_t)g] = bp;
                    runs[3 * (uint64_t)g + 1] = hi;
                    runs[3 * (uint64_t)g + 2] = i;
                } else {
                    const uint32_t q = atomicAdd(&s_n, 1u);
                    s_lo[q] = bp;
                    s_hi[q] = hi;
                    s_v[q] = i;
                }
            }
        }
        __syncthreads();
        const uint32_t cnt = s_n;
        for (uint32_t q = 0; q < cnt; ++q)
            for (uint64_t x = s_lo[q] + threadIdx.x; x <= s_hi[q]; x += blockDim.x) start[x] = s_v[q];
        __syncthreads();
        if (threadIdx.x == 0) s_n = 0;
        __syncthreads();
    }
}

// the listed long runs of empty buckets, every run over the whole grid
__global__ __launch_bounds__(256) void bucket_fill_kernel(const uint64_t *__restrict__ runs,
                                                          const uint32_t *__restrict__ nruns, uint32_t cap,
                                                          uint64_t *__restrict__ start) {
    const uint32_t m = min(*nruns, cap);
    const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint32_t q = 0; q < m; ++q) {
        const uint64_t lo = runs[3 * (uint64_t)q], hi = runs[3 * (uint64_t)q + 1], v = runs[3 * (uint64_t)q + 2];
        for (uint64_t x = lo + t; x <= hi; x += T) start[x] = v;
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

template <int L>
struct DummyTraits {
    static constexpr int BLOCK = 256;
    static constexpr int PER = L == 1 ? 4 : 2;   // consecutive edges per thread
    static constexpr int TILE = BLOCK * PER;
    static constexpr int CAP = TILE * 5 / 4;     // staged real edges (the 4 sink ranges hold ~TILE)
    static constexpr int WTILE = 4096;           // edges per tile of the count / write passes
};

/*
 * K5 (sink pass) over the sorted real edges x (2-bit keys), one join of the reference's two
 * dummy scans:
 *   sink   -- add_dummy_sink_kmers (boss_chunk_construct.cpp:54-98): the target node a_2..a_K
 *             of x has no real out-edge  <=>  no y with y >> 2 == to_next(x, 0) >> 2;
 *   in-edge marks -- add_dummy_source_kmers (:123-168) emits a source for the first edge x of
 *             a node with no real y such that y's chars 2..k equal x's chars 1..k-1 and y's label
 *             is a_k: exactly "no real edge targets x's node".  So when the sink probe of x finds
 *             its target node, it marks that node's first edge in in_flag, and the count/write
 *             passes read source = first edge && !in_flag.
 * flags[i] = sink | first-edge-of-node << 1.
 *
 * This is the GPU form of the reference's per-character merge iterators.  A workgroup takes
 * TILE consecutive edges, PER consecutive ones per thread.  The sink probes of label c are
 * sorted (to_next is monotone on the edges of one label), so all edges they can hit lie in one
 * contiguous key range, found from the bucket index.  The 4 ranges (about TILE edges together)
 * are staged in LDS and every probe binary-searches its range there.  The kernel is bound by the
 * edges in flight per CU, which LDS caps: 10 bytes per edge (CAP = 1.25 TILE keys, no staged
 * bucket slices) instead of 20 (2 TILE keys + a bucket-start slice): 2.66 -> 2.21 ms at configs[1]
 * (8 edges per thread instead of 4: 2.59 ms).
 * A range that does not fit falls back to bucketed searches in global memory.
 */
// ABL (timing ablations for tools/stage_bench only; 0 in the product): bit 0 = no in_flag stores,
// bit 1 = no flags stores, bit 2 = no staging and no search (every edge a sink), bit 3 = staging
// but no search
// q (the multi-GPU build, run_pipeline_dist): the probes look up a separate sorted array q[0..nq) --
// the edges of other ranks whose nodes this rank's edges target -- whose bucket index is `start`;
// in_flag then marks q's edges.  Without q the probes look up keys itself.
template <int L, int ABL = 0>
__global__ __launch_bounds__(256) void dummy_sink_kernel(
    const Key<L> *__restrict__ keys, uint64_t n, unsigned K, const uint64_t *__restrict__ start,
    unsigned bshift, uint8_t *__restrict__ flags, uint8_t *__restrict__ in_flag,
    const Key<L> *__restrict__ q = nullptr, uint64_t nq = 0) {
    // (round 5) the tile's edges come in as 16-byte loads, a thread's PER flag bytes go out as one
    // store, and the in-edge marks of staged edges are set in LDS first and written over the staged
    // ranges in order (consecutive lanes, consecutive bytes) instead of one scattered byte per probe
    using T = DummyTraits<L>;
    const Key<L> *__restrict__ look = q ? q : keys;
    const uint64_t nl = q ? nq : n;
    constexpr int PER = T::PER;
    __shared__ Key<L> s_r[T::CAP];
    __shared__ uint32_t s_hit[(T::CAP + 3) / 4];  // in-edge marks of the staged edges (bytes)
    __shared__ uint64_t s_lo[4];
    __shared__ uint32_t s_cnt[4], s_off[4];
    const uint32_t tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * T::TILE;
    const uint32_t tn = (uint32_t)min((uint64_t)T::TILE, n - base);
    const Key<L> m3 = Key<L>::from(3);
    uint8_t *s_hitb = reinterpret_cast<uint8_t *>(s_hit);

    if (L != 1 && tid < 4) {
        // key range of the sink probes of label c = tid, read off the bucket index
        const Key<L> c = shl(Key<L>::from(tid), 2 * (K - 1));
        const Key<L> lo = (shr(keys[base], 2) | c) & ~m3;
        const Key<L> hi = shr(keys[base + tn - 1], 2) | c | m3;
        const uint64_t blo = bits_at(shr(lo, bshift), 0, 32), bhi = bits_at(shr(hi, bshift), 0, 32);
        const uint64_t a = start[blo], b = start[bhi + 1];
        s_lo[tid] = a;
        s_cnt[tid] = (uint32_t)min(b - a, (uint64_t)0xFFFFFFFFu);
    }
    for (uint32_t i = tid; i < (uint32_t)(T::CAP + 3) / 4; i += 256) s_hit[i] = 0;
    const uint32_t j0 = tid * PER;
    Key<L> x[PER];
    uint32_t first = 0;
    {
        Key<L> prev = base + j0 > 0 && j0 < tn ? keys[base + j0 - 1] : Key<L>::zero();
        const Key<L> *src = keys + base + j0;
        if constexpr (L == 1 && PER == 4) {
            if (j0 + PER <= tn && (((uintptr_t)src) & 15) == 0) {
                const ulonglong2 a = *(const ulonglong2 *)src, b = *(const ulonglong2 *)(src + 2);
                x[0] = Key<L>::from(a.x), x[1] = Key<L>::from(a.y), x[2] = Key<L>::from(b.x), x[3] = Key<L>::from(b.y);
            } else {
#pragma unroll
                for (int q2 = 0; q2 < PER; ++q2) x[q2] = j0 + q2 < tn ? src[q2] : Key<L>::zero();
            }
        } else {
#pragma unroll
            for (int q2 = 0; q2 < PER; ++q2) x[q2] = j0 + q2 < tn ? src[q2] : Key<L>::zero();
        }
#pragma unroll
        for (int q2 = 0; q2 < PER; ++q2) {
            if (j0 + q2 < tn) {
                if (base + j0 + q2 == 0 || shr(prev, 2) != shr(x[q2], 2)) first |= 1u << q2;
                prev = x[q2];
            }
        }
    }
    if constexpr (L == 1) {
        // (round 5) wave w finds and stages label class w on its own, into its quarter of s_r: no block-wide
        // pass over the four range sizes and two barriers fewer before the search (a class over a quarter,
        // ~5e-4 of them at configs[1], takes the global searches)
        constexpr uint32_t QC = T::CAP / 4;
        const uint32_t w = tid >> 6, lane = tid & 63;
        uint32_t alo = 0, ahi = 0, cnt = 0;
        if (lane == 0) {
            const Key<L> c = shl(Key<L>::from(w), 2 * (K - 1));
            const Key<L> lo = (shr(keys[base], 2) | c) & ~m3;
            const Key<L> hi = shr(keys[base + tn - 1], 2) | c | m3;
            const uint64_t blo = bits_at(shr(lo, bshift), 0, 32), bhi = bits_at(shr(hi, bshift), 0, 32);
            const uint64_t a = start[blo], b = start[bhi + 1];
            alo = (uint32_t)a, ahi = (uint32_t)(a >> 32);
            cnt = (uint32_t)min(b - a, (uint64_t)0xFFFFFFFFu);
        }
        const uint64_t a = (uint64_t)__shfl(alo, 0, 64) | ((uint64_t)__shfl(ahi, 0, 64) << 32);
        cnt = __shfl(cnt, 0, 64);
        const uint32_t off = cnt <= QC ? w * QC : ~0u;
        if (lane == 0) {
            s_lo[w] = a;
            s_cnt[w] = cnt;
            s_off[w] = off;
        }
        if (off != ~0u && !(ABL & 4)) {
            if ((((uintptr_t)look) & 15) == 0) {
                // the class's <= QC + 1 keys from the even index at or below a: all of a lane's 16-byte loads in
                // flight before its LDS stores (a rolled loop waited for each load before issuing the next)
                constexpr int NI = (int)((QC + 1 + 127) / 128);
                const uint64_t a0 = a & ~1ull, e = a + cnt;
                ulonglong2 v[NI];
#pragma unroll
                for (int q = 0; q < NI; ++q) {
                    const uint64_t i = a0 + 2ull * lane + 128ull * q;
                    if (i < e && i + 1 < nl) v[q] = *(const ulonglong2 *)(look + i);  // (never past the last key)
                }
#pragma unroll
                for (int q = 0; q < NI; ++q) {
                    const uint64_t i = a0 + 2ull * lane + 128ull * q;
                    if (i >= e) continue;
                    if (i + 1 < nl) {
                        if (i >= a) s_r[off + (uint32_t)(i - a)] = Key<L>::from(v[q].x);
                        if (i + 1 < e) s_r[off + (uint32_t)(i + 1 - a)] = Key<L>::from(v[q].y);
                    } else if (i >= a) {
                        s_r[off + (uint32_t)(i - a)] = look[i];
                    }
                }
            } else {
                for (uint32_t j = lane; j < cnt; j += 64) s_r[off + j] = look[a + j];
            }
        }
        __syncthreads();
    } else {
    __syncthreads();
    if (tid == 0) {
        uint32_t cum = 0;
        for (int c = 0; c < 4; ++c) {
            s_off[c] = ~0u;  // ~0 = global fallback
            if ((uint64_t)cum + s_cnt[c] <= (uint64_t)T::CAP) {
                s_off[c] = cum;
                cum += s_cnt[c];
            }
        }
    }
    __syncthreads();
    if constexpr (L != 1) {
        // (round 6) the staged classes fill s_r[0 .. sum of their counts) one after another: a thread's
        // positions tid + 256 k are mapped to their class and loaded all at once, limb by limb (a rolled
        // loop per class waited for each 16-byte load before issuing the next: configs[2]'s sink pass)
        if (!(ABL & 4)) {
            constexpr int NJ = (T::CAP + 255) / 256;
            uint64_t lv[NJ * L];
            uint32_t okm = 0;
#pragma unroll
            for (int k2 = 0; k2 < NJ; ++k2) {
                const uint32_t p = tid + 256u * k2;
                uint64_t idx = 0;
                bool ok = false;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const uint32_t o = s_off[c];
                    if (o != ~0u && p >= o && p - o < s_cnt[c]) {
                        ok = true;
                        idx = s_lo[c] + (p - o);
                    }
                }
#pragma unroll
                for (int w = 0; w < L; ++w) lv[k2 * L + w] = 0;
                if (ok) {
                    okm |= 1u << k2;
                    const Key<L> v = look[idx];
#pragma unroll
                    for (int w = 0; w < L; ++w) lv[k2 * L + w] = v.w[w];
                }
            }
#pragma unroll
            for (int k2 = 0; k2 < NJ; ++k2)
                if ((okm >> k2) & 1u) {
#pragma unroll
                    for (int w = 0; w < L; ++w) s_r[tid + 256u * k2].w[w] = lv[k2 * L + w];
                }
        }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if (L != 1 || (ABL & 4)) break;  // (u64: the per-wave classes above; wider keys: the flat staging)
        if (s_off[c] == ~0u) continue;
        const uint64_t a = s_lo[c];
        const uint32_t off = s_off[c], cnt = s_cnt[c];
        if constexpr (L == 1) {
            if ((((uintptr_t)look) & 15) == 0) {
                // 16-byte loads from the even index at or below a (half the load instructions)
                const uint64_t a0 = a & ~1ull, e = a + cnt;
                for (uint64_t i = a0 + 2ull * tid; i < e; i += 512) {
                    if (i + 1 < nl) {  // (never past the array's last key)
                        const ulonglong2 v = *(const ulonglong2 *)(look + i);
                        if (i >= a) s_r[off + (uint32_t)(i - a)] = Key<L>::from(v.x);
                        if (i + 1 < e) s_r[off + (uint32_t)(i + 1 - a)] = Key<L>::from(v.y);
                    } else if (i >= a) {
                        s_r[off + (uint32_t)(i - a)] = look[i];
                    }
                }
                continue;
            }
        }
        for (uint32_t j = tid; j < cnt; j += 256) s_r[off + j] = look[a + j];
    }
    __syncthreads();
    }
    uint32_t fw = 0;  // this thread's flag bytes, byte q = edge j0 + q
#pragma unroll
    for (int q2 = 0; q2 < PER; ++q2) {
        if (j0 + q2 >= tn) continue;
        if (ABL & 12) {
            fw |= (uint32_t)((uint8_t)(1u | (((first >> q2) & 1u) << 1)) ^ (uint8_t)s_r[q2 & 7].w[0]) << (8 * q2);
            continue;
        }
        const uint32_t c = (uint32_t)(x[q2].w[0] & 3);
        // to_next(x, K, 0): node a_2..a_K, label 0 (kmer_boss.hpp:147-169)
        const Key<L> p = (shr(x[q2], 2) | shl(Key<L>::from(c), 2 * (K - 1))) & ~m3;
        bool hit = false;
        const uint32_t off = s_off[c];
        if (off != ~0u) {
            const uint32_t cnt = s_cnt[c];
            uint32_t lo = 0, hi = cnt;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_r[off + mid] < p) lo = mid + 1; else hi = mid;
            }
            if (lo < cnt && shr(s_r[off + lo], 2) == shr(p, 2)) {
                hit = true;
                if (!(ABL & 1)) s_hitb[off + lo] = 1;
            }
        } else {
            const uint64_t i = lower_bound_bucketed(look, start, bshift, p);
            if (i < nl && shr(look[i], 2) == shr(p, 2)) {
                hit = true;
                if (!(ABL & 1)) in_flag[i] = 1;
            }
        }
        fw |= ((hit ? 0u : 1u) | (((first >> q2) & 1u) << 1)) << (8 * q2);
    }
    if (!(ABL & 2)) {
        uint8_t *fo = flags + base + j0;
        if (j0 + PER <= tn && (((uintptr_t)fo) & (PER - 1)) == 0) {
            if constexpr (PER == 4) *(uint32_t *)fo = fw;
            else *(uint16_t *)fo = (uint16_t)fw;
        } else {
#pragma unroll
            for (int q2 = 0; q2 < PER; ++q2)
                if (j0 + q2 < tn) fo[q2] = (uint8_t)(fw >> (8 * q2));
        }
    } else if (fw == 12345u) {
        flags[0] = 1;  // keep the search
    }
    if (ABL & 13) return;
    __syncthreads();
    // the marks of the staged edges, in order over each staged range (only 1s: the ranges of
    // neighbouring tiles overlap at their ends)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint32_t off = s_off[c];
        if (off == ~0u) continue;
        uint8_t *dst = in_flag + s_lo[c];
        for (uint32_t j = tid; j < s_cnt[c]; j += 256)
            if (s_hitb[off + j]) dst[j] = 1;
    }
}

// the 16 flag bytes of edges i0 .. i0 + 15 (i0 a multiple of 16; zero past n)
__device__ __forceinline__ void load_flags16(const uint8_t *__restrict__ f, uint64_t i0, uint64_t n,
                                             uint32_t (&w)[4]) {
    if (i0 + 16 <= n) {
        const uint4 v = *(const uint4 *)(f + i0);
        w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            w[q] = 0;
#pragma unroll
            for (int bb = 0; bb < 4; ++bb)
                if (i0 + 4 * q + bb < n) w[q] |= (uint32_t)f[i0 + 4 * q + bb] << (8 * bb);
        }
    }
}

// sinks (low 16 bits) and sources (high 16 bits) among edges i0 .. i0 + 15, bit j = edge i0 + j
__device__ __forceinline__ uint32_t dummy_masks16(const uint8_t *__restrict__ flags,
                                                  const uint8_t *__restrict__ in_flag, uint64_t i0,
                                                  uint64_t n) {
    uint32_t fw[4], iw[4];
    load_flags16(flags, i0, n, fw);
    load_flags16(in_flag, i0, n, iw);
    uint32_t sink = 0, src = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t f = (fw[j / 4] >> (8 * (j % 4))) & 0xFFu;
        const uint32_t in = (iw[j / 4] >> (8 * (j % 4))) & 0xFFu;
        sink |= (f & 1u) << j;
        src |= ((f >> 1) & ~in & 1u) << j;
    }
    return sink | src << 16;
}

// K6a: per-tile dummy counts (WTILE edges per workgroup, 16 consecutive per thread)
__global__ __launch_bounds__(256) void dummy_count_kernel(const uint8_t *__restrict__ flags,
                                                          const uint8_t *__restrict__ in_flag,
                                                          uint64_t n, unsigned k,
                                                          uint32_t *__restrict__ tcnt) {
    __shared__ uint32_t s_scan[256 / 64 + 1];
    const uint64_t i0 = (uint64_t)blockIdx.x * 4096 + threadIdx.x * 16;
    const uint32_t m = dummy_masks16(flags, in_flag, i0, n);
    const uint32_t cnt = __popc(m & 0xFFFFu) + __popc(m >> 16) * k;
    uint32_t total;
    block_exclusive_sum<256>(cnt, s_scan, &total);
    if (threadIdx.x == 0) tcnt[blockIdx.x] = total;
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
 * K6b (write pass): the workgroup's dummies go to its range of the scanned tile counts -- order
 * inside it is free, the dummies are sorted next.  Sinks first: lift(to_next(x,0)) with the label
 * char cleared to $ (:94), one per sink edge, by its owner thread.  Then every (source, level)
 * pair is an independent item spread over the whole workgroup: level 1 is lift(to_prev(x,0))
 * with char 1 cleared to $ (:165); level 1 + j is its j-fold to_prev(., $) (:286-303), in closed
 * form (node chars shifted up j places, label = the level-1 word's char K - j).
 */
// ------------------------------------------------------------------ dummy keys as dense ranks
//
// Every dummy edge of the construction (sinks boss_chunk_construct.cpp:54-98, sources of every
// level :123-168, 286-306), read from its most significant char down, is r_1 .. r_m $^(k-m) c: m
// real node chars, the $ run of a source of level k - m, then the label c (real for a source; $ for
// a sink, where m = k).  In the lifted order ($ < A < C < G < T) these strings are the leaves of a
// trie whose subtree below d real chars holds T(k) = 1, T(d) = 4 + 4 T(d + 1) = (7 4^(k-d) - 4) / 3
// strings (the 4 sources that stop there, then the A, C, G, T subtrees), so a dummy's rank among
// all of them is
//     4 m + sum_p r_p T(p) + (m < k ? c : 0)  =  4 m + (7 W - 4 S) / 3 + (m < k ? c : 0),
// W = the real chars as a left-aligned 2-bit word (r_1 highest, 4^(k-p) for r_p), S = their sum.
// The rank is an order-preserving injection into [0, T(0)), 62 bits at k = 30, so the dummy sort runs
// on u64 keys (8 LSD passes) instead of the 3(k+1)-bit lifted keys (k = 30: 93 bits, 12 passes over
// 16-byte keys).  Valid for k <= 30 (7 4^k < 2^64).  A key outside that shape raises *bad (the
// caller then sorts the lifted keys).

__host__ __device__ inline uint64_t dummy_rank_space(unsigned k) {  // T(0)
    return (7ull * (1ull << (2 * k)) - 4) / 3;
}

// The same ranks in 128 bits for 30 < k <= 62 (7 4^62 < 2^128): BASELINE configs[2]'s k = 63 build
// (k = 62) sorts 16-byte ranks (16 LSD passes) instead of its 32-byte lifted keys (24 passes).
// dummy_rank_limbs(k): limbs of the rank word (1: u64, 2: u128, 0: no rank form, sort the lifted keys).
typedef unsigned __int128 u128;
__host__ __device__ constexpr int dummy_rank_limbs(unsigned k) { return k <= 30 ? 1 : k <= 62 ? 2 : 0; }
template <int LR>
struct RankWordT {
    typedef uint64_t type;
};
template <>
struct RankWordT<2> {
    typedef u128 type;
};
template <int LR>
using RankWord = typename RankWordT<LR>::type;

// the inverse of 3 modulo 2^64 / 2^128: (7 W - 4 S) / 3 is exact (4^j = 1 mod 3, so W = S mod 3), and an
// exact quotient is the product with the inverse (no 128-bit division on the device)
template <typename R>
__host__ __device__ constexpr R inv3() {
    if constexpr (sizeof(R) == 16) return ((u128)0xAAAAAAAAAAAAAAAAull << 64) | 0xAAAAAAAAAAAAAAABull;
    else return (R)0xAAAAAAAAAAAAAAABull;
}
template <typename R>
__host__ __device__ inline R dummy_rank_space_t(unsigned k) {  // T(0) = (7 4^k - 4) / 3
    return (((R)7 << (2 * k)) - 4) * inv3<R>();
}
// bits of the rank space (host): the LSD passes of the rank sort cover them
inline unsigned dummy_rank_bits(unsigned k) {
    const u128 t = dummy_rank_space_t<u128>(k);
    const uint64_t hi = (uint64_t)(t >> 64), lo = (uint64_t)t;
    return hi ? 128 - (unsigned)__builtin_clzll(hi) : 64 - (unsigned)__builtin_clzll(lo);
}

template <int LR>
__device__ __forceinline__ Key<LR> rank_key(RankWord<LR> v) {
    Key<LR> r;
    r.w[0] = (uint64_t)v;
    if constexpr (LR == 2) r.w[1] = (uint64_t)(v >> 64);
    return r;
}
template <int LR>
__device__ __forceinline__ RankWord<LR> rank_word(const Key<LR> &k) {
    if constexpr (LR == 2) return ((u128)k.w[1] << 64) | k.w[0];
    else return k.w[0];
}
// a 2-bit key of at most 2 limbs as one integer (the rank path: 2K <= 128)
template <int L>
__device__ __forceinline__ u128 key_u128(const Key<L> &k) {
    static_assert(L <= 2, "rank path keys are at most 128 bits");
    if constexpr (L == 2) return ((u128)k.w[1] << 64) | k.w[0];
    else return k.w[0];
}

// the lifted key as one 128-bit integer (k <= 30: 3 (k + 1) <= 93 bits)
template <int L3>
__device__ __forceinline__ unsigned __int128 lifted128(const Key<L3> &x) {
    if constexpr (L3 == 1) return x.w[0];
    else return ((unsigned __int128)x.w[1] << 64) | x.w[0];
}

// sum of the 2-bit chars of a word
__device__ __forceinline__ uint64_t char_sum2(uint64_t w) {
    return (uint64_t)__popcll(w & 0x5555555555555555ull) + 2ull * (uint64_t)__popcll(w & 0xAAAAAAAAAAAAAAAAull);
}
__device__ __forceinline__ uint64_t char_sum2(u128 w) { return char_sum2((uint64_t)w) + char_sum2((uint64_t)(w >> 64)); }

// rank of the dummy with m real node chars forming the 2-bit word W (r_1 highest, $ run below) and
// label c (0..3; ignored for a sink, m = k)
__device__ __forceinline__ uint64_t dummy_rank(uint64_t W, unsigned m, unsigned k, uint32_t c) {
    return 4ull * m + (7 * W - 4 * char_sum2(W)) / 3 + (m < k ? (uint64_t)c : 0ull);
}
template <typename R>
__device__ __forceinline__ R dummy_rank_t(R W, unsigned m, unsigned k, uint32_t c) {
    return (R)(4u * m) + (7 * W - 4 * (R)char_sum2(W)) * inv3<R>() + (R)(m < k ? c : 0u);
}

// The source levels with few real chars (m <= DUMMY_BITMAP_M: levels k - m) repeat: a level-(k - m)
// dummy is fixed by the source node's first m + 1 chars, so ~S sources share at most 4^(m+1) of them.
// In the dense-rank path they are not written one per (source, level) but set one bit each in a bitmap
// over (m, first m chars, next char) -- (4^(DUMMY_BITMAP_M + 2) - 4) / 3 bits, 175 KB -- whose set
// bits dummy_bitmap_ranks_kernel appends as ranks: the sort takes ~S (k - DUMMY_BITMAP_M - 1) + the
// distinct few instead of S k keys.
constexpr unsigned DUMMY_BITMAP_M = 9;
constexpr unsigned DUMMY_BITMAP_LDS = 6;  // levels with <= 6 real chars: 21844 bits, an LDS copy per tile
__host__ __device__ constexpr uint64_t dummy_bitmap_base(unsigned m) {  // bits of the levels with < m real chars
    return ((1ull << (2 * (m + 1))) - 4) / 3;
}

// RANKS (k <= 62): the dummies as their dense ranks (dummy_rank, u64 for k <= 30: LR = 1, u128 for
// k <= 62: LR = 2) straight from the 2-bit edge -- a sink's real chars are the edge's target node
// (x >> 2 with the label moved on top), a level-l source's are the edge's first k - l node chars shifted
// up l places -- instead of lifted keys.
// bitmap (RANKS, LR = 1): the levels above kbig (m = k - level <= DUMMY_BITMAP_M) go to the bitmap
// instead (the count pass counted kbig levels per source); nullptr: every level written (kbig = k)
template <int L2, int L3, bool RANKS = false, int LR = 1>
__global__ __launch_bounds__(256) void dummy_write_kernel(
    const Key<L2> *__restrict__ keys, const uint8_t *__restrict__ flags,
    const uint8_t *__restrict__ in_flag, uint64_t n, unsigned K,
    const uint64_t *__restrict__ toff, Key<L3> *__restrict__ out, unsigned kbig = 0,
    uint32_t *__restrict__ bitmap = nullptr) {
    static_assert(!RANKS || LR == 1 || L2 <= 2, "u128 ranks: 2-bit keys of at most 128 bits");
    uint64_t *rout = reinterpret_cast<uint64_t *>(out);
    Key<2> *rout2 = reinterpret_cast<Key<2> *>(out);
    __shared__ uint32_t s_scan[256 / 64 + 1];
    __shared__ uint16_t s_src[4096];  // tile-relative edge index of each source
    const uint32_t tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * 4096;
    const uint64_t i0 = t0 + tid * 16;
    const unsigned k = K - 1;
    const uint32_t m = dummy_masks16(flags, in_flag, i0, n);
    // one scan of packed (sinks, sources): both fit 13 bits per tile
    const uint32_t packed = __popc(m & 0xFFFFu) | (uint32_t)__popc(m >> 16) << 16;
    uint32_t total;
    const uint32_t off = block_exclusive_sum<256>(packed, s_scan, &total);
    const uint32_t nsink = total & 0xFFFFu, nsrc = total >> 16;
    if (!nsink && !nsrc) return;
    const uint64_t base = toff[blockIdx.x];
    uint32_t so = off & 0xFFFFu, qo = off >> 16;
    const Key<L2> full = Key<L2>::lowmask(2 * K);
    const Key<L3> full3 = Key<L3>::lowmask(3 * K);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        if ((m >> j) & 1u) {
            const Key<L2> x = keys[i0 + j];
            const Key<L2> t = (shr(x, 2) | shl(Key<L2>::from(x.w[0] & 3), 2 * (K - 1))) &
                              ~Key<L2>::from(3);
            if constexpr (RANKS && LR == 2) rout2[base + so++] = rank_key<2>(dummy_rank_t<u128>(key_u128(t) >> 2, k, k, 0));
            else if constexpr (RANKS) rout[base + so++] = dummy_rank(t.w[0] >> 2, k, k, 0);
            else out[base + so++] = lift_fast<L3>(t, K) & ~Key<L3>::from(7);
        }
        if ((m >> (16 + j)) & 1u) s_src[qo++] = (uint16_t)(tid * 16 + j);
    }
    __syncthreads();
    if constexpr (RANKS && LR == 2) {
        Key<2> *o = rout2 + base + nsink;
        for (uint32_t it = tid; it < nsrc * k; it += 256) {
            const uint32_t q = it / k, lev = it - q * k + 1;  // level 1 .. k
            const u128 node = key_u128(keys[t0 + s_src[q]]) >> 2;  // a_1 .. a_k, a_1 lowest
            const u128 low = node & ((((u128)1) << (2 * (k - lev))) - 1);  // a_1 .. a_(k - lev)
            o[it] = rank_key<2>(dummy_rank_t<u128>(low << (2 * lev), k - lev, k, (uint32_t)(node >> (2 * (k - lev))) & 3u));
        }
        return;
    }
    if constexpr (RANKS) {
        uint64_t *o = rout + base + nsink;
        const unsigned kb = bitmap ? kbig : k;
        for (uint32_t it = tid; it < nsrc * kb; it += 256) {
            const uint32_t q = it / kb, lev = it - q * kb + 1;  // level 1 .. kb
            const uint64_t node = keys[t0 + s_src[q]].w[0] >> 2;  // a_1 .. a_k, a_1 lowest
            const uint64_t low = node & ((1ull << (2 * (k - lev))) - 1);  // a_1 .. a_(k - lev)
            o[it] = dummy_rank(low << (2 * lev), k - lev, k, (uint32_t)(node >> (2 * (k - lev))) & 3u);
        }
        if (bitmap) {
            // the levels with <= DUMMY_BITMAP_LDS real chars (a few thousand bits that every tile's sources
            // hit) gather in an LDS copy first and reach the global bitmap once per word and tile; the
            // others set their bits directly.  Either way a word already holding the bits (an agent-scope
            // load, past the non-coherent L1) takes no atomic (0.28 -> 0.49 ms for the write pass when every
            // (source, level) item took a global atomic on a few hot words)
            constexpr unsigned ML = DUMMY_BITMAP_LDS;
            constexpr uint32_t WL = (uint32_t)((dummy_bitmap_base(ML + 1) + 31) / 32);
            __shared__ uint32_t s_bm[WL];
            for (uint32_t w = tid; w < WL; w += 256) s_bm[w] = 0;
            __syncthreads();
            const unsigned ks = k - kb;  // levels kb + 1 .. k: m = k - level real chars, m <= DUMMY_BITMAP_M
            for (uint32_t it = tid; it < nsrc * ks; it += 256) {
                const uint32_t q = it / ks, m = it - q * ks;  // m = 0 .. ks - 1
                const uint64_t node = keys[t0 + s_src[q]].w[0] >> 2;
                const uint64_t low = node & ((1ull << (2 * m)) - 1);
                const uint64_t idx = dummy_bitmap_base(m) + (low << 2 | ((node >> (2 * m)) & 3u));
                const uint32_t bit = 1u << (idx & 31);
                if (m <= ML) {
                    atomicOr(&s_bm[idx >> 5], bit);
                } else if (!(__hip_atomic_load(&bitmap[idx >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit)) {
                    atomicOr(&bitmap[idx >> 5], bit);
                }
            }
            __syncthreads();
            for (uint32_t w = tid; w < WL; w += 256) {
                const uint32_t v = s_bm[w];
                if (v && (v & ~__hip_atomic_load(&bitmap[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))
                    atomicOr(&bitmap[w], v);
            }
        }
        return;
    }
    Key<L3> *o = out + base + nsink;
    for (uint32_t it = tid; it < nsrc * k; it += 256) {
        const uint32_t q = it / k, lev = it - q * k;
        const Key<L2> x = keys[t0 + s_src[q]];
        const Key<L2> prev = (shl(x & ~Key<L2>::from(3), 2) & full) | shr(x, 2 * (K - 1));
        const Key<L3> d1 = lift_fast<L3>(prev, K) & ~Key<L3>::from(7 << 3);
        o[it] = lev == 0 ? d1
                         : (shl(d1 & ~Key<L3>::from(7), 3 * lev) & full3) |
                               Key<L3>::from(char_at(d1, K - lev, 3));
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

// outputs per merge workgroup: the two staged runs and the output image fit 32 KB of LDS, so
// several workgroups share a CU and hide the loads
template <int LO>
struct MergeTraits {
    static constexpr int TILE = LO == 1 ? 2048 : LO == 2 ? 1024 : 512;
};

// diagonal split of every tile boundary (one thread each, all in flight together)
template <int LO, int LA, bool LIFT, int TILE = MergeTraits<LO>::TILE>
__global__ void merge_partition_kernel(const Key<LA> *__restrict__ a, uint64_t na,
                                       const Key<LO> *__restrict__ b, uint64_t nb, unsigned K,
                                       uint64_t ntiles, uint64_t *__restrict__ splits) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntiles) return;
    const uint64_t diag = min(na + nb, t * (uint64_t)TILE);
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
    constexpr int TILE = MergeTraits<LO>::TILE, ITEMS = TILE / 256;
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

/*
 * K7 + K8 without materialising the merge ("split emit").  The stream rows are the lifted real
 * edges A (2-bit keys, sorted) and the sorted distinct dummies B, interleaved in key order behind
 * the main dummy row.  Two facts of the reference's construction make each row's W and last
 * depend on its own array only:
 *  - no dummy shares a node with a real edge: a sink exists only for a node that no real edge
 *    leaves (boss_chunk_construct.cpp:63-97), and a source's node starts with $ (:123-168).  So
 *    `last` of a real row compares it with the next real edge, and a dummy's with the next dummy;
 *  - no dummy shares (chars 2..k, label) with a real edge: a level-1 source exists only when no
 *    real edge has its chars 2..k and label (:148-166), higher levels have $ at char 2, and sinks
 *    carry the label $.  So the W "minus" flag (boss_chunk.cpp:91-103) of a real row looks at
 *    real rows only, and a dummy's at dummies only.
 * dummy_rank_kernel checks both facts for every dummy against its group-mates in A, and also
 * flags a redundant dummy sink (a row initialize_chunk skips).  Any hit raises *skip, and the
 * caller then runs the exact unfused path (merge_kernel + the compacting emit_kernel).
 *
 * unlift_floor: the 2-bit X with #{A : lift(A) < b} = #{A : A < X}.  Walking b's chars from the
 * top, lift(A) and b compare as A's char + 1 against b's char until b's first $, where every A
 * that matched so far is bigger (lifted chars are >= 1).  So X = b's chars - 1 above that $,
 * zeros from it down.
 */
// 21 2-bit digits (bits 2d, 2d + 1) spread to 3-bit slots (bits 3d, 3d + 1): five mask-and-shift steps,
// the units whose index has bit s set moving up 2^s places, highest s first (so no unit passes another)
struct SpreadMasks {
    uint64_t m[5];
};
__host__ __device__ constexpr SpreadMasks make_spread_masks() {
    SpreadMasks r{};
    int pos[21] = {};
    for (int d = 0; d < 21; ++d) pos[d] = 2 * d;
    for (int s = 4, i = 0; s >= 0; --s, ++i) {
        uint64_t mk = 0;
        for (int d = 0; d < 21; ++d)
            if ((d >> s) & 1) {
                mk |= 3ull << pos[d];
                pos[d] += 1 << s;
            }
        r.m[i] = mk;
    }
    return r;
}
// the same units at their positions after each spread step (compress21 runs the steps backwards)
__host__ __device__ constexpr SpreadMasks make_compress_masks() {
    SpreadMasks r{};
    int pos[21] = {};
    for (int d = 0; d < 21; ++d) pos[d] = 2 * d;
    for (int s = 4, i = 0; s >= 0; --s, ++i) {
        uint64_t mk = 0;
        for (int d = 0; d < 21; ++d)
            if ((d >> s) & 1) {
                pos[d] += 1 << s;
                mk |= 3ull << pos[d];
            }
        r.m[i] = mk;
    }
    return r;
}
// 21 values in 3-bit slots (low 2 bits each) packed to 2-bit digits: spread21 inverted
__device__ __forceinline__ uint64_t compress21(uint64_t x) {
    constexpr SpreadMasks M = make_compress_masks();
#pragma unroll
    for (int i = 4; i >= 0; --i) x = (x & ~M.m[i]) | ((x & M.m[i]) >> (16 >> i));
    return x;
}
__device__ __forceinline__ uint64_t spread21(uint64_t x) {
    constexpr SpreadMasks M = make_spread_masks();
#pragma unroll
    for (int i = 0; i < 5; ++i) x = (x & ~M.m[i]) | ((x & M.m[i]) << (16 >> i));
    return x;
}

template <int L2, int L3>
__device__ __forceinline__ Key<L2> unlift_floor(const Key<L3> &b, unsigned K) {
    // (round 5) by 21-slot pieces instead of char by char: every slot minus 1 (a $ stays 0), packed to
    // 2-bit digits (compress21), then the digits at and below the highest $ slot cleared -- the walk
    // cost one 3-bit extract and one shifted OR of a K-char key per char (configs[2]: 54 ms of
    // dummy_rank_kernel for 6.6e8 dummies)
    constexpr uint64_t ONES = 0x1249249249249249ull;  // 001 in every 3-bit slot (21 slots)
    Key<L2> x = Key<L2>::zero();
    int zs = -1;  // the highest $ slot
#pragma unroll
    for (int pi = 0; pi < 5; ++pi) {  // K <= 105 chars
        const unsigned s0 = 21u * pi;
        if (s0 >= K || 63 * pi >= 64 * L3) break;
        const unsigned ns = K - s0 < 21u ? K - s0 : 21u;
        const uint64_t vm = ns == 21u ? (1ull << 63) - 1 : (1ull << (3 * ns)) - 1;
        const uint64_t v = shr(b, 63 * pi).w[0] & vm;
        const uint64_t nz = (v | (v >> 1) | (v >> 2)) & ONES & vm;
        const uint64_t z = ~nz & ONES & vm;
        if (z) zs = (int)s0 + (63 - __clzll((long long)z)) / 3;
        if (2 * s0 < 64 * L2) x = x | shl(Key<L2>::from(compress21(v - nz)), 2 * s0);
    }
    if (zs >= 0) x = x & ~Key<L2>::lowmask(2 * (unsigned)(zs + 1));
    return x;
}

// per dummy j: its output row pos[j] (row0 = output row of the first merged row) and its
// W | last << 4 byte; *root_same = the main dummy row and B[0] share the all-$ node
template <int L2, int L3>
__global__ __launch_bounds__(256) void dummy_rank_kernel(
    const Key<L2> *__restrict__ a, uint64_t na, const Key<L3> *__restrict__ b, uint64_t nb, unsigned K,
    const uint64_t *__restrict__ bstart, unsigned bshift, uint64_t row0, uint64_t *__restrict__ pos,
    uint8_t *__restrict__ wl, uint32_t *__restrict__ skip, uint32_t *__restrict__ root_same) {
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= nb) return;
    const unsigned k = K - 1;
    const Key<L3> x = b[j];
    const Key<L2> X = unlift_floor<L2, L3>(x, K);
    uint64_t r;
    if (bstart) {
        r = lower_bound_bucketed(a, bstart, bshift, X);
    } else {
        uint64_t lo = 0, hi = na;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (a[mid] < X) lo = mid + 1; else hi = mid;
        }
        r = lo;
    }
    pos[j] = row0 + j + r;
    const Key<L3> node = shr(x, 3), grp = shr(x, 6);
    const uint32_t c = (uint32_t)(x.w[0] & 7);
    bool bad = false;
    // the real edges of x's chars-2..k group sit next to r (at most 16: 4 first chars x 4 labels); a
    // dummy with $ in char slot 2 (a source of level >= 2) has no real edge in its group: real edges
    // have no $ (skipped: two lifted real edges a dummy)
    const bool near = K < 3 || char_at(x, 2, 3) != 0;
    for (uint64_t i = r; near && i < na && i < r + 16; ++i) {
        const Key<L3> y = lift_fast<L3>(a[i], K);
        if (shr(y, 6) != grp) break;
        bad |= shr(y, 3) == node || (c && (uint32_t)(y.w[0] & 7) == c);
    }
    for (uint64_t i = r; near && i > 0 && i + 16 > r; --i) {
        const Key<L3> y = lift_fast<L3>(a[i - 1], K);
        if (shr(y, 6) != grp) break;
        bad |= shr(y, 3) == node || (c && (uint32_t)(y.w[0] & 7) == c);
    }
    uint32_t w = c;
    if (c) {  // "minus" among the dummies of the group (at most 25 rows)
        for (uint64_t p = j; p > 0; --p) {
            const Key<L3> y = b[p - 1];
            if (shr(y, 6) != grp) break;
            if ((uint32_t)(y.w[0] & 7) == c) { w = c + 5; break; }
        }
    }
    const bool same_next = j + 1 < nb && shr(b[j + 1], 3) == node;
    if (same_next && c == 0 && char_at(x, k, 3) > 0) bad = true;  // redundant sink (boss_chunk.cpp:78-86)
    wl[j] = (uint8_t)(w | (same_next ? 0u : 1u) << 4);
    if (j == 0 && node == Key<L3>::zero()) *root_same = 1;
    if (bad) atomicOr(skip, 1u);
}

template <int L2>
struct SplitEmitTraits {
    static constexpr int TILE = L2 <= 2 ? 2048 : 1024;  // output rows per workgroup
    static constexpr int PER = 8;                        // consecutive rows per thread
    static constexpr int BLOCK = TILE / PER;
    static constexpr int HALO = 16;                      // real edges staged before the tile
};

// jsplit[t] = #dummies whose output row is < t * TILE (one binary search per tile boundary)
template <int TILE>
__global__ void split_points_kernel(const uint64_t *__restrict__ pos, uint64_t nb, uint64_t ntiles,
                                    uint64_t *__restrict__ jsplit) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntiles) return;
    const uint64_t o = t * (uint64_t)TILE;
    uint64_t lo = 0, hi = nb;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (pos[mid] < o) lo = mid + 1; else hi = mid;
    }
    jsplit[t] = lo;
}

/*
 * The output rows [o0, o0 + TILE): row 0 is the leading all-zero row, row 1 the main dummy (when
 * `root`), then the merged stream.  The tile's dummies are the pos[] entries in range (bitmask
 * in LDS); the real edges between them are a contiguous run of A, staged in LDS with HALO edges
 * before it (a chars-2..k group holds at most 16 real edges, so the "minus" look-back never
 * leaves LDS) and one after it (the `last` compare).  A thread owns PER consecutive rows, so W
 * and last leave as one aligned 8-byte store each.
 */
template <int L2, bool COUNTED>
__global__ __launch_bounds__(SplitEmitTraits<L2>::BLOCK) void split_emit_kernel(
    const Key<L2> *__restrict__ a, const uint32_t *__restrict__ ac, uint64_t na,
    const uint64_t *__restrict__ pos, const uint8_t *__restrict__ wl, const uint64_t *__restrict__ jsplit,
    uint64_t nout, uint32_t root, const uint32_t *__restrict__ root_same, uint32_t wmax,
    uint8_t *__restrict__ W, uint8_t *__restrict__ last, uint32_t *__restrict__ weights) {
    using T = SplitEmitTraits<L2>;
    constexpr int TILE = T::TILE, PER = T::PER, HALO = T::HALO, BLOCK = T::BLOCK;
    __shared__ Key<L2> s_a[TILE + HALO + 1];
    __shared__ uint8_t s_bwl[TILE];
    __shared__ uint32_t s_bm[TILE / 32];
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    const uint32_t tid = threadIdx.x;
    const uint64_t o0 = (uint64_t)blockIdx.x * TILE;
    const uint64_t o1 = min(nout, o0 + TILE);
    const uint64_t j0 = jsplit[blockIdx.x], j1 = jsplit[blockIdx.x + 1];
    const uint32_t nbt = (uint32_t)(j1 - j0);
    const uint64_t lead = 1 + root;  // output rows before the merged stream
    const uint64_t m0 = o0 > lead ? o0 - lead : 0, m1 = o1 > lead ? o1 - lead : 0;
    const uint64_t i0 = m0 - j0;                  // first real edge of the tile
    const uint64_t i1 = m1 - j1;                  // one past its last
    // stage A[i0 - HALO, i1 + 1) (clipped to [0, na))
    const int64_t g0 = (int64_t)i0 - HALO;
    const uint32_t ns = (uint32_t)(i1 - i0) + HALO + 1;
    if constexpr (L2 == 1) {
        // all of a thread's staging loads in flight before the LDS stores (a rolled loop waited for each
        // load before issuing the next: one 8-byte load per wave in flight).  u64 keys only: the wider
        // keys' register array spilled (configs[2]: lift + merge 52 -> 67 ms)
        constexpr int SQ = (TILE + HALO + 1 + BLOCK - 1) / BLOCK;
        Key<L2> st[SQ];
#pragma unroll
        for (int q = 0; q < SQ; ++q) {
            const uint32_t qq = tid + q * BLOCK;
            const int64_t g = g0 + qq;
            if (qq < ns && g >= 0 && g < (int64_t)na) st[q] = a[g];
        }
#pragma unroll
        for (int q = 0; q < SQ; ++q) {
            const uint32_t qq = tid + q * BLOCK;
            const int64_t g = g0 + qq;
            if (qq < ns && g >= 0 && g < (int64_t)na) s_a[qq] = st[q];
        }
    } else {
        // wider keys: three loads in flight per thread at a time (configs[2]'s u128 edges), held limb by limb
        // (an array of keys went to scratch memory)
        constexpr int CH = 3;
        for (uint32_t b0 = 0; b0 < ns; b0 += CH * BLOCK) {
            uint64_t st[CH * L2];
#pragma unroll
            for (int q = 0; q < CH; ++q) {
                const uint32_t qq = b0 + tid + q * BLOCK;
                const int64_t g = g0 + qq;
                if (qq < ns && g >= 0 && g < (int64_t)na) {
                    const Key<L2> v = a[g];
#pragma unroll
                    for (int w = 0; w < L2; ++w) st[q * L2 + w] = v.w[w];
                }
            }
#pragma unroll
            for (int q = 0; q < CH; ++q) {
                const uint32_t qq = b0 + tid + q * BLOCK;
                const int64_t g = g0 + qq;
                if (qq < ns && g >= 0 && g < (int64_t)na) {
#pragma unroll
                    for (int w = 0; w < L2; ++w) s_a[qq].w[w] = st[q * L2 + w];
                }
            }
        }
    }
    for (uint32_t q = tid; q < TILE / 32; q += BLOCK) s_bm[q] = 0;
    __syncthreads();
    for (uint32_t q = tid; q < nbt; q += BLOCK) {
        const uint32_t off = (uint32_t)(pos[j0 + q] - o0);
        s_bwl[q] = wl[j0 + q];
        atomicOr(&s_bm[off >> 5], 1u << (off & 31));
    }
    __syncthreads();
    const uint32_t r0 = tid * PER;
    const uint32_t bits = (s_bm[r0 >> 5] >> (r0 & 31)) & 0xFFu;
    uint32_t tot;
    const uint32_t bq0 = block_exclusive_sum<BLOCK>((uint32_t)__popc(bits), s_scan, &tot);
    uint64_t wpack = 0, lpack = 0;
    uint32_t wt[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        wt[q] = 0;
        const uint64_t o = o0 + r0 + q;
        if (o >= o1) continue;
        uint32_t ww = 0, ll = 0;
        const uint32_t bq = bq0 + (uint32_t)__popc(bits & ((1u << q) - 1));
        if (o < lead) {
            ll = o == 0 ? 0u : (*root_same ? 0u : 1u);  // leading row; main dummy row
        } else if ((bits >> q) & 1u) {
            const uint32_t v = s_bwl[bq];
            ww = v & 15u;
            ll = v >> 4;
        } else {
            const uint64_t ia = (o - lead) - (j0 + bq);
            const uint32_t li = (uint32_t)(ia - i0) + HALO;
            const Key<L2> x = s_a[li];
            const uint32_t c = (uint32_t)(x.w[0] & 3);
            const Key<L2> grp = shr(x, 4);
            bool minus = false;
            const uint32_t back = (uint32_t)min<uint64_t>(ia, HALO - 1);
            for (uint32_t p = 1; p <= back; ++p) {
                const Key<L2> y = s_a[li - p];
                if (shr(y, 4) != grp) break;
                if ((uint32_t)(y.w[0] & 3) == c) { minus = true; break; }
            }
            ww = c + 1 + (minus ? 5u : 0u);
            ll = ia + 1 < na && shr(s_a[li + 1], 2) == shr(x, 2) ? 0u : 1u;
            if (COUNTED) {
                const uint32_t cnt = ac[ia];
                wt[q] = cnt < wmax ? cnt : wmax;
            }
        }
        wpack |= (uint64_t)ww << (8 * q);
        lpack |= (uint64_t)ll << (8 * q);
    }
    const uint64_t ob = o0 + r0;
    if (ob + PER <= o1) {
        *(uint64_t *)(W + ob) = wpack;
        *(uint64_t *)(last + ob) = lpack;
        if (COUNTED) {
            *(uint4 *)(weights + ob) = make_uint4(wt[0], wt[1], wt[2], wt[3]);
            *(uint4 *)(weights + ob + 4) = make_uint4(wt[4], wt[5], wt[6], wt[7]);
        }
    } else {
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            if (ob + q >= o1) break;
            W[ob + q] = (uint8_t)(wpack >> (8 * q));
            last[ob + q] = (uint8_t)(lpack >> (8 * q));
            if (COUNTED) weights[ob + q] = wt[q];
        }
    }
}

// F[c] = #stream rows whose last node char < c: the root ($), lifted A (char + 1) and B, by
// binary search on each sorted array (f_bounds_kernel without the materialised stream)
template <int LO, int LA>
__global__ void f_bounds_split_kernel(const Key<LA> *__restrict__ a, uint64_t na, const Key<LO> *__restrict__ b,
                                      uint64_t nb, unsigned K, uint64_t root, unsigned long long *__restrict__ F) {
    const uint32_t c = threadIdx.x;
    if (c >= 5) return;
    const unsigned k = K - 1;
    uint64_t lo = 0, hi = na;  // A: 2-bit char k + 1 < c
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (char_at(a[mid], k, 2) + 1 < c) lo = mid + 1; else hi = mid;
    }
    uint64_t fa = lo;
    lo = 0;
    hi = nb;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (char_at(b[mid], k, 3) < c) lo = mid + 1; else hi = mid;
    }
    F[c] = fa + lo + (root && c > 0 ? 1 : 0);
}

__global__ void set_root_row_kernel(uint64_t *key_words, int limbs, uint32_t *count) {
    for (int i = 0; i < limbs; ++i) key_words[i] = 0;  // the main dummy KMER(0)
    if (count) *count = 0;
}

/*
 * K8 fast path: the same rows as emit_kernel below when no row is a redundant dummy sink, which
 * is the normal case (the dummy unique leaves at most one sink per node and a sink's node has no
 * other out-edge); a skip row sets *skip and the caller reruns the compacting emit_kernel.
 * Row r goes to output r + 1 (row 0 of the output is the leading all-$ row).  A thread owns 8
 * consecutive OUTPUTS, so W and last leave as one aligned 8-byte store each and the weights as
 * two 16-byte stores; rows r-1 and r+1 come from the same sliding window of keys, and the
 * same-group look-back for the W "minus" flag rarely leaves the window.
 */
template <int L3, bool COUNTED>
__global__ __launch_bounds__(256) void emit_fast_kernel(
    const Key<L3> *__restrict__ s, const uint32_t *__restrict__ sc, uint64_t m, unsigned k,
    uint32_t wmax, uint8_t *__restrict__ W, uint8_t *__restrict__ last,
    uint32_t *__restrict__ weights, uint32_t *__restrict__ skip) {
    constexpr int PER = 8;
    const uint64_t o0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * PER;
    if (o0 > m) return;
    // window: rows o0 - 2 .. o0 + PER - 1 (row r = output o - 1)
    Key<L3> win[PER + 2];
#pragma unroll
    for (int j = 0; j < PER + 2; ++j) {
        const int64_t r = (int64_t)o0 - 2 + j;
        win[j] = r >= 0 && r < (int64_t)m ? s[r] : Key<L3>::zero();
    }
    uint64_t wpack = 0, lpack = 0;
    uint32_t wt[PER];
    bool skipped = false;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        wt[j] = 0;
        const int64_t r = (int64_t)o0 - 1 + j;
        if (r < 0 || r >= (int64_t)m) continue;
        const Key<L3> key = win[j + 1];
        const uint32_t c = (uint32_t)(key.w[0] & 7);
        const Key<L3> node = shr(key, 3);
        const bool same_next = r + 1 < (int64_t)m && shr(win[j + 2], 3) == node;
        if (same_next && c == 0 && char_at(key, k, 3) > 0) skipped = true;
        uint32_t ww = c;
        if (c) {
            // an earlier row of the same chars-2..k group with the same label -> "minus"
            const Key<L3> grp = shr(key, 6);
            int64_t p = r - 1;
            bool done = false;
#pragma unroll
            for (int q = j; q >= 0; --q) {  // window rows r-1 .. o0-2
                if (done || p < 0) break;
                const Key<L3> y = win[q];
                if (shr(y, 6) != grp) done = true;
                else if ((uint32_t)(y.w[0] & 7) == c) { ww = c + 5; done = true; }
                --p;
            }
            for (; !done && p >= 0; --p) {
                const Key<L3> y = s[p];
                if (shr(y, 6) != grp) break;
                if ((uint32_t)(y.w[0] & 7) == c) { ww = c + 5; break; }
            }
        }
        wpack |= (uint64_t)ww << (8 * j);
        lpack |= (uint64_t)(same_next ? 0 : 1) << (8 * j);
        if (COUNTED) {
            const uint32_t cnt = sc[r];
            wt[j] = (cnt && ww && char_at(key, 1, 3)) ? (cnt < wmax ? cnt : wmax) : 0;
        }
    }
    if (skipped) atomicOr(skip, 1u);
    if (o0 + PER <= m + 1) {
        *(uint64_t *)(W + o0) = wpack;
        *(uint64_t *)(last + o0) = lpack;
        if (COUNTED) {
            *(uint4 *)(weights + o0) = make_uint4(wt[0], wt[1], wt[2], wt[3]);
            *(uint4 *)(weights + o0 + 4) = make_uint4(wt[4], wt[5], wt[6], wt[7]);
        }
    } else {
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            if (o0 + j > m) break;
            W[o0 + j] = (uint8_t)(wpack >> (8 * j));
            last[o0 + j] = (uint8_t)(lpack >> (8 * j));
            if (COUNTED) weights[o0 + j] = wt[j];
        }
    }
}

// F[c] = number of stream rows whose last node char is < c (the stream is sorted by that char)
template <int L3>
__global__ void f_bounds_kernel(const Key<L3> *__restrict__ s, uint64_t m, unsigned k,
                                unsigned long long *__restrict__ F) {
    const uint32_t c = threadIdx.x;
    if (c >= 5) return;
    uint64_t lo = 0, hi = m;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (char_at(s[mid], k, 3) < c) lo = mid + 1; else hi = mid;
    }
    F[c] = lo;
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


template <int L3, int LR = 1>
__global__ void dummy_encode_kernel(const Key<L3> *__restrict__ in, uint64_t n, unsigned k,
                                    Key<LR> *__restrict__ out, uint32_t *__restrict__ bad) {
    using R = RankWord<LR>;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    bool err = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        const Key<L3> v = in[i];
        R W = 0;
        unsigned m = 0, top_dollar = 0;  // highest node position holding $
        for (unsigned j = 1; j <= k; ++j) {
            const uint32_t ch = char_at(v, j, 3);
            if (ch) {
                W |= (R)(ch - 1) << (2 * (j - 1));
                ++m;
            } else {
                top_dollar = j;
            }
        }
        const uint32_t c = (uint32_t)v.w[0] & 7u;
        // the $ run must be exactly node positions 1 .. k - m, the label real iff m < k
        err |= top_dollar != k - m || (m < k) != (c != 0) || c > 4 || shr(v, 3 * (k + 1)) != Key<L3>::zero();
        out[i] = rank_key<LR>(dummy_rank_t<R>(W, m, k, c - 1));
    }
    if (err) atomicOr(bad, 1u);
}

// the bitmap's dummies (dummy_write_kernel) appended as ranks at out[*cursor ..): one thread per word,
// one atomic per word with set bits (the order is free: the ranks are sorted next)
__global__ void dummy_bitmap_ranks_kernel(const uint32_t *__restrict__ bitmap, uint64_t nwords, unsigned k,
                                          unsigned ms, uint64_t *__restrict__ out,
                                          unsigned long long *__restrict__ cursor) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += gs) {
        uint32_t v = bitmap[w];
        if (!v) continue;
        uint64_t o = atomicAdd(cursor, (unsigned long long)__popc(v));
        while (v) {
            const uint32_t b = __ffs(v) - 1;
            v &= v - 1;
            const uint64_t idx = w * 32 + b;
            unsigned m = 0;
            while (m + 1 < ms && dummy_bitmap_base(m + 1) <= idx) ++m;
            const uint64_t r = idx - dummy_bitmap_base(m);  // low << 2 | c
            out[o++] = dummy_rank((r >> 2) << (2 * (k - m)), m, k, (uint32_t)(r & 3u));
        }
    }
}

// the inverse of an odd a modulo 2^64 / 2^128 (Newton: every step doubles the correct low bits)
template <typename R>
__host__ __device__ constexpr R inv_odd(R a) {
    R x = a;  // a * a = 1 mod 8 for odd a
    for (int i = 0; i < 7; ++i) x *= (R)2 - a * x;
    return x;
}

// The rank of a source dummy with m <= k - 5 real chars inverted in closed form: 3 r = 12 m + 7 W - 4 S + 3 c
// with 7 W a multiple of 4^(k - m) >= 2^10 and 0 <= 12 m - 4 S + 3 c < 2^10, so the low 10 bits of 3 r are
// eps = 12 m - 4 S + 3 c, W = (3 r - eps) / 7 (exact: times the inverse of 7), S = the digit sum of W, and
// eps + 4 S = 12 m + 3 c gives m and c.  A candidate whose digits lie in [k - m, k) has rank r, so it is
// the dummy (the rank is a bijection); anything else (sinks, the last 4 source levels) returns false and
// takes the char-by-char walk.  Writes the lifted key: real char p (digit k - p of W) + 1 at char slot
// k - p + 1, the label c + 1 at slot 0.
template <int L3, typename R>
__device__ __forceinline__ bool dummy_decode_fast(R r, unsigned k, Key<L3> &out) {
    constexpr R INV7 = inv_odd<R>((R)7);
    const R V = r * (R)3;
    const uint32_t eps = (uint32_t)V & 1023u;
    const R W = (V - (R)eps) * INV7;
    const uint32_t t = eps + 4u * (uint32_t)char_sum2(W);
    const uint32_t m = t / 12u, c = (t % 12u) / 3u;
    if (t % 3u || m + 5 > k || (W >> (2 * k)) != 0) return false;
    const unsigned lo = k - m;  // the lowest real digit
    if ((W & (((R)1 << (2 * lo)) - 1)) != 0) return false;
    constexpr uint64_t ONES = 0x1249249249249249ull & ((1ull << 63) - 1);  // 001 in every 3-bit slot
    Key<L3> x = Key<L3>::from((uint64_t)(c + 1));
#pragma unroll
    for (int pi = 0; pi < 3; ++pi) {
        const unsigned d0 = 21u * pi;  // digits d0 .. d0 + 20
        if (d0 >= k || 63 * pi + 3 >= 64 * L3) break;
        const uint64_t chunk = (uint64_t)(W >> (2 * d0)) & ((1ull << 42) - 1);
        const unsigned a = lo > d0 ? lo - d0 : 0u, b = k - d0 < 21u ? k - d0 : 21u;  // valid digits [a, b)
        const uint64_t ones = a < b ? (ONES & ((b == 21u ? ~0ull : (1ull << (3 * b)) - 1)) & ~((1ull << (3 * a)) - 1)) : 0ull;
        x = x | shl(Key<L3>::from(spread21(chunk) + ones), 63 * pi + 3);
    }
    out = x;
    return true;
}

// the char-by-char walk down the rank trie (any dummy: sinks, every source level)
template <int L3, typename R>
__device__ __forceinline__ Key<L3> dummy_decode_walk(R r, unsigned k, R T) {
    // the real chars r_1, r_2, ... enter at the bottom of x one by one (r_p ends up at node
    // position k - p + 1); then one shift leaves the $ run and the label below them
    Key<L3> x = Key<L3>::zero();
    unsigned m = 0;
    uint64_t label = 0;  // $ for a sink
    for (unsigned p = 1; p <= k; ++p) {
        if (r < 4) {  // a source of level k - (p - 1): its label
            label = (uint64_t)r + 1;
            break;
        }
        r -= 4;
        T = (T - 4) >> 2;  // T(p): strings below one real char at depth p
        const R rp = (R)(r >= T) + (R)(r >= 2 * T) + (R)(r >= 3 * T);
        r -= rp * T;
        x = shl(x, 3) | Key<L3>::from((uint64_t)rp + 1);
        ++m;
    }
    return shl(x, 3 * (k - m) + 3) | Key<L3>::from(label);
}

// Every block decodes a contiguous chunk of the dummies 256 at a time in closed form; the ones it
// leaves (sinks, the last 4 source levels: ~8 % at configs[2]) go to an LDS list that the whole block
// walks when it fills and at the chunk's end.  Walked where they lie, those few lanes held nearly every
// wave in the walk's ~k-step loop (63 ms for 6.6e8 dummies at configs[2] with or without the closed
// form), and a global list cost one atomic per wave on one counter (+58 ms).
template <int L3, int LR = 1>
__global__ __launch_bounds__(256) void dummy_decode_kernel(const Key<LR> *__restrict__ in, uint64_t n_, unsigned k,
                                                           Key<L3> *__restrict__ out,
                                                           const unsigned long long *__restrict__ n_dev = nullptr) {
    const uint64_t n = n_dev ? *n_dev : n_;  // n_dev: the count as the unique pass left it on the device
    using R = RankWord<LR>;
    constexpr uint32_t LCAP = 2048;
    __shared__ uint32_t s_list[LCAP];
    __shared__ uint32_t s_n;
    const R T0 = dummy_rank_space_t<R>(k);
    const uint64_t per = ((n + gridDim.x - 1) / gridDim.x + 255) & ~255ull;
    const uint64_t c0 = (uint64_t)blockIdx.x * per, c1 = min(n, c0 + per);
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    for (uint64_t base = c0; base < c1; base += 256) {
        const uint64_t i = base + threadIdx.x;
        bool walk = false;
        if (i < c1) {
            Key<L3> f;
            if (dummy_decode_fast<L3, R>(rank_word<LR>(in[i]), k, f)) out[i] = f;
            else walk = true;
        }
        const uint64_t bal = __ballot(walk);
        if (bal) {
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)bal) - 1;
            uint32_t pos = 0;
            if (__lane_id() == leader) pos = atomicAdd(&s_n, (uint32_t)__popcll(bal));
            pos = __shfl(pos, leader, 64);
            if (walk) s_list[pos + popc_below(bal)] = (uint32_t)(i - c0);
        }
        __syncthreads();
        const uint32_t cnt = s_n;
        if (cnt > LCAP - 256 || base + 256 >= c1) {  // (block-uniform: read after the barrier)
            for (uint32_t j = threadIdx.x; j < cnt; j += 256) {
                const uint64_t x = c0 + s_list[j];
                out[x] = dummy_decode_walk<L3, R>(rank_word<LR>(in[x]), k, T0);
            }
            __syncthreads();
            if (threadIdx.x == 0) s_n = 0;
            __syncthreads();
        }
    }
}

}  // namespace mtg
