// range_extract.hpp -- K1 of the range-batched (bounded-memory) build.
//
// The build collects the k-mers one key range at a time (boss_pipeline.hip: collect_ranges), so
// every range re-scans the whole read buffer.  The scans must be cheap: a window is assigned to a
// range by the top RB_CHARS chars of its key alone, which roll along the read in registers (as in
// the fused extraction's pass A), and only the windows of the current range build their full key, straight
// from a 2-bit packed copy of the tile in LDS.
//   count pass  -- per tile, how many k-mers fall in each of the 4^RB_CHARS top-char bins (u16);
//                  their column sums balance the ranges, their row sums over a range's bins are
//                  the write offsets;
//   write pass  -- per range: the k-mers whose bin lies in it, at the tile's scanned offset.
// The k-mers are the extractor's (kmer_extractor.cpp:165-237, 472-507): windows with an invalid
// char are skipped (drag_and_mark_segments, common/algorithms.hpp:50-67); canonical mode emits
// BOTH strands (the real-edge set of CANONICAL_ONLY, see collect_ranges).
#pragma once

#include "boss_kernels.hpp"
#include "extract_partition.hpp"

namespace mtg {

constexpr unsigned RB_CHARS = 4;                 // top node chars that pick a window's bin
constexpr uint32_t RB_BINS = 1u << (2 * RB_CHARS);  // 256

// the bins one range (or one round of the multi-GPU batched build: one bin interval per owner
// rank) collects, as a 256-bit set passed by value
struct BinSet {
    uint32_t m[RB_BINS / 32];
    __host__ __device__ bool has(uint32_t b) const { return (m[b >> 5] >> (b & 31)) & 1u; }
    __host__ void add(uint32_t lo, uint32_t hi) {
        for (uint32_t b = lo; b < hi; ++b) m[b >> 5] |= 1u << (b & 31);
    }
    __host__ uint32_t size() const {
        uint32_t s = 0;
        for (uint32_t w : m) s += (uint32_t)__builtin_popcount(w);
        return s;
    }
};

template <int L>
struct RangeTraits {
    static constexpr int BLOCK = 256;
    static constexpr int PPT = 16;               // consecutive windows per thread
    static constexpr int TILE = BLOCK * PPT;     // windows per workgroup
    static constexpr int SPAN = TILE + ExtractTraits<L>::MAXK;
    static constexpr int PACK = SPAN / 16 + 2 * L + 2;  // u32 words of 16 2-bit chars (+ read slack)
};

// plain (co-lex) word of the K chars starting at char r of a packed tile: sum c_{r+i} << 2i
template <int L>
__device__ __forceinline__ Key<L> packed_plain(const uint32_t *s_pack, uint32_t r, unsigned K) {
    const uint32_t bit = 2 * r, w = bit >> 5, b = bit & 31;
    Key<L> x;
#pragma unroll
    for (int i = 0; i < L; ++i) {
        const uint64_t lo = (uint64_t)s_pack[w + 2 * i] | (uint64_t)s_pack[w + 2 * i + 1] << 32;
        const uint64_t hi = s_pack[w + 2 * i + 2];
        x.w[i] = b ? (lo >> b) | (hi << (64 - b)) : lo;
    }
    return x & Key<L>::lowmask(2 * K);
}

// One thread's PPT windows starting at tile-relative char r0: the valid mask and each window's
// forward / reverse-complement top-char bins (the top 2*RB_CHARS bits of the 2-bit BOSS key:
// a_{K-1} .. a_{K-4} of the forward k-mer, comp(a_2) .. comp(a_5) for its reverse complement).
// Needs K >= RB_CHARS + 1.
template <int PPT>
__device__ __forceinline__ uint32_t window_bins(const uint8_t *s_code, uint32_t r0, uint64_t p0, uint64_t npos,
                                                unsigned K, uint8_t (&fb)[PPT], uint8_t (&rb)[PPT]) {
    constexpr unsigned C = RB_CHARS;
    const uint8_t *w0 = s_code + r0;
    int64_t last_bad = -1;
    for (unsigned i = 0; i < K; ++i)
        if (w0[i] == 4) last_bad = i;
    uint32_t f = 0, r = 0;
#pragma unroll
    for (unsigned q = 0; q < C; ++q) {
        f = (f << 2) | (w0[K - 2 - q] & 3u);
        r = (r << 2) | (3u - (w0[1 + q] & 3u));
    }
    uint32_t prev = w0[K - 1];
    uint32_t mask = 0;
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        if (p0 + j >= npos) break;
        if (j) {
            const uint32_t c = w0[j + K - 1];
            if (c == 4) last_bad = j + K - 1;
            f = (f >> 2) | ((prev & 3u) << (2 * C - 2));
            r = ((r << 2) & (RB_BINS - 1)) | (3u - (w0[j + C] & 3u));
            prev = c;
        }
        fb[j] = (uint8_t)f;
        rb[j] = (uint8_t)r;
        if (last_bad < (int64_t)j) mask |= 1u << j;
    }
    return mask;
}

// count pass: tbins[tile * RB_BINS + b] = k-mers of the tile in bin b (both strands when
// `both`), at most 2 * TILE = 8192 per tile (u16)
template <int L>
__global__ __launch_bounds__(256) void range_count_kernel(const uint8_t *__restrict__ seq, uint64_t seq_len,
                                                          unsigned K, int both, uint16_t *__restrict__ tbins) {
    using T = RangeTraits<L>;
    constexpr int BLOCK = T::BLOCK, PPT = T::PPT, TILE = T::TILE;
    __shared__ __align__(16) uint8_t s_code[T::SPAN];
    __shared__ uint32_t s_h[RB_BINS];
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < RB_BINS; i += BLOCK) s_h[i] = 0;
    const uint64_t npos = seq_len >= K ? seq_len - K + 1 : 0;
    const uint64_t base = (uint64_t)blockIdx.x * TILE;
    stage_codes<BLOCK>(seq, base, min(seq_len, base + TILE + K - 1), s_code, tid);
    __syncthreads();
    const uint64_t p0 = base + (uint64_t)tid * PPT;
    if (p0 < npos) {
        uint8_t fb[PPT], rb[PPT];
        const uint32_t m = window_bins<PPT>(s_code, tid * PPT, p0, npos, K, fb, rb);
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            if (!((m >> j) & 1u)) continue;
            atomicAdd(&s_h[fb[j]], 1u);
            if (both) atomicAdd(&s_h[rb[j]], 1u);
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < RB_BINS; i += BLOCK) tbins[(uint64_t)blockIdx.x * RB_BINS + i] = (uint16_t)s_h[i];
}

// column sums of the per-tile bins (the bins' global histogram)
__global__ __launch_bounds__(256) void range_bins_reduce_kernel(const uint16_t *__restrict__ tbins, uint64_t tiles,
                                                                unsigned long long *__restrict__ hist) {
    static_assert(RB_BINS == 256, "one bin per thread");
    unsigned long long s = 0;
    for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) s += tbins[t * RB_BINS + threadIdx.x];
    if (s) atomicAdd(&hist[threadIdx.x], s);
}

// one range's k-mers per tile: the tile's counts over the bins of `sel`; one wave per tile
// (each lane sums 4 bins of the tile's 512-byte row, then a wave reduction)
__global__ __launch_bounds__(256) void range_tile_counts_kernel(const uint16_t *__restrict__ tbins, uint64_t tiles,
                                                                BinSet sel, uint32_t *__restrict__ tcnt) {
    static_assert(RB_BINS == 256, "4 bins per lane");
    const uint64_t t = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    if (t >= tiles) return;
    const uint2 v = reinterpret_cast<const uint2 *>(tbins + t * RB_BINS)[lane];
    uint32_t word = 0;  // constant-index selects: no dynamic indexing into the kernel argument
#pragma unroll
    for (int i = 0; i < (int)(RB_BINS / 32); ++i)
        if ((lane >> 3) == (uint32_t)i) word = sel.m[i];
    const uint32_t bits = (word >> (4 * (lane & 7))) & 0xFu;
    uint32_t s = ((bits & 1u) ? (v.x & 0xFFFFu) : 0u) + ((bits & 2u) ? (v.x >> 16) : 0u) +
                 ((bits & 4u) ? (v.y & 0xFFFFu) : 0u) + ((bits & 8u) ? (v.y >> 16) : 0u);
#pragma unroll
    for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) tcnt[t] = s;
}

// write pass of the bins of `sel`: the tile's k-mers in them at toff[tile]
template <int L, bool COUNTED>
__global__ __launch_bounds__(256) void range_write_kernel(
    const uint8_t *__restrict__ seq, uint64_t seq_len, unsigned K, int both,
    const uint64_t *__restrict__ read_starts, const uint32_t *__restrict__ read_counts, uint64_t n_reads,
    const uint64_t *__restrict__ rid_at, uint32_t cmax, BinSet sel, const uint64_t *__restrict__ toff, Key<L> *__restrict__ out,
    uint32_t *__restrict__ out_counts) {
    using T = RangeTraits<L>;
    constexpr int BLOCK = T::BLOCK, PPT = T::PPT, TILE = T::TILE;
    __shared__ __align__(16) uint8_t s_code[T::SPAN];
    __shared__ uint32_t s_pack[T::PACK];
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    __shared__ uint16_t s_item[2 * TILE];
    __shared__ uint32_t s_sel[RB_BINS / 32];
    const uint32_t tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < (int)(RB_BINS / 32); ++i)
        if (tid == (uint32_t)i) s_sel[i] = sel.m[i];
    const uint64_t npos = seq_len >= K ? seq_len - K + 1 : 0;
    const uint64_t base = (uint64_t)blockIdx.x * TILE;
    const uint64_t span_end = min(seq_len, base + TILE + K - 1);
    const uint32_t span = (uint32_t)(span_end - base);
    stage_codes<BLOCK>(seq, base, span_end, s_code, tid);
    __syncthreads();
    for (uint32_t q = tid; q < (uint32_t)T::PACK; q += BLOCK) {  // 16 chars per word, invalid -> 0
        uint32_t v = 0;
        if (16 * q < span) {
            const uint4 c = reinterpret_cast<const uint4 *>(s_code)[q];
            const uint32_t cw[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const uint32_t ch = 16 * q + i < span ? (cw[i >> 2] >> (8 * (i & 3))) & 3u : 0u;
                v |= ch << (2 * i);
            }
        }
        s_pack[q] = v;
    }
    __syncthreads();
    const uint64_t p0 = base + (uint64_t)tid * PPT;
    uint32_t emit = 0;  // bit j: forward k-mer of window j, bit 16 + j: its reverse complement
    if (p0 < npos) {
        uint8_t fb[PPT], rb[PPT];
        const uint32_t m = window_bins<PPT>(s_code, tid * PPT, p0, npos, K, fb, rb);
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            if (!((m >> j) & 1u)) continue;
            if ((s_sel[fb[j] >> 5] >> (fb[j] & 31)) & 1u) emit |= 1u << j;
            if (both && (s_sel[rb[j] >> 5] >> (rb[j] & 31)) & 1u) emit |= 1u << (16 + j);
        }
    }
    // compact the tile's emitted k-mers into an LDS list (window << 1 | strand), then build and
    // write them densely: every lane of every wave has a k-mer, and the stores are coalesced
    uint32_t total;
    const uint32_t off = block_exclusive_sum<BLOCK>(__popc(emit), s_scan, &total);
    {
        uint32_t q = off;
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const uint32_t w = tid * PPT + j;
            if ((emit >> j) & 1u) s_item[q++] = (uint16_t)(w << 1);
            if ((emit >> (16 + j)) & 1u) s_item[q++] = (uint16_t)(w << 1 | 1u);
        }
    }
    __syncthreads();
    const uint64_t gb = toff[blockIdx.x];
    const Key<L> low = Key<L>::lowmask(2 * (K - 1));
    for (uint32_t i = tid; i < total; i += BLOCK) {
        const uint32_t it = s_item[i], w = it >> 1;
        const Key<L> f = plain_to_boss(packed_plain<L>(s_pack, w, K), K, low);
        out[gb + i] = (it & 1u) ? revcomp2(f, K) : f;
        if (COUNTED) {
            uint32_t c = 1;
            if (read_counts) c = read_counts[read_of(read_starts, n_reads, rid_at, base + w)];  // window base + w
            out_counts[gb + i] = c < cmax ? c : cmax;
        }
    }
}

}  // namespace mtg
