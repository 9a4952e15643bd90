// suffix_extract.hpp -- K1 of the suffix-filtered route (build --suffix-len: one BOSS chunk per
// node suffix, concatenated afterwards).
//
// With a non-empty filter suffix the reference collects (k+1)-mers over the BOSS alphabet $ACGT
// (3 bits a char) straight from `$`-padded read segments (KmerExtractorBOSS::sequence_to_kmers,
// kmer/kmer_extractor.cpp:316-381): every maximal run of valid chars of length >= K = k + 1 is
// read as $^(K-1) segment $, so it yields K - 1 source-dummy windows, its real windows and one
// sink window; only windows whose node ends with the suffix are kept (KMerBOSS::match_suffix,
// kmer/kmer_boss.hpp:107-112).  In BOTH mode (both strands, boss_chunk_construct.cpp:960-971) the
// reverse complement of every read is padded and scanned the same way (kmer_collector.cpp:40-52).
// The chunk is then initialize_chunk over the sorted set, with no dummy reconstruction
// (boss_chunk_construct.cpp:1001-1013).
//
// Window map: a segment [s, e) of the read buffer (e = the invalid char after it) has len + 1
// padded windows; the forward window ending at padded position w ends at buffer position s + w,
// so every position p in [s, e] ends exactly one forward window (chars p-K+1 .. p; positions
// before s and position e read as $).  The reverse-complement read's padded windows map onto the
// same positions: the rc window owned by p holds comp(char p+K-2-i) at window position i
// (positions >= e and position s-1 read as $).  A workgroup stages its tile of positions with a
// HALO of chars on both sides in LDS, which holds every char a window or its segment test reads.
#pragma once

#include "boss_kernels.hpp"

namespace mtg {

constexpr int SUFFIX_MAX = 88;  // suffix chars carried in the kernel arguments (< K <= 85)

struct SuffixSpec {
    uint32_t n;                 // suffix length (0 < n < K)
    uint8_t c[SUFFIX_MAX];      // BOSS codes: $ = 0, A C G T = 1..4, first char first
};

struct SuffixTraits {
    static constexpr int BLOCK = 256;
    static constexpr int PPT = 4;
    static constexpr int TILE = BLOCK * PPT;  // positions per workgroup
    static constexpr int HALO = 96;           // >= K + 1 chars each side (K <= 85)
    static constexpr int SPAN = TILE + 2 * HALO;
};

// BOSS key of the window(s) owned by local position x of the staged codes (2-bit codes, 4 =
// invalid).  Returns bit 0: forward window emitted, bit 1: reverse-complement window emitted.
template <int L3>
__device__ __forceinline__ uint32_t suffix_windows(const uint8_t *s_code, int x, unsigned K, bool both,
                                                   const SuffixSpec &suf, Key<L3> *fwd, Key<L3> *rcw) {
    const bool vp = s_code[x] < 4, vprev = s_code[x - 1] < 4;
    if (!vp && !vprev) return 0;  // neither inside a segment nor its terminating char
    constexpr int FAR_LO = -(1 << 20), FAR_HI = 1 << 20;
    int sl = FAR_LO;  // segment start (local), FAR_LO when it lies K or more chars back
    for (int q = x - 1; q >= x - (int)K; --q)
        if (s_code[q] >= 4) { sl = q + 1; break; }
    int el = FAR_HI;  // segment end (first invalid char at or after x), FAR_HI when > x + K
    for (int q = x; q <= x + (int)K; ++q)
        if (s_code[q] >= 4) { el = q; break; }
    if (sl != FAR_LO && el != FAR_HI && el - sl < (int)K) return 0;  // segment shorter than K
    uint32_t m = 0;
    // forward: window char i at position x-K+1+i; label = char K-1
    {
        Key<L3> key = Key<L3>::zero();
        bool ok = true;
        for (unsigned i = 0; i < K; ++i) {
            const int q = x - (int)K + 1 + (int)i;
            const uint32_t c = (q < sl || q == el) ? 0u : (uint32_t)s_code[q] + 1u;
            const unsigned slot = i + 1 == K ? 0u : i + 1;
            if (i + 1 < K && i + 1 + suf.n >= K && suf.c[i + 1 + suf.n - K] != c) ok = false;
            key = key | shl(Key<L3>::from(c), 3 * slot);
        }
        if (ok) { *fwd = key; m |= 1u; }
    }
    if (both) {
        Key<L3> key = Key<L3>::zero();
        bool ok = true;
        for (unsigned i = 0; i < K; ++i) {
            const int q = x + (int)K - 2 - (int)i;
            const uint32_t c = (q >= el || q < sl) ? 0u : 4u - (uint32_t)s_code[q];
            const unsigned slot = i + 1 == K ? 0u : i + 1;
            if (i + 1 < K && i + 1 + suf.n >= K && suf.c[i + 1 + suf.n - K] != c) ok = false;
            key = key | shl(Key<L3>::from(c), 3 * slot);
        }
        if (ok) { *rcw = key; m |= 2u; }
    }
    return m;
}

// stage codes [base - HALO, base + TILE + HALO) of the buffer; outside [0, seq_len) -> invalid
__device__ __forceinline__ void suffix_stage(const uint8_t *__restrict__ seq, uint64_t seq_len, uint64_t base,
                                             uint8_t *s_code, uint32_t tid) {
    using T = SuffixTraits;
    for (int i = (int)tid; i < T::SPAN; i += T::BLOCK) {
        const int64_t p = (int64_t)base - T::HALO + i;
        s_code[i] = (p >= 0 && (uint64_t)p < seq_len) ? encode_dna(seq[p]) : (uint8_t)4;
    }
}

// COUNT_ONLY: tcnt[tile] = windows kept by the tile; else write them at toff[tile] (+ counts:
// the read's count, clamped, kmer_collector.cpp:74-104)
template <int L3, bool COUNTED, bool COUNT_ONLY>
__global__ __launch_bounds__(256) void suffix_extract_kernel(
    const uint8_t *__restrict__ seq, uint64_t seq_len, unsigned K, int both, SuffixSpec suf,
    const uint64_t *__restrict__ read_starts, const uint32_t *__restrict__ read_counts, uint64_t n_reads,
    const uint64_t *__restrict__ rid_at,
    uint32_t cmax, uint32_t *__restrict__ tcnt, const uint64_t *__restrict__ toff, Key<L3> *__restrict__ out,
    uint32_t *__restrict__ out_counts) {
    using T = SuffixTraits;
    __shared__ uint8_t s_code[T::SPAN];
    __shared__ uint32_t s_scan[T::BLOCK / 64 + 1];
    const uint32_t tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * T::TILE;
    const uint64_t npos = seq_len + 1;  // position seq_len ends a final unterminated segment
    suffix_stage(seq, seq_len, base, s_code, tid);
    __syncthreads();
    Key<L3> fw[T::PPT], rw[T::PPT];
    uint32_t ms[T::PPT];
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < T::PPT; ++j) {
        const uint64_t p = base + (uint64_t)tid * T::PPT + j;
        ms[j] = p < npos ? suffix_windows<L3>(s_code, T::HALO + (int)(tid * T::PPT + j), K, both != 0, suf,
                                              &fw[j], &rw[j])
                         : 0u;
        cnt += __popc(ms[j]);
    }
    uint32_t total;
    const uint32_t off = block_exclusive_sum<T::BLOCK>(cnt, s_scan, &total);
    if (COUNT_ONLY) {
        if (tid == 0) tcnt[blockIdx.x] = total;
        return;
    }
    uint64_t o = toff[blockIdx.x] + off;
#pragma unroll
    for (int j = 0; j < T::PPT; ++j) {
        if (!ms[j]) continue;
        uint32_t c = 1;
        if (COUNTED && read_counts)  // the read holding position p: last start <= p
            c = read_counts[read_of(read_starts, n_reads, rid_at, base + (uint64_t)tid * T::PPT + j)];
        c = c < cmax ? c : cmax;
        if (ms[j] & 1u) {
            out[o] = fw[j];
            if (COUNTED) out_counts[o] = c;
            ++o;
        }
        if (ms[j] & 2u) {
            out[o] = rw[j];
            if (COUNTED) out_counts[o] = c;
            ++o;
        }
    }
}

}  // namespace mtg
