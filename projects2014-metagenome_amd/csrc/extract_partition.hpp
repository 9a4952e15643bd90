// extract_partition.hpp -- K1 fused with the first MSD partition level of K2 (2-bit u64 keys).
//
// The unfused path writes every extracted k-mer in window order (K1) and then reads and scatters
// it again by its top digit (K2 level 1): 2 x 9.6 GB of HBM traffic at the bench size.  Here the
// extraction kernel itself scatters the k-mers into their level-1 buckets, so that pass and its
// histogram pass disappear.  Bucket starts must be known before the scatter, hence two passes
// over the read bytes (1.5 GB each at the bench size):
//   A  extract_hist_fast_kernel -- extract, histogram of the top HB bits (HB = 12), no writes;
//   B  extract_partition_kernel -- extract again, rank by bucket in LDS, reserve one run per
//                                  (tile, bucket) with a cursor atomic, write the runs.
// The window logic is slide_windows (boss_kernels.hpp), shared with extract_kernel, so both
// produce the same k-mers (kmer_extractor.cpp:165-237, 472-507).
#pragma once

#include "boss_kernels.hpp"
#include "msd_sort.hpp"

namespace mtg {

constexpr unsigned FUSED_HB = 12;  // histogram bits of pass A (>= any level-1 digit)
constexpr uint32_t FUSED_SEL_WORDS = 32;  // a level-1 bucket mask of a collect round (<= 1024 buckets)

// Stage a tile's read bytes as 2-bit codes (4 = invalid) in LDS: one dword load, four encodes and
// one dword LDS store per thread step when the bytes are 4-aligned, byte loads for the tail.
template <int BLOCK>
__device__ __forceinline__ void stage_codes(const uint8_t *__restrict__ seq, uint64_t base, uint64_t span_end,
                                            uint8_t *s_code, uint32_t tid) {
    const uint32_t n = span_end > base ? (uint32_t)(span_end - base) : 0u;
    uint32_t done = 0;
    if ((((uintptr_t)(seq + base)) & 3) == 0) {
        const uint32_t nw = n >> 2;
        const uint32_t *src = reinterpret_cast<const uint32_t *>(seq + base);
        for (uint32_t i = tid; i < nw; i += BLOCK) {
            const uint32_t v = src[i];
            reinterpret_cast<uint32_t *>(s_code)[i] = encode_dna(v & 0xff) | encode_dna((v >> 8) & 0xff) << 8 |
                                                      encode_dna((v >> 16) & 0xff) << 16 | encode_dna(v >> 24) << 24;
        }
        done = nw << 2;
    }
    for (uint32_t i = done + tid; i < n; i += BLOCK) s_code[i] = encode_dna(seq[base + i]);
}

// 16 read bytes -> 16 2-bit codes (invalid -> 0) and a 16-bit invalid-char mask
__device__ __forceinline__ void pack16(const uint4 v, uint32_t &pk, uint32_t &iv) {
    const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
    pk = 0;
    iv = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t c = encode_dna((vv[q] >> (8 * r)) & 0xffu);
            pk |= (c & 3u) << (2 * (4 * q + r));
            iv |= (c >> 2) << (4 * q + r);
        }
}

// packed word w of a tile (chars base + 16 w ..), bytes past seq_len invalid
__device__ __forceinline__ void pack_word(const uint8_t *__restrict__ seq, uint64_t seq_len, uint64_t p,
                                          uint32_t &pk, uint32_t &iv) {
    if (((((uintptr_t)(seq + p)) & 15) == 0) && p + 16 <= seq_len) {
        pack16(*reinterpret_cast<const uint4 *>(seq + p), pk, iv);
        return;
    }
    pk = 0;
    iv = 0;
    for (int i = 0; i < 16; ++i) {
        const uint32_t c = p + i < seq_len ? encode_dna(seq[p + i]) : 4u;
        pk |= (c & 3u) << (2 * i);
        iv |= (c >> 2) << i;
    }
}

// reverse complement of a packed word: char i -> position 15 - i, code c -> 3 - c
__device__ __forceinline__ uint32_t rc_word(uint32_t w) {
    uint32_t x = __builtin_bitreverse32(w);
    x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
    return ~x;
}

// A: one LDS histogram per workgroup over its tiles (grid-stride), one row per workgroup.
// The top HB bits of a 2-bit BOSS key are its node's last HB/2 chars a_{K-1} .. a_{K-HB/2}
// (kmer_boss.hpp:58-72), and top(min(fwd, rc)) = min(top(fwd), top(rc)) (the tops decide the
// comparison unless they are equal), so a window needs only those chars of each strand: rc's
// top chars are comp(a_2) .. comp(a_{HB/2+1}).  Needs K - 1 >= HB/2 (callers check).
// The tile is packed once (pack16); per window the forward top a_{K-6} .. a_{K-1} and the rc top
// comp(a_7) .. comp(a_2) are constant-offset 12-bit fields of two precomputed 64/96-bit words,
// validity a field of the invalid-char mask (round 2: 1.85 -> ~1.2 ms, VALU-bound before).
// Row r counts the per_row consecutive tiles [r * per_row, (r + 1) * per_row): rps consecutive rows
// then cover one stripe of pass B's tiles (stripe_cursor_kernel).
// OTHER (the multi-GPU build): also rows_other, the histogram of the top bits of the other strand's
// key of every canonical window (its reverse complement: max(fwd, rc)), so the owner ranges can be
// balanced on the real edges (both strands) as well as on the canonical k-mers.
// KC (both fused passes): the window length K as a compile-time constant (0 = the runtime argument);
// the host instantiates KC = 31, the k = 30 BOSS build of BASELINE configs[1] / [3], so the 64-bit masks
// and shifts of the window loop fold into immediates
// CM (both fused passes): the canonical mode as a compile-time constant (-1 = the runtime argument):
// a runtime mode split every window's code into branches around the hash-canonical test, and the 16
// windows of a thread could not be scheduled together
template <bool OTHER = false, int KC = 0, int CM = -1>
__global__ __launch_bounds__(256) void extract_hist_fast_kernel(const uint8_t *__restrict__ seq, uint64_t seq_len,
                                                                unsigned K_, int canonical_, uint64_t ntiles,
                                                                uint64_t per_row, uint32_t *__restrict__ rows,
                                                                uint32_t *__restrict__ rows_other = nullptr,
                                                                uint32_t tstride = 1) {
    // tstride > 1: a sample -- row r counts every tstride-th of its tiles (the speculative level-1
    // layout of fused_pass_b_spec sizes its segments from it)
    const unsigned K = KC ? (unsigned)KC : K_;
    const int canonical = CM >= 0 ? CM : canonical_;
    constexpr int BLOCK = 256, PPT = 16, TILE = BLOCK * PPT, NW = BLOCK + 2;
    constexpr uint32_t NB = 1u << FUSED_HB;
    static_assert(FUSED_HB == 12, "6-char tops");
    __shared__ uint32_t s_pack[NW];
    __shared__ uint32_t s_inv[NW];
    __shared__ uint32_t s_h[NB];
    __shared__ uint32_t s_o[OTHER ? NB : 1];
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < NB; i += BLOCK) {
        s_h[i] = 0;
        if (OTHER) s_o[i] = 0;
    }
    const uint64_t npos = seq_len >= K ? seq_len - K + 1 : 0;
    const uint64_t maskK = (1ull << K) - 1;
    const unsigned fs = 2 * (K - 7);  // K >= 7 (callers check K - 1 >= 6)
    // the raw bytes of word tid of the next tile, loaded while the current tile is counted
    uint4 pre = make_uint4(0, 0, 0, 0);
    bool have = false;
    auto fetch = [&](uint64_t t) {
        const uint64_t p = t * TILE + 16ull * tid;
        have = t < ntiles && ((((uintptr_t)(seq + p)) & 15) == 0) && p + 16 <= seq_len;
        if (have) pre = *reinterpret_cast<const uint4 *>(seq + p);
    };
    const uint64_t t0 = (uint64_t)blockIdx.x * per_row, t1 = min(ntiles, t0 + per_row);
    fetch(t0);
    for (uint64_t tile = t0; tile < t1; tile += tstride) {
        const uint64_t base = tile * TILE;
        uint32_t pk, iv;
        if (have) pack16(pre, pk, iv);
        else pack_word(seq, seq_len, base + 16ull * tid, pk, iv);
        __syncthreads();  // the previous tile's words are read
        s_pack[tid] = pk;
        s_inv[tid] = iv;
        if (tid < NW - BLOCK) {
            uint32_t a, b;
            pack_word(seq, seq_len, base + 16ull * (BLOCK + tid), a, b);
            s_pack[BLOCK + tid] = a;
            s_inv[BLOCK + tid] = b;
        }
        __syncthreads();
        if (tile + tstride < t1) fetch(tile + tstride);
        else have = false;
        const uint64_t p0 = base + 16ull * tid;
        if (p0 >= npos) continue;
        const uint32_t nwin = (uint32_t)min<uint64_t>(PPT, npos - p0);
        const uint32_t w0 = s_pack[tid], w1 = s_pack[tid + 1], w2 = s_pack[tid + 2];
        const uint64_t inv = (uint64_t)s_inv[tid] | ((uint64_t)s_inv[tid + 1] << 16) | ((uint64_t)s_inv[tid + 2] << 32);
        // F = chars K-7 .. of the span (window j's forward top = F >> 2j)
        uint32_t flo, fhi;
        if (fs < 32) {
            flo = __builtin_amdgcn_alignbit(w1, w0, fs);
            fhi = __builtin_amdgcn_alignbit(w2, w1, fs);
        } else {
            flo = __builtin_amdgcn_alignbit(w2, w1, fs - 32);
            fhi = w2 >> (fs - 32);
        }
        // Q = the reverse complement of the 48 chars: char t at bits 2 (47 - t); window j's rc top
        // comp(a_7) .. comp(a_2) = chars j + 6 .. j + 1 = Q >> 2 (41 - j)
        const uint32_t q1 = rc_word(w1), q2 = rc_word(w0);
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const uint32_t f = (j ? __builtin_amdgcn_alignbit(fhi, flo, 2 * j) : flo) & (NB - 1);
            const int sr = 2 * (41 - j);  // 52 .. 82
            const uint32_t r = (sr >= 64 ? (q2 >> (sr - 64)) : __builtin_amdgcn_alignbit(q2, q1, sr - 32)) & (NB - 1);
            const bool ok = (uint32_t)j < nwin && ((inv >> j) & maskK) == 0;
            if (ok) {
                const bool rc = take_rc_top(canonical, f, r);
                atomicAdd(&s_h[rc ? r : f], 1u);
                if (OTHER) atomicAdd(&s_o[rc ? f : r], 1u);
            }
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < NB; i += BLOCK) {
        rows[(uint64_t)blockIdx.x * NB + i] = s_h[i];
        if (OTHER) rows_other[(uint64_t)blockIdx.x * NB + i] = s_o[i];
    }
}

// A for windows of up to 64 chars (u128 keys; BASELINE configs[2]: K = 63): the same histogram of the
// canonical keys' top 12 bits as extract_hist_fast_kernel, from five packed words per thread (a thread's
// 16 windows span 15 + K <= 79 chars); the forward top of window j is chars j + K - 7 .. j + K - 2, a
// 12-bit field of a funnel-shifted pair of words, validity the K-bit field of the 80-bit invalid mask.
// KC: K as a compile-time constant (0: the runtime K_).
template <int KC = 0>
__global__ __launch_bounds__(256) void extract_hist_wide_kernel(const uint8_t *__restrict__ seq, uint64_t seq_len,
                                                                unsigned K_, int canonical, uint64_t ntiles,
                                                                uint64_t per_row, uint32_t *__restrict__ rows,
                                                                uint32_t tstride = 1) {
    const unsigned K = KC ? (unsigned)KC : K_;
    constexpr int BLOCK = 256, PPT = 16, TILE = BLOCK * PPT, NW = BLOCK + 5;
    constexpr uint32_t NB = 1u << FUSED_HB;
    __shared__ uint32_t s_pack[NW];
    __shared__ uint32_t s_inv[NW];
    __shared__ uint32_t s_h[NB];
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < NB; i += BLOCK) s_h[i] = 0;
    const uint64_t npos = seq_len >= K ? seq_len - K + 1 : 0;
    const uint64_t maskK = K >= 64 ? ~0ull : (1ull << K) - 1;
    const unsigned fs = 2 * (K - 7);  // bit offset of window 0's forward top in the thread's span
    const unsigned qs = fs >> 5, bs = fs & 31;
    const uint64_t t0 = (uint64_t)blockIdx.x * per_row, t1 = min(ntiles, t0 + per_row);
    for (uint64_t tile = t0; tile < t1; tile += tstride) {
        const uint64_t base = tile * TILE;
        __syncthreads();  // the previous tile's words are read
        for (uint32_t w = tid; w < (uint32_t)NW; w += BLOCK) {
            uint32_t a, b;
            pack_word(seq, seq_len, base + 16ull * w, a, b);
            s_pack[w] = a;
            s_inv[w] = b;
        }
        __syncthreads();
        const uint64_t p0 = base + 16ull * tid;
        if (p0 >= npos) continue;
        const uint32_t nwin = (uint32_t)min<uint64_t>(PPT, npos - p0);
        uint32_t w[6];
#pragma unroll
        for (int q = 0; q < 5; ++q) w[q] = s_pack[tid + q];
        w[5] = 0;
        const u128 inv = (u128)s_inv[tid] | ((u128)s_inv[tid + 1] << 16) | ((u128)s_inv[tid + 2] << 32) |
                         ((u128)s_inv[tid + 3] << 48) | ((u128)s_inv[tid + 4] << 64);
        // the words at qs, qs + 1, qs + 2 (a select chain: no dynamic register indexing)
        uint32_t x0 = w[0], x1 = w[1], x2 = w[2];
#pragma unroll
        for (unsigned q = 1; q < 4; ++q)
            if (qs == q) x0 = w[q], x1 = w[q + 1], x2 = w[q + 2];
        const uint32_t flo = bs ? __builtin_amdgcn_alignbit(x1, x0, bs) : x0;
        const uint32_t fhi = bs ? __builtin_amdgcn_alignbit(x2, x1, bs) : x1;
        const uint32_t q1 = rc_word(w[1]), q2 = rc_word(w[0]);
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const uint32_t f = (j ? __builtin_amdgcn_alignbit(fhi, flo, 2 * j) : flo) & (NB - 1);
            const int sr = 2 * (41 - j);  // 52 .. 82
            const uint32_t r = (sr >= 64 ? (q2 >> (sr - 64)) : __builtin_amdgcn_alignbit(q2, q1, sr - 32)) & (NB - 1);
            const bool ok = (uint32_t)j < nwin && ((uint64_t)(inv >> j) & maskK) == 0;
            if (ok) atomicAdd(&s_h[take_rc_top(canonical, f, r) ? r : f], 1u);
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < NB; i += BLOCK) rows[(uint64_t)blockIdx.x * NB + i] = s_h[i];
}

template <bool COUNTED, int BLOCK_ = COUNTED ? 512 : 1024>
struct FusedTraits {
    static constexpr int BLOCK = BLOCK_;  // the LDS tile: BLOCK * PPT keys (16 K at 1024 threads)
    static constexpr int PPT = ExtractTraits<1>::PPT;
    static constexpr int TILE = BLOCK * PPT;
};
// pass B's workgroup for L-limb keys: 512 threads (8 K windows) for u64, 256 (4 K windows, 64 KB of
// u128 keys in LDS) for u128
template <int L>
constexpr int fused_block() { return L == 1 ? 512 : 256; }

// B: extract one tile, order its k-mers by the top b bits in LDS, write one run per bucket at
// cursor[bucket] (the bucket starts of pass A's histogram).  L-limb keys (u128: BASELINE configs[2]'s
// k = 63 rounds); KC: the window length as a compile-time constant (0: the runtime K)
template <int L, bool COUNTED, int BLOCK_, int KC = 0>
__global__ __launch_bounds__(BLOCK_) void extract_partition_kernel(
    const uint8_t *__restrict__ seq, uint64_t seq_len, unsigned K_, int canonical,
    const uint64_t *__restrict__ read_starts, const uint32_t *__restrict__ read_counts, uint64_t n_reads,
    const uint64_t *__restrict__ rid_at, uint32_t cmax, unsigned b, uint64_t per_stripe, unsigned long long *__restrict__ cursor,
    const unsigned long long *__restrict__ bend, Key<L> *__restrict__ kout, uint32_t *__restrict__ vout,
    uint32_t *__restrict__ error, const uint32_t *__restrict__ sel = nullptr) {
    const unsigned K = KC ? (unsigned)KC : K_;
    using F = FusedTraits<COUNTED, BLOCK_>;
    constexpr int BLOCK = F::BLOCK, PPT = F::PPT, TILE = F::TILE;
    constexpr int NBMAX = 512;
    constexpr int PER = NBMAX / BLOCK > 0 ? NBMAX / BLOCK : 1;
    static_assert(ExtractTraits<L>::PPT == PPT, "16 windows per thread");
    __shared__ __align__(16) uint8_t s_code[TILE + ExtractTraits<L>::MAXK];
    __shared__ Key<L> s_keys[TILE];
    __shared__ uint32_t s_vals[COUNTED ? TILE : 1];
    __shared__ uint32_t s_cnt[NBMAX];  // bucket counts, then the buckets' offsets in the tile
    __shared__ unsigned long long s_gbase[NBMAX];
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    __shared__ uint32_t s_sel[FUSED_SEL_WORDS];

    const uint32_t tid = threadIdx.x;
    const uint32_t nb = 1u << b;
    const uint64_t npos = seq_len >= K ? seq_len - K + 1 : 0;
    // XCD-contiguous tiles (device_common.hpp: xcd_tile); stripe = tile / per_stripe
    const uint64_t tile = xcd_tile((npos + TILE - 1) / TILE);
    if (tile * TILE >= npos) return;
    for (uint32_t i = tid; i < nb; i += BLOCK) s_cnt[i] = 0;
    if (sel && tid < FUSED_SEL_WORDS) s_sel[tid] = sel[tid];
    const uint64_t base = tile * TILE;
    const uint64_t span_end = min(seq_len, base + TILE + K - 1);
    stage_codes<BLOCK>(seq, base, span_end, s_code, tid);
    __syncthreads();
    Key<L> kk[PPT];
    uint32_t cc[PPT];
    uint32_t m = slide_windows<L, COUNTED, PPT, true>(s_code, tid * PPT, base + (uint64_t)tid * PPT, npos, K,
                                                      canonical, read_starts, read_counts, n_reads, rid_at, cmax, kk, cc);
    if (sel) {  // one round of a batched collect: only the level-1 buckets of its mask
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const uint32_t pb = key_prefix(kk[j], 2 * K, b);
            if (!((s_sel[pb >> 5] >> (pb & 31)) & 1u)) m &= ~(1u << j);
        }
    }
    uint32_t r[PPT];
#pragma unroll
    for (int j = 0; j < PPT; ++j)
        r[j] = (m & (1u << j)) ? atomicAdd(&s_cnt[key_prefix(kk[j], 2 * K, b)], 1u) : 0u;
    __syncthreads();
    uint32_t c[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid * PER + q;
        c[q] = i < nb ? s_cnt[i] : 0;
        sum += c[q];
    }
    uint32_t total;
    uint32_t off = block_exclusive_sum<BLOCK>(sum, s_scan, &total);
    __syncthreads();  // every count is read before the offsets overwrite them
    // (the run reservations stay in flight across the LDS scatter, as in extract_partition_fast_kernel)
    unsigned long long gq[PER], be[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid * PER + q;
        gq[q] = 0, be[q] = 0;
        if (i < nb) {
            s_cnt[i] = off;
            const size_t ci = (size_t)(tile / per_stripe) * nb + i;  // this tile's stripe
            if (c[q]) {
                gq[q] = atomicAdd(&cursor[ci], (unsigned long long)c[q]);
                be[q] = bend[ci];
            }
        }
        off += c[q];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        if (m & (1u << j)) {
            const uint32_t pos = s_cnt[key_prefix(kk[j], 2 * K, b)] + r[j];
            s_keys[pos] = kk[j];
            if (COUNTED) s_vals[pos] = cc[j];
        }
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid * PER + q;
        if (i < nb) {
            unsigned long long g = gq[q];
            if (c[q] && g + c[q] > be[q]) {  // pass A counted this bucket differently: never
                atomicOr(error, 2u);          // write past its range (the host raises)
                g = ~0ull;
            }
            s_gbase[i] = g;
        }
    }
    __syncthreads();
    for (uint32_t p = tid; p < total; p += BLOCK) {
        const Key<L> key = s_keys[p];
        const uint32_t lb = key_prefix(key, 2 * K, b);
        if (s_gbase[lb] == ~0ull) continue;
        const uint64_t o = s_gbase[lb] + (p - s_cnt[lb]);
        kout[o] = key;
        if (COUNTED) vout[o] = s_vals[p];
    }
}

// Pass B without counts for K <= 32 (u64 keys), VALU-lean: the tile's read bytes are packed once
// in LDS (16 chars a word: 2-bit codes + a 16-bit invalid-char mask), and each thread forms its 16
// windows from three packed words with constant-offset funnel shifts (v_alignbit), the reverse
// complement by sliding one char a window, validity from the invalid-char mask -- no per-window
// LDS reads and no per-window branches.  Same k-mers as slide_windows (forward and rc plain words,
// plain_to_boss, rc < fwd picks rc), so the same output as extract_partition_kernel<false>.
// NB: the widest digit's bucket count (1024: a 10-bit level 1, so that inputs of ~2e9 k-mers keep a
// 2-level plan).  The bucket counts live in the run-base array until the scan has read them, and the
// in-tile offsets are u16, so NB = 1024 still fits two workgroups per CU (78 KB of LDS).
template <int BLOCK, int NB = 512, int KC = 0, int CM = -1>
__global__ __launch_bounds__(BLOCK) void extract_partition_fast_kernel(
    const uint8_t *__restrict__ seq, uint64_t seq_len, unsigned K_, int canonical_, unsigned b,
    uint64_t per_stripe, unsigned long long *__restrict__ cursor, const unsigned long long *__restrict__ bend,
    Key<1> *__restrict__ kout, uint32_t *__restrict__ error, const uint32_t *__restrict__ sel = nullptr,
    uint32_t *__restrict__ povf = nullptr, const long long *__restrict__ bdelta = nullptr) {
    // povf (the speculative level-1 layout): a reservation past its segment's end writes nothing and
    // raises *povf instead of the error word -- the caller then runs the exact passes A and B
    // bdelta (the collect rounds' one pass B): bucket i's keys go bdelta[i] elements away from their
    // layout position (each round's buckets into that round's buffer)
    const unsigned K = KC ? (unsigned)KC : K_;
    const int canonical = CM >= 0 ? CM : canonical_;
    constexpr int PPT = 16, TILE = BLOCK * PPT, NW = BLOCK + 2;  // +2 words: the last thread's overhang
    constexpr int NBMAX = NB;
    constexpr int PER = NBMAX / BLOCK > 0 ? NBMAX / BLOCK : 1;
    static_assert(TILE <= 65536, "u16 in-tile offsets");
    __shared__ uint32_t s_pack[NW];
    __shared__ uint32_t s_inv[NW];
    __shared__ uint64_t s_keys[TILE];
    __shared__ unsigned long long s_gbase[NBMAX];  // the run bases; first the u32 bucket counts (s_cnt)
    __shared__ uint16_t s_off[NBMAX];              // the buckets' offsets in the tile
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    __shared__ uint32_t s_sel[FUSED_SEL_WORDS];
    uint32_t *s_cnt = reinterpret_cast<uint32_t *>(s_gbase);

    const uint32_t tid = threadIdx.x;
    const uint32_t nb = 1u << b;
    const uint64_t npos = seq_len >= K ? seq_len - K + 1 : 0;
    // XCD-contiguous tiles (device_common.hpp: xcd_tile); stripe = tile / per_stripe
    const uint64_t tile = xcd_tile((npos + TILE - 1) / TILE);
    if (tile * TILE >= npos) return;
    for (uint32_t i = tid; i < nb; i += BLOCK) s_cnt[i] = 0;
    if (sel && tid < FUSED_SEL_WORDS) s_sel[tid] = sel[tid];
    const uint64_t base = tile * TILE;
    const bool aligned = (((uintptr_t)(seq + base)) & 15) == 0;
    for (uint32_t w = tid; w < (uint32_t)NW; w += BLOCK) {  // word w = chars base + 16 w ..
        const uint64_t p = base + 16ull * w;
        uint32_t pk = 0, iv = 0;
        if (aligned && p + 16 <= seq_len) {
            const uint4 v = *reinterpret_cast<const uint4 *>(seq + p);
            const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t c = encode_dna((vv[q] >> (8 * r)) & 0xffu);
                    pk |= (c & 3u) << (2 * (4 * q + r));
                    iv |= (c >> 2) << (4 * q + r);
                }
        } else {
            for (int i = 0; i < 16; ++i) {
                const uint32_t c = p + i < seq_len ? encode_dna(seq[p + i]) : 4u;
                pk |= (c & 3u) << (2 * i);
                iv |= (c >> 2) << i;
            }
        }
        s_pack[w] = pk;
        s_inv[w] = iv;
    }
    __syncthreads();

    // this thread's windows p0 + j (j < 16): chars 16 tid .. 16 tid + 47 of the tile
    const uint32_t w0 = s_pack[tid], w1 = s_pack[tid + 1], w2 = s_pack[tid + 2];
    const uint64_t inv = (uint64_t)s_inv[tid] | ((uint64_t)s_inv[tid + 1] << 16) | ((uint64_t)s_inv[tid + 2] << 32);
    const uint64_t p0 = base + 16ull * tid;
    const uint32_t nwin = p0 < npos ? (uint32_t)min<uint64_t>(PPT, npos - p0) : 0u;
    const uint64_t maskK = (1ull << K) - 1;                         // K <= 32 chars
    const uint64_t maskP = K >= 32 ? ~0ull : ((1ull << (2 * K)) - 1);  // 2K bits
    const uint64_t lowNode = (1ull << (2 * (K - 1))) - 1;
    const unsigned sh = 2 * (K - 1);
    // E: the chars entering windows 1..16 (char K + j - 1 for window j) as 2-bit groups
    uint32_t E;
    {
        const unsigned s2 = 2 * K;  // 2 .. 64
        if (s2 < 32) E = __builtin_amdgcn_alignbit(w1, w0, s2);
        else if (s2 < 64) E = __builtin_amdgcn_alignbit(w2, w1, s2 - 32);
        else E = w2;
    }
    const uint64_t P0 = ((uint64_t)w0 | ((uint64_t)w1 << 32)) & maskP;
    uint64_t R = reverse_pairs64(~P0) >> (64 - 2 * K);  // rc of window 0, plain
    uint64_t kk[PPT];
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        const uint32_t lo32 = j ? __builtin_amdgcn_alignbit(w1, w0, 2 * j) : w0;
        const uint32_t hi32 = j ? __builtin_amdgcn_alignbit(w2, w1, 2 * j) : w1;
        const uint64_t P = (((uint64_t)hi32 << 32) | lo32) & maskP;
        if (j) R = ((R << 2) | (3u - ((E >> (2 * (j - 1))) & 3u))) & maskP;
        const uint64_t f = ((P & lowNode) << 2) | (P >> sh);
        const uint64_t r = ((R & lowNode) << 2) | (R >> sh);
        const bool rc = canonical == 2 ? take_rc_top(2, (uint32_t)(f >> (2 * K - 12)), (uint32_t)(r >> (2 * K - 12))) ||
                                             ((f >> (2 * K - 12)) == (r >> (2 * K - 12)) && r < f)
                                       : canonical && r < f;
        kk[j] = rc ? r : f;
        m |= (uint32_t)((uint32_t)j < nwin && ((inv >> j) & maskK) == 0) << j;
    }
    const unsigned bshift = 2 * K - b;
    if (sel) {  // one round of a batched collect: only the level-1 buckets of its mask
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const uint32_t pb = (uint32_t)(kk[j] >> bshift);
            if (!((s_sel[pb >> 5] >> (pb & 31)) & 1u)) m &= ~(1u << j);
        }
    }
    uint32_t r[PPT];
#pragma unroll
    for (int j = 0; j < PPT; ++j)
        r[j] = (m & (1u << j)) ? atomicAdd(&s_cnt[(uint32_t)(kk[j] >> bshift)], 1u) : 0u;
    __syncthreads();
    uint32_t c[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid * PER + q;
        c[q] = i < nb ? s_cnt[i] : 0;
        sum += c[q];
    }
    uint32_t total;
    uint32_t off = block_exclusive_sum<BLOCK>(sum, s_scan, &total);
    __syncthreads();  // every count is read before the run bases overwrite them
    // (round 5) the run reservations are issued here and consumed after the LDS scatter below, so their
    // round trip to the cursors overlaps the scatter instead of stalling the workgroup before it
    unsigned long long gq[PER], be[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid * PER + q;
        gq[q] = 0, be[q] = 0;
        if (i < nb) {
            s_off[i] = (uint16_t)off;
            const size_t ci = (size_t)(tile / per_stripe) * nb + i;  // this tile's stripe
            if (c[q]) {
                gq[q] = atomicAdd(&cursor[ci], (unsigned long long)c[q]);
                be[q] = bend[ci];
            }
        }
        off += c[q];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PPT; ++j)
        if (m & (1u << j)) s_keys[s_off[(uint32_t)(kk[j] >> bshift)] + r[j]] = kk[j];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid * PER + q;
        if (i < nb) {
            unsigned long long g = gq[q];
            if (c[q] && g + c[q] > be[q]) {  // pass A counted this bucket differently: never
                atomicOr(povf ? povf : error, povf ? 1u : 2u);  // write past its range
                g = ~0ull;
            } else if (bdelta) {
                g += (unsigned long long)bdelta[i];
            }
            s_gbase[i] = g;
        }
    }
    __syncthreads();
    for (uint32_t p = tid; p < total; p += BLOCK) {
        const uint64_t key = s_keys[p];
        const uint32_t lb = (uint32_t)(key >> bshift);
        if (s_gbase[lb] == ~0ull) continue;
        kout[s_gbase[lb] + (p - s_off[lb])].w[0] = key;
    }
}

// Pass B for u128 windows (33 <= K <= 64, BASELINE configs[2]'s k = 63), VALU-lean like the u64 kernel
// above: the tile is packed once (16 chars a word + an invalid mask), a thread's 16 windows span five
// words, and window j's forward plain word is four funnel shifts of them (v_alignbit by 2j); the rc word
// slides one char a window (two 64-bit halves); the BOSS rotation drops the top char with a shift and
// puts it in the label; validity is the K-bit field of the 80-bit invalid mask.  Same k-mers as
// slide_windows<2> (forward and rc plain words, plain_to_boss, rc < fwd picks rc), so the same output as
// extract_partition_kernel<2>.  canonical: 0 / 1 only (the routed u128 collect is not fused).
// PPT = 8 (round 6): 8 windows a thread on 512-thread tiles of the same 4096 windows -- a thread starts at
// char 8 t, half-way into a packed word, so its five words are funnel-shifted by 16 bits from six.  Twice the
// waves per CU at the same LDS (the tile's 64 KB of staged keys held 16 windows a thread at 256 threads:
// 8 waves a CU; configs[2]'s pass B ran at 2.1 TB/s of writes)
template <int BLOCK, int KC = 0, int PPT_ = 16>
__global__ __launch_bounds__(BLOCK) void extract_partition_fast2_kernel(
    const uint8_t *__restrict__ seq, uint64_t seq_len, unsigned K_, int canonical, unsigned b,
    uint64_t per_stripe, unsigned long long *__restrict__ cursor, const unsigned long long *__restrict__ bend,
    Key<2> *__restrict__ kout, uint32_t *__restrict__ error, const uint32_t *__restrict__ sel = nullptr,
    const long long *__restrict__ bdelta = nullptr) {
    // bdelta: as in extract_partition_fast_kernel (the collect rounds' one pass B for configs[2]'s two rounds)
    const unsigned K = KC ? (unsigned)KC : K_;
    static_assert(PPT_ == 16 || PPT_ == 8, "16 or 8 windows a thread");
    constexpr int PPT = PPT_, TILE = BLOCK * PPT, NW = TILE / 16 + 5;  // +5 words: a thread's windows reach 15 + 63 chars on
    constexpr int NBMAX = 512;
    constexpr int PER = NBMAX / BLOCK > 0 ? NBMAX / BLOCK : 1;
    static_assert(TILE <= 65536, "u16 in-tile offsets");
    __shared__ uint32_t s_pack[NW];
    __shared__ uint32_t s_inv[NW];
    __shared__ ulonglong2 s_keys[TILE];
    __shared__ unsigned long long s_gbase[NBMAX];  // the run bases; first the u32 bucket counts (s_cnt)
    __shared__ uint16_t s_off[NBMAX];
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    __shared__ uint32_t s_sel[FUSED_SEL_WORDS];
    uint32_t *s_cnt = reinterpret_cast<uint32_t *>(s_gbase);

    const uint32_t tid = threadIdx.x;
    const uint32_t nb = 1u << b;
    const uint64_t npos = seq_len >= K ? seq_len - K + 1 : 0;
    const uint64_t tile = xcd_tile((npos + TILE - 1) / TILE);
    if (tile * TILE >= npos) return;
    for (uint32_t i = tid; i < nb; i += BLOCK) s_cnt[i] = 0;
    if (sel && tid < FUSED_SEL_WORDS) s_sel[tid] = sel[tid];
    const uint64_t base = tile * TILE;
    for (uint32_t w = tid; w < (uint32_t)NW; w += BLOCK) {
        uint32_t pk, iv;
        pack_word(seq, seq_len, base + 16ull * w, pk, iv);
        s_pack[w] = pk;
        s_inv[w] = iv;
    }
    __syncthreads();

    uint32_t w[5];
    uint64_t invlo, invhi;
    if constexpr (PPT == 16) {
#pragma unroll
        for (int q = 0; q < 5; ++q) w[q] = s_pack[tid + q];
        invlo = (uint64_t)s_inv[tid] | ((uint64_t)s_inv[tid + 1] << 16) | ((uint64_t)s_inv[tid + 2] << 32) |
                ((uint64_t)s_inv[tid + 3] << 48);
        invhi = s_inv[tid + 4];
    } else {
        // the thread's chars start at 8 t: word t / 2, char 8 (t & 1) -- five words from six, shifted by hc chars
        const uint32_t wi = tid >> 1, hc = 8u * (tid & 1u);
        uint32_t x[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) x[q] = s_pack[wi + q];
#pragma unroll
        for (int q = 0; q < 5; ++q) w[q] = __builtin_amdgcn_alignbit(x[q + 1], x[q], 2 * hc);
        const uint64_t a = (uint64_t)s_inv[wi] | ((uint64_t)s_inv[wi + 1] << 16) | ((uint64_t)s_inv[wi + 2] << 32) |
                           ((uint64_t)s_inv[wi + 3] << 48);
        const uint64_t bh = (uint64_t)s_inv[wi + 4] | ((uint64_t)s_inv[wi + 5] << 16);
        invlo = hc ? (a >> hc) | (bh << (64 - hc)) : a;
        invhi = hc ? bh >> hc : bh;
    }
    const uint64_t p0 = base + (uint64_t)PPT * tid;
    const uint32_t nwin = p0 < npos ? (uint32_t)min<uint64_t>(PPT, npos - p0) : 0u;
    const uint64_t maskK = K >= 64 ? ~0ull : (1ull << K) - 1;
    const unsigned hb = 2 * K - 64;                                   // bits of the high half (2 .. 64)
    const uint64_t mhi = hb >= 64 ? ~0ull : (1ull << hb) - 1;
    // E: the chars entering windows 1..16 (char K + j - 1 for window j), 2 bits each
    uint32_t E;
    {
        const unsigned qe = K >> 4, se = 2 * (K & 15);
        uint32_t a = w[2], c2 = w[3];
        if (qe == 3) a = w[3], c2 = w[4];
        if (qe == 4) a = w[4], c2 = 0;
        E = se ? __builtin_amdgcn_alignbit(c2, a, se) : a;
    }
    // R: the rc plain word of window 0 = the reversed, complemented chars of P0, shifted down to 2K bits
    uint64_t rlo, rhi;
    {
        const uint64_t plo = (uint64_t)w[0] | ((uint64_t)w[1] << 32), phi = ((uint64_t)w[2] | ((uint64_t)w[3] << 32)) & mhi;
        const uint64_t xl = reverse_pairs64(~phi), xh = reverse_pairs64(~plo);  // (~P) reversed, 128 bits
        const unsigned sh = 128 - 2 * K;                                         // 0 .. 62
        rlo = sh ? (xl >> sh) | (xh << (64 - sh)) : xl;
        rhi = (sh ? xh >> sh : xh) & mhi;
    }
    const unsigned tsh = 2 * K - 66;  // the top char's bit in the high half
    const unsigned bs = 2 * K - b;    // the level-1 digit: key bits [bs, 2K)
    ulonglong2 kk[PPT];
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        const uint32_t d0 = j ? __builtin_amdgcn_alignbit(w[1], w[0], 2 * j) : w[0];
        const uint32_t d1 = j ? __builtin_amdgcn_alignbit(w[2], w[1], 2 * j) : w[1];
        const uint32_t d2 = j ? __builtin_amdgcn_alignbit(w[3], w[2], 2 * j) : w[2];
        const uint32_t d3 = j ? __builtin_amdgcn_alignbit(w[4], w[3], 2 * j) : w[3];
        const uint64_t plo = (uint64_t)d0 | ((uint64_t)d1 << 32), phi = ((uint64_t)d2 | ((uint64_t)d3 << 32)) & mhi;
        if (j) {
            rhi = ((rhi << 2) | (rlo >> 62)) & mhi;
            rlo = (rlo << 2) | (3u - ((E >> (2 * (j - 1))) & 3u));
        }
        // plain -> BOSS: the 2K-bit word shifted up one char (its top char falls off) with that char as the label
        const uint64_t flo = (plo << 2) | ((phi >> tsh) & 3u), fhi = ((phi << 2) | (plo >> 62)) & mhi;
        const uint64_t qlo = (rlo << 2) | ((rhi >> tsh) & 3u), qhi = ((rhi << 2) | (rlo >> 62)) & mhi;
        const bool rc = canonical && (qhi < fhi || (qhi == fhi && qlo < flo));
        kk[j] = rc ? make_ulonglong2(qlo, qhi) : make_ulonglong2(flo, fhi);
        const uint64_t iw = j ? (invlo >> j) | (invhi << (64 - j)) : invlo;
        m |= (uint32_t)((uint32_t)j < nwin && (iw & maskK) == 0) << j;
    }
    auto digit = [&](const ulonglong2 &x) -> uint32_t {
        return (uint32_t)(bs >= 64 ? x.y >> (bs - 64) : (x.x >> bs) | (x.y << (64 - bs)));
    };
    if (sel) {  // one round of a batched collect: only the level-1 buckets of its mask
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const uint32_t pb = digit(kk[j]);
            if (!((s_sel[pb >> 5] >> (pb & 31)) & 1u)) m &= ~(1u << j);
        }
    }
    uint32_t r[PPT];
#pragma unroll
    for (int j = 0; j < PPT; ++j) r[j] = (m & (1u << j)) ? atomicAdd(&s_cnt[digit(kk[j])], 1u) : 0u;
    __syncthreads();
    uint32_t c[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid * PER + q;
        c[q] = i < nb ? s_cnt[i] : 0;
        sum += c[q];
    }
    uint32_t total;
    uint32_t off = block_exclusive_sum<BLOCK>(sum, s_scan, &total);
    __syncthreads();  // every count is read before the run bases overwrite them
    // (the run reservations stay in flight across the LDS scatter, as in extract_partition_fast_kernel)
    unsigned long long gq[PER], be[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid * PER + q;
        gq[q] = 0, be[q] = 0;
        if (i < nb) {
            s_off[i] = (uint16_t)off;
            const size_t ci = (size_t)(tile / per_stripe) * nb + i;  // this tile's stripe
            if (c[q]) {
                gq[q] = atomicAdd(&cursor[ci], (unsigned long long)c[q]);
                be[q] = bend[ci];
            }
        }
        off += c[q];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PPT; ++j)
        if (m & (1u << j)) s_keys[s_off[digit(kk[j])] + r[j]] = kk[j];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid * PER + q;
        if (i < nb) {
            unsigned long long g = gq[q];
            if (c[q] && g + c[q] > be[q]) {  // pass A counted this bucket differently: never
                atomicOr(error, 2u);          // write past its range
                g = ~0ull;
            } else if (bdelta) {
                g += (unsigned long long)bdelta[i];
            }
            s_gbase[i] = g;
        }
    }
    __syncthreads();
    for (uint32_t p = tid; p < total; p += BLOCK) {
        const ulonglong2 key = s_keys[p];
        const uint32_t lb = digit(key);
        if (s_gbase[lb] == ~0ull) continue;
        *reinterpret_cast<ulonglong2 *>(&kout[s_gbase[lb] + (p - s_off[lb])]) = key;
    }
}

// Pass B's write cursors, one set per stripe.  All tiles scatter into the same 2^b level-1
// buckets, so one cursor per bucket would take every tile's atomic (146 k tiles x 512 buckets at
// the bench size, all on 512 words).  A pass-B tile is rps pass-A tiles; stripe s is the pass-B
// tiles [s C, (s + 1) C), and pass A's row r counts the pass-A tiles [r C, (r + 1) C), so with
// nrows = rps S rows, rows rps s .. rps s + rps - 1 count exactly stripe s: stripe s of bucket i
// starts at the bucket's start plus the stripe counts of stripes < s.  Contiguous stripes keep the
// runs of neighbouring tiles (which one XCD runs together, xcd_tile) next to each other in a
// bucket.  One workgroup per bucket, S <= 4 * 256.  Buckets outside the mask `sel` (not in this
// round of a batched collect) get empty stripes.
__global__ __launch_bounds__(256) void stripe_cursor_kernel(const uint32_t *__restrict__ rows, uint32_t nrows,
                                                            unsigned hb, unsigned b, uint32_t stripes, uint32_t rps,
                                                            const unsigned long long *__restrict__ bstart,
                                                            unsigned long long *__restrict__ cursor,
                                                            unsigned long long *__restrict__ bend,
                                                            const uint32_t *__restrict__ sel = nullptr) {
    __shared__ uint64_t s_scan[256 / 64 + 1];
    constexpr int PER = 4;
    const uint32_t i = blockIdx.x, nb = 1u << b, f = 1u << (hb - b), nbh = 1u << hb;
    const bool in = !sel || ((sel[i >> 5] >> (i & 31)) & 1u);
    uint32_t h[PER];
    uint64_t sum = 0;  // a bucket of a large input may hold more than 2^32 k-mers
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t st = threadIdx.x * PER + q;
        h[q] = 0;
        if (st < stripes && in) {
            const uint32_t r1 = stripes == 1 ? nrows : min(rps * st + rps, nrows);  // one stripe: every row
            for (uint32_t r = rps * st; r < r1; ++r)
                for (uint32_t j = 0; j < f; ++j) h[q] += rows[(size_t)r * nbh + i * f + j];
        }
        sum += h[q];
    }
    uint64_t total;
    uint64_t off = block_exclusive_sum_u64<256>(sum, s_scan, &total);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t st = threadIdx.x * PER + q;
        if (st < stripes) {
            cursor[(size_t)st * nb + i] = bstart[i] + off;
            bend[(size_t)st * nb + i] = bstart[i] + off + h[q];
        }
        off += h[q];
    }
}

// after pass B every cursor must sit exactly at its bucket's end (fewer keys than pass A counted
// would leave holes); sets error bit 2 otherwise
__global__ void cursor_check_kernel(const unsigned long long *__restrict__ cursor,
                                    const unsigned long long *__restrict__ bend, uint32_t nb,
                                    uint32_t *__restrict__ error) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nb && cursor[i] != bend[i]) atomicOr(error, 2u);
}

/*
 * The speculative level-1 layout (fused_pass_b_spec): pass A counts only every SA-th tile of each
 * row, and pass B scatters into segments sized from that sample, one per (bucket, stripe), bucket-
 * major, each rounded up to whole level-2 tiles (TILE2 keys) so that every level-2 tile lies inside
 * one segment: its keys are a prefix of the tile (tvalid[tile] of them) and the level-2 pass
 * (msd_hist_kernel / msd_partition_kernel with tvalid) reads the padded array without compaction.
 * caps[i * S + s] = the segment of bucket i, stripe s: the sampled count times SA with 1/slack + 3
 * sigma + 1024 of slack.  One workgroup per bucket, one thread per stripe (S <= 256).
 */
__global__ __launch_bounds__(256) void spec_l1_caps_kernel(const uint32_t *__restrict__ rows, uint32_t nrows,
                                                           unsigned hb, unsigned b, uint32_t stripes, uint32_t rps,
                                                           float sa, uint32_t tile2, uint32_t *__restrict__ caps,
                                                           bool tiny = false, uint32_t slack = 16) {
    // tiny (tests): half the sampled count, rounded down -- every populated stripe overflows
    // 256 / S threads per stripe, each over a share of its rows, summed by shuffles (one thread per stripe
    // walking its 128 rows serially: 0.13 ms for the launch)
    const uint32_t i = blockIdx.x, f = 1u << (hb - b), nbh = 1u << hb;
    const uint32_t tps = min(256u / max(stripes, 1u), 64u), s = threadIdx.x / tps, q = threadIdx.x % tps;
    uint64_t cnt = 0;
    if (s < stripes) {
        const uint32_t r1 = min(rps * s + rps, nrows);
        for (uint32_t r = rps * s + q; r < r1; r += tps)
            for (uint32_t j = 0; j < f; ++j) cnt += rows[(size_t)r * nbh + i * f + j];
    }
    for (uint32_t o = 1; o < tps; o <<= 1) cnt += __shfl_xor(cnt, (int)o, 64);
    if (s >= stripes || q) return;
    const double est = (double)cnt * (double)sa;  // sa: tiles per sampled tile
    uint64_t cap = (uint64_t)(est + est / slack + 3.0 * sqrt(est * sa) + 1024.0);
    cap = tiny ? (uint64_t)(est / 2) / tile2 * tile2 : (cap + tile2 - 1) / tile2 * tile2;
    caps[(size_t)i * stripes + s] = (uint32_t)min(cap, (uint64_t)0xFFFFFFFFu / tile2 * tile2);
}

// segment starts (scan of caps, bucket-major) -> pass B's per-stripe cursors and ends (stripe-major)
__global__ void spec_l1_cursor_kernel(const uint64_t *__restrict__ start, const uint32_t *__restrict__ caps,
                                      uint32_t nb, uint32_t stripes, unsigned long long *__restrict__ cursor,
                                      unsigned long long *__restrict__ bend) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)nb * stripes) return;
    const uint32_t i = (uint32_t)(t / stripes), s = (uint32_t)(t % stripes);
    cursor[(size_t)s * nb + i] = start[t];
    bend[(size_t)s * nb + i] = start[t] + caps[t];
}

// after the speculative pass B: every segment's fill (its cursor minus its start), the exact level-1
// counts h1 (zeroed by the caller), the total in *total, and tvalid of the segment's level-2 tiles
__global__ void spec_l1_finish_kernel(const uint64_t *__restrict__ start, const uint32_t *__restrict__ caps,
                                      const unsigned long long *__restrict__ cursor, uint32_t nb, uint32_t stripes,
                                      uint32_t tile2, uint32_t *__restrict__ h1, uint32_t *__restrict__ tvalid,
                                      unsigned long long *__restrict__ total) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)nb * stripes) return;
    const uint32_t i = (uint32_t)(t / stripes), s = (uint32_t)(t % stripes);
    const uint64_t st = start[t], cap = caps[t];
    const uint64_t fill = min((uint64_t)cursor[(size_t)s * nb + i] - st, cap);  // past cap: overflow, flagged
    if (fill) {
        atomicAdd(&h1[i], (uint32_t)fill);
        atomicAdd(total, (unsigned long long)fill);
    }
    for (uint64_t o = 0; o < cap; o += tile2)
        tvalid[(st + o) / tile2] = (uint32_t)(fill > o ? min(fill - o, (uint64_t)tile2) : 0);
}

// duplication estimate straight from the read bytes (the keys do not exist yet): the k-mer at
// m evenly spaced window starts, when valid, into the fingerprint table of estimate_dup
template <int L>
__global__ void dup_sample_reads_kernel(const uint8_t *__restrict__ seq, uint64_t seq_len, unsigned K,
                                        int canonical, uint32_t m, unsigned long long *__restrict__ table,
                                        uint32_t mask, unsigned long long *__restrict__ stats) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint64_t npos = seq_len - K + 1;
    // window starts at multiples of 8 bytes, read as 8-byte words (the byte-by-byte loads were a latency
    // chain of K loads per thread: 0.26 ms for 2^19 windows)
    const uint64_t p = (uint64_t)((double)j * ((double)npos / m)) & ~7ull;
    const unsigned nw = (K + 7) / 8;
    const bool wide = ((((uintptr_t)(seq + p)) & 7) == 0) && p + 8ull * nw <= seq_len;
    Key<L> P = Key<L>::zero(), R = Key<L>::zero();
    uint64_t wv = 0;
    for (unsigned i = 0; i < K; ++i) {
        uint32_t byte;
        if (wide) {
            if ((i & 7) == 0) wv = *(const uint64_t *)(seq + p + i);
            byte = (uint32_t)(wv >> (8 * (i & 7))) & 0xFFu;
        } else {
            byte = seq[p + i];
        }
        const uint32_t c = encode_dna(byte);
        if (c == 4) return;
        P = P | shl(Key<L>::from(c), 2 * i);
        R = R | shl(Key<L>::from(3 - c), 2 * (K - 1 - i));
    }
    const Key<L> low = Key<L>::lowmask(2 * (K - 1));
    Key<L> f = plain_to_boss(P, K, low);
    if (canonical) {
        const Key<L> r = plain_to_boss(R, K, low);
        if (r < f) f = r;
    }
    uint64_t h = 0x9e3779b97f4a7c15ull;
#pragma unroll
    for (int i = 0; i < L; ++i) {
        h ^= f.w[i];
        h ^= h >> 33;
        h *= 0xff51afd7ed558ccdull;
        h ^= h >> 33;
        h *= 0xc4ceb9fe1a85ec53ull;
        h ^= h >> 33;
    }
    h |= 1;
    atomicAdd(&stats[1], 1ull);  // valid samples
    uint32_t slot = (uint32_t)(h >> 32) & mask;
    while (true) {
        const unsigned long long prev = atomicCAS(&table[slot], 0ull, (unsigned long long)h);
        if (prev == 0) return;
        if (prev == h) {
            atomicAdd(&stats[0], 1ull);  // repeats
            return;
        }
        slot = (slot + 1) & mask;
    }
}

}  // namespace mtg
