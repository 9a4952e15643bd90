// superkmer.hpp -- exchange 0 of the multi-GPU build: every rank's windows go to a collect owner
// as super-k-mers (runs of consecutive windows with the same owner, 2 bits per char), not as keys.
//
// The collect owner of a window (a K-mer, K = k + 1) is a hash of its canonical minimizer: the
// smallest mix32 hash over the window's canonical M-mers (min of the forward and reverse-complement
// 2-bit codes; forward only in basic mode).  A window and its reverse complement have the same
// canonical M-mers, so every canonical k-mer -- every key the owner's collect extracts -- lives at
// exactly one owner, and the owners' sorted distinct sets are disjoint.  Consecutive windows share
// their minimizer for ~(K - M + 1) / 2 positions, so a 150-char read travels as ~12 runs of ~40
// chars: ~140 bytes packed (28 chars + a char count per 64-bit word) instead of the 120 x 8 bytes of
// its keys (6x less exchange volume at k = 30), and the hash spreads the owners' windows evenly (the
// key-prefix ranges of the routed collect were balanced on canonical keys, which pile up at small
// prefixes).  A run's last word holds at most 27 chars, so every word unpacks on its own into 28
// bytes (chars, then '$'): the received words become an ordinary read buffer of 28 bytes per word,
// every run ending in a separator, and the owner runs the single build's collect on it; the distinct keys then go to their BOSS-range owners
// as sorted runs (boss_pipeline.hip: run_pipeline_dist).  KMC's partitioning by signatures is the
// same idea; the reference has no multi-machine collect (cli/build.cpp:106-148 splits by suffix).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "boss_kernels.hpp"
#include "device_common.hpp"
#include "extract_partition.hpp"

namespace mtg {

constexpr int SK_BLOCK = 256;
constexpr int SK_PER = 16;                       // consecutive windows per thread
constexpr int SK_TILE = SK_BLOCK * SK_PER;       // windows per workgroup
constexpr int SK_KMAX = 512;                     // K bound of the path (LDS window overhang)
constexpr int SK_RUN_MAX = 256;                  // a run starts at least every 256 windows
constexpr uint8_t SK_NONE = 0xFF;                // window with an invalid char
constexpr int SK_MAX_OWNERS = 64;

__device__ __forceinline__ uint32_t sk_mix32(uint32_t h) {  // murmur3 finaliser
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

/*
 * own[p] = collect owner of window p (chars p .. p + K - 1 of seq), SK_NONE when the window holds
 * an invalid char.  One workgroup per SK_TILE windows: the tile's chars (2-bit codes) and the hashes
 * of its M-mers are staged in LDS; thread t takes windows 16t .. 16t + 15, whose minima share the
 * middle of their M-mer range: min(window j) = min(suffix-min of the first 15 - j ... , the shared
 * middle, prefix-min of the last j), w + 15 LDS reads for 16 windows instead of 16 w.  The owner is
 * a second hash of that minimum (the minimum itself is skewed towards 0: owner 0 took most windows).
 * Thread t reads LDS at 16 t + j, so both arrays are padded (one word per 16 hashes, one word per 16
 * chars): 17 t / 5 t words apart, every lane of a wave on its own bank.
 */
__device__ __forceinline__ uint32_t sk_hpad(uint32_t i) { return i + (i >> 4); }
__device__ __forceinline__ uint32_t sk_cpad(uint32_t i) { return i + ((i >> 4) << 2); }

__global__ __launch_bounds__(SK_BLOCK) void sk_owner_kernel(const uint8_t *__restrict__ seq, uint64_t seq_len,
                                                           unsigned K, unsigned M, int canonical, uint32_t P,
                                                           uint8_t *__restrict__ own) {
    constexpr int NC = SK_TILE + SK_KMAX;
    __shared__ uint8_t s_code[NC + NC / 4 + 16];
    __shared__ uint32_t s_h[NC + NC / 16 + 1];
    const uint32_t tid = threadIdx.x;
    const uint64_t npos = seq_len - K + 1;  // host: seq_len >= K
    const uint64_t base = (uint64_t)blockIdx.x * SK_TILE;
    const uint32_t nchars = (uint32_t)min((uint64_t)(SK_TILE + K - 1), seq_len - base);
    for (uint32_t i = tid; i < nchars; i += SK_BLOCK) s_code[sk_cpad(i)] = (uint8_t)encode_dna(seq[base + i]);
    __syncthreads();
    // M-mer hashes at tile positions 0 .. nh - 1 (an M-mer with an invalid char never enters a valid window)
    const uint32_t nh = nchars >= M ? nchars - M + 1 : 0;
    const uint32_t mmask = (uint32_t)((1ull << (2 * M)) - 1);
    auto roll = [&](uint32_t i0, uint32_t n) {  // hashes of positions i0 .. i0 + n - 1 (< nh)
        uint32_t f = 0, r = 0;
        for (unsigned j = 0; j + 1 < M; ++j) {
            const uint32_t x = s_code[sk_cpad(i0 + j)] & 3u;
            f = (f << 2) | x;
            r = (r >> 2) | ((3u - x) << (2 * (M - 1)));
        }
        for (uint32_t q = 0; q < n; ++q) {
            const uint32_t i = i0 + q;
            const uint32_t x = s_code[sk_cpad(i + M - 1)] & 3u;
            f = ((f << 2) | x) & mmask;
            r = (r >> 2) | ((3u - x) << (2 * (M - 1)));
            s_h[sk_hpad(i)] = sk_mix32(canonical && r < f ? r : f);
        }
    };
    for (uint32_t i0 = tid * SK_PER; i0 < nh; i0 += SK_BLOCK * SK_PER) roll(i0, min((uint32_t)SK_PER, nh - i0));
    __syncthreads();
    const unsigned w = K - M + 1;  // M-mers per window
    const uint32_t r0 = tid * SK_PER;
    if (base + r0 >= npos) return;
    // validity: the last invalid char at or before the window's end
    int32_t last_bad = -1;
    uint32_t valid = 0;
    {
        const uint32_t end = min((uint32_t)(r0 + SK_PER + K - 1), nchars);
        for (uint32_t i = r0; i < end; ++i) {
            if (s_code[sk_cpad(i)] > 3) last_bad = (int32_t)i;
            if (i + 1 >= r0 + K) {
                const uint32_t j = i + 1 - K - r0;  // window r0 + j ends at i
                if (last_bad < (int32_t)(r0 + j)) valid |= 1u << j;
            }
        }
    }
    uint32_t mins[SK_PER];
    if (w >= SK_PER) {
        // every window j contains M-mers [r0 + 15, r0 + w - 1]
        uint32_t mid = 0xFFFFFFFFu;
        for (uint32_t i = r0 + SK_PER - 1; i < r0 + w && i < nh; ++i) mid = min(mid, s_h[sk_hpad(i)]);
        uint32_t suf = 0xFFFFFFFFu;
#pragma unroll
        for (int j = SK_PER - 2; j >= 0; --j) {  // suffix minima of M-mers r0 + j .. r0 + 14
            if (r0 + j < nh) suf = min(suf, s_h[sk_hpad(r0 + j)]);
            mins[j] = suf;
        }
        mins[SK_PER - 1] = 0xFFFFFFFFu;
        uint32_t pre = 0xFFFFFFFFu;
#pragma unroll
        for (int j = 1; j < SK_PER; ++j) {  // prefix minima of M-mers r0 + w .. r0 + w + j - 1
            const uint32_t i = r0 + w + j - 1;
            if (i < nh) pre = min(pre, s_h[sk_hpad(i)]);
            mins[j] = min(mins[j], pre);
        }
#pragma unroll
        for (int j = 0; j < SK_PER; ++j) mins[j] = min(mins[j], mid);
    } else {
#pragma unroll
        for (int j = 0; j < SK_PER; ++j) {
            uint32_t m = 0xFFFFFFFFu;
            for (uint32_t i = r0 + j; i < r0 + j + w && i < nh; ++i) m = min(m, s_h[sk_hpad(i)]);
            mins[j] = m;
        }
    }
    // 16 owner bytes, stored as 4 words
    uint32_t ob[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < SK_PER; ++j) {
        const uint32_t o = (valid >> j) & 1u ? (uint32_t)(((uint64_t)sk_mix32(mins[j] ^ 0x9e3779b9u) * P) >> 32)
                                             : (uint32_t)SK_NONE;
        ob[j >> 2] |= o << (8 * (j & 3));
    }
    const uint64_t p0 = base + r0;
    if (p0 + SK_PER <= npos) {
        *(uint4 *)(own + p0) = make_uint4(ob[0], ob[1], ob[2], ob[3]);
    } else {
        for (int j = 0; j < SK_PER && p0 + j < npos; ++j) own[p0 + j] = (uint8_t)(ob[j >> 2] >> (8 * (j & 3)));
    }
}

/*
 * The runs, one pass counting and one writing (routed by owner like route_count / route_write):
 * COUNT: tcnt[o * ntiles + tile] = runs of owner o starting in the tile, tcnt[(P + o) * ntiles +
 * tile] = their packed 64-bit words.
 * WRITE: run -> words[woff ..] = its chars, 28 per word (2 bits each, bits 0..55) with the word's
 * char count in bits 56..60, ceil((len + 1) / 28) words so the last one holds <= 27; with per-read
 * counts also nwords[slot] / cnt[slot] = its word count and its read's count.  slot / woff come from
 * the scanned offsets (toff: runs, toffw: words, both owner-major) plus an LDS cursor (order inside a
 * tile's share is free: the owner sorts).
 * A run starts where the owner changes and at every multiple of SK_RUN_MAX windows, so no run
 * leaves its tile (SK_TILE is a multiple).  Round 5: the tile's run boundaries are a bitmap in LDS
 * (one 16-bit field per thread), so a run's end is the next set bit (at most 16 fields on); and its
 * chars are a 2-bit image of the tile in LDS (16 chars a word), so each output word is three LDS reads
 * and two funnel shifts instead of 28 byte reads and shifts (the char-by-char pack was 5.9 ms of an
 * 8-rank build's 2.5 M-read rank, twice the routed collect's compute).
 */
static_assert(SK_TILE % SK_RUN_MAX == 0, "runs must not cross tiles");
constexpr uint32_t SK_WCH = 28;  // chars per packed word

template <bool COUNT_ONLY>
__global__ __launch_bounds__(SK_BLOCK) void sk_runs_kernel(const uint8_t *__restrict__ own, uint64_t npos,
                                                          const uint8_t *__restrict__ seq, unsigned K, uint32_t P,
                                                          uint64_t ntiles, uint32_t *__restrict__ tcnt,
                                                          const uint64_t *__restrict__ toff,
                                                          const uint64_t *__restrict__ toffw,
                                                          const uint64_t *__restrict__ read_starts,
                                                          const uint32_t *__restrict__ read_counts, uint64_t n_reads,
                                                          const uint64_t *__restrict__ rid_at,
                                                          uint64_t *__restrict__ words, uint32_t *__restrict__ nwords,
                                                          uint32_t *__restrict__ cnt) {
    constexpr int NC = SK_TILE + SK_KMAX;
    constexpr int NWC = NC / 16 + 3;  // 2-bit image words (+ the overhang of a word's 3-word read)
    __shared__ uint8_t s_own[SK_TILE + 1];
    __shared__ uint16_t s_bnd[SK_BLOCK + 1];       // run boundaries: bit j of field t = window 16 t + j
    __shared__ uint32_t s_pk[COUNT_ONLY ? 1 : NWC];
    // one 64-bit cursor per owner: runs << 40 | words, so a run's slot and word offset come from
    // one atomic (the receiver finds the runs' first words from the word counts in slot order)
    __shared__ unsigned long long s_cur[SK_MAX_OWNERS];
    __shared__ uint64_t s_rbase[SK_MAX_OWNERS], s_wbase[SK_MAX_OWNERS];
    constexpr unsigned long long WMASK = (1ull << 40) - 1;
    const uint32_t tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * SK_TILE;
    const uint32_t tn = (uint32_t)min((uint64_t)SK_TILE, npos - base);
    for (uint32_t o = tid; o < P; o += SK_BLOCK) {
        s_cur[o] = 0;
        if (!COUNT_ONLY) {
            s_rbase[o] = toff[(uint64_t)o * ntiles + blockIdx.x];
            s_wbase[o] = toffw[(uint64_t)o * ntiles + blockIdx.x];
        }
    }
    const uint32_t r0 = tid * SK_PER;
    // this thread's 16 owner bytes (+ the one before them)
    uint8_t ob[SK_PER];
#pragma unroll
    for (int q = 0; q < SK_PER; ++q) ob[q] = r0 + q < tn ? own[base + r0 + q] : SK_NONE;
#pragma unroll
    for (int q = 0; q < SK_PER; ++q) s_own[r0 + q] = ob[q];
    if (!COUNT_ONLY) {
        const uint32_t nch = tn + K - 1;
        for (uint32_t wi = tid; wi < (uint32_t)NWC; wi += SK_BLOCK) {
            uint32_t pk = 0, iv;
            if (16 * wi < nch) pack_word(seq, base + nch, base + 16ull * wi, pk, iv);
            s_pk[wi] = pk;
        }
    }
    __syncthreads();
    // boundaries: window 0, every SK_RUN_MAX-th window, every owner change; the end of the tile
    const uint8_t prev0 = r0 ? s_own[r0 - 1] : SK_NONE;
    uint32_t bnd = 0;
#pragma unroll
    for (int q = 0; q < SK_PER; ++q) {
        const uint32_t r = r0 + q;
        const uint8_t pv = q ? ob[q - 1] : prev0;
        if (r < tn && (r % SK_RUN_MAX == 0 || ob[q] != pv)) bnd |= 1u << q;
        if (r >= tn) bnd |= 1u << q;  // past the tile: every position ends a run
    }
    s_bnd[tid] = (uint16_t)bnd;
    if (tid == 0) s_bnd[SK_BLOCK] = 0xFFFFu;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < SK_PER; ++q) {
        const uint32_t r = r0 + q;
        const uint8_t o = ob[q];
        if (r >= tn || o == SK_NONE || !((bnd >> q) & 1u)) continue;
        // the run's end: the next boundary after r (this thread's field first, then the next fields)
        uint32_t e;
        const uint32_t rest = bnd >> (q + 1);
        if (rest) {
            e = r + 1 + (uint32_t)__ffs(rest) - 1;
        } else {
            uint32_t t = tid + 1;
            while (!s_bnd[t]) ++t;
            e = 16 * t + (uint32_t)__ffs((uint32_t)s_bnd[t]) - 1;
        }
        e = min(e, tn);
        const uint32_t len = (e - r) + K - 1;
        const uint32_t nw = len / SK_WCH + 1;  // = ceil((len + 1) / 28)
        const unsigned long long old = atomicAdd(&s_cur[o], (1ull << 40) | (unsigned long long)nw);
        if (COUNT_ONLY) continue;
        const uint64_t slot = s_rbase[o] + (old >> 40);
        const uint64_t wo = s_wbase[o] + (old & WMASK);
        if (cnt) {
            nwords[slot] = nw;
            cnt[slot] = read_counts[read_of(read_starts, n_reads, rid_at, base + r)];
        }
        for (uint32_t wi = 0; wi < nw; ++wi) {
            const uint32_t c0 = r + wi * SK_WCH;  // first char of the word in the tile
            const uint32_t m = min(SK_WCH, len - wi * SK_WCH);
            const uint32_t q0 = c0 >> 4, sh = 2 * (c0 & 15);
            const uint32_t a = s_pk[q0], b = s_pk[q0 + 1], d = s_pk[q0 + 2];
            const uint32_t lo = sh ? __builtin_amdgcn_alignbit(b, a, sh) : a;
            const uint32_t hi = sh ? __builtin_amdgcn_alignbit(d, b, sh) : b;
            uint64_t v = (uint64_t)lo | ((uint64_t)hi << 32);
            v &= (1ull << (2 * m)) - 1;  // m <= 28: 56 bits at most
            words[wo + wi] = v | ((uint64_t)m << 56);
        }
    }
    if (COUNT_ONLY) {
        __syncthreads();
        for (uint32_t o = tid; o < P; o += SK_BLOCK) {
            tcnt[(uint64_t)o * ntiles + blockIdx.x] = (uint32_t)(s_cur[o] >> 40);
            tcnt[(uint64_t)(P + o) * ntiles + blockIdx.x] = (uint32_t)(s_cur[o] & WMASK);
        }
    }
}

// receiver: word x -> bytes [28 x, 28 x + 28): its chars, then '$' (coalesced: 7 words per thread)
__global__ void sk_unpack_kernel(const uint64_t *__restrict__ words, uint64_t n, uint32_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += stride) {
        const uint64_t v = words[x];
        const uint32_t m = (uint32_t)(v >> 56) & 31u;
#pragma unroll
        for (uint32_t q = 0; q < 7; ++q) {
            uint32_t b = 0;
#pragma unroll
            for (uint32_t t = 0; t < 4; ++t) {
                const uint32_t ci = q * 4 + t;
                const uint32_t ch = ci < m ? (0x54474341u >> (8 * ((uint32_t)(v >> (2 * ci)) & 3u))) & 0xFFu : (uint32_t)'$';
                b |= ch << (8 * t);
            }
            out[7 * x + q] = b;
        }
    }
}

// receiver (per-read counts): run j's first byte = 28 x its first word
__global__ void sk_starts_kernel(const uint64_t *__restrict__ wstart, uint64_t n, uint64_t *__restrict__ starts) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) starts[j] = SK_WCH * wstart[j];
}

}  // namespace mtg
