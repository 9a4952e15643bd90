/*
 * boss_oracle.c -- TEST INFRASTRUCTURE ONLY (see boss_oracle.h for scope and pinning).
 *
 * Plain-C, single-threaded restatement of the reference's in-memory BOSS construction
 * (CS1 in SURVEY.md).  The per-word-width bodies live in oracle_pipeline.inc; this file holds
 * the alphabet tables, a byte-wise LSD radix sort standing in for ips4o::parallel::sort (any
 * correct sort gives the same result: keys are totally ordered and equal keys are merged
 * commutatively), and the dispatch on k that the reference does in
 * boss_chunk_construct.cpp:1068-1079 / :1030-1036.
 */
#include "boss_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <omp.h>
#include <string.h>

static __thread char g_err[256];

static void set_error(const char *msg) {
    snprintf(g_err, sizeof(g_err), "%s", msg);
}

const char *oracle_last_error(void) { return g_err; }

static void *xmalloc(size_t n) {
    void *p = malloc(n ? n : 1);
    if (!p) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
    return p;
}

static void *xrealloc(void *p, size_t n) {
    p = realloc(p, n ? n : 1);
    if (!p) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
    return p;
}

/* kmer/alphabets.hpp:127-143 : A/a->0, C/c->1, G/g->2, T/t/U/u->3, everything else 4 */
static uint8_t kCharToDNA[128];
static const uint8_t kComplementDNA[5] = {3, 2, 1, 0, 4};

__attribute__((constructor)) static void init_tables(void) {
    for (int i = 0; i < 128; ++i) kCharToDNA[i] = 4;
    kCharToDNA['A'] = kCharToDNA['a'] = 0;
    kCharToDNA['C'] = kCharToDNA['c'] = 1;
    kCharToDNA['G'] = kCharToDNA['g'] = 2;
    kCharToDNA['T'] = kCharToDNA['t'] = 3;
    kCharToDNA['U'] = kCharToDNA['u'] = 3;
}

/*
 * Stable LSD radix sort over little-endian key bytes, with an optional u32 payload.
 * Passes whose byte is constant over all keys are skipped.  Large inputs run each pass on all
 * OpenMP threads: per-thread digit counts over contiguous chunks, offsets digit-major then
 * thread-minor, scatter in chunk order -- the same stable order as the serial pass, so the
 * result does not depend on the thread count (this is the CPU baseline's stand-in for
 * ips4o::parallel::sort; any correct sort gives the same sets).
 */
#define DEFINE_RADIX(ESZ)                                                                   \
    static void radix_sort_##ESZ(uint8_t *keys, uint32_t *cnt, size_t n) {                 \
        if (n < 2) return;                                                                 \
        uint8_t *tmp = (uint8_t *)xmalloc(n * ESZ);                                        \
        uint32_t *tcnt = cnt ? (uint32_t *)xmalloc(n * sizeof(uint32_t)) : NULL;           \
        int nt = 1;                                                                        \
        if (n >= ((size_t)1 << 20)) nt = omp_get_max_threads();                            \
        if (nt > 256) nt = 256;                                                            \
        size_t(*th)[256] = (size_t(*)[256])xmalloc((size_t)nt * ESZ * 256 * sizeof(size_t)); \
        memset(th, 0, (size_t)nt * ESZ * 256 * sizeof(size_t));                            \
        _Pragma("omp parallel num_threads(nt)")                                            \
        {                                                                                  \
            const int t = omp_get_thread_num();                                            \
            const size_t lo = n * t / nt, hi = n * (t + 1) / nt;                           \
            for (size_t i = lo; i < hi; ++i)                                               \
                for (int b = 0; b < ESZ; ++b) th[t * ESZ + b][keys[i * ESZ + b]]++;        \
        }                                                                                  \
        uint8_t *src = keys, *dst = tmp;                                                   \
        uint32_t *csrc = cnt, *cdst = tcnt;                                                \
        for (int b = 0; b < ESZ; ++b) {                                                    \
            int trivial = 0;                                                               \
            for (int d = 0; d < 256 && !trivial; ++d) {                                    \
                size_t tot = 0;                                                            \
                for (int t = 0; t < nt; ++t) tot += th[t * ESZ + b][d];                    \
                if (tot == n) trivial = 1;                                                 \
            }                                                                              \
            if (trivial) continue;                                                         \
            /* this pass's per-thread digit counts over the CURRENT order */              \
            size_t(*pc)[256] = (size_t(*)[256])xmalloc((size_t)nt * 256 * sizeof(size_t)); \
            memset(pc, 0, (size_t)nt * 256 * sizeof(size_t));                              \
            _Pragma("omp parallel num_threads(nt)")                                        \
            {                                                                              \
                const int t = omp_get_thread_num();                                        \
                const size_t lo = n * t / nt, hi = n * (t + 1) / nt;                       \
                for (size_t i = lo; i < hi; ++i) pc[t][src[i * ESZ + b]]++;                \
            }                                                                              \
            size_t s = 0;                                                                  \
            for (int d = 0; d < 256; ++d)                                                  \
                for (int t = 0; t < nt; ++t) {                                             \
                    const size_t c = pc[t][d];                                             \
                    pc[t][d] = s;                                                          \
                    s += c;                                                                \
                }                                                                          \
            _Pragma("omp parallel num_threads(nt)")                                        \
            {                                                                              \
                const int t = omp_get_thread_num();                                        \
                const size_t lo = n * t / nt, hi = n * (t + 1) / nt;                       \
                size_t *off = pc[t];                                                       \
                for (size_t i = lo; i < hi; ++i) {                                         \
                    size_t o = off[src[i * ESZ + b]]++;                                    \
                    memcpy(dst + o * ESZ, src + i * ESZ, ESZ);                             \
                    if (cnt) cdst[o] = csrc[i];                                            \
                }                                                                          \
            }                                                                              \
            free(pc);                                                                      \
            uint8_t *t = src; src = dst; dst = t;                                          \
            uint32_t *ct = csrc; csrc = cdst; cdst = ct;                                   \
        }                                                                                  \
        if (src != keys) {                                                                 \
            memcpy(keys, src, n * ESZ);                                                    \
            if (cnt) memcpy(cnt, csrc, n * sizeof(uint32_t));                              \
        }                                                                                  \
        free(th);                                                                          \
        free(tmp);                                                                         \
        free(tcnt);                                                                        \
    }

DEFINE_RADIX(8)
DEFINE_RADIX(16)
DEFINE_RADIX(32)

static void radix_sort_records(void *keys, size_t esz, uint32_t *cnt, size_t n) {
    switch (esz) {
        case 8: radix_sort_8((uint8_t *)keys, cnt, n); break;
        case 16: radix_sort_16((uint8_t *)keys, cnt, n); break;
        case 32: radix_sort_32((uint8_t *)keys, cnt, n); break;
        default: abort();
    }
}

/* KmerExtractorBOSS codes -- kmer/alphabets.hpp:68-77: A C G T/U (either case) -> 1..4, else 5 */
static uint8_t boss_code(char ch) {
    switch (ch) {
        case 'A': case 'a': return 1;
        case 'C': case 'c': return 2;
        case 'G': case 'g': return 3;
        case 'T': case 't': case 'U': case 'u': return 4;
        default: return 5;
    }
}

/* COMPL_TAB of common/seq_tools/reverse_complement.hpp on the chars that encode as valid: the
   table maps no other char onto A C G T U, so the rest stays invalid whatever it becomes */
static char compl_char(char ch) {
    switch (ch) {
        case 'A': return 'T'; case 'a': return 't';
        case 'C': return 'G'; case 'c': return 'g';
        case 'G': return 'C'; case 'g': return 'c';
        case 'T': case 'U': return 'A';
        case 't': case 'u': return 'a';
        default: return 'N';
    }
}

#include "oracle_words.h"

#define T2 u64
#define T3 u64
#include "oracle_pipeline.inc"
#undef T3
#define T3 u128
#include "oracle_pipeline.inc"
#undef T2
#undef T3
#define T2 u128
#define T3 u128
#include "oracle_pipeline.inc"
#undef T3
#define T3 u256
#include "oracle_pipeline.inc"
#undef T2
#undef T3
#define T2 u256
#define T3 u256
#include "oracle_pipeline.inc"
#undef T2
#undef T3

typedef int (*run_fn)(int, size_t, int, int, const char *, const uint64_t *, const uint64_t *,
                      uint64_t, const oracle_keys *, oracle_keys *, oracle_chunk *);

/* word choice: 2-bit by (k+1)*2 (boss_chunk_construct.cpp:1068-1079), lifted by (k+1)*3
 * (:1030-1036); k is the BOSS k, valid in [1, 84] (:1057-1062) */
static run_fn pick(uint64_t k) {
    uint64_t K = k + 1;
    if (k < 1 || k > 84) return NULL;
    if (3 * K <= 64) return run_u64_u64;
    if (2 * K <= 64) return run_u64_u128;
    if (3 * K <= 128) return run_u128_u128;
    if (2 * K <= 128) return run_u128_u256;
    return run_u256_u256;
}

static int dispatch(int stage, uint64_t k, int canonical, int bits_per_count, const char *seq,
                    const uint64_t *offsets, const uint64_t *counts, uint64_t n_seqs,
                    const oracle_keys *pre, oracle_keys *keys_out, oracle_chunk *chunk_out) {
    run_fn f = pick(k);
    if (!f) { set_error("k must be in [1, 84]"); return -1; }
    if (bits_per_count < 0 || bits_per_count > 32) {
        set_error("bits_per_count must be in [0, 32]");
        return -1;
    }
    if (keys_out) memset(keys_out, 0, sizeof(*keys_out));
    if (chunk_out) memset(chunk_out, 0, sizeof(*chunk_out));
    return f(stage, k, canonical, bits_per_count, seq, offsets, counts, n_seqs, pre, keys_out,
             chunk_out);
}

int oracle_collect(uint64_t k, int canonical, int bits_per_count, const char *seq,
                   const uint64_t *offsets, const uint64_t *counts, uint64_t n_seqs,
                   oracle_keys *out) {
    return dispatch(0, k, canonical, bits_per_count, seq, offsets, counts, n_seqs, NULL, out,
                    NULL);
}

int oracle_real_kmers(uint64_t k, int canonical, int bits_per_count, const char *seq,
                      const uint64_t *offsets, const uint64_t *counts, uint64_t n_seqs,
                      oracle_keys *out) {
    return dispatch(1, k, canonical, bits_per_count, seq, offsets, counts, n_seqs, NULL, out,
                    NULL);
}

int oracle_dummy_kmers(uint64_t k, int canonical, int bits_per_count, const char *seq,
                       const uint64_t *offsets, const uint64_t *counts, uint64_t n_seqs,
                       oracle_keys *out) {
    return dispatch(2, k, canonical, bits_per_count, seq, offsets, counts, n_seqs, NULL, out,
                    NULL);
}

int oracle_build_chunk(uint64_t k, int canonical, int bits_per_count, const char *seq,
                       const uint64_t *offsets, const uint64_t *counts, uint64_t n_seqs,
                       oracle_chunk *out) {
    return dispatch(3, k, canonical, bits_per_count, seq, offsets, counts, n_seqs, NULL, NULL,
                    out);
}

int oracle_build_chunk_from_kmers(uint64_t k, int canonical, int bits_per_count,
                                  const oracle_keys *kmers, oracle_chunk *out) {
    return dispatch(3, k, canonical, bits_per_count, NULL, NULL, NULL, 0, kmers, NULL, out);
}

int oracle_build_suffix_chunk(uint64_t k, int both_strands, int bits_per_count, const char *suffix,
                              const char *seq, const uint64_t *offsets, const uint64_t *counts,
                              uint64_t n_seqs, oracle_chunk *out) {
    if (k < 1 || k > 84) { set_error("k must be in [1, 84]"); return -1; }
    if (bits_per_count < 0 || bits_per_count > 32) {
        set_error("bits_per_count must be in [0, 32]");
        return -1;
    }
    size_t ns = suffix ? strlen(suffix) : 0;
    if (!ns || ns >= k + 1) { set_error("the suffix must be non-empty and shorter than k + 1"); return -1; }
    uint8_t enc[96];
    for (size_t i = 0; i < ns; ++i) enc[i] = suffix[i] == '$' ? 0 : boss_code(suffix[i]);
    memset(out, 0, sizeof(*out));
    const uint64_t K = k + 1;
    if (3 * K <= 64)
        return suffix_run_u64_u64(k, both_strands, bits_per_count, enc, ns, seq, offsets, counts, n_seqs, out);
    if (3 * K <= 128)
        return suffix_run_u128_u128(k, both_strands, bits_per_count, enc, ns, seq, offsets, counts, n_seqs, out);
    return suffix_run_u256_u256(k, both_strands, bits_per_count, enc, ns, seq, offsets, counts, n_seqs, out);
}

void oracle_pack_kmer(const uint8_t *codes, uint64_t len, uint32_t bits_per_char,
                      uint32_t limbs, uint64_t *out_words) {
    /* KMerBOSS(arr, k) for any L: arr[len-1] in the low bits, arr[0..len-2] above it */
    u256_t seq = u256_zero();
    for (int i = (int)len - 2; i >= 0; --i) {
        seq = u256_or(seq, u256_from(codes[i]));
        seq = u256_shl(seq, bits_per_char);
    }
    seq = u256_or(seq, u256_from(codes[len - 1]));
    for (uint32_t i = 0; i < limbs; ++i) out_words[i] = i < 4 ? seq.w[i] : 0;
}

void oracle_reverse_complement(uint64_t len, uint32_t limbs, const uint64_t *in_words,
                               uint64_t *out_words) {
    u256_t x = u256_zero();
    for (uint32_t i = 0; i < limbs && i < 4; ++i) x.w[i] = in_words[i];
    u256_t r = revcomp2_u256_u256(x, len);
    for (uint32_t i = 0; i < limbs; ++i) out_words[i] = i < 4 ? r.w[i] : 0;
}

void oracle_keys_free(oracle_keys *keys) {
    if (!keys) return;
    free(keys->words);
    free(keys->counts);
    keys->words = NULL;
    keys->counts = NULL;
    keys->n = 0;
}

void oracle_chunk_free(oracle_chunk *chunk) {
    if (!chunk) return;
    free(chunk->W);
    free(chunk->last);
    free(chunk->weights);
    chunk->W = chunk->last = NULL;
    chunk->weights = NULL;
    chunk->n = 0;
}
