/*
 * boss_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, single thread) of MetaGraph's `build` hot path:
 * k-mer extraction -> canonicalisation -> sort/unique (or sort/count) -> reverse-complement
 * augmentation -> dummy sink/source generation -> lift + merge -> BOSS::Chunk (W, last, F,
 * weights).  It is the CHECKER for the HIP implementation and the "port" CPU baseline in
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it;
 * the product library (libmtg_boss.so) never links or calls it.
 *
 * Parity pinning: the reference cannot be compiled in this image (sdsl-lite, ips4o, spdlog,
 * KMC submodules are empty), so this restatement is pinned by the reference's
 * own goldens: integration_tests/test_build.py & test_build_weighted.py node counts / average
 * weights on tests/data/transcripts_1000.fa, the KMerBOSS hex KATs of tests/test_kmer_boss.cpp,
 * the reverse-complement property of tests/kmer/test_transform.cpp, the dummy<=>zero-weight
 * invariant of tests/graph/succinct/test_boss_construct.cpp, and by an independent
 * definition-level Python builder (oracle/boss_definition.py).
 *
 * Key words are exchanged as little-endian arrays of 64-bit limbs.  The limb count per key
 * follows the reference's word choice (boss_chunk_construct.cpp:1068-1079 for 2-bit keys,
 * :1030-1036 for 3-bit lifted keys): 1, 2 or 4 limbs.
 */
#ifndef MTG_BOSS_ORACLE_H
#define MTG_BOSS_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_keys {
    uint64_t n;          /* number of keys */
    uint32_t limbs;      /* 64-bit limbs per key */
    uint64_t *words;     /* n * limbs, little-endian limbs */
    uint32_t *counts;    /* n counts (NULL when not counting) */
} oracle_keys;

typedef struct oracle_chunk {
    uint64_t k;          /* BOSS k (node length) */
    uint64_t n;          /* number of rows incl. the leading dummy row 0 */
    uint8_t *W;          /* n edge labels, 0..9 (label + 5 for "minus") */
    uint8_t *last;       /* n bits stored as bytes 0/1 */
    uint32_t *weights;   /* n weights (NULL when bits_per_count == 0) */
    uint64_t F[5];
    uint64_t n_real;     /* real (non-dummy) k-mers */
    uint64_t n_dummy_sink;
    uint64_t n_dummy_source;  /* all levels, deduplicated */
} oracle_chunk;

/*
 * Input: n_seqs sequences concatenated in `seq` with offsets[n_seqs + 1]; counts[n_seqs] or
 * NULL (all 1).  k = BOSS k (node length), so (k+1)-mers are extracted, exactly like
 * IBOSSChunkConstructor::initialize(k, canonical, bits_per_count, "").
 */
int oracle_collect(uint64_t k, int canonical, int bits_per_count,
                   const char *seq, const uint64_t *offsets, const uint64_t *counts,
                   uint64_t n_seqs, oracle_keys *out);

/* collect + add_reverse_complements (canonical) : the sorted real 2-bit k-mers */
int oracle_real_kmers(uint64_t k, int canonical, int bits_per_count,
                      const char *seq, const uint64_t *offsets, const uint64_t *counts,
                      uint64_t n_seqs, oracle_keys *out);

/* the sorted dummy k-mer array (3-bit lifted words) as fed to the final merge */
int oracle_dummy_kmers(uint64_t k, int canonical, int bits_per_count,
                       const char *seq, const uint64_t *offsets, const uint64_t *counts,
                       uint64_t n_seqs, oracle_keys *out);

/* full path: BOSS::Chunk arrays */
int oracle_build_chunk(uint64_t k, int canonical, int bits_per_count,
                       const char *seq, const uint64_t *offsets, const uint64_t *counts,
                       uint64_t n_seqs, oracle_chunk *out);

/* the same full path fed with pre-extracted real 2-bit keys (+counts), as the chunk
 * constructor sees them after KmerCollector::data(); keys need not be sorted/unique. */
int oracle_build_chunk_from_kmers(uint64_t k, int canonical, int bits_per_count,
                                  const oracle_keys *kmers, oracle_chunk *out);

/* the suffix-filtered route: IBOSSChunkConstructor::initialize(k, both_strands, bits_per_count,
 * suffix) + build_chunk (boss_chunk_construct.cpp:946-1013): BOSS::Chunk of the `$`-padded
 * (k+1)-mers whose node ends with `suffix` (chars of "$ACGT", shorter than k + 1) */
int oracle_build_suffix_chunk(uint64_t k, int both_strands, int bits_per_count, const char *suffix,
                              const char *seq, const uint64_t *offsets, const uint64_t *counts,
                              uint64_t n_seqs, oracle_chunk *out);

/* building blocks (unit-level KATs) */
void oracle_pack_kmer(const uint8_t *codes, uint64_t len, uint32_t bits_per_char,
                      uint32_t limbs, uint64_t *out_words);
void oracle_reverse_complement(uint64_t len, uint32_t limbs, const uint64_t *in_words,
                               uint64_t *out_words);

void oracle_keys_free(oracle_keys *keys);
void oracle_chunk_free(oracle_chunk *chunk);
const char *oracle_last_error(void);

#ifdef __cplusplus
}
#endif

#endif
