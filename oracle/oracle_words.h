/*
 * oracle_words.h -- TEST INFRASTRUCTURE ONLY (see boss_oracle.h).
 *
 * 64/128/256-bit unsigned words used as KMerBOSS storage, mirroring what the reference takes
 * from sdsl (uint64_t, sdsl::uint128_t = unsigned __int128, sdsl::uint256_t).  Every op is
 * named <type>_<op> so that oracle_pipeline.inc can be instantiated per word type, the way
 * the reference instantiates KMerBOSS<G, L> for G in {uint64_t, uint128_t, uint256_t}
 * (kmer/kmer_boss.hpp:29-120).
 */
#ifndef MTG_ORACLE_WORDS_H
#define MTG_ORACLE_WORDS_H

#include <stdint.h>
#include <string.h>

/* ---------------- 64 ---------------- */
typedef uint64_t u64_t;
#define U64_LIMBS 1
static inline u64_t u64_zero(void) { return 0; }
static inline u64_t u64_from(uint64_t x) { return x; }
static inline u64_t u64_shl(u64_t a, unsigned s) { return s >= 64 ? 0 : a << s; }
static inline u64_t u64_shr(u64_t a, unsigned s) { return s >= 64 ? 0 : a >> s; }
static inline u64_t u64_or(u64_t a, u64_t b) { return a | b; }
static inline u64_t u64_and(u64_t a, u64_t b) { return a & b; }
static inline u64_t u64_not(u64_t a) { return ~a; }
static inline u64_t u64_add(u64_t a, u64_t b) { return a + b; }
static inline int u64_lt(u64_t a, u64_t b) { return a < b; }
static inline int u64_eq(u64_t a, u64_t b) { return a == b; }
static inline uint64_t u64_low(u64_t a) { return a; }
static inline u64_t u64_lowmask(unsigned n) { return n >= 64 ? ~0ull : ((1ull << n) - 1); }
static inline void u64_store(u64_t a, uint64_t *w) { w[0] = a; }
static inline u64_t u64_load(const uint64_t *w) { return w[0]; }

/* ---------------- 128 ---------------- */
typedef unsigned __int128 u128_t;
#define U128_LIMBS 2
static inline u128_t u128_zero(void) { return 0; }
static inline u128_t u128_from(uint64_t x) { return x; }
static inline u128_t u128_shl(u128_t a, unsigned s) { return s >= 128 ? 0 : a << s; }
static inline u128_t u128_shr(u128_t a, unsigned s) { return s >= 128 ? 0 : a >> s; }
static inline u128_t u128_or(u128_t a, u128_t b) { return a | b; }
static inline u128_t u128_and(u128_t a, u128_t b) { return a & b; }
static inline u128_t u128_not(u128_t a) { return ~a; }
static inline u128_t u128_add(u128_t a, u128_t b) { return a + b; }
static inline int u128_lt(u128_t a, u128_t b) { return a < b; }
static inline int u128_eq(u128_t a, u128_t b) { return a == b; }
static inline uint64_t u128_low(u128_t a) { return (uint64_t)a; }
static inline u128_t u128_lowmask(unsigned n) {
    return n >= 128 ? ~(u128_t)0 : (((u128_t)1 << n) - 1);
}
static inline void u128_store(u128_t a, uint64_t *w) { w[0] = (uint64_t)a; w[1] = (uint64_t)(a >> 64); }
static inline u128_t u128_load(const uint64_t *w) { return ((u128_t)w[1] << 64) | w[0]; }

/* ---------------- 256 (w[0] least significant) ---------------- */
typedef struct { uint64_t w[4]; } u256_t;
#define U256_LIMBS 4
static inline u256_t u256_zero(void) { u256_t r = {{0, 0, 0, 0}}; return r; }
static inline u256_t u256_from(uint64_t x) { u256_t r = {{x, 0, 0, 0}}; return r; }
static inline u256_t u256_shl(u256_t a, unsigned s) {
    u256_t r = u256_zero();
    if (s >= 256) return r;
    unsigned q = s / 64, b = s % 64;
    for (int i = 3; i >= (int)q; --i) {
        uint64_t v = a.w[i - q] << b;
        if (b && i - (int)q - 1 >= 0) v |= a.w[i - q - 1] >> (64 - b);
        r.w[i] = v;
    }
    return r;
}
static inline u256_t u256_shr(u256_t a, unsigned s) {
    u256_t r = u256_zero();
    if (s >= 256) return r;
    unsigned q = s / 64, b = s % 64;
    for (int i = 0; i + (int)q < 4; ++i) {
        uint64_t v = a.w[i + q] >> b;
        if (b && i + q + 1 < 4) v |= a.w[i + q + 1] << (64 - b);
        r.w[i] = v;
    }
    return r;
}
static inline u256_t u256_or(u256_t a, u256_t b) {
    for (int i = 0; i < 4; ++i) a.w[i] |= b.w[i];
    return a;
}
static inline u256_t u256_and(u256_t a, u256_t b) {
    for (int i = 0; i < 4; ++i) a.w[i] &= b.w[i];
    return a;
}
static inline u256_t u256_not(u256_t a) {
    for (int i = 0; i < 4; ++i) a.w[i] = ~a.w[i];
    return a;
}
static inline u256_t u256_add(u256_t a, u256_t b) {
    u256_t r;
    unsigned __int128 c = 0;
    for (int i = 0; i < 4; ++i) {
        c += (unsigned __int128)a.w[i] + b.w[i];
        r.w[i] = (uint64_t)c;
        c >>= 64;
    }
    return r;
}
static inline int u256_lt(u256_t a, u256_t b) {
    for (int i = 3; i >= 0; --i)
        if (a.w[i] != b.w[i]) return a.w[i] < b.w[i];
    return 0;
}
static inline int u256_eq(u256_t a, u256_t b) {
    return a.w[0] == b.w[0] && a.w[1] == b.w[1] && a.w[2] == b.w[2] && a.w[3] == b.w[3];
}
static inline uint64_t u256_low(u256_t a) { return a.w[0]; }
static inline u256_t u256_lowmask(unsigned n) {
    u256_t r = u256_zero();
    for (int i = 0; i < 4; ++i) {
        if (n >= 64 * (unsigned)(i + 1)) r.w[i] = ~0ull;
        else if (n > 64 * (unsigned)i) r.w[i] = (1ull << (n - 64 * i)) - 1;
    }
    return r;
}
static inline void u256_store(u256_t a, uint64_t *w) { memcpy(w, a.w, 32); }
static inline u256_t u256_load(const uint64_t *w) { u256_t r; memcpy(r.w, w, 32); return r; }

#endif
