// keys.hpp -- k-mer words for the device pipeline.
//
// Key<L> is an L-limb little-endian unsigned integer (L = 1, 2, 4 -> 64/128/256 bits), the
// storage of KMerBOSS<G, 2> (tight 2-bit collector k-mers) and KMerBOSS<G, 3> (lifted $ACGT
// k-mers) of the reference (kmer/kmer_boss.hpp:29-120).  Integer order on the word is BOSS
// order, so every sort below is a plain unsigned sort.  Limb loops are fully unrolled: for
// L = 1 everything folds to scalar 64-bit ops.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mtg {

#define MTG_HD __host__ __device__ __forceinline__

template <int L>
struct alignas(L == 1 ? 8 : 16) Key {
    uint64_t w[L];

    static MTG_HD Key zero() {
        Key r;
#pragma unroll
        for (int i = 0; i < L; ++i) r.w[i] = 0;
        return r;
    }
    static MTG_HD Key from(uint64_t x) {
        Key r = zero();
        r.w[0] = x;
        return r;
    }
    static MTG_HD Key ones() {
        Key r;
#pragma unroll
        for (int i = 0; i < L; ++i) r.w[i] = ~0ull;
        return r;
    }
    // low n bits set
    static MTG_HD Key lowmask(unsigned n) {
        Key r;
#pragma unroll
        for (int i = 0; i < L; ++i) {
            unsigned lo = 64u * i;
            r.w[i] = n >= lo + 64 ? ~0ull : (n > lo ? ((1ull << (n - lo)) - 1) : 0ull);
        }
        return r;
    }
};

template <int L>
MTG_HD Key<L> operator|(Key<L> a, const Key<L> &b) {
#pragma unroll
    for (int i = 0; i < L; ++i) a.w[i] |= b.w[i];
    return a;
}
template <int L>
MTG_HD Key<L> operator&(Key<L> a, const Key<L> &b) {
#pragma unroll
    for (int i = 0; i < L; ++i) a.w[i] &= b.w[i];
    return a;
}
template <int L>
MTG_HD Key<L> operator~(Key<L> a) {
#pragma unroll
    for (int i = 0; i < L; ++i) a.w[i] = ~a.w[i];
    return a;
}
template <int L>
MTG_HD bool operator==(const Key<L> &a, const Key<L> &b) {
    bool eq = true;
#pragma unroll
    for (int i = 0; i < L; ++i) eq &= a.w[i] == b.w[i];
    return eq;
}
template <int L>
MTG_HD bool operator!=(const Key<L> &a, const Key<L> &b) { return !(a == b); }
template <int L>
MTG_HD bool operator<(const Key<L> &a, const Key<L> &b) {
    bool lt = false, decided = false;
#pragma unroll
    for (int i = L - 1; i >= 0; --i) {
        if (!decided && a.w[i] != b.w[i]) {
            lt = a.w[i] < b.w[i];
            decided = true;
        }
    }
    return lt;
}
template <int L>
MTG_HD bool operator>(const Key<L> &a, const Key<L> &b) { return b < a; }
template <int L>
MTG_HD bool operator<=(const Key<L> &a, const Key<L> &b) { return !(b < a); }

// a + b with carry (used for the lift: +1 per 3-bit char never carries across chars, but a
// char may straddle a limb boundary)
template <int L>
MTG_HD Key<L> operator+(const Key<L> &a, const Key<L> &b) {
    Key<L> r;
    uint64_t carry = 0;
#pragma unroll
    for (int i = 0; i < L; ++i) {
        uint64_t s = a.w[i] + b.w[i];
        uint64_t c1 = s < a.w[i];
        uint64_t s2 = s + carry;
        uint64_t c2 = s2 < s;
        r.w[i] = s2;
        carry = c1 | c2;
    }
    return r;
}

// limb i of a (0 outside [0, L)); a select chain, so a runtime i never indexes the array
// dynamically (which would put the key in scratch memory)
template <int L>
MTG_HD uint64_t limb(const Key<L> &a, int i) {
    uint64_t v = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) v = (i == j) ? a.w[j] : v;
    return v;
}

template <int L>
MTG_HD Key<L> shl(const Key<L> &a, unsigned s) {
    if (L == 1) return Key<L>::from(s >= 64 ? 0 : a.w[0] << s);
    Key<L> r;
    const int q = (int)(s >> 6);
    const unsigned b = s & 63;
#pragma unroll
    for (int i = 0; i < L; ++i) {
        uint64_t v = limb(a, i - q) << b;
        if (b) v |= limb(a, i - q - 1) >> (64 - b);
        r.w[i] = v;
    }
    return r;
}

template <int L>
MTG_HD Key<L> shr(const Key<L> &a, unsigned s) {
    if (L == 1) return Key<L>::from(s >= 64 ? 0 : a.w[0] >> s);
    Key<L> r;
    const int q = (int)(s >> 6);
    const unsigned b = s & 63;
#pragma unroll
    for (int i = 0; i < L; ++i) {
        uint64_t v = limb(a, i + q) >> b;
        if (b) v |= limb(a, i + q + 1) << (64 - b);
        r.w[i] = v;
    }
    return r;
}

// bits [pos, pos + n) as an integer, n <= 32
template <int L>
MTG_HD uint32_t bits_at(const Key<L> &a, unsigned pos, unsigned n) {
    const int q = (int)(pos >> 6);
    const unsigned b = pos & 63;
    uint64_t v = limb(a, q) >> b;
    if (b + n > 64) v |= limb(a, q + 1) << (64 - b);
    return (uint32_t)(v & ((1ull << n) - 1));
}

// character i of an L-bit-per-char KMerBOSS word (operator[], kmer_boss.hpp:188-194)
template <int L>
MTG_HD uint32_t char_at(const Key<L> &a, unsigned i, unsigned bits_per_char) {
    return bits_at(a, i * bits_per_char, bits_per_char);
}

// reverse the order of the 32 2-bit groups of a word
MTG_HD uint64_t reverse_pairs64(uint64_t v) {
    v = __builtin_bswap64(v);
    v = ((v >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((v & 0x0F0F0F0F0F0F0F0Full) << 4);
    v = ((v >> 2) & 0x3333333333333333ull) | ((v & 0x3333333333333333ull) << 2);
    return v;
}

// reverse complement of a tight 2-bit BOSS-layout (K)-mer (kmer_transform.hpp:14-35):
// label <- comp(a_1), pos 1 <- comp(a_K), pos i <- comp(a_{K+1-i})
template <int L>
MTG_HD Key<L> revcomp2(const Key<L> &x, unsigned K) {
    // plain layout P = a_1 at bits 0..1, ..., a_K at the top; the BOSS word is P rotated by
    // one char: boss = ((P & low(2(K-1))) << 2) | (P >> 2(K-1)).  rc in plain layout
    // reverses the char order and complements (3 - c = c ^ 3): complement all bits, reverse the
    // 2-bit groups of the whole L-limb word, and shift the K chars back down.
    const Key<L> P = shr(x, 2) | shl(Key<L>::from(x.w[0] & 3), 2 * (K - 1));
    const Key<L> C = ~P;
    Key<L> R;
#pragma unroll
    for (int i = 0; i < L; ++i) R.w[i] = reverse_pairs64(C.w[L - 1 - i]);
    R = shr(R, 64 * L - 2 * K);
    return shl(R & Key<L>::lowmask(2 * (K - 1)), 2) | shr(R, 2 * (K - 1));
}

// transform<3-bit>(2-bit word) + get_sentinel_delta (kmer_transform.hpp:38-47, :75-100):
// every char c -> c + 1 in a 3-bit slot.
template <int LO, int LI>
MTG_HD Key<LO> lift(const Key<LI> &x, unsigned K) {
    Key<LO> r = Key<LO>::zero();
    for (unsigned i = 0; i < K; ++i) {
        uint64_t c = bits_at(x, 2 * i, 2) + 1;
        r = r | shl(Key<LO>::from(c), 3 * i);
    }
    return r;
}

}  // namespace mtg
