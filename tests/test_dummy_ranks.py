"""The dense-rank form of the dummy keys (boss_kernels.hpp: dummy_encode_kernel /
dummy_decode_kernel) checked as arithmetic on the CPU: for every dummy string a small BOSS k
allows -- sinks r_1..r_k + label $, sources r_1..r_m $^(k-m) + a real label (the dummy edges of
boss_chunk_construct.cpp:54-168, 286-306) -- the rank is a bijection onto [0, T(0)) that preserves
the order of the lifted keys ($ACGT, 3 bits per char, the last node char most significant), and
the decode walk inverts it.  The GPU path is checked against the oracle in the -m gpu tests
(every k; MTG_DUMMY_SORT=lifted keeps the lifted sort)."""
import itertools

import pytest


def space(k):
    return (7 * 4 ** k - 4) // 3


def lifted(node_top_down, label, k):
    """node chars given most significant first (position k .. 1), values 0..4 ($ACGT)."""
    x = label
    for j, v in enumerate(reversed(node_top_down)):  # position 1 first
        x |= v << (3 * (j + 1))
    return x


def encode(x, k):
    W = S = m = top = 0
    for j in range(1, k + 1):
        v = (x >> (3 * j)) & 7
        if v:
            W |= (v - 1) << (2 * (j - 1))
            S += v - 1
            m += 1
        else:
            top = j
    c = x & 7
    assert top == k - m and (m < k) == (c != 0)
    return 4 * m + (7 * W - 4 * S) // 3 + (c - 1 if m < k else 0)


def decode(r, k):
    T = space(k)
    x = 0
    for p in range(1, k + 1):
        if r < 4:
            return x | (r + 1)
        r -= 4
        T = (T - 4) // 4
        rp = (r >= T) + (r >= 2 * T) + (r >= 3 * T)
        r -= rp * T
        x |= (rp + 1) << (3 * (k - p + 1))
    assert r == 0
    return x


def dummies(k):
    out = []
    for m in range(0, k + 1):
        for real in itertools.product(range(1, 5), repeat=m):
            node = list(real) + [0] * (k - m)
            labels = [0] if m == k else range(1, 5)
            out += [lifted(node, c, k) for c in labels]
    return out


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 6])
def test_rank_is_an_order_preserving_bijection(k):
    ds = sorted(dummies(k))
    ranks = [encode(x, k) for x in ds]
    assert ranks == list(range(space(k)))  # dense, in lifted order
    assert all(decode(r, k) == x for r, x in zip(ranks, ds))


def test_rank_fits_u64_up_to_k30():
    assert space(30) < 2 ** 64 and 7 * 4 ** 30 < 2 ** 64
    assert (space(30)).bit_length() == 62  # 8 LSD passes of 8 bits
    assert 7 * 4 ** 31 >= 2 ** 64  # k = 31 would overflow: the lifted sort takes over


def char_sum2(w):
    return sum((w >> (2 * i)) & 3 for i in range(32))


def rank_direct(W, m, k, c):
    return 4 * m + (7 * W - 4 * char_sum2(W)) // 3 + (c if m < k else 0)


@pytest.mark.parametrize("k", [1, 2, 5, 12, 30])
def test_ranks_straight_from_the_edge(k):
    # dummy_write_kernel<RANKS>: a sink's and every source level's rank from the 2-bit edge x
    # (node a_1..a_k at bits 2i, label a_K in the low bits) equal the rank of the lifted dummy the
    # reference builds (to_next + $ label, :54-98; to_prev + $ in char 1 and its levels, :123-168)
    import random
    rnd = random.Random(k)
    K = k + 1
    for _ in range(200):
        a = [rnd.randrange(4) for _ in range(K)]  # a[0] = a_1 ... a[K-1] = a_K
        node = sum(a[i] << (2 * i) for i in range(k))
        # sink: node a_2 .. a_K, label $
        sink = lifted([v + 1 for v in reversed(a[1:K])], 0, k)
        assert encode(sink, k) == rank_direct(sum(a[i + 1] << (2 * i) for i in range(k)), k, k, 0)
        for lev in range(1, k + 1):
            # level lev: node $^lev a_1 .. a_(k-lev) (a_1 at position lev + 1), label a_(k-lev+1)
            top_down = [v + 1 for v in reversed(a[:k - lev])] + [0] * lev
            src = lifted(top_down, a[k - lev] + 1, k)
            low = node & ((1 << (2 * (k - lev))) - 1)
            assert encode(src, k) == rank_direct(low << (2 * lev), k - lev, k, (node >> (2 * (k - lev))) & 3)


def bitmap_base(m):
    """bits of the source levels with fewer than m real chars (boss_kernels.hpp: dummy_bitmap_base)"""
    return (4 ** (m + 1) - 4) // 3


@pytest.mark.parametrize("k", [1, 2, 3, 5, 6])
def test_source_bitmap_index_is_the_rank(k):
    # dummy_write_kernel sets bit base(m) + (low << 2 | c) for the level-(k - m) source with first m real
    # chars `low` (a_1 lowest) and next char c; dummy_bitmap_ranks_kernel turns a set bit back into the
    # dense rank.  Over every (m, low, c) of the small levels: the bits are distinct, the walk finds m
    # again, and the rank is the encode of the lifted source (its real chars at node positions
    # k - m + 1 .. k, a_1 lowest of them, $ below, label c)
    ms = min(k, 10)
    seen = set()
    for m in range(ms):
        for low in range(4 ** m):
            for c in range(4):
                idx = bitmap_base(m) + (low << 2 | c)
                assert idx not in seen
                seen.add(idx)
                mm = 0
                while mm + 1 < ms and bitmap_base(mm + 1) <= idx:
                    mm += 1
                assert mm == m
                r = idx - bitmap_base(mm)
                # the lifted source: $ at node positions 1 .. k - m, a_i at position k - m + i
                x = c + 1
                for i in range(m):
                    x |= (((low >> (2 * i)) & 3) + 1) << (3 * (k - m + i + 1))
                W = (r >> 2) << (2 * (k - m))
                S = sum((low >> (2 * i)) & 3 for i in range(m))
                assert 4 * m + (7 * W - 4 * S) // 3 + (r & 3) == encode(x, k)
    assert len(seen) == bitmap_base(ms)


def _spread21(x):
    # dummy_decode_fast's spread21: 21 2-bit digits to 3-bit slots by five mask-and-shift steps
    pos = [2 * d for d in range(21)]
    for s in range(4, -1, -1):
        mk = 0
        for d in range(21):
            if (d >> s) & 1:
                mk |= 3 << pos[d]
                pos[d] += 1 << s
        x = (x & ~mk) | ((x & mk) << (1 << s))
    return x


def decode_closed_form(r, k, bits):
    """boss_kernels.hpp: dummy_decode_fast -- 3 r = 12 m + 7 W - 4 S + 3 c inverted through the low 10
    bits of 3 r (mod 2^bits, the device's u64 / u128 word); None where the kernel walks char by char."""
    M = (1 << bits) - 1
    V = (3 * r) & M
    eps = V & 1023
    W = ((V - eps) * pow(7, -1, 1 << bits)) & M
    t = eps + 4 * sum((W >> (2 * j)) & 3 for j in range(bits // 2))
    m, c = t // 12, (t % 12) // 3
    if t % 3 or m + 5 > k or W >> (2 * k):
        return None
    lo = k - m
    if W & ((1 << (2 * lo)) - 1):
        return None
    ones = 0x1249249249249249
    x = c + 1
    for pi in range(3):
        d0 = 21 * pi
        if d0 >= k:
            break
        a, b = max(lo - d0, 0), min(k - d0, 21)
        o = (ones & ((1 << (3 * b)) - 1) & ~((1 << (3 * a)) - 1)) if a < b else 0
        x |= (_spread21((W >> (2 * d0)) & ((1 << 42) - 1)) + o) << (63 * pi + 3)
    return x


@pytest.mark.parametrize("k", [5, 6, 7])
def test_closed_form_decode_every_dummy(k):
    # every dummy of a small k: the closed form returns the walk's key or defers to it (sinks and the
    # last 4 source levels only)
    for x in dummies(k):
        r = encode(x, k)
        got = decode_closed_form(r, k, 64)
        m = sum(1 for j in range(1, k + 1) if (x >> (3 * j)) & 7)
        if got is None:
            assert m > k - 5, (k, x)
        else:
            assert got == x == decode(r, k)


@pytest.mark.parametrize("k,bits", [(30, 64), (31, 128), (47, 128), (62, 128)])
def test_closed_form_decode_random_sources(k, bits):
    # random source dummies at the widths the device decodes (u64 ranks to k = 30, u128 to k = 62)
    import random
    rng = random.Random(k)
    for _ in range(3000):
        m = rng.randint(0, k - 1)
        node = [rng.randint(1, 4) for _ in range(m)] + [0] * (k - m)
        x = lifted(node, rng.randint(1, 4), k)
        got = decode_closed_form(encode(x, k), k, bits)
        assert got == x if m <= k - 5 else got is None
