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
