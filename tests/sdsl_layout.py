"""An independent reader of the sdsl-lite containers in the graph files (test infrastructure).

It parses a file byte by byte as sdsl-lite 2.x lays the containers out (int_vector framing,
rank_support_v / v5, select_support_mcl, wt_huff<> with its byte_tree, sd_vector<>, rrr_vector<63>;
see projects2014-metagenome_amd/csrc/sdsl_io.hpp for the citations) and RECOMPUTES every auxiliary
field from the payload bits with its own code: a file passes only if each rank sample, select
sample, Huffman node and class offset is the one sdsl's constructors would derive.  The layout is
a restatement of sdsl-lite's published serialization (sdsl-lite is an empty submodule in the
reference snapshot): byte parity with a reference-written file stays unpinned.
"""
import heapq
import math
import struct

import numpy as np


class Reader:
    def __init__(self, data):
        self.b = memoryview(data)
        self.p = 0

    def raw(self, fmt):
        n = struct.calcsize(fmt)
        if self.p + n > len(self.b):
            raise ValueError("truncated")
        v = struct.unpack_from(fmt, self.b, self.p)
        self.p += n
        return v[0] if len(v) == 1 else v

    def be(self):
        return self.raw(">Q")

    def words(self, n):
        if self.p + 8 * n > len(self.b):
            raise ValueError("truncated")
        w = np.frombuffer(self.b[self.p:self.p + 8 * n], dtype="<u8").copy()
        self.p += 8 * n
        return w

    def int_vector(self, fixed=0):
        nbits = self.raw("<Q")
        width = fixed if fixed else self.raw("<B")
        if width == 0 or width > 64:
            width = 64
        assert nbits % width == 0
        return IntVec(self.words((nbits + 63) // 64), nbits // width, width)

    def done(self):
        return self.p == len(self.b)


def hi1(x):
    return int(x).bit_length()


class IntVec:
    def __init__(self, words, n, width):
        self.words, self.n, self.width = words, n, width

    def bits(self):
        return np.unpackbits(self.words.view(np.uint8), bitorder="little")[:self.n * self.width]

    def values(self):
        if self.width == 64:
            return [int(x) for x in self.words[:self.n]]
        b = self.bits().reshape(self.n, self.width).astype(object)
        return [int(sum(int(v) << j for j, v in enumerate(row))) for row in b]


def pack(values, width):
    if width == 0 or width > 64:
        width = 64
    nbits = len(values) * width
    out = [0] * ((nbits + 63) // 64)
    for i, v in enumerate(values):
        v &= (1 << width) - 1
        pos = i * width
        out[pos >> 6] |= (v << (pos & 63)) & ((1 << 64) - 1)
        if (pos & 63) + width > 64:
            out[(pos >> 6) + 1] |= v >> (64 - (pos & 63))
    return out


def _popcounts(bits):
    nw = (len(bits) + 63) // 64
    padded = np.zeros(nw * 64, dtype=np.uint8)
    padded[:len(bits)] = bits
    return padded.reshape(nw, 64).sum(axis=1).astype(np.int64)


def rank_v(bits):
    """rank_support_v<1>: per 8 words (512 bits) the count before, and the counts before words 1..7
    of the block in 9-bit fields from bit 54 down."""
    if len(bits) == 0:
        return [0, 0]
    pc = _popcounts(bits)
    nw = len(pc)
    out = [0] * (((64 * nw >> 9) + 1) * 2)
    cum = 0
    for blk in range(0, nw, 8):
        out[2 * (blk // 8)] = cum
        second, s = 0, 0
        for j in range(1, 8):
            s += int(pc[blk + j - 1]) if blk + j - 1 < nw else 0
            if blk + j <= nw:  # counts recorded up to the end of the vector
                second |= s << (63 - 9 * j)
        out[2 * (blk // 8) + 1] = second
        cum += int(pc[blk:blk + 8].sum())
    if nw % 8 == 0:
        out[2 * (nw // 8)] = cum
        out[2 * (nw // 8) + 1] = 0
    return out


def rank_v5(bits):
    """rank_support_v5<1>: per 32 words the count before, and the counts before its 6-word blocks
    1..5 in 12-bit fields at 48, 36, .., 0."""
    if len(bits) == 0:
        return [0, 0]
    pc = _popcounts(bits)
    nw = len(pc)
    out = [0] * (((64 * nw >> 11) + 1) * 2)
    cum = 0
    for sb in range(0, nw, 32):
        out[2 * (sb // 32)] = cum
        second = 0
        for b in range(1, 6):
            if sb + 6 * b <= nw:
                second |= int(pc[sb:sb + 6 * b].sum()) << (60 - 12 * b)
        out[2 * (sb // 32) + 1] = second
        cum += int(pc[sb:sb + 32].sum())
    if nw % 32 == 0:
        out[2 * (nw // 32)] = cum
        out[2 * (nw // 32) + 1] = 0
    return out


def check_select_mcl(r, bits, b):
    """select_support_mcl<b>: parse and compare with the structure derived from the bits."""
    pos = np.flatnonzero(bits == b)
    args = r.raw("<Q")
    assert args == len(pos), (args, len(pos))
    if not args:
        return
    n = len(bits)
    logn = hi1(n if n else 1)
    logn4 = logn ** 4
    sb = (args + 4095) // 4096
    sup = r.int_vector()
    assert sup.width == logn and sup.n == sb
    assert sup.values() == [int(pos[4096 * s]) for s in range(sb)]
    flags = r.int_vector(1)
    longs = []
    for s in range(sb):
        p = pos[4096 * s:4096 * (s + 1)]
        longs.append(int(p[-1] - p[0]) > logn4)
    if any(longs):
        assert flags.n == sb and list(flags.bits()) == [int(not x) for x in longs]
    else:
        assert flags.n == 0
    for s in range(sb):
        p = [int(x) for x in pos[4096 * s:4096 * (s + 1)]]
        blk = r.int_vector()
        if longs[s]:
            assert blk.n == 4096 and blk.width == (hi1(p[-1]) or 64)
            assert blk.values() == p + [0] * (4096 - len(p))
        else:
            assert blk.n == 64 and blk.width == (hi1(p[-1] - p[0]) or 64)
            want = [p[j] - p[0] for j in range(0, len(p), 64)]
            assert blk.values() == want + [0] * (64 - len(want))


def bits_of(iv):
    return iv.bits()


def check_bit_vector_stat(r):
    bv = r.int_vector(1)
    bits = bits_of(bv)
    assert int(bv.words.sum() if False else 0) == 0 or True
    assert r.be() == int(bits.sum())
    rk = r.int_vector(64)
    assert rk.values() == rank_v5(bits)
    check_select_mcl(r, bits, 1)
    return bits


def huffman_tree(freq):
    """huff_shape + byte_tree, written from the description: a min-heap of (freq, id), leaves in
    symbol order; nodes numbered breadth first; child[0] = the first popped."""
    temp = []
    heap = []
    for s in range(256):
        if freq[s]:
            heapq.heappush(heap, (freq[s], len(temp)))
            temp.append({"freq": freq[s], "sym": s, "kids": None})
    while len(heap) > 1:
        f1, a = heapq.heappop(heap)
        f2, b = heapq.heappop(heap)
        heapq.heappush(heap, (f1 + f2, len(temp)))
        temp.append({"freq": f1 + f2, "sym": None, "kids": (a, b)})
    order = [len(temp) - 1]
    nodes = []
    i = 0
    while i < len(order):
        t = temp[order[i]]
        node = {"t": t, "children": None}
        if t["kids"]:
            node["children"] = (len(order), len(order) + 1)
            order.extend(t["kids"])
        nodes.append(node)
        i += 1
    parent = [0xFFFF] * len(nodes)
    for v, nd in enumerate(nodes):
        if nd["children"]:
            for c in nd["children"]:
                parent[c] = v
    return nodes, parent


def check_wt_huff(r, W):
    n = r.raw("<Q")
    assert n == len(W)
    sigma = r.raw("<Q")
    freq = np.bincount(np.asarray(W, dtype=np.int64), minlength=256)
    assert sigma == int((freq > 0).sum())
    nodes, parent = huffman_tree(freq)
    # codes: path from the root, bit d = branch at depth d
    code = {}
    for v, nd in enumerate(nodes):
        if not nd["children"]:
            w, l, u = 0, 0, v
            while u != 0:
                p = parent[u]
                w = (w << 1) | int(nodes[p]["children"][1] == u)
                l += 1
                u = p
            code[nd["t"]["sym"]] = (w, l)
    bv_pos, total = [], 0
    for nd in nodes:
        bv_pos.append(total)
        if nd["children"]:
            total += nd["t"]["freq"]
    seqs = {v: [] for v, nd in enumerate(nodes) if nd["children"]}
    for c in W:
        w, l = code[int(c)]
        v = 0
        for d in range(l):
            b = (w >> d) & 1
            seqs[v].append(b)
            v = nodes[v]["children"][b]
    want_bits = np.zeros(total, dtype=np.uint8)
    for v, s in seqs.items():
        want_bits[bv_pos[v]:bv_pos[v] + len(s)] = s
    bv = r.int_vector(1)
    bits = bits_of(bv)
    assert bv.n == total and np.array_equal(bits, want_bits)
    assert r.int_vector(64).values() == rank_v(bits)
    check_select_mcl(r, bits, 1)
    check_select_mcl(r, bits, 0)
    assert r.raw("<Q") == len(nodes)
    for v, nd in enumerate(nodes):
        pos, rank, par, c0, c1 = r.raw("<QQHHH")
        assert pos == bv_pos[v] and par == parent[v], (v, pos, bv_pos[v], par, parent[v])
        if nd["children"]:
            assert (c0, c1) == nd["children"] and rank == int(bits[:pos].sum())
        else:
            assert (c0, c1) == (0xFFFF, 0xFFFF) and rank == nd["t"]["sym"]
    leaf = [r.raw("<H") for _ in range(256)]
    path = [r.raw("<Q") for _ in range(256)]
    for s in range(256):
        if s in code:
            v = [i for i, nd in enumerate(nodes) if not nd["children"] and nd["t"]["sym"] == s][0]
            assert leaf[s] == v and path[s] == (code[s][0] | code[s][1] << 56)
        else:
            assert leaf[s] == 0xFFFF and path[s] == 0


def check_sd_vector(r, setpos, size):
    assert r.raw("<Q") == size
    wl = r.raw("<B")
    m = len(setpos)
    logm, logn = hi1(m), hi1(size)
    if logm == logn:
        logm -= 1
    assert wl == logn - logm
    low = r.int_vector()
    assert low.n == m and low.width == (wl or 64)
    assert low.values() == [int(p) & ((1 << low.width) - 1) for p in setpos]
    high = r.int_vector(1)
    want = np.zeros(m + (1 << logm), dtype=np.uint8)
    for j, p in enumerate(setpos):
        want[(int(p) >> wl) + j] = 1
    hb = bits_of(high)
    assert np.array_equal(hb, want)
    check_select_mcl(r, hb, 1)
    check_select_mcl(r, hb, 0)


def bin_to_nr(block, n=63):
    k = bin(block).count("1")
    if block == 0 or block == (1 << n) - 1:
        return 0
    nr, nn = 0, n
    while block:
        if block & 1:
            nr += math.comb(nn - 1, k)
            k -= 1
        block >>= 1
        nn -= 1
    return nr


def check_rrr_vector(r, bits):
    size = len(bits)
    assert r.raw("<Q") == size
    nblocks = (size + 63) // 63
    blocks = []
    for i in range(nblocks):
        seg = bits[63 * i:63 * i + 63]
        blocks.append(int(sum(int(b) << j for j, b in enumerate(seg))))
    bt = [bin(x).count("1") for x in blocks]
    space = [0 if math.comb(63, k) <= 1 else (math.comb(63, k) - 1).bit_length() for k in range(64)]
    nsuper = (nblocks + 31) // 32
    inv = [0] * nsuper
    for s in range(nsuper):
        i = 32 * s
        if 63 * i + 63 <= size and i + 32 <= nblocks:
            inv[s] = int(sum(1 for j in range(i, i + 32) if bt[j] > 31) > 16)
    stored = [63 - bt[i] if inv[i // 32] else bt[i] for i in range(nblocks)]
    btv = r.int_vector()
    assert btv.width == 6 and btv.values() == stored
    total_space = sum(space[bt[i]] for i in range(nblocks) if 63 * i < size)
    btnr = r.int_vector(1)
    assert btnr.n == max(total_space, 64)
    nb_bits = bits_of(btnr)
    p = 0
    ptrs, ranks, s_rank = [], [], 0
    for i in range(nblocks):
        if 63 * i >= size:
            break
        if i % 32 == 0:
            ptrs.append(p)
            ranks.append(s_rank)
        sp = space[bt[i]]
        got = int(sum(int(b) << j for j, b in enumerate(nb_bits[p:p + sp])))
        assert got == (bin_to_nr(blocks[i]) if sp else 0), i
        p += sp
        s_rank += bt[i]
    btnrp = r.int_vector()
    assert btnrp.width == (hi1(total_space) or 64)
    assert btnrp.values() == ptrs + [0] * (btnrp.n - len(ptrs)) and btnrp.n == nsuper
    rk = r.int_vector()
    want_n = nsuper + int(size % (32 * 63) > 0)
    assert rk.n == want_n and rk.width == (hi1(s_rank) or 64)
    want = ranks + [0] * (want_n - len(ranks))
    want[-1] = s_rank
    assert rk.values() == want
    iv = r.int_vector(1)
    assert list(bits_of(iv)) == inv


def check_bit_vector_small(r, bits):
    tag = r.be()
    if tag == 1:  # SD_VECTOR
        ones = int(bits.sum())
        inverted = ones > len(bits) // 2
        setpos = np.flatnonzero(bits == (0 if inverted else 1))
        check_sd_vector(r, setpos, len(bits))
        assert r.raw("<B") == int(inverted)
    else:
        assert tag == 0, tag  # RRR_VECTOR
        check_rrr_vector(r, bits)
    return tag


def check_dbg(path, W, last_bits):
    """The whole .dbg: F, k, state, W (wt_huff + logsigma), last (bit_vector_stat), mode, index."""
    r = Reader(open(path, "rb").read())
    assert r.be() == 5
    F = [r.be() for _ in range(5)]
    k, state = r.be(), r.be()
    check_wt_huff(r, W)
    assert r.be() == 4
    got_last = check_bit_vector_stat(r)
    assert np.array_equal(got_last, last_bits)
    mode = r.be()
    L = r.be()
    r.words(2 * 4 ** L if L else 0)
    assert r.done()
    return F, k, state, mode, L
