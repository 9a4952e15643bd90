"""The graph files of `metagraph build` (the .dbg writer), on CPU: libmtg_boss.so's
host writer/reader (csrc/dbg_io.hpp) on chunks built by the oracle.

Pinned here: the round trip of every BOSS array, the suffix-range index against its definition
(boss.cpp:3091-3161 via tighten_range: the co-lex range of the nodes ending with each suffix),
the valid-edge mask of --mask-dummy against its definition (neither a dummy sink nor a $-prefixed
source, dbg_succinct.cpp:839-870), and `nodes (k)` after masking against the reference's
integration goldens (integration_tests/test_build.py:42-130: 591997 / 1159851).  The bytes of the
sdsl containers inside the files are restated, not pinned (no sdsl-lite, no golden .dbg file)."""
import importlib
import itertools
import os

import numpy as np
import pytest

import oracle_ctypes as O
from oracle import boss_definition as D
from test_oracle_goldens import CONSTRUCT_SEQS

boss = importlib.import_module("projects2014-metagenome_amd.boss")


def _chunk(k, seqs, canonical=False, bits=0):
    c = O.build_chunk(k, seqs, canonical=canonical, bits_per_count=bits)
    return boss.Chunk(k, np.asarray(c.W, np.uint8), np.asarray(c.last, np.uint8),
                      np.asarray(c.F, np.uint64), None if c.weights is None else np.asarray(c.weights),
                      n_real=c.n_real, bits_per_count=bits)


def _expected_ranges(k, rows, L):
    # rows: the definition builder's sorted row strings (node + label); BOSS row = index + 1
    code = {"A": 1, "C": 2, "G": 3, "T": 4}
    n = len(rows) + 1
    out = [(n, 0)] * (4 ** L)
    for i, r in enumerate(rows):
        suf = r[:k][k - L:]
        if "$" in suf:
            continue
        idx = sum((code[ch] - 1) * 4 ** j for j, ch in enumerate(suf))
        lo, hi = out[idx]
        out[idx] = (min(lo, i + 1), max(hi, i + 1))
    for i in range(1, len(out)):  # boss.cpp:3153-3159
        if not out[i][1]:
            out[i] = (out[i - 1][1] + 1, out[i - 1][1])
    return np.array(out, dtype=np.uint64)


@pytest.mark.parametrize("k", [1, 2, 3, 5, 8, 12, 20])
@pytest.mark.parametrize("canonical", [False, True])
def test_roundtrip_index_and_mask_match_definition(tmp_path, k, canonical):
    ch = _chunk(k, CONSTRUCT_SEQS, canonical, 8)
    ref = D.boss_table(k, CONSTRUCT_SEQS, canonical, 8)
    assert list(ch.W) == ref["W"]  # the oracle chunk is the definition's table
    base = str(tmp_path / "g")
    nv = ch.write_dbg(base, canonical=canonical, mask_dummy=True)
    f = boss.DbgFile(base)
    assert f.k == k and f.state == 3 and f.mode == int(canonical)
    assert np.array_equal(f.W, ch.W) and np.array_equal(f.last, ch.last)
    assert np.array_equal(f.F, ch.F)
    L = min(10, k)
    assert f.suffix_length == L
    assert np.array_equal(f.ranges, _expected_ranges(k, ref["rows"], L))
    valid = np.array([0] + [int(r[k] != "$" and r[0] != "$") for r in ref["rows"]], np.uint8)
    assert np.array_equal(f.valid, valid)
    assert nv == f.n_valid == valid.sum() == ref["n_real"]
    assert os.path.getsize(base + ".dbg.weights") > 0


def test_random_reads_index_and_mask(tmp_path):
    rng = np.random.default_rng(3)
    genome = "".join(rng.choice(list("ACGT"), size=3000))
    reads = []
    for _ in range(200):
        s = int(rng.integers(0, 2900))
        reads.append(genome[s:s + 100])
    for k, L in ((6, -1), (15, 4), (15, 0), (31, 7)):
        ch = _chunk(k, reads, True)
        ref = D.boss_table(k, reads, True)
        base = str(tmp_path / ("r%d_%d" % (k, L)))
        nv = ch.write_dbg(base, canonical=True, mask_dummy=True, suffix_length=L)
        f = boss.DbgFile(base)
        LL = min(10, k) if L < 0 else L
        assert f.suffix_length == LL
        if LL:
            assert np.array_equal(f.ranges, _expected_ranges(k, ref["rows"], LL))
        assert nv == ref["n_real"]
        assert not os.path.exists(base + ".dbg.weights")


@pytest.mark.parametrize("canonical,nodes", [(False, 591997), (True, 1159851)])
def test_nodes_after_mask_dummy_match_goldens(tmp_path, transcripts_1000, canonical, nodes):
    # `metagraph build --mask-dummy -k 20` then `stats`: nodes (k)
    ch = _chunk(19, transcripts_1000, canonical, 8)
    base = str(tmp_path / "t")
    assert ch.write_dbg(base, canonical=canonical, mask_dummy=True) == nodes
    f = boss.DbgFile(base)
    assert f.n_valid == nodes and int(f.valid.sum()) == nodes
    assert np.array_equal(f.W, ch.W) and np.array_equal(f.last, ch.last)


def test_weights_file_is_the_int_vector_of_the_chunk(tmp_path):
    ch = _chunk(5, CONSTRUCT_SEQS, False, 12)
    base = str(tmp_path / "w")
    ch.write_dbg(base)
    raw = open(base + ".dbg.weights", "rb").read()
    nbits = int(np.frombuffer(raw[:8], "<u8")[0])
    assert nbits == 12 * len(ch.W) and raw[8] == 12
    words = np.frombuffer(raw[9:], "<u8")
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:nbits].reshape(-1, 12)
    vals = (bits.astype(np.uint64) << np.arange(12, dtype=np.uint64)).sum(axis=1)
    assert np.array_equal(vals, np.asarray(ch.weights, np.uint64))


def test_corrupt_file_raises(tmp_path):
    ch = _chunk(4, CONSTRUCT_SEQS)
    base = str(tmp_path / "c")
    ch.write_dbg(base)
    data = open(base + ".dbg", "rb").read()
    open(base + ".dbg", "wb").write(data[:len(data) // 2])
    with pytest.raises(RuntimeError):
        boss.DbgFile(base)


@pytest.mark.gpu
@pytest.mark.parametrize("canonical,nodes", [(False, 591997), (True, 1159851)])
def test_gpu_chunk_to_dbg_goldens(tmp_path, transcripts_1000, canonical, nodes):
    ctor = boss.IBOSSChunkConstructor.initialize(19, both_strands=canonical, bits_per_count=8)
    ctor.add_sequences(transcripts_1000)
    ch = ctor.build_chunk()
    base = str(tmp_path / "g")
    assert ch.write_dbg(base, canonical=canonical, mask_dummy=True) == nodes
    want = _chunk(19, transcripts_1000, canonical, 8)
    f = boss.DbgFile(base)
    assert np.array_equal(f.W, want.W) and np.array_equal(f.last, want.last)
    assert np.array_equal(f.F, want.F) and f.n_valid == nodes


# ---- the sdsl-lite layout, checked field by field by an independent reader (tests/sdsl_layout.py)

import ctypes  # noqa: E402

import sdsl_layout as S  # noqa: E402


def _write(tmp_path, kind, data, nbits, name):
    path = str(tmp_path / name)
    buf = np.ascontiguousarray(data)
    rc = boss.lib().mtg_sdsl_write(os.fsencode(path), kind, buf.ctypes.data_as(ctypes.c_void_p), nbits)
    assert rc == 0, boss.lib().mtg_last_error()
    return open(path, "rb").read()


def _packed(bits):
    words = np.zeros((len(bits) + 63) // 64 + 1, np.uint64)
    if len(bits):
        pb = np.packbits(np.asarray(bits, np.uint8), bitorder="little")
        words.view(np.uint8)[:len(pb)] = pb
    return words


def _bit_cases():
    rng = np.random.default_rng(5)
    yield "one", np.array([1], np.uint8)
    yield "zero", np.array([0], np.uint8)
    for n in (63, 64, 65, 126, 511, 512, 513, 2047, 2048, 2049, 2016, 4032, 6000, 64 * 32 * 3):
        yield "dense%d" % n, (rng.random(n) < 0.6).astype(np.uint8)
    yield "words8", (rng.random(512 * 5) < 0.5).astype(np.uint8)
    yield "mostly_ones", (rng.random(200000) < 0.97).astype(np.uint8)
    yield "mostly_zeros", (rng.random(200000) < 0.02).astype(np.uint8)
    sparse = np.zeros(3_000_000, np.uint8)  # superblocks of 4096 ones spanning > logn^4 bits (long form)
    sparse[rng.choice(3_000_000, 9000, replace=False)] = 1
    yield "long_superblocks", sparse
    mixed = np.zeros(400000, np.uint8)  # one dense superblock, then sparse ones
    mixed[:5000] = 1
    mixed[rng.choice(np.arange(5000, 400000), 5000, replace=False)] = 1
    yield "mixed", mixed
    yield "all_ones_2016", np.ones(2016, np.uint8)


@pytest.mark.parametrize("name,bits", list(_bit_cases()))
def test_sdsl_bit_containers_layout(tmp_path, name, bits):
    words = _packed(bits)
    n = len(bits)
    r = S.Reader(_write(tmp_path, 0, words, n, name + ".stat"))
    assert np.array_equal(S.check_bit_vector_stat(r), bits) and r.done()
    r = S.Reader(_write(tmp_path, 3, words, n, name + ".sd"))
    S.check_sd_vector(r, np.flatnonzero(bits), n)
    assert r.done()
    r = S.Reader(_write(tmp_path, 4, words, n, name + ".rrr"))
    S.check_rrr_vector(r, bits)
    assert r.done()
    r = S.Reader(_write(tmp_path, 1, words, n, name + ".small"))
    S.check_bit_vector_small(r, bits)
    assert r.done()


@pytest.mark.parametrize("case", ["one_symbol", "two", "skewed", "boss_like", "all_256", "ties"])
def test_sdsl_wt_huff_layout(tmp_path, case):
    rng = np.random.default_rng(9)
    if case == "one_symbol":
        W = np.zeros(1, np.uint8)
    elif case == "two":
        W = np.array([0, 3, 3, 0, 3], np.uint8)
    elif case == "skewed":
        W = rng.choice(10, size=50000, p=[.01, .2, .3, .2, .19, .02, .02, .02, .02, .02]).astype(np.uint8)
    elif case == "boss_like":
        W = rng.integers(0, 10, size=100003).astype(np.uint8)
    elif case == "all_256":
        W = rng.integers(0, 256, size=70000).astype(np.uint8)
    else:  # equal frequencies everywhere: the heap's (frequency, id) tie rule decides the shape
        W = np.repeat(np.arange(7, dtype=np.uint8), 64)
        rng.shuffle(W)
    r = S.Reader(_write(tmp_path, 2, W, len(W), case + ".wt"))
    S.check_wt_huff(r, W)
    assert r.done()


@pytest.mark.parametrize("k,canonical", [(3, False), (12, True), (19, False), (19, True)])
def test_dbg_file_layout(tmp_path, transcripts_1000, k, canonical):
    # the whole .dbg and .edgemask of real graphs, field by field
    seqs = transcripts_1000 if k == 19 else CONSTRUCT_SEQS
    ch = _chunk(k, seqs, canonical, 8)
    base = str(tmp_path / "g")
    ch.write_dbg(base, canonical=canonical, mask_dummy=True)
    last = np.asarray(ch.last, np.uint8)
    F, kk, state, mode, L = S.check_dbg(base + ".dbg", np.asarray(ch.W, np.uint8), last)
    assert list(F) == [int(x) for x in ch.F] and kk == k and state == 3 and mode == int(canonical)
    f = boss.DbgFile(base)
    r = S.Reader(open(base + ".edgemask", "rb").read())
    S.check_bit_vector_small(r, np.asarray(f.valid, np.uint8))
    assert r.done()
