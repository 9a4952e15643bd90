"""The range-batched build (the bounded-memory path of BASELINE configs[2]; the reference's disk
container, boss_chunk_construct.cpp:664-933): k-mers collected one key range at a time (both
strands in canonical mode), then the single-pass dummy and emit stages.  Bit-exact against the
oracle (oracle/, boss_chunk_construct.cpp:54-356 + boss_chunk.cpp:32-133) on the same reads."""
import importlib

import numpy as np
import pytest

import oracle_ctypes as O
from test_gpu_parity import _random_reads, assert_same
from test_oracle_goldens import CONSTRUCT_SEQS

boss = importlib.import_module("projects2014-metagenome_amd.boss")

pytestmark = pytest.mark.gpu


def _build(k, seqs, canonical, bits, counts=None, **kw):
    ctor = boss.IBOSSChunkConstructor.initialize(k, both_strands=canonical, bits_per_count=bits, **kw)
    if counts is None:
        ctor.add_sequences(seqs)
    else:
        ctor.add_sequences(list(zip(seqs, counts)))
    got = ctor.build_chunk()
    return got, ctor.timings()


def _check(k, seqs, canonical, bits, counts=None, **kw):
    got, t = _build(k, seqs, canonical, bits, counts, **kw)
    want = O.build_chunk(k, seqs, canonical=canonical, bits_per_count=bits, counts=counts)
    assert_same(got, want, "k=%d canonical=%s bits=%d" % (k, canonical, bits))
    return got, t


@pytest.mark.parametrize("ranges", [2, 3, 7])
@pytest.mark.parametrize("k", [4, 11, 20, 30, 31, 40, 62, 63])
def test_ranges_random_reads(monkeypatch, ranges, k):
    monkeypatch.setenv("MTG_RANGES", str(ranges))
    reads = _random_reads(1000 + k, 400, 150, 5000, n_rate=0.005, lower=True)
    for canonical in (False, True):
        _, t = _check(k, reads, canonical, 8 if k % 2 else 0)
        assert t.n_batches == ranges


@pytest.mark.parametrize("k", [1, 2, 5, 9, 13, 24])
def test_ranges_construct_seqs_palindromes(monkeypatch, k):
    # even DBG k (odd BOSS k here + 1) has palindromes: both-strand extraction doubles their counts
    monkeypatch.setenv("MTG_RANGES", "4")
    for canonical in (False, True):
        for bits in (0, 2, 8):
            _check(k, CONSTRUCT_SEQS, canonical, bits)
    _check(k + 1 if k % 2 == 0 else k, ["ACGT" * 40, "AATT" * 30, "GC" * 70], True, 3)


def test_ranges_counts_saturate(monkeypatch):
    monkeypatch.setenv("MTG_RANGES", "5")
    rng = np.random.default_rng(8)
    seqs = _random_reads(9, 500, 14, 200)
    counts = rng.integers(1, 400, size=len(seqs)).tolist()
    for bits in (4, 8, 16, 32):
        for canonical in (False, True):
            _check(11, seqs, canonical, bits, counts)


def test_ranges_transcripts_goldens(monkeypatch, transcripts_1000):
    monkeypatch.setenv("MTG_RANGES", "6")
    for canonical, nodes in ((False, 591997), (True, 1159851)):
        got, t = _check(19, transcripts_1000, canonical, 8)
        assert got.n_real == nodes and t.n_batches == 6


def test_memory_budget_plans_ranges(transcripts_1000):
    # a 16 MB budget cannot hold the single pass of 1.5 M u64 windows: the build batches itself
    got, t = _check(30, transcripts_1000, True, 0, memory_preallocated=16e6)
    assert t.n_batches >= 2
    got2, t2 = _check(30, transcripts_1000, True, 0)
    assert t2.n_batches == 1 and np.array_equal(got.W, got2.W)


def test_disk_container_is_the_batched_build(transcripts_1000):
    got, t = _check(62, transcripts_1000[:300], True, 8, container_type=boss.CONTAINER_VECTOR_DISK)
    assert t.n_batches >= 2


def test_ranges_k63_u256_dummies(monkeypatch):
    # k = 63 / 64: u128 2-bit keys, u256 lifted dummies
    monkeypatch.setenv("MTG_RANGES", "3")
    reads = _random_reads(63, 3000, 150, 60000, n_rate=0.001)
    for canonical in (False, True):
        _check(62, reads, canonical, 8)
        _check(63, reads, canonical, 0)


def test_ranges_empty_and_tiny(monkeypatch):
    monkeypatch.setenv("MTG_RANGES", "9")
    for k in (1, 5, 31, 40):
        _check(k, [], False, 0)
        _check(k, ["A" * k], True, 8)
        _check(k, ["N" * 100, "$" * 50, "."], False, 8)


def test_config2_default_planner_many_ranges(monkeypatch):
    # configs[2]'s shape (k = 63, u128 keys, genome-sampled 150 bp reads) at 2 M reads, with a
    # memory budget that makes the DEFAULT range planner (no MTG_RANGES) cut the collection into >= 8
    # key ranges; bit for bit vs the oracle.  (The default collect of such a build is the canonical
    # rounds of the fused extraction since round 5 -- test_gpu_rounds.py; MTG_COLLECT=ranges keeps
    # this path, which the disk container and the multi-GPU u128 build still take.)
    import bench
    monkeypatch.setenv("MTG_COLLECT", "ranges")
    asc = bench.make_reads_host_codes(2_000_000, 150, 4321, "genome", 10.0)
    data = asc.reshape(-1)
    off = np.arange(len(asc) + 1, dtype=np.uint64) * asc.shape[1]
    ctor = boss.IBOSSChunkConstructor.initialize(62, both_strands=True, num_threads=8, memory_preallocated=5e9)
    ctor.add_packed(data, off)
    got = ctor.build_chunk()
    t = ctor.timings()
    assert t.n_batches >= 8, t.n_batches
    assert t.n_extracted == len(asc) * (150 - 63 + 1)
    reads = [asc[i].tobytes() for i in range(len(asc))]
    want = O.build_chunk(62, reads, canonical=True, bits_per_count=0)
    assert_same(got, want, "configs[2] shape, %d ranges" % t.n_batches)
