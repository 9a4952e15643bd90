"""Canonical key rounds of the fused K1 (boss_pipeline.hip: collect_rounds_fused): a build too big
for one pass (BASELINE configs[3]'s per-GPU share) runs pass A of the fused extraction once and
collects the canonical k-mers in rounds of level-1 buckets of the whole input's MSD plan, then runs
the one-pass rc, dummy and emit stages on the whole canonical set -- the bounded-memory role of the
reference's disk container (boss_chunk_construct.cpp:664-933).  Bit-exact against the oracle
(oracle/, boss_chunk_construct.cpp:54-356 + boss_chunk.cpp:32-133) on the same reads."""
import importlib

import numpy as np
import pytest

import oracle_ctypes as O
import bench
from test_gpu_parity import _random_reads, assert_same

boss = importlib.import_module("projects2014-metagenome_amd.boss")

pytestmark = pytest.mark.gpu

ROUNDS = 2  # timings.collect_mode of collect_rounds_fused (1: key ranges re-scanning the reads)


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


@pytest.fixture
def small_fused(monkeypatch):
    # the fused K1 (and so the rounds) on inputs below its default 4 M-window threshold
    monkeypatch.setenv("MTG_FUSED_MIN", "0")
    return monkeypatch


@pytest.mark.parametrize("rounds", [2, 3, 7])
@pytest.mark.parametrize("k", [6, 11, 12, 20, 30, 31])
def test_rounds_random_reads(small_fused, rounds, k):
    # k = 11 / 31 (even K = k + 1): palindromes drop out of the rc set, doubling their counts
    small_fused.setenv("MTG_RANGES", str(rounds))
    reads = _random_reads(2000 + k, 400, 150, 5000, n_rate=0.005, lower=True)
    for canonical in (False, True):
        for bits in (0, 8):
            _, t = _check(k, reads, canonical, bits)
            assert t.collect_mode == ROUNDS and t.n_batches == rounds, (t.collect_mode, t.n_batches)


@pytest.mark.parametrize("k", [20, 31])
def test_rounds_pass_b_per_round_knob(small_fused, k):
    # two rounds of the u64 pass B run as one pass writing each round's buckets into its own buffer;
    # (the default; MTG_ROUNDS_ONE_B=1); 0: a pass B per round (the masked scan)
    small_fused.setenv("MTG_RANGES", "2")
    reads = _random_reads(3000 + k, 400, 150, 5000, n_rate=0.005, lower=True)
    for one_b in ("1", "0"):
        small_fused.setenv("MTG_ROUNDS_ONE_B", one_b)
        for canonical in (False, True):
            for bits in (0, 8):
                _, t = _check(k, reads, canonical, bits)
                assert t.collect_mode == ROUNDS and t.n_batches == 2, (t.collect_mode, t.n_batches)


@pytest.mark.parametrize("knob,value", [("MTG_ROUND_INDEX", "0"), ("MTG_ROUND_BITS", "0"), ("MTG_ROUNDS_ONE_B", "0"),
                                         ("MTG_SPEC_MID", "0"), ("MTG_SPEC_CAPS", "tiny")])
def test_rounds_2m_knobs_off(monkeypatch, knob, value):
    # the batched collect's defaults each switched off in turn on 1 M genome reads of 3 MSD levels in 2
    # rounds: the canonical set's bucket index written by the rounds' gathers (MTG_ROUND_INDEX), one final
    # bit fewer in a sparse round (MTG_ROUND_BITS), one pass B for both rounds (MTG_ROUNDS_ONE_B), the
    # speculative middle level (MTG_SPEC_MID); halved speculative capacities (MTG_SPEC_CAPS=tiny) make the
    # middle and final levels overflow and fall back to the exact ones
    monkeypatch.setenv("MTG_RANGES", "2")
    monkeypatch.setenv("MTG_MSD_LEVELS", "3")
    monkeypatch.setenv(knob, value)
    asc = bench.make_reads_host_codes(1_000_000, 150, 4242, "genome", 10.0)
    ctor = boss.IBOSSChunkConstructor.initialize(30, both_strands=True, num_threads=8)
    ctor.add_packed(asc.reshape(-1), np.arange(len(asc) + 1, dtype=np.uint64) * 150)
    got = ctor.build_chunk()
    t = ctor.timings()
    assert t.collect_mode == ROUNDS and t.n_batches == 2
    reads = [asc[i].tobytes() for i in range(len(asc))]
    assert_same(got, O.build_chunk(30, reads, canonical=True), "1M reads k=31, 2 rounds, %s=%s" % (knob, value))
    if knob == "MTG_SPEC_CAPS":
        assert t.spec_fallbacks > 0, t.spec_fallbacks


def test_rounds_counts_saturate(small_fused):
    small_fused.setenv("MTG_RANGES", "4")
    rng = np.random.default_rng(18)
    seqs = _random_reads(19, 300, 60, 2000)
    counts = rng.integers(1, 400, size=len(seqs)).tolist()
    for bits in (4, 8, 16, 32):
        for canonical in (False, True):
            _, t = _check(15, seqs, canonical, bits, counts)
            assert t.collect_mode == ROUNDS


def test_rounds_transcripts_goldens(small_fused, transcripts_1000):
    small_fused.setenv("MTG_RANGES", "5")
    for canonical, nodes in ((False, 591997), (True, 1159851)):
        got, t = _check(19, transcripts_1000, canonical, 8)
        assert got.n_real == nodes and t.collect_mode == ROUNDS and t.n_batches == 5


def test_rounds_memory_budget_plans(small_fused, transcripts_1000):
    # a 16 MB budget cannot hold the one-pass build of 1.5 M u64 windows: the build plans its rounds
    got, t = _check(30, transcripts_1000, True, 0, memory_preallocated=16e6)
    assert t.collect_mode == ROUNDS and t.n_batches >= 2, (t.collect_mode, t.n_batches)
    got2, t2 = _check(30, transcripts_1000, True, 0)
    assert t2.n_batches == 1 and t2.collect_mode == 0 and np.array_equal(got.W, got2.W)


def test_range_scan_knob(small_fused, transcripts_1000):
    # MTG_COLLECT=ranges keeps the key-range collect (both strands, re-scanned reads) for the same input
    small_fused.setenv("MTG_RANGES", "3")
    small_fused.setenv("MTG_COLLECT", "ranges")
    _, t = _check(30, transcripts_1000, True, 8)
    assert t.collect_mode == 1 and t.n_batches == 3


# 2 M genome-sampled reads at k = 31 (the bench generator): a 2-level plan whose speculative final
# level runs in every round, then the speculative rc level of the fused merge over the whole
# canonical set; basic mode and counts take the other branches
@pytest.mark.parametrize("canonical,bits", [(True, 0), (False, 0), (True, 8)])
def test_rounds_bench_generator_2m(monkeypatch, canonical, bits):
    monkeypatch.setenv("MTG_RANGES", "3")
    asc = bench.make_reads_host_codes(2_000_000, 150, 12345, "genome", 10.0)
    ctor = boss.IBOSSChunkConstructor.initialize(30, both_strands=canonical, bits_per_count=bits, num_threads=8)
    ctor.add_packed(asc.reshape(-1), np.arange(len(asc) + 1, dtype=np.uint64) * 150)
    got = ctor.build_chunk()
    t = ctor.timings()
    assert t.collect_mode == ROUNDS and t.n_batches == 3
    assert t.n_extracted == 2_000_000 * 120
    if not bits:
        assert t.spec_levels >= 3 and t.spec_fallbacks == 0, (t.spec_levels, t.spec_fallbacks)
    reads = [asc[i].tobytes() for i in range(len(asc))]
    want = O.build_chunk(30, reads, canonical=canonical, bits_per_count=bits)
    assert_same(got, want, "2M reads k=31 canonical=%s bits=%d, 3 rounds" % (canonical, bits))


# a 3-level plan in every round (configs[3]'s share plans 10 + 16 + 22 bits): forced on 2 M reads.  The
# speculative level 3 partitions into the rounds' level-1 array (c.spec_into) and its local unique writes
# over its own buckets; MTG_SPEC_INPLACE=0 gives it two buffers of its own, MTG_WS_CARVE=1 makes every
# workspace request a piece carved off a kept block where one holds it (the allocator's no-room path)
@pytest.mark.parametrize("spec3,knobs", [("0", {}), ("1", {}), ("1", {"MTG_WS_CARVE": "1"}),
                                         ("1", {"MTG_SPEC_INPLACE": "0"})])
@pytest.mark.parametrize("canonical", [False, True])
def test_rounds_three_msd_levels(monkeypatch, canonical, spec3, knobs):
    if knobs and not canonical:
        pytest.skip("the knob cases run on the canonical build")
    monkeypatch.setenv("MTG_RANGES", "3")
    monkeypatch.setenv("MTG_MSD_LEVELS", "3")
    monkeypatch.setenv("MTG_SPEC3", spec3)
    for name, v in knobs.items():
        monkeypatch.setenv(name, v)
    asc = bench.make_reads_host_codes(2_000_000, 150, 12345, "genome", 10.0)
    ctor = boss.IBOSSChunkConstructor.initialize(30, both_strands=canonical, num_threads=8)
    ctor.add_packed(asc.reshape(-1), np.arange(len(asc) + 1, dtype=np.uint64) * 150)
    got = ctor.build_chunk()
    t = ctor.timings()
    assert t.collect_mode == ROUNDS and t.n_batches == 3
    if spec3 == "1":  # every round's level 3 speculative, none fell back
        assert t.spec_levels >= 3 and t.spec_fallbacks == 0, (t.spec_levels, t.spec_fallbacks)
    reads = [asc[i].tobytes() for i in range(len(asc))]
    want = O.build_chunk(30, reads, canonical=canonical)
    assert_same(got, want, "2M reads k=31 canonical=%s, 3 rounds of 3 MSD levels, MTG_SPEC3=%s %s" %
                (canonical, spec3, knobs))
    if knobs:  # a second build on the same constructor: the kept (and carved) blocks handed out again
        ctor.add_packed(asc.reshape(-1), np.arange(len(asc) + 1, dtype=np.uint64) * 150)  # (a build consumes its reads)
        again = ctor.build_chunk()
        assert_same(again, want, "the same constructor's second build, %s" % knobs)


# configs[3]'s shape at a size the oracle finishes: 20 M genome-sampled reads (2.4e9 windows) under a
# memory_preallocated budget that the DEFAULT planner answers with rounds (no MTG_RANGES), the
# device path's arrays bit for bit against the oracle (~70 s of oracle time on the box's 16 threads)
@pytest.mark.timeout(900)
def test_rounds_20m_reads_memory_planned_vs_oracle():
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    n_reads, L = 20_000_000, 150
    seq = bench.make_reads_device(torch, n_reads, L, 1000, "genome", 10.0, dev)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    ctor = boss.IBOSSChunkConstructor.initialize(30, both_strands=True, memory_preallocated=3.5e10)
    dc = ctor.build_device(seq.data_ptr(), seq.numel())
    t = ctor.timings()
    assert t.collect_mode == ROUNDS and t.n_batches >= 2, (t.collect_mode, t.n_batches)
    assert t.n_extracted == n_reads * (L - 31 + 1)
    L_ = boss.lib()
    W = np.empty(dc.n, dtype=np.uint8)
    last = np.empty(dc.n, dtype=np.uint8)
    assert L_.mtg_memcpy_d2h(W.ctypes.data, dc.W, dc.n) == 0
    assert L_.mtg_memcpy_d2h(last.ctypes.data, dc.last, dc.n) == 0
    F = np.array([int(f) for f in dc.F], dtype=np.uint64)
    n_real = dc.n_real
    del ctor
    host = seq.cpu().numpy()
    del seq
    want = O.build_chunk_packed(30, host, np.arange(n_reads + 1, dtype=np.uint64) * (L + 1), canonical=True)
    assert len(W) == len(want.W)
    assert np.array_equal(W, want.W) and np.array_equal(last, want.last)
    assert np.array_equal(F, want.F) and n_real == want.n_real


# u128 windows (BOSS k 32..63, K = 33..64: BASELINE configs[2]'s k = 63 is BOSS k = 62): the wide pass A
# (extract_hist_wide_kernel), the generic pass B on u128 keys and the exact later MSD levels in every
# round, then the one-pass rc / dummy (dense u128 ranks) / emit stages; k = 62 takes the kernels with
# K = 63 compiled in, the others the runtime K
@pytest.mark.parametrize("rounds", [2, 5])
@pytest.mark.parametrize("k", [32, 33, 47, 62, 63])
def test_rounds_u128_random_reads(small_fused, rounds, k):
    small_fused.setenv("MTG_RANGES", str(rounds))
    reads = _random_reads(3000 + k, 300, 150, 6000, n_rate=0.005, lower=True)
    for canonical in (False, True):
        for bits in (0, 16):
            _, t = _check(k, reads, canonical, bits)
            assert t.collect_mode == ROUNDS and t.n_batches == rounds, (t.collect_mode, t.n_batches)


@pytest.mark.parametrize("k", [33, 62, 63])
def test_rounds_u128_pass_b_per_round_knob(small_fused, k):
    # configs[2]'s two u128 rounds share one packed-word pass B (extract_partition_fast2_kernel with per-bucket
    # destinations: round 1's buckets into KA2); MTG_ROUNDS_ONE_B=0: a pass B per round.  Counted builds take
    # the generic pass B, one per round
    small_fused.setenv("MTG_RANGES", "2")
    reads = _random_reads(7000 + k, 300, 150, 6000, n_rate=0.005, lower=True)
    for one_b in ("1", "0"):
        small_fused.setenv("MTG_ROUNDS_ONE_B", one_b)
        for canonical in (False, True):
            for bits in (0, 16):
                _, t = _check(k, reads, canonical, bits)
                assert t.collect_mode == ROUNDS and t.n_batches == 2, (t.collect_mode, t.n_batches)


@pytest.mark.parametrize("k", [32, 47, 62, 63])
def test_rounds_u128_generic_pass_b(small_fused, k):
    # MTG_FAST2=0: the uncounted u128 rounds' pass B as the generic extract_partition_kernel<2> (slide_windows)
    # instead of the packed-word extract_partition_fast2_kernel; the same chunk
    small_fused.setenv("MTG_RANGES", "3")
    small_fused.setenv("MTG_FAST2", "0")
    reads = _random_reads(5000 + k, 300, 150, 6000, n_rate=0.005, lower=True)
    for canonical in (False, True):
        _, t = _check(k, reads, canonical, 0)
        assert t.collect_mode == ROUNDS and t.n_batches == 3


def test_rounds_u128_counts_saturate(small_fused):
    small_fused.setenv("MTG_RANGES", "3")
    rng = np.random.default_rng(41)
    seqs = _random_reads(43, 300, 100, 3000)
    counts = rng.integers(1, 400, size=len(seqs)).tolist()
    for bits in (4, 8, 32):
        for canonical in (False, True):
            _, t = _check(40, seqs, canonical, bits, counts)
            assert t.collect_mode == ROUNDS


# configs[2]'s shape (k = 63, u128) at a size the oracle finishes: 10 M genome-sampled reads under a
# memory_preallocated budget that the DEFAULT planner answers with u128 rounds (no MTG_RANGES), bit for
# bit against the oracle
@pytest.mark.timeout(1200)
def test_rounds_u128_10m_reads_memory_planned_vs_oracle():
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    n_reads, L = 10_000_000, 150
    seq = bench.make_reads_device(torch, n_reads, L, 1000, "genome", 10.0, dev)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    ctor = boss.IBOSSChunkConstructor.initialize(62, both_strands=True, memory_preallocated=3.0e10)
    dc = ctor.build_device(seq.data_ptr(), seq.numel())
    t = ctor.timings()
    assert t.collect_mode == ROUNDS and t.n_batches >= 2, (t.collect_mode, t.n_batches)
    assert t.n_extracted == n_reads * (L - 63 + 1)
    L_ = boss.lib()
    W = np.empty(dc.n, dtype=np.uint8)
    last = np.empty(dc.n, dtype=np.uint8)
    assert L_.mtg_memcpy_d2h(W.ctypes.data, dc.W, dc.n) == 0
    assert L_.mtg_memcpy_d2h(last.ctypes.data, dc.last, dc.n) == 0
    F = np.array([int(f) for f in dc.F], dtype=np.uint64)
    n_real = dc.n_real
    del ctor
    host = seq.cpu().numpy()
    del seq
    want = O.build_chunk_packed(62, host, np.arange(n_reads + 1, dtype=np.uint64) * (L + 1), canonical=True)
    assert len(W) == len(want.W)
    assert np.array_equal(W, want.W) and np.array_equal(last, want.last)
    assert np.array_equal(F, want.F) and n_real == want.n_real
