"""Parity of the multi-GPU build with the single-build oracle (through the C ABI).

P ranks run in one process on the one GPU of the box (include/mtg_boss.h: mtg_comm_create_local,
one host thread per rank, the same exchange steps as RCCL with device copies).  Every rank
builds from its own share of the reads; the rank chunks, concatenated in rank order with
BOSS::Chunk::extend (boss_chunk.cpp:230-270), must equal the oracle's chunk of ALL reads bit for
bit -- the range partition, the three exchanges (k-mers, sink / in-edge queries, dummy sources)
and the per-rank emission together reproduce the single build.
"""
import importlib
import threading

import numpy as np
import pytest

import oracle_ctypes as O
from test_gpu_parity import _random_reads, assert_same
from test_oracle_goldens import CONSTRUCT_SEQS

boss = importlib.import_module("projects2014-metagenome_amd.boss")

pytestmark = pytest.mark.gpu


def dist_chunks(k, shares, canonical=False, bits=0, counts=None, ctors_out=None, **kw):
    """Per-rank chunks of one build: shares[r] = the reads of rank r (kw: constructor options)."""
    P = len(shares)
    comms = boss.Comm.local_group(P)
    ctors = [boss.IBOSSChunkConstructor.initialize(k, both_strands=canonical, bits_per_count=bits, **kw)
             for _ in range(P)]
    if ctors_out is not None:
        ctors_out.extend(ctors)
    for r in range(P):
        if counts is None:
            if shares[r]:
                ctors[r].add_sequences(shares[r])
        elif shares[r]:
            ctors[r].add_sequences(list(zip(shares[r], counts[r])))
    out, errs = [None] * P, []

    def run(r):
        try:
            out[r] = ctors[r].build_chunk(comm=comms[r])
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append((r, e))

    ts = [threading.Thread(target=run, args=(r,)) for r in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not errs, errs
    assert all(c is not None for c in out)
    return out


def check_dist(k, seqs, P, canonical=False, bits=0, counts=None, split="round_robin", ctors_out=None, **kw):
    if split == "round_robin":
        shares = [seqs[r::P] for r in range(P)]
        cshares = None if counts is None else [counts[r::P] for r in range(P)]
    else:  # everything on the last rank: the others only own ranges
        shares = [[] for _ in range(P - 1)] + [list(seqs)]
        cshares = None if counts is None else [[] for _ in range(P - 1)] + [list(counts)]
    chunks = dist_chunks(k, shares, canonical, bits, cshares, ctors_out, **kw)
    got = boss.concatenate(chunks)
    want = O.build_chunk(k, seqs, canonical=canonical, bits_per_count=bits, counts=counts)
    assert_same(got, want, "k=%d P=%d canonical=%s bits=%d" % (k, P, canonical, bits))
    return chunks


@pytest.mark.parametrize("P", [1, 2, 3])
@pytest.mark.parametrize("canonical", [False, True])
def test_dist_construct_seqs_every_k(P, canonical):
    for k in range(1, 85):
        check_dist(k, CONSTRUCT_SEQS, P, canonical, bits=8 if k % 3 == 0 else 0)


@pytest.mark.parametrize("canonical,nodes", [(False, 591997), (True, 1159851)])
def test_dist_transcripts_k20(transcripts_1000, canonical, nodes):
    chunks = check_dist(19, transcripts_1000, 4, canonical, bits=8)
    assert sum(c.n_real for c in chunks) == nodes
    # the ranges are balanced: no rank owns more than twice its share of the real edges
    assert max(c.n_real for c in chunks) < 2 * nodes / 4


@pytest.mark.parametrize("k", [2, 15, 30, 31, 32, 45, 63, 64, 70])
def test_dist_random_reads(k):
    reads = _random_reads(100 + k, 400, 150, 4000, n_rate=0.01, lower=True)
    check_dist(k, reads, 3, canonical=k % 2 == 1, bits=8 if k % 2 else 0)
    check_dist(k, reads, 2, canonical=k % 2 == 0, bits=16)


def test_dist_counts_saturate_across_ranks():
    # the same k-mers on every rank: counts add across ranks and saturate at the owner
    rng = np.random.default_rng(11)
    seqs = _random_reads(9, 400, 12, 120)
    counts = rng.integers(1, 200, size=len(seqs)).tolist()
    for bits in (4, 8, 16):
        for canonical in (False, True):
            check_dist(11, seqs, 4, canonical, bits, counts)


def test_dist_superkmer_read_counts(monkeypatch):
    # exchange 0 carries every run's read count: per-read counts of k >= 19 builds go through it
    monkeypatch.setenv("MTG_DIST_COLLECT", "superkmer")
    rng = np.random.default_rng(12)
    seqs = _random_reads(13, 1500, 150, 9000, n_rate=0.003, lower=True)
    counts = rng.integers(1, 90, size=len(seqs)).tolist()
    for k, P, canonical, bits in ((25, 4, True, 8), (40, 3, False, 16), (19, 8, True, 4)):
        check_dist(k, seqs, P, canonical, bits, counts)


@pytest.mark.parametrize("env", [{"MTG_DIST_COLLECT": "superkmer"}, {"MTG_DIST_COLLECT": "local"},
                                 {"MTG_ROUTED_CANON": "min"}, {"MTG_DIST_SINKS": "query"},
                                 {"MTG_DIST_SINKS": "query", "MTG_DIST_COLLECT": "superkmer"}])
def test_dist_collect_modes(monkeypatch, env):
    # every collect of the multi-GPU build (MTG_DIST_COLLECT; the routed default with min(fwd, rc)
    # canonical keys instead of the hashed-top choice) is exact, and so is the sink join by routed
    # queries (MTG_DIST_SINKS=query) that the pulled edge slices replaced
    for name, v in env.items():
        monkeypatch.setenv(name, v)
    reads = _random_reads(21, 2000, 150, 20000, n_rate=0.005, lower=True)
    for k, P, canonical, bits in ((30, 3, True, 8), (31, 2, False, 0), (19, 4, True, 16)):
        check_dist(k, reads, P, canonical, bits)


def test_dist_empty_and_lopsided_ranks():
    reads = _random_reads(5, 300, 150, 3000)
    for P in (2, 5, 8):
        check_dist(30, reads, P, True, 8, split="last")
    check_dist(30, [], 3, True, 8)
    check_dist(5, ["ACGT" * 10], 4, False, 0)
    check_dist(1, CONSTRUCT_SEQS, 4, True, 8)


@pytest.mark.parametrize("sinks", ["pull", "query"])
def test_dist_large_multi_tile(monkeypatch, sinks):
    # (8, True) is configs[3]'s shape: canonical, BOSS k = 30 (k = 31), the default routed collect on 8
    # ranks; the default pulled sink join and the routed queries it replaced
    monkeypatch.setenv("MTG_DIST_SINKS", sinks)
    reads = _random_reads(77, 30000, 150, 400000, n_rate=0.0005)
    for P, canonical in ((2, True), (4, True), (8, False), (8, True)):
        check_dist(30, reads, P, canonical, bits=8)


def test_dist_timings_report_exchange():
    reads = _random_reads(3, 2000, 150, 20000)
    P = 2
    comms = boss.Comm.local_group(P)
    ctors = [boss.IBOSSChunkConstructor.initialize(30, both_strands=True) for _ in range(P)]
    for r in range(P):
        ctors[r].add_sequences(reads[r::P])
    ts = [threading.Thread(target=lambda r=r: ctors[r].build_chunk(comm=comms[r])) for r in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    for c in ctors:
        t = c.timings()
        assert t.world == P and t.exchange_ms > 0 and t.n_sent > 0


def test_dist_rccl_single_rank():
    # the RCCL communicator itself (a one-rank group on this box's one GPU)
    comm = boss.Comm.rccl(boss.Comm.unique_id(), 1, 0, 0)
    assert comm.rank == 0 and comm.size == 1
    reads = _random_reads(8, 500, 150, 5000)
    ctor = boss.IBOSSChunkConstructor.initialize(30, both_strands=True, bits_per_count=8)
    ctor.add_sequences(reads)
    got = ctor.build_chunk(comm=comm)
    assert_same(got, O.build_chunk(30, reads, canonical=True, bits_per_count=8), "rccl P=1")


# ------------------------------------------------------------ the batched (bounded-memory) collect
#
# A rank share too big for one pass (configs[3]: 125 M reads per GPU) is collected in rounds.  The
# default for u64 keys (BOSS k 6..31) is the routed collect's rounds: every owner's level-1 buckets
# cut into `rounds` sub-intervals, pass B of the fused K1 keeping one sub-interval of every owner per
# round (boss_pipeline.hip: dist_collect_routed), canonical k-mers only.  Otherwise -- and with
# MTG_COLLECT=ranges -- owner ranges on the top-char bins of the range kernels, each cut into `rounds`
# batches; per round every rank extracts both strands of every owner's batch, dedupes, and the
# owners merge the P runs (collect_ranges_dist).  MTG_RANGES forces the rounds on small inputs.

@pytest.mark.parametrize("collect", ["routed", "ranges"])
@pytest.mark.parametrize("P,rounds", [(1, 2), (2, 2), (2, 5), (3, 3), (4, 7)])
def test_dist_rounds_random_reads(monkeypatch, P, rounds, collect):
    monkeypatch.setenv("MTG_RANGES", str(rounds))
    if collect == "ranges":
        monkeypatch.setenv("MTG_COLLECT", "ranges")
    for k, canonical, bits in ((30, True, 8), (31, False, 0), (45, True, 16), (63, True, 0),
                               (70, False, 8), (4, True, 8), (5, False, 0), (7, True, 4), (6, True, 0)):
        reads = _random_reads(200 + k, 600, 150, 6000, n_rate=0.005, lower=True)
        ctors = []
        check_dist(k, reads, P, canonical, bits, ctors_out=ctors)
        # BOSS k >= 5: batched (bins of 4 node chars leave the k - 1 >= 4 chars of every emission
        # group on one rank); routed rounds for BOSS k 6..31 (collect_mode 2), else key ranges (1)
        want = rounds if k >= 5 else 1
        mode = 2 if collect == "routed" and 6 <= k <= 31 else 1 if k >= 5 else 0
        assert all(c.timings().n_batches == want for c in ctors), (k, [c.timings().n_batches for c in ctors])
        assert all(c.timings().collect_mode == mode for c in ctors), (k, [c.timings().collect_mode for c in ctors])


@pytest.mark.parametrize("canonical,nodes", [(False, 591997), (True, 1159851)])
def test_dist_rounds_transcripts_k20(monkeypatch, transcripts_1000, canonical, nodes):
    monkeypatch.setenv("MTG_RANGES", "6")
    chunks = check_dist(19, transcripts_1000, 4, canonical, bits=8)
    assert sum(c.n_real for c in chunks) == nodes


def test_dist_rounds_counts_saturate_and_lopsided(monkeypatch):
    monkeypatch.setenv("MTG_RANGES", "4")
    rng = np.random.default_rng(12)
    seqs = _random_reads(19, 400, 40, 200)
    counts = rng.integers(1, 200, size=len(seqs)).tolist()
    for bits in (4, 8, 16):
        check_dist(11, seqs, 3, bits % 8 == 0, bits, counts)
    reads = _random_reads(6, 300, 150, 3000)
    for P in (2, 5):
        check_dist(30, reads, P, True, 8, split="last")
    check_dist(30, [], 3, True, 8)
    check_dist(30, ["ACGT" * 10], 4, False, 0)
    check_dist(12, CONSTRUCT_SEQS, 3, True, 8)


def test_dist_rounds_planned_from_memory_budget():
    # no MTG_RANGES: a budget far below the single-pass footprint plans the rounds itself
    reads = _random_reads(31, 4000, 150, 40000, n_rate=0.001)
    ctors = []
    check_dist(30, reads, 2, True, 8, ctors_out=ctors, memory_preallocated=4e6)
    assert all(c.timings().n_batches >= 2 for c in ctors)
    ctors = []
    check_dist(30, reads[:200], 2, False, 0, ctors_out=ctors, container_type=boss.CONTAINER_VECTOR_DISK)
    assert all(c.timings().n_batches >= 2 for c in ctors)


@pytest.mark.parametrize("collect", ["routed", "ranges"])
def test_dist_rounds_large_multi_tile(monkeypatch, collect):
    # (8, True): configs[3]'s shape (canonical, k = 31, 8 ranks) in rounds
    monkeypatch.setenv("MTG_RANGES", "3")
    if collect == "ranges":
        monkeypatch.setenv("MTG_COLLECT", "ranges")
    reads = _random_reads(78, 30000, 150, 400000, n_rate=0.0005)
    for P, canonical in ((2, True), (4, False), (8, True)):
        check_dist(30, reads, P, canonical, bits=8)


@pytest.mark.parametrize("pieces", ["1", "2", "7"])
def test_dist_exchange_pieces(monkeypatch, pieces):
    # exchange 1 of the routed collect in pieces on the exchange stream, each piece sorted while the next
    # is in flight (routed_pieces; 4 by default, 1 = one exchange then the sort): exact for every count,
    # with counted keys, on lopsided ranks, and the overlap is reported
    monkeypatch.setenv("MTG_DIST_PIECES", pieces)
    reads = _random_reads(91, 20000, 150, 300000, n_rate=0.0005)
    for P, canonical, bits in ((2, True, 0), (3, True, 8), (5, False, 16)):
        ctors = []
        check_dist(30, reads, P, canonical, bits, ctors_out=ctors)
        for c in ctors:
            t = c.timings()
            assert t.exchange_ms > 0 and t.exchange_hidden_ms >= 0
            if pieces == "1":
                assert t.exchange_hidden_ms == 0
    check_dist(30, reads[:3000], 4, True, 8, split="last")


@pytest.mark.parametrize("pieces", ["1", "4"])
@pytest.mark.parametrize("rounds", ["2", "5"])
def test_dist_rounds_exchange_pipelined(monkeypatch, pieces, rounds):
    # the routed rounds with each round's exchange in flight under the next round's pass B and the
    # previous round's owner sort (routed_rounds_pipelined: alternating send / receive buffers ordered
    # by stream events), and the serial rounds (MTG_DIST_PIECES=1): both exact, counted and not
    monkeypatch.setenv("MTG_RANGES", rounds)
    monkeypatch.setenv("MTG_DIST_PIECES", pieces)
    reads = _random_reads(93, 12000, 150, 200000, n_rate=0.0005)
    for P, canonical, bits in ((2, True, 0), (3, True, 8), (4, False, 16)):
        ctors = []
        check_dist(30, reads, P, canonical, bits, ctors_out=ctors)
        for c in ctors:
            t = c.timings()
            assert t.n_batches == int(rounds) and t.collect_mode == 2
            assert t.exchange_ms > 0 and t.exchange_hidden_ms >= 0
            if pieces == "1":
                assert t.exchange_hidden_ms == 0
    check_dist(30, reads[:2000], 3, True, 8, split="last")
