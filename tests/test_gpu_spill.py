"""The spilled build (f3, the disk container of `metagraph build --disk-swap`): when not even the real
edges fit memory_preallocated, build_chunk keeps one key range's edges in HBM at a time and the
rest in host memory or in files under swap_dir (boss_pipeline.hip: run_pipeline_spill; the
reference's SortedSetDisk + construct_boss_chunk_disk, boss_chunk_construct.cpp:664-933).  The
chunk must equal the oracle's bit for bit, with budgets far below the real-edge set."""
import importlib
import os

import numpy as np
import pytest

import oracle_ctypes as O
from test_gpu_parity import _random_reads, assert_same
from test_oracle_goldens import CONSTRUCT_SEQS

boss = importlib.import_module("projects2014-metagenome_amd.boss")

pytestmark = pytest.mark.gpu


def _spilled(k, seqs, canonical, bits, counts=None, swap_dir="/tmp/", disk_cap=0, budget=1e5):
    ctor = boss.IBOSSChunkConstructor.initialize(k, both_strands=canonical, bits_per_count=bits,
                                                 memory_preallocated=budget,
                                                 container_type=boss.CONTAINER_VECTOR_DISK,
                                                 swap_dir=swap_dir, disk_cap_bytes=disk_cap)
    if counts is None:
        ctor.add_sequences(seqs)
    else:
        ctor.add_sequences(list(zip(seqs, counts)))
    got = ctor.build_chunk()
    return got, ctor.timings()


@pytest.mark.parametrize("k,canonical,bits", [(30, True, 8), (31, False, 0), (20, True, 0), (45, True, 16),
                                              (63, False, 8), (5, True, 8), (12, False, 4)])
def test_spill_random_reads(k, canonical, bits):
    reads = _random_reads(300 + k, 4000, 150, 40000, n_rate=0.002, lower=True)
    got, t = _spilled(k, reads, canonical, bits)
    assert t.spilled_bytes > 0 and t.n_batches >= 2
    # the budget is far below the real edges alone
    assert t.n_real * 8 > 4 * 1e5 or k < 10
    assert_same(got, O.build_chunk(k, reads, canonical=canonical, bits_per_count=bits),
                "spill k=%d canonical=%s bits=%d" % (k, canonical, bits))


def test_spill_transcripts_goldens(transcripts_1000):
    for canonical, nodes in ((False, 591997), (True, 1159851)):
        got, t = _spilled(19, transcripts_1000, canonical, 8, budget=1e6)
        assert t.spilled_bytes > 0 and got.n_real == nodes and nodes * 8 > 4 * 1e6
        assert_same(got, O.build_chunk(19, transcripts_1000, canonical=canonical, bits_per_count=8), "transcripts")


def test_spill_files_under_swap_dir(tmp_path):
    # with a disk cap the blocks go to files under swap_dir (removed after the build), up to the cap
    reads = _random_reads(41, 3000, 150, 30000)
    got, t = _spilled(30, reads, True, 8, swap_dir=str(tmp_path), disk_cap=10**9)
    assert t.spilled_bytes > 0
    assert os.listdir(tmp_path) == []
    assert_same(got, O.build_chunk(30, reads, canonical=True, bits_per_count=8), "swap files")
    # a cap below the spill: the rest stays in RAM, same chunk
    got2, t2 = _spilled(30, reads, True, 8, swap_dir=str(tmp_path), disk_cap=100000)
    assert t2.spilled_bytes == t.spilled_bytes
    assert np.array_equal(got2.W, got.W) and np.array_equal(got2.last, got.last)


def test_spill_counts_saturate_and_degenerate(monkeypatch):
    rng = np.random.default_rng(5)
    seqs = _random_reads(7, 500, 60, 600)
    counts = rng.integers(1, 300, size=len(seqs)).tolist()
    for bits in (4, 8, 16):
        got, _ = _spilled(11, seqs, bits != 8, bits, counts, budget=2e4)
        assert_same(got, O.build_chunk(11, seqs, canonical=bits != 8, bits_per_count=bits, counts=counts),
                    "spill counts bits=%d" % bits)
    # forced on tiny inputs: empty ranges, a single read, the test strings of the reference
    monkeypatch.setenv("MTG_SPILL", "1")
    monkeypatch.setenv("MTG_RANGES", "7")
    for k, seqs in ((30, ["ACGT" * 10]), (5, CONSTRUCT_SEQS), (8, CONSTRUCT_SEQS)):
        for canonical in (False, True):
            ctor = boss.IBOSSChunkConstructor.initialize(k, both_strands=canonical, bits_per_count=8)
            ctor.add_sequences(seqs)
            got = ctor.build_chunk()
            assert ctor.timings().spilled_bytes > 0
            assert_same(got, O.build_chunk(k, seqs, canonical=canonical, bits_per_count=8), "forced k=%d" % k)


def test_spill_not_for_device_builds():
    # the device entry keeps its arrays in HBM: it never spills
    reads = _random_reads(3, 500, 150, 5000)
    data = b"".join(r + b"$" for r in reads)
    L = boss.lib()
    d = L.mtg_device_alloc(0, len(data))
    try:
        assert L.mtg_memcpy_h2d(d, data, len(data)) == 0
        ctor = boss.IBOSSChunkConstructor.initialize(30, both_strands=True, memory_preallocated=1e5,
                                                     container_type=boss.CONTAINER_VECTOR_DISK)
        dc = ctor.build_device(d, len(data))
        assert ctor.timings().spilled_bytes == 0 and dc.n > 1
    finally:
        L.mtg_device_free(d)
