"""The suffix-filtered route on the MI355X: suffix_extract_kernel + LSD sort of
the lifted keys + emit, through the C ABI, bit for bit against the oracle's restatement
(oracle_build_suffix_chunk, itself pinned to the definition in test_suffix_route.py).  The chunks
of all suffixes, concatenated and pruned (`concatenate --clear-dummy`), reach the reference's
integration goldens."""
import importlib
import random

import numpy as np
import pytest

import oracle_ctypes as O
from test_oracle_goldens import CONSTRUCT_SEQS

boss = importlib.import_module("projects2014-metagenome_amd.boss")

pytestmark = pytest.mark.gpu


def gpu_suffix_chunk(k, seqs, suffix, both=False, bits=0, counts=None):
    ctor = boss.IBOSSChunkConstructor.initialize(k, both_strands=both, bits_per_count=bits, filter_suffix=suffix)
    if counts is None:
        ctor.add_sequences(seqs)
    else:
        ctor.add_sequences(list(zip(seqs, counts)))
    return ctor.build_chunk()


def same(got, want, ctx):
    assert len(got.W) == len(want.W), ctx
    assert np.array_equal(got.W, want.W), ctx
    assert np.array_equal(got.last, want.last), ctx
    assert np.array_equal(got.F, want.F), ctx
    if want.weights is None:
        assert got.weights is None, ctx
    else:
        assert np.array_equal(got.weights, want.weights), ctx


def check(k, seqs, suffix, both=False, bits=0, counts=None):
    got = gpu_suffix_chunk(k, seqs, suffix, both, bits, counts)
    want = O.build_suffix_chunk(k, seqs, suffix, both, bits, counts)
    same(got, want, "k=%d suffix=%r both=%s bits=%d" % (k, suffix, both, bits))
    return got


def random_reads(seed, n, lo, hi, alphabet="ACGTACGTACGTACGTNacgu"):
    rng = random.Random(seed)
    return ["".join(rng.choice(alphabet) for _ in range(rng.randint(lo, hi))) for _ in range(n)]


@pytest.mark.parametrize("both", [False, True])
@pytest.mark.parametrize("bits", [0, 8])
def test_construct_seqs_every_k(both, bits):
    for k in range(1, 85):
        for suf in boss.generate_suffixes(1):
            check(k, CONSTRUCT_SEQS, suf, both, bits)
        if k >= 2:
            for suf in ("$$", "$A", "CA", "TT"):
                check(k, CONSTRUCT_SEQS, suf, both, bits)


def test_random_reads_counts_and_saturation():
    seqs = random_reads(5, 3000, 1, 400)
    counts = [1 + (i * 7919) % 70000 for i in range(len(seqs))]
    for k, bits in ((5, 8), (31, 16), (42, 32), (63, 8)):
        for suf in ("$", "G", "$T", "AC"):
            check(k, seqs, suf, True, bits, counts)
            check(k, seqs, suf, False, bits, counts)


def test_many_tiles_both_strands():
    # ~3.6 M positions: thousands of extraction tiles, tile-edge segments, deep LSD sorts
    seqs = random_reads(9, 24000, 100, 200, "ACGT" * 30 + "N")
    for suf in boss.generate_suffixes(2)[:6]:
        check(31, seqs, suf, True, 0)


@pytest.mark.parametrize("both,nodes", [(False, 591997), (True, 1159851)])
def test_transcripts_suffix_chunks_concatenate_to_goldens(tmp_path, transcripts_1000, both, nodes):
    chunks = [gpu_suffix_chunk(19, transcripts_1000, suf, both) for suf in boss.generate_suffixes(2)]
    cat = boss.concatenate(chunks)
    want = [O.build_suffix_chunk(19, transcripts_1000, suf, both) for suf in boss.generate_suffixes(2)]
    assert np.array_equal(cat.W, np.concatenate([want[0].W] + [w.W[1:] for w in want[1:]]))
    assert np.array_equal(cat.last, np.concatenate([want[0].last] + [w.last[1:] for w in want[1:]]))
    assert cat.write_dbg(str(tmp_path / "g"), canonical=both, mask_dummy=True, prune=True) == nodes


def test_suffix_route_has_no_multi_gpu_form():
    comms = boss.Comm.local_group(1)
    ctor = boss.IBOSSChunkConstructor.initialize(10, filter_suffix="A")
    ctor.add_sequences(CONSTRUCT_SEQS)
    with pytest.raises(RuntimeError, match="no multi-GPU form"):
        ctor.build_chunk(comm=comms[0])
