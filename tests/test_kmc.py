"""KMC1 database input (BASELINE config 5): the decoder pinned by the reference's own fixtures,
and the device build from a database against the oracle and the reference's node counts
(integration_tests/test_build.py:176-268: nodes (k) 469983 / 802920 at k = 11)."""
import collections
import importlib
import os

import numpy as np
import pytest

import kmc_oracle
import oracle_ctypes as O
from conftest import GOLDEN

boss = importlib.import_module("projects2014-metagenome_amd.boss")

SINGLE = os.path.join(GOLDEN, "transcripts_1000_kmc_counters.kmc_suf")
BOTH = os.path.join(GOLDEN, "transcripts_1000_kmc_counters_both_strands.kmc_suf")
RC = bytes.maketrans(b"ACGT", b"TGCA")


def _fasta_kmers(seqs, k):
    c = collections.Counter()
    for s in seqs:
        for i in range(len(s) - k + 1):
            w = s[i:i + k]
            if not w.strip(b"ACGT"):
                c[w] += 1
    return c


def test_kmc_headers():
    h = kmc_oracle.read_header(SINGLE)
    assert (h["k"], h["lut_len"], h["counter_size"], h["total"]) == (11, 7, 1, 469983)
    assert not h["both_strands"]
    h = kmc_oracle.read_header(BOTH)
    assert (h["k"], h["total"], h["both_strands"]) == (11, 401460, True)


def test_kmc_decoder_matches_the_reads(transcripts_1000):
    # the fixture databases are KMC's 11-mer counts of transcripts_1000.fa (counter: 1 byte)
    seqs = [s if isinstance(s, bytes) else s.encode() for s in transcripts_1000]
    fwd = _fasta_kmers(seqs, 11)
    single = dict(kmc_oracle.read_kmers(SINGLE))
    assert single.keys() == fwd.keys()
    assert all(single[w] == min(n, 255) for w, n in fwd.items())
    canon = collections.Counter()
    for w, n in fwd.items():
        canon[min(w, w[::-1].translate(RC))] += n
    both = dict(kmc_oracle.read_kmers(BOTH))
    assert both.keys() == canon.keys()
    assert all(both[w] == min(n, 255) for w, n in canon.items())
    # call_both_from_canonical adds the reverse complements of a canonical database only
    assert len(kmc_oracle.read_kmers(BOTH, True)) == 2 * 401460
    assert len(kmc_oracle.read_kmers(SINGLE, True)) == 469983


def test_kmc_count_filter():
    recs = kmc_oracle.read_kmers(SINGLE)
    got = kmc_oracle.read_kmers(SINGLE, min_count=3, max_count=100)
    assert len(got) == sum(1 for _, c in recs if 3 <= c < 100)
    assert kmc_oracle.read_kmers(SINGLE, min_count=5, max_count=5) == []


@pytest.mark.gpu
def test_kmc_add_rejects_missing_database():
    ctor = boss.IBOSSChunkConstructor.initialize(10)
    with pytest.raises(RuntimeError, match="KMC"):
        ctor.add_kmc("/nonexistent/db.kmc_suf")


def _gpu_kmc(k, path, canonical, bits, **kw):
    ctor = boss.IBOSSChunkConstructor.initialize(k, both_strands=canonical, bits_per_count=bits)
    ctor.add_kmc(path, **kw)
    return ctor.build_chunk()


def _oracle_kmc(k, path, canonical, bits, call_both=None, **kw):
    if call_both is None:
        call_both = not canonical
    recs = kmc_oracle.read_kmers(path, call_both, **kw)
    return O.build_chunk(k, [s for s, _ in recs], canonical=canonical, bits_per_count=bits,
                         counts=[c for _, c in recs])


# test_build_weighted.py:155-273: --count-kmers (width 8) => nnz weights and avg weight
@pytest.mark.parametrize("path,canonical,nodes,avg", [(SINGLE, False, 469983, "3.15029"),
                                                      (BOTH, False, 802920, "3.68754"),
                                                      (SINGLE, True, 802920, "3.68754"),
                                                      (BOTH, True, 802920, "3.68754")])
def test_oracle_kmc_weighted_goldens(path, canonical, nodes, avg):
    c = _oracle_kmc(10, path, canonical, 8)
    assert c.n_real == nodes
    w = c.weights[1:].astype(np.float64)
    nz = w[w > 0]
    assert (len(nz), "{:.6g}".format(nz.mean())) == (nodes, avg)


@pytest.mark.gpu
@pytest.mark.parametrize("path,canonical,nodes", [(SINGLE, False, 469983), (BOTH, False, 802920),
                                                  (SINGLE, True, 802920), (BOTH, True, 802920)])
def test_build_from_kmc_goldens(path, canonical, nodes):
    # test_build_from_kmc / _both / _canonical / _both_canonical (test_build.py:176-268)
    got = _gpu_kmc(10, path, canonical, 8)
    assert got.n_real == nodes
    want = _oracle_kmc(10, path, canonical, 8)
    for a in ("W", "last", "F", "weights"):
        assert np.array_equal(getattr(got, a), getattr(want, a)), a


@pytest.mark.gpu
def test_build_from_kmc_other_k_and_filters():
    # k-mers of another length are sequences like any other (parse_sequences.hpp:82-87)
    for k, canonical, bits, kw in ((5, False, 16, {}), (14, True, 0, {}),
                                   (10, False, 8, dict(min_count=3, max_count=50))):
        got = _gpu_kmc(k, SINGLE, canonical, bits, **kw)
        want = _oracle_kmc(k, SINGLE, canonical, bits, **kw)
        assert np.array_equal(got.W, want.W) and np.array_equal(got.last, want.last)
        assert np.array_equal(got.F, want.F)
        if bits:
            assert np.array_equal(got.weights, want.weights)


@pytest.mark.gpu
def test_build_from_kmc_mixed_with_reads(transcripts_1000):
    ctor = boss.IBOSSChunkConstructor.initialize(10, both_strands=True, bits_per_count=8)
    reads = transcripts_1000[:50]
    ctor.add_sequences(reads)
    ctor.add_kmc(BOTH)
    got = ctor.build_chunk()
    recs = kmc_oracle.read_kmers(BOTH, False)
    want = O.build_chunk(10, list(reads) + [s for s, _ in recs], canonical=True, bits_per_count=8,
                         counts=[1] * len(reads) + [c for _, c in recs])
    assert np.array_equal(got.W, want.W) and np.array_equal(got.weights, want.weights)
