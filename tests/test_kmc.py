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


# ---------------------------------------------------------------- the builder's KMC1 writer
#
# BASELINE config 5 builds from a KMC database of k = 31 counts.  KMC itself is not in the image,
# so the builder writes its own databases (mtg_kmc_write_device: GPU k-mer counting, KMC record
# order and header); kmc_oracle -- pinned on the reference's fixtures above -- reads them back.

def _device_reads(reads):
    data = b"".join((r if isinstance(r, bytes) else r.encode()) + b"$" for r in reads)
    L = boss.lib()
    d = L.mtg_device_alloc(0, max(len(data), 1))
    assert d
    assert L.mtg_memcpy_h2d(d, data, len(data)) == 0
    return d, len(data)


def _lex_counts(reads, k, canonical):
    c = collections.Counter()
    for s in reads:
        s = s if isinstance(s, bytes) else s.encode()
        s = s.upper().replace(b"U", b"T")
        for i in range(len(s) - k + 1):
            w = s[i:i + k]
            if w.strip(b"ACGT"):
                continue
            if canonical:
                w = min(w, w[::-1].translate(RC))
            c[w] += 1
    return c


def _write_db(tmp_path, reads, k, canonical, cs=1, name="db"):
    d, n = _device_reads(reads)
    try:
        ctor = boss.IBOSSChunkConstructor.initialize(max(k - 1, 1))
        base = str(tmp_path / name)
        total = ctor.write_kmc(d, n, base, k, canonical=canonical, counter_size=cs)
    finally:
        boss.lib().mtg_device_free(d)
    return base, total


@pytest.mark.gpu
@pytest.mark.parametrize("k,canonical,cs", [(31, True, 1), (31, False, 2), (11, True, 1), (32, True, 4),
                                            (15, False, 1), (3, True, 1)])
def test_kmc_writer_roundtrip(tmp_path, k, canonical, cs):
    from test_gpu_parity import _random_reads
    reads = _random_reads(40 + k, 3000, 150, 30000, n_rate=0.002, lower=True)
    reads += [b"ACGT" * 40, b"A" * 200]  # palindromes and a saturating count
    base, total = _write_db(tmp_path, reads, k, canonical, cs)
    want = _lex_counts(reads, k, canonical)
    h = kmc_oracle.read_header(base)
    assert (h["k"], h["counter_size"], h["total"], h["both_strands"]) == (k, cs, len(want), canonical)
    assert (h["k"] - h["lut_len"]) % 4 == 0
    got = kmc_oracle.read_kmers(base)
    cmax = (1 << (8 * cs)) - 1
    assert [w for w, _ in got] == sorted(want)  # KMC record order: lexicographic
    assert all(c == min(want[w], cmax) for w, c in got)


@pytest.mark.gpu
def test_kmc_writer_empty_and_short(tmp_path):
    base, total = _write_db(tmp_path, [b"ACGTN", b"NNNN"], 11, True)
    assert total == 0 and kmc_oracle.read_kmers(base) == []
    assert kmc_oracle.read_header(base)["total"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("canonical,bits", [(True, 8), (False, 16), (True, 0)])
def test_build_from_written_kmc_k31(tmp_path, canonical, bits):
    # configs[4]: k = 31 --count-kmers on a KMC database of the reads' canonical counts, through both
    # inputs: add_kmc (the file, decoded at build time) and the device-resident decode
    from test_gpu_parity import _random_reads
    reads = _random_reads(77, 6000, 150, 60000, n_rate=0.0005)
    base, total = _write_db(tmp_path, reads, 31, True)
    got = _gpu_kmc(30, base, canonical, bits)
    want = _oracle_kmc(30, base, canonical, bits)
    for a in ("W", "last", "F") + (("weights",) if bits else ()):
        assert np.array_equal(getattr(got, a), getattr(want, a)), a
    dr = boss.DeviceReads(base, call_both_from_canonical=not canonical)
    assert dr.n_reads == total * (1 if canonical else 2)
    ctor = boss.IBOSSChunkConstructor.initialize(30, both_strands=canonical, bits_per_count=bits)
    dc = ctor.build_device(*dr.build_args())
    L = boss.lib()
    W = np.empty(dc.n, dtype=np.uint8)
    L.mtg_memcpy_d2h(W.ctypes.data, dc.W, dc.n)
    assert np.array_equal(W, want.W) and list(dc.F) == list(want.F)
    if bits:
        wt = np.empty(dc.n, dtype=np.uint32)
        L.mtg_memcpy_d2h(wt.ctypes.data, dc.weights, dc.n * 4)
        assert np.array_equal(wt, want.weights)


@pytest.mark.gpu
@pytest.mark.parametrize("P,rounds", [(1, 0), (2, 0), (3, 0), (4, 0), (2, 3), (4, 5), (8, 0), (8, 3)])
def test_dist_build_from_kmc_k31(tmp_path, monkeypatch, P, rounds):
    # configs[4] across ranks: every rank counts its own reads into its own database; the ranks'
    # records meet at their owners, where the counts add with saturation (the count-aggregating
    # merge), and the concatenated rank chunks equal the oracle's build of all records
    import threading
    from test_gpu_parity import _random_reads
    if rounds:
        monkeypatch.setenv("MTG_RANGES", str(rounds))
    reads = _random_reads(91, 4000, 150, 20000, n_rate=0.0005)
    bases = [_write_db(tmp_path, reads[r::P], 31, True, name="r%d" % r)[0] for r in range(P)]
    for canonical, bits in ((True, 8), (False, 16)):
        comms = boss.Comm.local_group(P)
        ctors = [boss.IBOSSChunkConstructor.initialize(30, both_strands=canonical, bits_per_count=bits)
                 for _ in range(P)]
        for r in range(P):
            ctors[r].add_kmc(bases[r])
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
        got = boss.concatenate(out)
        recs = [rec for b in bases for rec in kmc_oracle.read_kmers(b, not canonical)]
        want = O.build_chunk(30, [s for s, _ in recs], canonical=canonical, bits_per_count=bits,
                             counts=[c for _, c in recs])
        for a in ("W", "last", "F", "weights"):
            assert np.array_equal(getattr(got, a), getattr(want, a)), (a, canonical, bits)
        if rounds:
            assert all(c.timings().n_batches == rounds for c in ctors)


# configs[4] at its full single-GPU size: the KMC1 database of the canonical k = 31 counts of 10 M
# genome-sampled reads (~1.9e8 records, written by the GPU counter), decoded into HBM, built with
# --count-kmers --count-width 8 and compared bit for bit (W, last, F, weights) with the oracle's build
# of every decoded record with its count (kmc_parser.cpp:27-62, sorted_multiset.cpp:54-84)
@pytest.mark.gpu
@pytest.mark.timeout(1200)
def test_config4_full_kmc_database_vs_oracle(tmp_path):
    torch = pytest.importorskip("torch")
    import bench
    dev = torch.device("cuda", 0)
    n_reads, L = 10_000_000, 150
    seq = bench.make_reads_device(torch, n_reads, L, 1000, "genome", 10.0, dev)
    torch.cuda.synchronize()
    base = str(tmp_path / "cfg5")
    ctor = boss.IBOSSChunkConstructor.initialize(30, both_strands=True, bits_per_count=8)
    total = ctor.write_kmc(seq.data_ptr(), seq.numel(), base, 31, canonical=True)
    del seq
    torch.cuda.empty_cache()
    assert total > 100_000_000, total
    dr = boss.DeviceReads(base)
    assert dr.n_reads == total
    dc = ctor.build_device(*dr.build_args())
    t = ctor.timings()
    assert t.n_extracted == total
    Lb = boss.lib()
    W = np.empty(dc.n, dtype=np.uint8)
    last = np.empty(dc.n, dtype=np.uint8)
    wt = np.empty(dc.n, dtype=np.uint32)
    assert Lb.mtg_memcpy_d2h(W.ctypes.data, dc.W, dc.n) == 0
    assert Lb.mtg_memcpy_d2h(last.ctypes.data, dc.last, dc.n) == 0
    assert Lb.mtg_memcpy_d2h(wt.ctypes.data, dc.weights, dc.n * 4) == 0
    F = np.array([int(f) for f in dc.F], dtype=np.uint64)
    n_real = dc.n_real
    n = dr.n_reads
    hseq = np.empty(dr.seq_len, dtype=np.uint8)
    starts = np.empty(n + 1, dtype=np.uint64)
    counts = np.empty(n, dtype=np.uint32)
    assert Lb.mtg_memcpy_d2h(hseq.ctypes.data, dr.seq, dr.seq_len) == 0
    assert Lb.mtg_memcpy_d2h(starts.ctypes.data, dr.read_starts, n * 8) == 0
    assert Lb.mtg_memcpy_d2h(counts.ctypes.data, dr.counts, n * 4) == 0
    starts[n] = dr.seq_len
    del dr, ctor
    # the decoded buffer is the database: record i is 31 chars + '$' at i * 32 with its count
    assert np.array_equal(starts[:n], np.arange(n, dtype=np.uint64) * 32)
    assert counts.min() >= 1
    want = O.build_chunk_packed(30, hseq, starts, canonical=True, bits_per_count=8, counts=counts)
    assert len(W) == len(want.W)
    assert np.array_equal(W, want.W) and np.array_equal(last, want.last)
    assert np.array_equal(F, want.F) and n_real == want.n_real
    assert np.array_equal(wt, want.weights)
