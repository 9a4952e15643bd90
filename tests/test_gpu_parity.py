"""Parity of the MI355X path (through the C ABI) with the CPU restatement (oracle/).

Bit-exact on every BOSS array: W, last, F and weights, over the reference's own test inputs
(test_boss_construct.cpp sequences for every k in [1, 84], transcripts_1000.fa goldens) and
seeded random reads that exercise invalid characters, read boundaries, per-read counts,
counter saturation and every key-width boundary (2-bit 64/128 and lifted 64/128/256 bits).
"""
import importlib

import numpy as np
import pytest

import oracle_ctypes as O
from test_oracle_goldens import CONSTRUCT_SEQS

boss = importlib.import_module("projects2014-metagenome_amd.boss")

pytestmark = pytest.mark.gpu


def gpu_chunk(k, seqs, canonical=False, bits=0, counts=None):
    ctor = boss.IBOSSChunkConstructor.initialize(k, both_strands=canonical, bits_per_count=bits)
    if counts is None:
        ctor.add_sequences(seqs)
    else:
        ctor.add_sequences(list(zip(seqs, counts)))
    return ctor.build_chunk()


def assert_same(got, want, ctx=""):
    assert len(got.W) == len(want.W), ctx
    assert np.array_equal(got.W, want.W), ctx
    assert np.array_equal(got.last, want.last), ctx
    assert np.array_equal(got.F, want.F), ctx
    if want.weights is None:
        assert got.weights is None, ctx
    else:
        assert np.array_equal(got.weights, want.weights), ctx
    assert got.n_real == want.n_real, ctx


def check(k, seqs, canonical=False, bits=0, counts=None):
    got = gpu_chunk(k, seqs, canonical, bits, counts)
    want = O.build_chunk(k, seqs, canonical=canonical, bits_per_count=bits, counts=counts)
    assert_same(got, want, "k=%d canonical=%s bits=%d" % (k, canonical, bits))
    return got


@pytest.mark.parametrize("canonical", [False, True])
@pytest.mark.parametrize("bits", [0, 8])
def test_construct_seqs_every_k(canonical, bits):
    # ConstructionEQAppending / ...Canonical / DummyKmersZeroWeight inputs, k in [1, 84]
    for k in range(1, 85):
        check(k, CONSTRUCT_SEQS, canonical, bits)


@pytest.mark.parametrize("canonical,nodes", [(False, 591997), (True, 1159851)])
def test_transcripts_k20(transcripts_1000, canonical, nodes):
    got = check(19, transcripts_1000, canonical, 8)
    assert got.n_real == nodes
    w = got.weights[1:].astype(np.float64)
    avg = "{:.6g}".format(w[w > 0].mean())
    assert avg == ("2.53761" if canonical else "2.48587")


@pytest.mark.parametrize("k", [1, 3, 11, 30, 31, 32, 40, 41, 42, 63, 64, 84])
def test_transcripts_key_widths(transcripts_1000, k):
    check(k, transcripts_1000[:200], canonical=(k % 2 == 0), bits=16)


@pytest.mark.parametrize("width", [2, 3, 6, 8, 12, 16, 32])
def test_transcripts_k4_count_width(transcripts_1000, width):
    got = check(3, transcripts_1000, False, width)
    assert got.n_real == 256


def _random_reads(seed, n, length, genome_len, n_rate=0.0, lower=False):
    rng = np.random.default_rng(seed)
    genome = rng.integers(0, 4, size=genome_len, dtype=np.uint8)
    alpha = np.frombuffer(b"ACGT", dtype=np.uint8)
    reads = []
    for _ in range(n):
        s = int(rng.integers(0, genome_len - length))
        r = alpha[genome[s:s + length]].copy()
        if rng.random() < 0.5:
            r = np.frombuffer(bytes(r)[::-1], dtype=np.uint8).copy()
            r = np.array([{65: 84, 67: 71, 71: 67, 84: 65}[x] for x in r], dtype=np.uint8)
        if n_rate:
            m = rng.random(length) < n_rate
            r[m] = ord("N")
        if lower:
            r[rng.random(length) < 0.3] |= 0x20
        reads.append(bytes(r))
    return reads


@pytest.mark.parametrize("k", [2, 15, 20, 30, 31, 32, 45, 63, 64, 70])
@pytest.mark.parametrize("canonical", [False, True])
def test_random_reads_with_invalid_chars(k, canonical):
    reads = _random_reads(k, 300, 150, 3000, n_rate=0.01, lower=True)
    check(k, reads, canonical, bits=8 if k % 2 else 0)


def test_per_read_counts_and_saturation():
    rng = np.random.default_rng(5)
    seqs = _random_reads(9, 500, 12, 200)
    counts = rng.integers(1, 400, size=len(seqs)).tolist()
    for bits in (4, 8, 16, 32):
        for canonical in (False, True):
            check(11, seqs, canonical, bits, counts)
    counts = [2**32 - 5] * len(seqs)
    check(11, seqs, True, 32, counts)


def test_empty_and_degenerate_inputs():
    for k in (1, 5, 31, 40):
        check(k, [], False, 0)
        check(k, ["A" * k], True, 8)
        check(k, ["N" * 100, "$" * 50, "."], False, 8)
        check(k, ["A" * 100], False, 8)
        check(k, ["ACGT" * 50, "acgu" * 50], True, 8)


def test_cg_repeat_large_counts():
    for k, width in ((3, 32), (28, 32), (34, 16), (69, 32)):
        got = check(k, [b"CG" * 10**6], False, width)
        assert got.n_real == 2


def test_large_multi_tile():
    # enough k-mers for hundreds of sort tiles and look-back chains
    reads = _random_reads(77, 30000, 150, 400000, n_rate=0.0005)
    for canonical in (False, True):
        check(30, reads, canonical, bits=8)
        check(30, reads, canonical, bits=0)


def test_fused_extract_small_inputs(monkeypatch):
    # K1 fused with the first partition level on inputs it would skip by size, u64 k >= 7
    monkeypatch.setenv("MTG_FUSED_MIN", "0")
    reads = _random_reads(41, 2000, 150, 30000, n_rate=0.002, lower=True)
    for k in range(6, 32):
        check(k, reads, canonical=k % 2 == 1, bits=8 if k % 3 else 0)


def test_device_build_matches_host_build():
    reads = _random_reads(3, 1000, 150, 20000)
    k = 30
    data = b"".join(r + b"$" for r in reads)
    L = boss.lib()
    d = L.mtg_device_alloc(0, len(data))
    try:
        assert L.mtg_memcpy_h2d(d, data, len(data)) == 0
        ctor = boss.IBOSSChunkConstructor.initialize(k, both_strands=True)
        dc = ctor.build_device(d, len(data))
        W = np.empty(dc.n, dtype=np.uint8)
        last = np.empty(dc.n, dtype=np.uint8)
        L.mtg_memcpy_d2h(W.ctypes.data, dc.W, dc.n)
        L.mtg_memcpy_d2h(last.ctypes.data, dc.last, dc.n)
        want = O.build_chunk(k, reads, canonical=True)
        assert np.array_equal(W, want.W) and np.array_equal(last, want.last)
        assert list(dc.F) == list(want.F)
        t = ctor.timings()
        assert t.n_rows == dc.n and t.total_ms > 0
    finally:
        L.mtg_device_free(d)


def test_trim_keeps_device_chunk_and_next_build():
    # mtg_boss_ctor_trim frees the idle workspace blocks and the stage buffers but keeps the device
    # chunk arrays (W, last, weights) valid; a second build on the same constructor is exact again
    reads = _random_reads(5, 3000, 150, 40000, n_rate=0.001)
    k = 30
    data = b"".join(r + b"$" for r in reads)
    L = boss.lib()
    d = L.mtg_device_alloc(0, len(data))
    try:
        assert L.mtg_memcpy_h2d(d, data, len(data)) == 0
        want = O.build_chunk(k, reads, canonical=True, bits_per_count=8)
        ctor = boss.IBOSSChunkConstructor.initialize(k, both_strands=True, bits_per_count=8)
        for rep in range(2):
            dc = ctor.build_device(d, len(data))
            ctor.trim()
            assert ctor.timings().cached_bytes == 0
            W = np.empty(dc.n, dtype=np.uint8)
            last = np.empty(dc.n, dtype=np.uint8)
            wt = np.empty(dc.n, dtype=np.uint32)
            L.mtg_memcpy_d2h(W.ctypes.data, dc.W, dc.n)
            L.mtg_memcpy_d2h(last.ctypes.data, dc.last, dc.n)
            L.mtg_memcpy_d2h(wt.ctypes.data, dc.weights, dc.n * 4)
            assert np.array_equal(W, want.W) and np.array_equal(last, want.last), rep
            assert np.array_equal(wt, want.weights), rep
            assert list(dc.F) == list(want.F), rep
    finally:
        L.mtg_device_free(d)


@pytest.mark.parametrize("env", [{"MTG_EMIT": "slow"}, {"MTG_SORT": "lsd"}, {"MTG_FUSED_MIN": "0"}, {"MTG_DUMMY_SORT": "lifted"},
                                 {"MTG_FUSED": "0"}, {"MTG_FUSED_EMIT": "0"}, {"MTG_DUMMY_BITMAP": "1"},
                                 {"MTG_RC_FUSE": "0"}])
def test_alternate_device_paths(transcripts_1000, monkeypatch, env):
    # the unfused merge + emit, the compacting emit kernel, the unfused K1 and the LSD sorts
    # stay bit-exact too
    for key, val in env.items():
        monkeypatch.setenv(key, val)
    for k, canonical, bits in [(19, True, 8), (30, False, 0), (40, True, 16), (3, False, 8)]:
        check(k, transcripts_1000[:400], canonical, bits)
    check(5, CONSTRUCT_SEQS, True, 8)


def test_chunk_files_roundtrip(tmp_path, transcripts_1000):
    # the device-built chunk through <base>.dbg.chunk{,.W,.last,.weights} and back
    # (BOSS::Chunk::serialize / load, boss_chunk.cpp:330-386)
    for k, canonical, bits in [(19, True, 8), (30, False, 0)]:
        got = gpu_chunk(k, transcripts_1000[:300], canonical, bits)
        name = got.serialize(str(tmp_path / ("g%d" % k)))
        back = boss.Chunk.load(name)
        want = O.build_chunk(k, transcripts_1000[:300], canonical=canonical, bits_per_count=bits)
        assert back.k == k and back.bits_per_count == bits
        assert np.array_equal(back.W, want.W) and np.array_equal(back.last, want.last)
        assert list(back.F) == list(want.F)
        assert (back.weights is None) if not bits else np.array_equal(back.weights, want.weights)


def test_concurrent_adds_and_stage_growth():
    # host_stage.hpp: many adder threads at once (each batch reserves a 32-char-aligned range,
    # packs 2-bit codes + the valid mask, DMAs its pieces to the device mirror), many small
    # batches (the pinned buffers and the mirror grow under in-flight copies), single reads with
    # counts, reads of every length mod 32 with N / lowercase / U, all in one build
    import threading
    rng = np.random.default_rng(77)
    batches = []
    for b in range(48):
        n = int(rng.integers(1, 300))
        lens = rng.integers(0, 460, size=n)  # ~1.7 M chars: the 1 M-char first buffer grows
        reads = []
        for L in lens:
            r = rng.choice(np.frombuffer(b"ACGTacgtUuNn", dtype=np.uint8), size=int(L),
                           p=[0.22, 0.22, 0.22, 0.22, 0.02, 0.02, 0.02, 0.02, 0.01, 0.01, 0.01, 0.01])
            reads.append(r.tobytes())
        counts = rng.integers(1, 70, size=n).tolist()
        batches.append((reads, counts))
    for canonical, bits in ((True, 8), (False, 0)):
        ctor = boss.IBOSSChunkConstructor.initialize(20, both_strands=canonical, bits_per_count=bits,
                                                     num_threads=4)

        def worker(j):
            for b in range(j, len(batches), 6):
                reads, counts = batches[b]
                if b % 3 == 0:
                    ctor.add_sequences(list(zip(reads, counts)) if bits else reads)
                elif b % 3 == 1:
                    for r, c in zip(reads[:5], counts[:5]):
                        ctor.add_sequence(r, c if bits else 1)
                    ctor.add_sequences(list(zip(reads[5:], counts[5:])) if bits else reads[5:])
                else:
                    off = np.zeros(len(reads) + 1, dtype=np.uint64)
                    off[1:] = np.cumsum([len(r) for r in reads])
                    ctor.add_packed(b"".join(reads), off,
                                    np.array(counts, dtype=np.uint64) if bits else None)

        th = [threading.Thread(target=worker, args=(j,)) for j in range(6)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        got = ctor.build_chunk()
        seqs = [r for reads, _ in batches for r in reads]
        cnts = [c for _, counts in batches for c in counts] if bits else None
        want = O.build_chunk(20, seqs, canonical=canonical, bits_per_count=bits, counts=cnts)
        assert_same(got, want, "concurrent adds canonical=%s bits=%d" % (canonical, bits))
