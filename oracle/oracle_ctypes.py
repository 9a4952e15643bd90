"""TEST INFRASTRUCTURE ONLY -- ctypes view of oracle/liboracle_boss.so (the C restatement).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It is the checker, never the product path.  See oracle/boss_oracle.h for what is restated and
how parity is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_boss.so")


class OracleKeys(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("limbs", ctypes.c_uint32),
                ("words", ctypes.POINTER(ctypes.c_uint64)),
                ("counts", ctypes.POINTER(ctypes.c_uint32))]


class OracleChunk(ctypes.Structure):
    _fields_ = [("k", ctypes.c_uint64), ("n", ctypes.c_uint64),
                ("W", ctypes.POINTER(ctypes.c_uint8)),
                ("last", ctypes.POINTER(ctypes.c_uint8)),
                ("weights", ctypes.POINTER(ctypes.c_uint32)),
                ("F", ctypes.c_uint64 * 5),
                ("n_real", ctypes.c_uint64), ("n_dummy_sink", ctypes.c_uint64),
                ("n_dummy_source", ctypes.c_uint64)]


def build():
    """Compile the oracle with its own Makefile (gcc only)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        seq_args = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                    ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                    ctypes.c_uint64]
        for name in ("oracle_collect", "oracle_real_kmers", "oracle_dummy_kmers"):
            f = getattr(L, name)
            f.argtypes = seq_args + [ctypes.POINTER(OracleKeys)]
            f.restype = ctypes.c_int
        L.oracle_build_chunk.argtypes = seq_args + [ctypes.POINTER(OracleChunk)]
        L.oracle_build_chunk.restype = ctypes.c_int
        L.oracle_build_suffix_chunk.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_char_p] + seq_args[3:] + [ctypes.POINTER(OracleChunk)]
        L.oracle_build_suffix_chunk.restype = ctypes.c_int
        L.oracle_build_chunk_from_kmers.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                                    ctypes.POINTER(OracleKeys),
                                                    ctypes.POINTER(OracleChunk)]
        L.oracle_build_chunk_from_kmers.restype = ctypes.c_int
        L.oracle_pack_kmer.argtypes = [ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint64,
                                       ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_reverse_complement.argtypes = [ctypes.c_uint64, ctypes.c_uint32,
                                                ctypes.POINTER(ctypes.c_uint64),
                                                ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_keys_free.argtypes = [ctypes.POINTER(OracleKeys)]
        L.oracle_chunk_free.argtypes = [ctypes.POINTER(OracleChunk)]
        L.oracle_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


def pack_sequences(seqs):
    """list[str|bytes] -> (concatenated bytes, offsets uint64[n+1])."""
    bs = [s.encode() if isinstance(s, str) else bytes(s) for s in seqs]
    offsets = np.zeros(len(bs) + 1, dtype=np.uint64)
    if bs:
        offsets[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    return b"".join(bs), offsets


def _seq_call(fn, k, canonical, bits, seqs, counts, out):
    data, offsets = pack_sequences(seqs)
    cnt = None
    if counts is not None:
        cnt = np.ascontiguousarray(counts, dtype=np.uint64)
    rc = fn(k, int(canonical), int(bits), data,
            offsets.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
            cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)) if cnt is not None else None,
            len(seqs), ctypes.byref(out))
    if rc != 0:
        raise RuntimeError(lib().oracle_last_error().decode())


def _keys_to_numpy(keys):
    n, limbs = keys.n, keys.limbs
    words = np.ctypeslib.as_array(keys.words, shape=(max(n * limbs, 1),))[:n * limbs]
    words = words.reshape(n, limbs).copy()
    counts = None
    if keys.counts:
        counts = np.ctypeslib.as_array(keys.counts, shape=(max(n, 1),))[:n].copy()
    lib().oracle_keys_free(ctypes.byref(keys))
    return words, counts


def collect(k, seqs, canonical=False, bits_per_count=0, counts=None):
    """Sorted unique (k+1)-mers (2-bit KMerBOSS words) as KmerCollector::data() returns them."""
    out = OracleKeys()
    _seq_call(lib().oracle_collect, k, canonical, bits_per_count, seqs, counts, out)
    return _keys_to_numpy(out)


def real_kmers(k, seqs, canonical=False, bits_per_count=0, counts=None):
    out = OracleKeys()
    _seq_call(lib().oracle_real_kmers, k, canonical, bits_per_count, seqs, counts, out)
    return _keys_to_numpy(out)


def dummy_kmers(k, seqs, canonical=False, bits_per_count=0, counts=None):
    out = OracleKeys()
    _seq_call(lib().oracle_dummy_kmers, k, canonical, bits_per_count, seqs, counts, out)
    return _keys_to_numpy(out)[0]


class Chunk:
    """BOSS::Chunk arrays as initialize_chunk (boss_chunk.cpp:32-133) produces them."""

    def __init__(self, c):
        n = c.n
        self.k = c.k
        self.W = np.ctypeslib.as_array(c.W, shape=(n,)).copy()
        self.last = np.ctypeslib.as_array(c.last, shape=(n,)).copy()
        self.weights = (np.ctypeslib.as_array(c.weights, shape=(n,)).copy()
                        if c.weights else None)
        self.F = np.array(list(c.F), dtype=np.uint64)
        self.n_real = c.n_real
        self.n_dummy_sink = c.n_dummy_sink
        self.n_dummy_source = c.n_dummy_source
        lib().oracle_chunk_free(ctypes.byref(c))


def build_chunk(k, seqs, canonical=False, bits_per_count=0, counts=None):
    out = OracleChunk()
    _seq_call(lib().oracle_build_chunk, k, canonical, bits_per_count, seqs, counts, out)
    return Chunk(out)


def build_chunk_packed(k, data, offsets, canonical=False, bits_per_count=0, counts=None):
    """build_chunk on one packed buffer (uint8 array or bytes; sequence i = data[off[i]:off[i+1]]),
    for inputs too big for a list of Python strings (the bench-size parity checks)."""
    buf = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray))
                               else data, dtype=np.uint8)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    cnt = None if counts is None else np.ascontiguousarray(counts, dtype=np.uint64)
    out = OracleChunk()
    rc = lib().oracle_build_chunk(k, int(canonical), int(bits_per_count), buf.ctypes.data_as(ctypes.c_char_p),
                                  off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                  cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)) if cnt is not None else None,
                                  len(off) - 1, ctypes.byref(out))
    if rc != 0:
        raise RuntimeError(lib().oracle_last_error().decode())
    return Chunk(out)


def build_suffix_chunk(k, seqs, suffix, both_strands=False, bits_per_count=0, counts=None):
    """The suffix-filtered route (boss_chunk_construct.cpp:946-1013) for one filter suffix."""
    data, offsets = pack_sequences(seqs)
    cnt = None if counts is None else np.ascontiguousarray(counts, dtype=np.uint64)
    out = OracleChunk()
    rc = lib().oracle_build_suffix_chunk(
        k, int(bool(both_strands)), bits_per_count, suffix.encode(), data,
        offsets.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
        cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)) if cnt is not None else None,
        len(seqs), ctypes.byref(out))
    if rc != 0:
        raise RuntimeError(lib().oracle_last_error().decode())
    return Chunk(out)


def build_chunk_from_kmers(k, words, counts=None, canonical=False, bits_per_count=0):
    words = np.ascontiguousarray(words, dtype=np.uint64)
    if words.ndim == 1:
        words = words.reshape(-1, 1)
    keys = OracleKeys()
    keys.n = words.shape[0]
    keys.limbs = words.shape[1]
    keys.words = words.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    cnt = None
    if counts is not None:
        cnt = np.ascontiguousarray(counts, dtype=np.uint32)
        keys.counts = cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    out = OracleChunk()
    rc = lib().oracle_build_chunk_from_kmers(k, int(canonical), int(bits_per_count),
                                             ctypes.byref(keys), ctypes.byref(out))
    if rc != 0:
        raise RuntimeError(lib().oracle_last_error().decode())
    return Chunk(out)


def pack_kmer(codes, bits_per_char, limbs):
    arr = np.ascontiguousarray(codes, dtype=np.uint8)
    out = np.zeros(limbs, dtype=np.uint64)
    lib().oracle_pack_kmer(arr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), len(arr),
                           bits_per_char, limbs,
                           out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    return out


def reverse_complement(words, length):
    w = np.ascontiguousarray(words, dtype=np.uint64)
    out = np.zeros_like(w)
    lib().oracle_reverse_complement(length, len(w),
                                    w.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    return out
