"""Host-side mirror of the reference's chunk-constructor interface over libmtg_boss.so.

Same names, argument meaning and error behaviour as
graph/representation/succinct/boss_chunk_construct.hpp:18-34 (IBOSSChunkConstructor) and
boss_chunk.hpp:19-104 (BOSS::Chunk), so tests read like the reference's own:

    ctor = IBOSSChunkConstructor.initialize(k, both_strands, bits_per_count)
    ctor.add_sequences(["ACGT...", ...])
    chunk = ctor.build_chunk()          # chunk.W, chunk.last, chunk.F, chunk.weights

The constructor runs entirely on the MI355X through the C ABI (include/mtg_boss.h).  There is
no CPU fallback: a missing library or device raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmtg_boss.so")

CONTAINER_VECTOR = 0
CONTAINER_VECTOR_DISK = 1


class _Params(ctypes.Structure):
    _fields_ = [("k", ctypes.c_uint64), ("both_strands", ctypes.c_int),
                ("bits_per_count", ctypes.c_uint8), ("filter_suffix", ctypes.c_char_p),
                ("num_threads", ctypes.c_uint64), ("memory_preallocated", ctypes.c_double),
                ("container_type", ctypes.c_int), ("swap_dir", ctypes.c_char_p),
                ("disk_cap_bytes", ctypes.c_uint64), ("device_id", ctypes.c_int)]


class _Chunk(ctypes.Structure):
    _fields_ = [("k", ctypes.c_uint64), ("alph_size", ctypes.c_uint64), ("n", ctypes.c_uint64),
                ("W", ctypes.POINTER(ctypes.c_uint8)), ("last", ctypes.POINTER(ctypes.c_uint64)),
                ("weights", ctypes.POINTER(ctypes.c_uint32)), ("F", ctypes.c_uint64 * 5),
                ("bits_per_count", ctypes.c_uint8), ("n_real", ctypes.c_uint64),
                ("n_dummy", ctypes.c_uint64)]


class _DeviceChunk(ctypes.Structure):
    _fields_ = [("k", ctypes.c_uint64), ("n", ctypes.c_uint64),
                ("W", ctypes.c_void_p), ("last", ctypes.c_void_p), ("weights", ctypes.c_void_p),
                ("F", ctypes.c_uint64 * 5), ("n_real", ctypes.c_uint64),
                ("n_dummy", ctypes.c_uint64)]


class _DeviceReads(ctypes.Structure):
    _fields_ = [("seq", ctypes.c_void_p), ("seq_len", ctypes.c_uint64), ("read_starts", ctypes.c_void_p),
                ("counts", ctypes.c_void_p), ("n_reads", ctypes.c_uint64), ("device_id", ctypes.c_int)]


_ALLREDUCE_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t)
_ALLGATHER_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                 ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t)
_ALLTOALLV_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                 ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64))


class _CommCallbacks(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("rank", ctypes.c_int), ("world", ctypes.c_int),
                ("allreduce_sum_u64", _ALLREDUCE_CB), ("allgather_u64", _ALLGATHER_CB),
                ("alltoallv", _ALLTOALLV_CB)]


class _DbgFile(ctypes.Structure):
    _fields_ = [(name, ctypes.c_uint64) for name in ("k", "n")] + \
               [("F", ctypes.c_uint64 * 5)] + \
               [(name, ctypes.c_uint64) for name in ("state", "mode", "suffix_length", "n_ranges")] + \
               [("W", ctypes.POINTER(ctypes.c_uint8)), ("last", ctypes.POINTER(ctypes.c_uint64)),
                ("ranges", ctypes.POINTER(ctypes.c_uint64)), ("valid", ctypes.POINTER(ctypes.c_uint64)),
                ("n_valid", ctypes.c_uint64)]


class Timings(ctypes.Structure):
    _fields_ = [(name, ctypes.c_double) for name in
                ("total_ms", "extract_ms", "sort_ms", "unique_ms", "rc_ms", "dummy_ms",
                 "merge_ms", "emit_ms", "radix_pass_ms", "radix_bytes")] + \
               [(name, ctypes.c_uint64) for name in
                ("radix_launches", "n_positions", "n_extracted", "n_unique", "n_real",
                 "n_dummy", "n_rows")] + \
               [("exchange_ms", ctypes.c_double), ("n_sent", ctypes.c_uint64),
                ("world", ctypes.c_uint64)] + \
               [(name, ctypes.c_double) for name in
                ("stage_ms", "h2d_ms", "d2h_ms", "host_total_ms")] + \
               [("n_batches", ctypes.c_uint64), ("peak_bytes", ctypes.c_uint64),
                ("input_ms", ctypes.c_double), ("spilled_bytes", ctypes.c_uint64)] + \
               [(name, ctypes.c_uint64) for name in ("spec_levels", "spec_fine_levels", "spec_fallbacks",
                                                      "collect_mode", "sent_bytes", "spec_l1",
                                                      "cached_bytes")] + \
               [("exchange_hidden_ms", ctypes.c_double), ("coresident", ctypes.c_uint64)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


# exported C-ABI symbols (must match include/mtg_boss.h)
EXPORTS = ("mtg_boss_abi_version", "mtg_last_error", "mtg_boss_ctor_create",
           "mtg_boss_ctor_destroy", "mtg_boss_ctor_get_k", "mtg_boss_ctor_add_sequences",
           "mtg_boss_ctor_add_sequence", "mtg_boss_ctor_add_packed", "mtg_boss_ctor_build_chunk",
           "mtg_boss_chunk_free", "mtg_boss_build_device", "mtg_boss_last_timings",
           "mtg_device_alloc", "mtg_device_free", "mtg_memcpy_h2d", "mtg_memcpy_d2h",
           "mtg_device_count", "mtg_device_synchronize", "mtg_comm_get_unique_id",
           "mtg_comm_create_rccl", "mtg_comm_create_local", "mtg_comm_destroy", "mtg_comm_rank",
           "mtg_comm_size", "mtg_boss_ctor_build_chunk_dist", "mtg_boss_build_device_dist",
           "mtg_dist_bounds", "mtg_device_identity", "mtg_dist_coresident", "mtg_boss_ctor_add_kmc", "mtg_dna_encode_table",
           "mtg_boss_write_dbg", "mtg_sdsl_write", "mtg_boss_read_dbg", "mtg_dbg_file_free",
           "mtg_boss_ctor_add_fasta", "mtg_device_copy", "mtg_kmc_load_device",
           "mtg_device_reads_free", "mtg_kmc_write_device", "mtg_host_pool_bytes",
           "mtg_host_pool_trim", "mtg_comm_create_callbacks", "mtg_comm_local_held_ms",
           "mtg_boss_ctor_trim")

COMM_ID_BYTES = 128

_lib = None


def lib():
    """Load libmtg_boss.so (built by __graft_entry__.build()); raise if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libmtg_boss.so is not built (run __graft_entry__.build()); "
                               "the BOSS constructor has no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        L.mtg_boss_abi_version.restype = ctypes.c_int
        L.mtg_last_error.restype = ctypes.c_char_p
        L.mtg_boss_ctor_create.argtypes = [P(_Params)]
        L.mtg_boss_ctor_create.restype = ctypes.c_void_p
        L.mtg_boss_ctor_destroy.argtypes = [ctypes.c_void_p]
        L.mtg_boss_ctor_get_k.argtypes = [ctypes.c_void_p]
        L.mtg_boss_ctor_get_k.restype = ctypes.c_uint64
        L.mtg_boss_ctor_add_sequences.argtypes = [ctypes.c_void_p, P(ctypes.c_char_p),
                                                  P(ctypes.c_uint64), P(ctypes.c_uint64),
                                                  ctypes.c_size_t]
        L.mtg_boss_ctor_add_sequence.argtypes = [ctypes.c_void_p, ctypes.c_char_p,
                                                 ctypes.c_uint64, ctypes.c_uint64]
        L.mtg_boss_ctor_add_packed.argtypes = [ctypes.c_void_p, ctypes.c_char_p,
                                               P(ctypes.c_uint64), P(ctypes.c_uint64),
                                               ctypes.c_size_t]
        L.mtg_boss_ctor_build_chunk.argtypes = [ctypes.c_void_p, P(_Chunk)]
        L.mtg_boss_chunk_free.argtypes = [P(_Chunk)]
        L.mtg_boss_build_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                            ctypes.c_void_p, P(_DeviceChunk)]
        L.mtg_boss_last_timings.argtypes = [ctypes.c_void_p, P(Timings)]
        L.mtg_device_alloc.argtypes = [ctypes.c_int, ctypes.c_uint64]
        L.mtg_device_alloc.restype = ctypes.c_void_p
        L.mtg_device_free.argtypes = [ctypes.c_void_p]
        L.mtg_memcpy_h2d.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        L.mtg_memcpy_d2h.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        L.mtg_device_count.restype = ctypes.c_int
        L.mtg_device_synchronize.argtypes = [ctypes.c_int]
        L.mtg_comm_get_unique_id.argtypes = [ctypes.c_char_p]
        L.mtg_comm_create_rccl.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int]
        L.mtg_comm_create_rccl.restype = ctypes.c_void_p
        L.mtg_comm_create_local.argtypes = [ctypes.c_int, P(ctypes.c_void_p)]
        L.mtg_comm_destroy.argtypes = [ctypes.c_void_p]
        L.mtg_comm_rank.argtypes = [ctypes.c_void_p]
        L.mtg_comm_size.argtypes = [ctypes.c_void_p]
        L.mtg_comm_local_held_ms.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.mtg_comm_local_held_ms.restype = ctypes.c_double
        L.mtg_boss_ctor_build_chunk_dist.argtypes = [ctypes.c_void_p, ctypes.c_void_p, P(_Chunk)]
        L.mtg_boss_build_device_dist.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_uint64, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_uint64,
                                                 ctypes.c_void_p, P(_DeviceChunk)]
        L.mtg_boss_ctor_add_kmc.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64,
                                             ctypes.c_uint64, ctypes.c_int]
        L.mtg_dist_bounds.argtypes = [P(ctypes.c_uint64), ctypes.c_uint64, ctypes.c_int,
                                      P(ctypes.c_uint64)]
        L.mtg_device_identity.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.mtg_device_identity.restype = ctypes.c_uint64
        L.mtg_dist_coresident.argtypes = [P(ctypes.c_uint64), ctypes.c_int, ctypes.c_int]
        L.mtg_dist_coresident.restype = ctypes.c_uint32
        L.mtg_dna_encode_table.argtypes = [ctypes.c_char_p]
        L.mtg_boss_ctor_add_fasta.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.mtg_device_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.mtg_boss_write_dbg.argtypes = [P(_Chunk), ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int64, P(ctypes.c_uint64)]
        L.mtg_boss_read_dbg.argtypes = [ctypes.c_char_p, P(_DbgFile)]
        L.mtg_sdsl_write.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64]
        L.mtg_kmc_load_device.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                          ctypes.c_int, P(_DeviceReads)]
        L.mtg_device_reads_free.argtypes = [P(_DeviceReads)]
        L.mtg_host_pool_bytes.restype = ctypes.c_uint64
        L.mtg_comm_create_callbacks.argtypes = [P(_CommCallbacks)]
        L.mtg_comm_create_callbacks.restype = ctypes.c_void_p
        L.mtg_kmc_write_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint,
                                           ctypes.c_int, ctypes.c_uint, ctypes.c_uint, ctypes.c_char_p,
                                           P(ctypes.c_uint64)]
        L.mtg_dbg_file_free.argtypes = [P(_DbgFile)]
        L.mtg_boss_ctor_trim.argtypes = [ctypes.c_void_p]
        for name in EXPORTS:
            getattr(L, name)
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise RuntimeError(lib().mtg_last_error().decode() or "error %d" % rc)


class _ChunkBlocks:
    """Owner of one mtg_boss_chunk's pinned host arrays: numpy views keep it alive, and it
    releases the arrays (mtg_boss_chunk_free) when the last view is gone."""

    def __init__(self, c):
        self._c = c

    def view(self, ptr, n, dtype):
        size = int(n) * np.dtype(dtype).itemsize
        if size == 0:
            return np.zeros(0, dtype=dtype)
        buf = (ctypes.c_uint8 * size).from_address(ctypes.cast(ptr, ctypes.c_void_p).value)
        buf._owner = self
        return np.frombuffer(buf, dtype=dtype)

    def __del__(self):
        c, self._c = getattr(self, "_c", None), None
        if c is not None and _lib is not None:
            _lib.mtg_boss_chunk_free(ctypes.byref(c))


class Chunk:
    """BOSS::Chunk (boss_chunk.hpp:19-104): W (0..9), last (0/1), F[5], weights, k.  `last`
    may be given as packed words (last_words, the ABI's layout) and is unpacked on first use."""

    def __init__(self, k, W, last, F, weights=None, n_real=None, n_dummy=None, bits_per_count=0,
                 last_words=None):
        self.k = k
        self.alph_size = 5
        self.bits_per_count = bits_per_count
        self.W = W
        self._last = last
        self._last_words = last_words
        self.F = F
        self.weights = weights
        self.n_real = n_real
        self.n_dummy = n_dummy

    @property
    def last(self):
        if self._last is None:
            self._last = unpack_last(self._last_words, len(self.W))
        return self._last

    @last.setter
    def last(self, value):
        self._last = value
        self._last_words = None

    def size(self):
        return len(self.W)

    def serialize(self, outbase):
        """BOSS::Chunk::serialize (boss_chunk.cpp:372-386): <outbase>.dbg.chunk{,.W,.last,.weights}."""
        from . import chunk_io
        return chunk_io.serialize(self, outbase)

    @classmethod
    def load(cls, infbase):
        """BOSS::Chunk::load (boss_chunk.cpp:330-370); raises ValueError on a corrupted chunk."""
        from . import chunk_io
        k, alph, W, last, F, weights, bits = chunk_io.load(infbase)
        if alph != 5:
            raise ValueError("ERROR: only the DNA alphabet of size 5 is supported")
        return cls(k, W, last, F, weights, bits_per_count=bits)

    def write_dbg(self, outbase, canonical=False, mask_dummy=False, suffix_length=-1, prune=False):
        """The files `metagraph build` writes from this chunk (cli/build.cpp:323-352):
        <outbase>.dbg, <outbase>.edgemask (mask_dummy) and <outbase>.dbg.weights (weighted).
        prune=True is `metagraph concatenate --clear-dummy` (cli/build.cpp:400-405): the
        redundant source dummies of suffix-built chunks are erased before writing, the mask is
        written, and no weights file (build_boss_from_chunks takes none).
        Returns the valid edges after masking (`nodes (k)` of `metagraph stats`), else rows - 1."""
        W = np.ascontiguousarray(self.W, dtype=np.uint8)
        last = self._last_words if self._last_words is not None else pack_last(self.last)
        F = (ctypes.c_uint64 * 5)(*[int(f) for f in self.F])
        c = _Chunk(k=self.k, alph_size=5, n=len(W), F=F, bits_per_count=self.bits_per_count or 0)
        c.W = W.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        c.last = last.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        wts = None
        if self.weights is not None and self.bits_per_count:
            wts = np.ascontiguousarray(self.weights, dtype=np.uint32)
            c.weights = wts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        nv = ctypes.c_uint64(0)
        _check(lib().mtg_boss_write_dbg(ctypes.byref(c), os.fsencode(outbase), int(bool(canonical)),
                                        2 if prune else int(bool(mask_dummy)), int(suffix_length),
                                        ctypes.byref(nv)))
        return nv.value

    def extend(self, other):
        """BOSS::Chunk::extend (boss_chunk.cpp:230-270): append rows after index 0, sum F."""
        if self.alph_size != other.alph_size or self.k != other.k:
            raise RuntimeError("ERROR: trying to concatenate incompatible graph chunks")
        if len(other.W) == 1:
            return
        if (self.weights is None) != (other.weights is None):
            raise RuntimeError("ERROR: trying to concatenate weighted and unweighted blocks")
        self.W = np.concatenate([self.W, other.W[1:]])
        self.last = np.concatenate([self.last, other.last[1:]])
        self.F = self.F + other.F
        if self.weights is not None:
            self.weights = np.concatenate([self.weights, other.weights[1:]])


def generate_suffixes(length):
    """KmerExtractorBOSS::generate_suffixes (kmer/kmer_extractor.cpp:402-416): the node suffixes
    of `build --suffix-len` in BOSS order (last char slowest, common/utils/string_utils.cpp:82-95),
    keeping those whose '$'s form a prefix.  Building one chunk per suffix (filter_suffix) and
    concatenating them in this order gives the graph (cli/build.cpp:102-155)."""
    out = [""]
    while len(out[0]) < length:
        head = out.pop(0)
        out.extend(c + head for c in "$ACGT")
    res = []
    for s in out:
        j = s.rfind("$")
        if j < 0 or s[:j + 1] == "$" * (j + 1):
            res.append(s)
    return res


class BOSSChunkConstructor:
    def __init__(self, handle, k, bits_per_count, canonical=False):
        self._h = handle
        self._k = k
        self._bits = bits_per_count
        self._canonical = canonical

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h and _lib is not None:
            _lib.mtg_boss_ctor_destroy(h)

    def get_k(self):
        return lib().mtg_boss_ctor_get_k(self._h)

    def add_sequence(self, seq, count=1):
        b = seq.encode() if isinstance(seq, str) else bytes(seq)
        _check(lib().mtg_boss_ctor_add_sequence(self._h, b, len(b), count))

    def add_sequences(self, seqs, counts=None):
        """add_sequences(vector<string>&&) / add_sequences(vector<pair<string,uint64_t>>&&)."""
        if len(seqs) and isinstance(seqs[0], tuple):
            counts = [c for _, c in seqs]
            seqs = [s for s, _ in seqs]
        bs = [s.encode() if isinstance(s, str) else bytes(s) for s in seqs]
        if not bs:
            return
        offsets = np.zeros(len(bs) + 1, dtype=np.uint64)
        offsets[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
        cnt = None if counts is None else np.ascontiguousarray(counts, dtype=np.uint64)
        _check(lib().mtg_boss_ctor_add_packed(
            self._h, b"".join(bs), offsets.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
            cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)) if cnt is not None else None,
            len(bs)))

    def add_packed(self, data, offsets, counts=None):
        """n sequences back to back in one buffer (bytes or uint8 array), offsets[n + 1]."""
        buf = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8)
                                   if isinstance(data, (bytes, bytearray)) else data, dtype=np.uint8)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = len(off) - 1
        if n <= 0:
            return
        cnt = None if counts is None else np.ascontiguousarray(counts, dtype=np.uint64)
        _check(lib().mtg_boss_ctor_add_packed(
            self._h, buf.ctypes.data_as(ctypes.c_char_p),
            off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
            cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)) if cnt is not None else None, n))

    def add_fasta(self, path):
        """A FASTA / FASTQ file (plain or .gz): parse_sequences' FASTA branch
        (cli/parse_sequences.hpp:103-151), split into records on the device at build time."""
        _check(lib().mtg_boss_ctor_add_fasta(self._h, os.fsencode(path)))

    def add_fasta_files(self, paths, threads=None):
        """push_sequences (cli/build.cpp:31-56): one host thread per file."""
        from concurrent.futures import ThreadPoolExecutor
        paths = list(paths)
        with ThreadPoolExecutor(max_workers=threads or max(1, min(len(paths), os.cpu_count() or 1))) as ex:
            for f in [ex.submit(self.add_fasta, p) for p in paths]:
                f.result()

    def add_kmc(self, kmc_path, min_count=1, max_count=2**32 - 1,
                call_both_from_canonical=None):
        """KMC1 database input (cli/parse_sequences.hpp:50-101, seq_io/kmc_parser.cpp:27-62).
        call_both_from_canonical defaults to what `metagraph build` passes: not canonical."""
        if call_both_from_canonical is None:
            call_both_from_canonical = not self._canonical
        _check(lib().mtg_boss_ctor_add_kmc(self._h, os.fsencode(kmc_path), min_count, max_count,
                                           int(bool(call_both_from_canonical))))

    def write_kmc(self, d_seq, seq_len, outbase, k, canonical=True, counter_size=1, lut_len=None):
        """Count the k-mers of device-resident reads on the GPU and write them as a KMC1 database
        (<outbase>.kmc_pre / .kmc_suf), the input BASELINE config 5 feeds `metagraph build`.
        Returns the records written."""
        if lut_len is None:
            # KMC's prefix length: at most 11 bases, leaving at least one suffix byte
            lut_len = next((L for L in range(min(k, 11), -1, -1) if (k - L) % 4 == 0 and k - L >= 4), k)
        n = ctypes.c_uint64(0)
        _check(lib().mtg_kmc_write_device(self._h, d_seq, seq_len, k, int(bool(canonical)), counter_size,
                                          lut_len, os.fsencode(outbase), ctypes.byref(n)))
        return n.value

    def build_chunk(self, comm=None):
        """BOSS::Chunk of everything added; with `comm`, this rank's range of the global build
        (concatenate the ranks' chunks in rank order with Chunk.extend)."""
        c = _Chunk()
        if comm is None:
            _check(lib().mtg_boss_ctor_build_chunk(self._h, ctypes.byref(c)))
        else:
            _check(lib().mtg_boss_ctor_build_chunk_dist(self._h, comm.handle, ctypes.byref(c)))
        n = c.n
        # zero-copy views of the chunk's pinned host blocks; the blocks are released when the
        # last view is gone (_ChunkBlocks)
        owner = _ChunkBlocks(c)
        W = owner.view(c.W, n, np.uint8)
        words = owner.view(c.last, (n + 63) // 64, np.uint64)
        weights = owner.view(c.weights, n, np.uint32) if c.weights else None
        F = np.array(list(c.F), dtype=np.uint64)
        return Chunk(c.k, W, None, F, weights, c.n_real, c.n_dummy, self._bits, last_words=words)

    def build_device(self, d_seq, seq_len, d_read_starts=None, d_counts=None, n_reads=0,
                     stream=None, comm=None):
        """Whole path on a device-resident read buffer; returns the device chunk descriptor
        (with `comm`: this rank's range of the multi-GPU build)."""
        c = _DeviceChunk()
        if comm is None:
            _check(lib().mtg_boss_build_device(self._h, d_seq, seq_len, d_read_starts, d_counts,
                                               n_reads, stream, ctypes.byref(c)))
        else:
            _check(lib().mtg_boss_build_device_dist(self._h, comm.handle, d_seq, seq_len,
                                                    d_read_starts, d_counts, n_reads, stream,
                                                    ctypes.byref(c)))
        return c

    def timings(self):
        t = Timings()
        _check(lib().mtg_boss_last_timings(self._h, ctypes.byref(t)))
        return t

    def trim(self):
        """Free the device memory held between builds -- idle workspace blocks and the last build's stage
        buffers; its device chunk arrays stay valid (mtg_boss_ctor_trim)."""
        _check(lib().mtg_boss_ctor_trim(self._h))


class IBOSSChunkConstructor:
    @staticmethod
    def initialize(k, both_strands=False, bits_per_count=0, filter_suffix="", num_threads=1,
                   memory_preallocated=0, container_type=CONTAINER_VECTOR, swap_dir="/tmp/",
                   disk_cap_bytes=int(1e9), device_id=0):
        """IBOSSChunkConstructor::initialize (boss_chunk_construct.cpp:1134-1178).

        k is the BOSS k (node length, = DBG k - 1).  Invalid k / count width raise like the
        reference's exit(1) / runtime_error; there is no CPU fallback for other containers.
        """
        if k < 1 or k > 84:
            raise ValueError("For succinct graph, k must be between 2 and 85")
        if bits_per_count > 32:
            raise RuntimeError("Error: trying to allocate too many bits per k-mer count")
        p = _Params(k, int(bool(both_strands)), bits_per_count,
                    filter_suffix.encode() if filter_suffix else None, num_threads,
                    float(memory_preallocated), container_type,
                    swap_dir.encode() if swap_dir else None, int(disk_cap_bytes), device_id)
        h = lib().mtg_boss_ctor_create(ctypes.byref(p))
        if not h:
            raise RuntimeError(lib().mtg_last_error().decode())
        return BOSSChunkConstructor(h, k, bits_per_count, bool(both_strands))


class BOSSConstructor(BOSSChunkConstructor):
    """BOSSConstructor (boss_construct.hpp:12-53): (k, canonical, bits_per_count, ...)."""

    def __new__(cls, k, canonical=False, bits_per_count=0, filter_suffix="", num_threads=1,
                memory_preallocated=0, container_type=CONTAINER_VECTOR):
        return IBOSSChunkConstructor.initialize(k, canonical, bits_per_count, filter_suffix,
                                                num_threads, memory_preallocated,
                                                container_type)


class DeviceReads:
    """A KMC1 database decoded into device memory (mtg_kmc_load_device): the read buffer, per-read
    starts and counts that build_device takes, as add_kmc would decode them at build time."""

    def __init__(self, kmc_path, min_count=1, max_count=2**32 - 1, call_both_from_canonical=False,
                 device_id=0):
        self._r = _DeviceReads()
        _check(lib().mtg_kmc_load_device(os.fsencode(kmc_path), min_count, max_count,
                                         int(bool(call_both_from_canonical)), device_id,
                                         ctypes.byref(self._r)))

    seq = property(lambda self: self._r.seq)
    seq_len = property(lambda self: self._r.seq_len)
    read_starts = property(lambda self: self._r.read_starts)
    counts = property(lambda self: self._r.counts)
    n_reads = property(lambda self: self._r.n_reads)

    def build_args(self):
        """(d_seq, seq_len, d_read_starts, d_counts, n_reads) for build_device."""
        return self.seq, self.seq_len, self.read_starts, self.counts, self.n_reads

    def __del__(self):
        r, self._r = getattr(self, "_r", None), None
        if r is not None and _lib is not None:
            _lib.mtg_device_reads_free(ctypes.byref(r))


class Comm:
    """Exchange group of a multi-GPU build (include/mtg_boss.h: mtg_comm_*)."""

    def __init__(self, handle):
        self.handle = handle

    def __del__(self):
        h, self.handle = getattr(self, "handle", None), None
        if h and _lib is not None:
            _lib.mtg_comm_destroy(h)

    @property
    def rank(self):
        return lib().mtg_comm_rank(self.handle)

    @property
    def size(self):
        return lib().mtg_comm_size(self.handle)

    def held_ms(self, reset=False):
        """Serial local groups (MTG_LOCAL_SERIAL=1): this rank's device time in ms; -1 otherwise."""
        return lib().mtg_comm_local_held_ms(self.handle, 1 if reset else 0)

    @staticmethod
    def unique_id():
        """128 opaque bytes (ncclGetUniqueId) that rank 0 broadcasts to the others."""
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        _check(lib().mtg_comm_get_unique_id(buf))
        return buf.raw

    @staticmethod
    def rccl(unique_id, world, rank, device_id):
        """One rank of an RCCL group over xGMI (one process per GPU)."""
        h = lib().mtg_comm_create_rccl(bytes(unique_id), world, rank, device_id)
        if not h:
            raise RuntimeError(lib().mtg_last_error().decode())
        return Comm(h)

    @staticmethod
    def callbacks(rank, world, allreduce_sum_u64, allgather_u64, alltoallv):
        """One rank of a build whose exchanges run through Python functions on host numpy arrays
        (mtg_comm_create_callbacks): allreduce_sum_u64(buf) in place; allgather_u64(send) -> array
        of world * len(send); alltoallv(send_bytes, scounts) -> received bytes in rank order."""
        def ar(_u, buf, n):
            try:
                a = np.ctypeslib.as_array(buf, shape=(n,)) if n else np.zeros(0, dtype=np.uint64)
                a[:] = allreduce_sum_u64(a.copy())
                return 0
            except Exception:  # noqa: BLE001 -- reported to the library as a failed exchange
                return 1

        def ag(_u, send, recv, n):
            try:
                a = np.ctypeslib.as_array(send, shape=(n,)).copy() if n else np.zeros(0, dtype=np.uint64)
                out = np.ctypeslib.as_array(recv, shape=(n * world,)) if n else None
                got = allgather_u64(a)
                if n:
                    out[:] = got
                return 0
            except Exception:  # noqa: BLE001
                return 1

        def a2a(_u, send, scnt, recv, rcnt):
            try:
                sc = np.ctypeslib.as_array(scnt, shape=(world,)).copy()
                rc = np.ctypeslib.as_array(rcnt, shape=(world,)).copy()
                st, rt = int(sc.sum()), int(rc.sum())
                sb = np.frombuffer((ctypes.c_uint8 * st).from_address(send), dtype=np.uint8) if st else \
                    np.zeros(0, dtype=np.uint8)
                got = alltoallv(sb.copy(), sc, rc)
                if rt:
                    np.frombuffer((ctypes.c_uint8 * rt).from_address(recv), dtype=np.uint8)[:] = got
                return 0
            except Exception:  # noqa: BLE001
                return 1

        cb = _CommCallbacks(None, rank, world, _ALLREDUCE_CB(ar), _ALLGATHER_CB(ag), _ALLTOALLV_CB(a2a))
        h = lib().mtg_comm_create_callbacks(ctypes.byref(cb))
        if not h:
            raise RuntimeError(lib().mtg_last_error().decode())
        c = Comm(h)
        c._keep = cb  # the C function pointers must outlive the communicator
        return c

    @staticmethod
    def torch_distributed(group=None):
        """This process's rank of a build exchanging over an initialised torch.distributed group
        (e.g. gloo between processes that share one GPU): host-staged, see callbacks()."""
        f = torch_exchange_functions(group)
        import torch.distributed as dist
        return Comm.callbacks(dist.get_rank(group), dist.get_world_size(group), *f)

    @staticmethod
    def local_group(world):
        """`world` ranks inside this process on one device (one host thread per rank)."""
        arr = (ctypes.c_void_p * world)()
        _check(lib().mtg_comm_create_local(world, arr))
        return [Comm(arr[r]) for r in range(world)]


def torch_exchange_functions(group=None):
    """The three exchange functions of Comm.callbacks over torch.distributed CPU tensors (gloo)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)

    def allreduce(a):
        t = torch.from_numpy(a.view(np.int64).copy())  # sums wrap like uint64
        dist.all_reduce(t, group=group)
        return t.numpy().view(np.uint64)

    def allgather(a):
        t = torch.from_numpy(a.view(np.int64).copy())
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t, group=group)
        return np.concatenate([o.numpy().view(np.uint64) for o in out])

    def alltoallv(send, scounts, rcounts):
        out = torch.empty(int(rcounts.sum()), dtype=torch.uint8)
        dist.all_to_all_single(out, torch.from_numpy(send), [int(c) for c in rcounts],
                               [int(c) for c in scounts], group=group)
        return out.numpy()

    return allreduce, allgather, alltoallv


def dist_bounds(hist, world):
    """The range split of the multi-GPU build: bounds[0..world] over len(hist) prefixes."""
    h = np.ascontiguousarray(hist, dtype=np.uint64)
    out = np.zeros(world + 1, dtype=np.uint64)
    _check(lib().mtg_dist_bounds(h.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), len(h), world,
                                 out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))))
    return out


def coresident(hosts_and_buses, rank):
    """Ranks that share rank's GPU, from every rank's (host name, PCI bus id) -- the count a
    multi-GPU build plans its HBM share with (timings' coresident)."""
    ids = np.array([lib().mtg_device_identity(h.encode(), b.encode()) for h, b in hosts_and_buses],
                   dtype=np.uint64)
    return int(lib().mtg_dist_coresident(ids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), len(ids), rank))


def concatenate(chunks):
    """Rank chunks -> one chunk, BOSS::Chunk::extend in rank order (boss_chunk.cpp:230-270)."""
    first = chunks[0]
    out = Chunk(first.k, first.W.copy(), first.last.copy(), first.F.copy(),
                None if first.weights is None else first.weights.copy(), first.n_real,
                first.n_dummy, first.bits_per_count)
    for ch in chunks[1:]:
        out.extend(ch)
        out.n_real += ch.n_real
        out.n_dummy += ch.n_dummy
    return out


def concatenate_files(chunk_filenames):
    """BOSS::Chunk::build_boss_from_chunks (boss_chunk.cpp:286-327) up to initialize_boss: load
    the `.dbg.chunk` files in order and extend the first with the rest."""
    if not chunk_filenames:
        raise ValueError("no graph chunks")
    full = None
    for name in chunk_filenames:
        ch = Chunk.load(name)
        if full is None:
            full = ch
        else:
            full.extend(ch)
    return full


class DbgFile:
    """A `.dbg` (+ `.edgemask`) as mtg_boss_read_dbg parses it: k, F, state, mode, W, last,
    the suffix-range index (n_ranges x 2: first and last edge) and the valid-edge mask."""

    def __init__(self, outbase):
        f = _DbgFile()
        _check(lib().mtg_boss_read_dbg(os.fsencode(outbase), ctypes.byref(f)))
        try:
            self.k, self.n, self.state, self.mode = f.k, f.n, f.state, f.mode
            self.F = np.array(list(f.F), dtype=np.uint64)
            self.suffix_length = f.suffix_length
            self.W = np.ctypeslib.as_array(f.W, shape=(f.n,)).copy()
            self.last = unpack_last(np.ctypeslib.as_array(f.last, shape=((f.n + 63) // 64,)), f.n)
            self.ranges = (np.ctypeslib.as_array(f.ranges, shape=(2 * f.n_ranges,)).reshape(-1, 2).copy()
                           if f.n_ranges else np.zeros((0, 2), dtype=np.uint64))
            self.valid = (unpack_last(np.ctypeslib.as_array(f.valid, shape=((f.n + 63) // 64,)), f.n)
                          if f.valid else None)
            self.n_valid = f.n_valid
        finally:
            lib().mtg_dbg_file_free(ctypes.byref(f))


def unpack_last(words, n):
    """Packed `last` (bit i of word i // 64, sdsl::bit_vector layout) -> n flags 0/1 (uint8)."""
    bits = np.unpackbits(np.ascontiguousarray(words, dtype="<u8").view(np.uint8), bitorder="little")
    return bits[:n].copy()


def pack_last(last):
    """n flags 0/1 -> packed words (inverse of unpack_last)."""
    b = np.packbits(np.asarray(last, dtype=np.uint8) & 1, bitorder="little")
    b = np.concatenate([b, np.zeros((-len(b)) % 8, dtype=np.uint8)])
    return b.view("<u8").copy()


def dna_encode_table():
    """The extractor's encode table as the library's device function computes it (256 bytes)."""
    buf = ctypes.create_string_buffer(256)
    lib().mtg_dna_encode_table(buf)
    return np.frombuffer(buf.raw, dtype=np.uint8).copy()


def host_pool_bytes():
    """Bytes of spare pinned host blocks the library keeps for reuse (bounded by 4 GiB)."""
    return lib().mtg_host_pool_bytes()


def host_pool_trim():
    lib().mtg_host_pool_trim()


def device_count():
    return lib().mtg_device_count()
