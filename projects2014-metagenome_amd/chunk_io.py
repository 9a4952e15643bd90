"""`.dbg.chunk` files: BOSS::Chunk::serialize / load (boss_chunk.cpp:330-386).

A chunk on disk is four files next to each other (kFileExtension = ".dbg.chunk",
boss_chunk.hpp:91):

  <base>.dbg.chunk          sdsl int_vector<> of F (64-bit entries; serialize_number_vector,
                            serialization.cpp:109-121), then alph_size and k as big-endian u64
                            (serialize_number, serialization.cpp:38-49)
  <base>.dbg.chunk.W        sdsl int_vector_buffer<> of W, width hi(2 * alph_size - 1) + 1 = 4
                            (get_W_width, boss_chunk.cpp:388-390)
  <base>.dbg.chunk.last     sdsl int_vector_buffer<1> of last
  <base>.dbg.chunk.weights  sdsl int_vector_buffer<> of weights, width bits_per_count (empty,
                            width 64, when the graph is unweighted: boss_chunk.cpp:140, 171-174)

sdsl's (non-plain) layout, as written by int_vector::serialize / int_vector_buffer::close:
u64 length in BITS, then one u8 width byte unless the width is fixed by the type (<1>), then the
elements bit-packed LSB-first into little-endian 64-bit words (int_vector_buffer pads its data to
a multiple of 8 bytes).  The sdsl-lite submodule is absent from the reference checkout and it
holds no serialized chunk, so the byte layout is restated from sdsl's published format and its
parity is UNPINNED; W / last / F / weights themselves are the pinned arrays (test_gpu_parity.py).
Host-side I/O only: the arrays come off the device already built.
"""
import os
import struct

import numpy as np

EXT = ".dbg.chunk"
ALPH_SIZE = 5
_PACK_BLOCK = 1 << 22  # elements per packing block (a multiple of 64: whole words per block)


def w_width(alph_size=ALPH_SIZE):
    """BOSS::Chunk::get_W_width (boss_chunk.cpp:388-390)."""
    return (2 * alph_size - 1).bit_length() if alph_size else 1


def make_suffix(base, ext=EXT):
    """utils::make_suffix: append `ext` unless `base` already ends with it."""
    return base if base.endswith(ext) else base + ext


def pack_bits(values, width):
    """Elements LSB-first at bit i * width of a little-endian bit stream (sdsl int_vector data)."""
    values = np.asarray(values)
    n = len(values)
    nbytes = (n * width + 7) // 8
    out = bytearray()
    if width in (8, 16, 32, 64):
        dt = {8: "<u1", 16: "<u2", 32: "<u4", 64: "<u8"}[width]
        out += values.astype(dt).tobytes()
    else:
        shifts = np.arange(width, dtype=np.uint64)
        for s in range(0, n, _PACK_BLOCK):
            v = values[s:s + _PACK_BLOCK].astype(np.uint64)
            bits = ((v[:, None] >> shifts) & np.uint64(1)).astype(np.uint8).ravel()
            out += np.packbits(bits, bitorder="little").tobytes()
    assert len(out) == nbytes
    return bytes(out)


def unpack_bits(data, n, width):
    """Inverse of pack_bits: n elements of `width` bits (uint64)."""
    if width in (8, 16, 32, 64):
        dt = {8: "<u1", 16: "<u2", 32: "<u4", 64: "<u8"}[width]
        return np.frombuffer(data, dtype=dt, count=n).astype(np.uint64)
    out = np.empty(n, dtype=np.uint64)
    weights = (np.uint64(1) << np.arange(width, dtype=np.uint64))
    buf = np.frombuffer(data, dtype=np.uint8, count=(n * width + 7) // 8)
    for s in range(0, n, _PACK_BLOCK):
        m = min(_PACK_BLOCK, n - s)
        # blocks start on byte boundaries: _PACK_BLOCK * width is a multiple of 8 bits
        b0 = s * width // 8
        bits = np.unpackbits(buf[b0:b0 + (m * width + 7) // 8], bitorder="little")[:m * width]
        out[s:s + m] = (bits.reshape(m, width).astype(np.uint64) * weights).sum(axis=1)
    return out


def _header(nbits, width, fixed_width):
    return struct.pack("<Q", nbits) + (b"" if fixed_width else struct.pack("<B", width))


def int_vector_buffer_bytes(values, width, fixed_width=False):
    """sdsl::int_vector_buffer file contents after close() (header, data padded to 8 bytes)."""
    n = len(values)
    data = pack_bits(values, width)
    if len(data) % 8:
        data += b"\0" * (8 - len(data) % 8)
    return _header(n * width, width, fixed_width) + data


def int_vector_bytes(values, width):
    """sdsl::int_vector<>::serialize: header, then ceil(bits / 64) whole words."""
    n = len(values)
    data = pack_bits(values, width)
    words = (n * width + 63) // 64
    data += b"\0" * (words * 8 - len(data))
    return _header(n * width, width, False) + data


def read_int_vector(buf, pos=0, fixed_width=None):
    """Parse one sdsl vector at buf[pos:]; returns (values, width, end position)."""
    if len(buf) < pos + 8:
        raise ValueError("truncated sdsl header")
    (nbits,) = struct.unpack_from("<Q", buf, pos)
    pos += 8
    if fixed_width is None:
        if len(buf) < pos + 1:
            raise ValueError("truncated sdsl header")
        width = buf[pos]
        pos += 1
    else:
        width = fixed_width
    if width == 0 or width > 64 or nbits % width:
        raise ValueError("bad sdsl width %d for %d bits" % (width, nbits))
    n = nbits // width
    nbytes = (nbits + 7) // 8
    if len(buf) < pos + nbytes:
        raise ValueError("truncated sdsl data")
    vals = unpack_bits(bytes(buf[pos:pos + nbytes]), n, width)
    return vals, width, pos + ((nbits + 63) // 64) * 8


def _write(path, data):
    with open(path, "wb") as f:
        f.write(data)


def _read(path):
    with open(path, "rb") as f:
        return f.read()


def serialize(chunk, outbase):
    """BOSS::Chunk::serialize (boss_chunk.cpp:372-386)."""
    fname = make_suffix(outbase)
    _write(fname + ".W", int_vector_buffer_bytes(chunk.W, w_width(chunk.alph_size)))
    _write(fname + ".last", int_vector_buffer_bytes(chunk.last, 1, fixed_width=True))
    if chunk.weights is None:
        weights = int_vector_buffer_bytes(np.zeros(0, dtype=np.uint64), 64)
    else:
        bits = getattr(chunk, "bits_per_count", 0) or 32
        weights = int_vector_buffer_bytes(chunk.weights, bits)
    _write(fname + ".weights", weights)
    F = np.asarray(chunk.F, dtype=np.uint64)
    _write(fname, int_vector_bytes(F, 64) + struct.pack(">QQ", chunk.alph_size, chunk.k))
    return fname


def load(infbase):
    """BOSS::Chunk::load (boss_chunk.cpp:330-370): (k, alph_size, W, last, F, weights, bits)
    or raises ValueError where the reference's load returns false."""
    fname = make_suffix(infbase)
    for suf in ("", ".W", ".last", ".weights"):
        if not os.path.exists(fname + suf):
            raise ValueError("ERROR: File corrupted. Cannot load graph chunk " + fname)
    W, _, _ = read_int_vector(_read(fname + ".W"))
    last, _, _ = read_int_vector(_read(fname + ".last"), fixed_width=1)
    weights, wbits, _ = read_int_vector(_read(fname + ".weights"))
    main = _read(fname)
    F, _, pos = read_int_vector(main)
    if len(main) < pos + 16:
        raise ValueError("ERROR: failed to load F vector")
    alph_size, k = struct.unpack_from(">QQ", main, pos)
    ok = (k and alph_size and len(W) == len(last) and len(F) == alph_size
          and (len(weights) == 0 or len(weights) == len(W)))
    if not ok:
        raise ValueError("ERROR: File corrupted. Cannot load graph chunk " + fname)
    return (int(k), int(alph_size), W.astype(np.uint8), last.astype(np.uint8), F,
            weights.astype(np.uint32) if len(weights) else None, int(wbits) if len(weights) else 0)
