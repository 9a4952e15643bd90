"""Writes tests/golden/capi_k20_fixture.bin, the expected chunk of tests/c/capi_min.c: the first
40 records of transcripts_1000.fa, BOSS k = 19 (DBG k = 20), canonical, 8-bit counts, built by
the oracle (oracle/, the C restatement of boss_chunk_construct.cpp:54-356 + boss_chunk.cpp:32-133,
pinned by the reference's goldens in tests/test_oracle_goldens.py).
Layout: b"MTGF", u64 n, u64 F[5], W[n] (u8), last as u64 words (bit i % 64 of word i / 64),
weights u32[n]; all little-endian."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import oracle_ctypes  # noqa: E402

RECORDS, KB, CANONICAL, BITS = 40, 19, True, 8


def fasta_head(path, n):
    seqs, cur = [], None
    for line in open(path):
        line = line.rstrip("\r\n")
        if line.startswith(">"):
            if len(seqs) == n:
                break
            seqs.append("")
        elif seqs:
            seqs[-1] += line
    return seqs[:n]


def main():
    src = os.path.join(HERE, "transcripts_1000.fa")
    seqs = fasta_head(src, RECORDS)
    with open(os.path.join(HERE, "capi_reads.fa"), "w") as f:
        for i, s in enumerate(seqs):
            f.write(">%d\n%s\n" % (i, s))
    c = oracle_ctypes.build_chunk(KB, seqs, canonical=CANONICAL, bits_per_count=BITS)
    n = len(c.W)
    bits = np.zeros(((n + 63) // 64) * 64, dtype=np.uint8)
    bits[:n] = c.last
    words = np.packbits(bits, bitorder="little").view("<u8")
    with open(os.path.join(HERE, "capi_k20_fixture.bin"), "wb") as f:
        f.write(b"MTGF")
        f.write(np.array([n], dtype="<u8").tobytes())
        f.write(np.asarray(c.F, dtype="<u8").tobytes())
        f.write(np.asarray(c.W, dtype=np.uint8).tobytes())
        f.write(words.tobytes())
        f.write(np.asarray(c.weights, dtype="<u4").tobytes())
    print("rows", n)


if __name__ == "__main__":
    main()
