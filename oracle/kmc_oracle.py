"""TEST INFRASTRUCTURE ONLY -- a CPU restatement of the KMC1 input path, for the parity tests.

Restates what `metagraph build <db>.kmc_suf` feeds the constructor: seq_io::read_kmers
(metagraph/src/seq_io/kmc_parser.cpp:27-62, over the KMC API's CKMCFile listing) and the build's
KMC branch (cli/parse_sequences.hpp:50-101): one sequence of k bases per record with the record's
count, plus the reverse complement when the database holds canonical k-mers and
call_both_from_canonical is set.  The KMC submodule is absent from the reference snapshot, so the
byte layout is the one documented in projects2014-metagenome_amd/csrc/kmc.hpp; it is pinned by
tests/test_kmc.py against the reference's own fixtures (every 11-mer of transcripts_1000.fa with
its count, and the canonical ones for the both-strands database).
"""
import struct

import numpy as np

_ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
_COMP = {ord("A"): ord("T"), ord("C"): ord("G"), ord("G"): ord("C"), ord("T"): ord("A")}


def _base(path):
    for suf in (".kmc_suf", ".kmc_pre"):
        if path.endswith(suf):
            return path[: -len(suf)]
    return path


def read_header(path):
    pre = open(_base(path) + ".kmc_pre", "rb").read()
    hsize = struct.unpack("<I", pre[-8:-4])[0]
    h = pre[-8 - hsize:-8]
    k, mode, counter_size, lut_len, min_count, max_count = struct.unpack("<6I", h[:24])
    total = struct.unpack("<Q", h[24:32])[0]
    flags = struct.unpack("<I", h[32:36])[0]
    return dict(k=k, mode=mode, counter_size=counter_size, lut_len=lut_len, min_count=min_count,
                max_count=max_count, total=total, both_strands=(flags & 1) == 0, pre=pre)


def read_kmers(path, call_both_from_canonical=False, min_count=1, max_count=2**32 - 1):
    """[(kmer bytes, count)] in database order (kmc_parser.cpp:38-62)."""
    if min_count >= max_count:
        return []
    h = read_header(path)
    k, lut_len, cs, total = h["k"], h["lut_len"], h["counter_size"], h["total"]
    lut = np.frombuffer(h["pre"], dtype=np.uint64, count=4 ** lut_len, offset=4)
    suf = open(_base(path) + ".kmc_suf", "rb").read()[4:-4]
    slen = (k - lut_len) // 4
    rec = np.frombuffer(suf, dtype=np.uint8).reshape(total, slen + cs)
    r = np.arange(total, dtype=np.uint64)
    prefix = np.searchsorted(lut, r, side="right") - 1
    codes = np.empty((total, k), dtype=np.uint8)
    for i in range(lut_len):
        codes[:, i] = (prefix >> (2 * (lut_len - 1 - i))) & 3
    for i in range(k - lut_len):
        codes[:, lut_len + i] = (rec[:, i // 4] >> (6 - 2 * (i % 4))) & 3
    counts = np.zeros(total, dtype=np.uint64)
    for b in range(cs):
        counts |= rec[:, slen + b].astype(np.uint64) << np.uint64(8 * b)
    lo = max(min_count, h["min_count"])  # CKMCFile::SetMinCount / SetMaxCount
    hi = min(max_count - 1, h["max_count"])
    seqs = _ACGT[codes]
    out = []
    both = call_both_from_canonical and h["both_strands"]
    for s, c in zip(seqs, counts.tolist()):
        if c < lo or c > hi:
            continue
        b = s.tobytes()
        out.append((b, c))
        if both:
            out.append((bytes(_COMP[x] for x in reversed(b)), c))
    return out
