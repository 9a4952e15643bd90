"""Sequence input for the `build` path: FASTA/FASTQ (optionally gzipped) records.

Mirrors what the reference hands to the chunk constructor: every record's sequence as one
string (kseq strips line breaks), in file order -- seq_io/sequence_io.cpp:364-405
(read_fasta_file_critical) driven by cli/parse_sequences.hpp:103-151.
"""
import gzip
import io


def _open(path):
    with open(path, "rb") as f:
        magic = f.read(2)
    if magic == b"\x1f\x8b":
        return io.BufferedReader(gzip.open(path, "rb"))
    return open(path, "rb")


def read_sequences(path):
    """Return the list of record sequences (bytes) of a FASTA or FASTQ file."""
    seqs = []
    with _open(path) as f:
        data = f.read()
    if not data:
        return seqs
    if data[:1] == b"@":
        lines = data.split(b"\n")
        i = 0
        while i < len(lines):
            if lines[i].startswith(b"@"):
                seq = []
                i += 1
                while i < len(lines) and not lines[i].startswith(b"+"):
                    seq.append(lines[i].strip())
                    i += 1
                seqs.append(b"".join(seq))
                n = sum(len(s) for s in seq)
                i += 1
                q = 0
                while i < len(lines) and q < n:
                    q += len(lines[i].strip())
                    i += 1
            else:
                i += 1
        return seqs
    cur = None
    for line in data.split(b"\n"):
        if line.startswith(b">"):
            if cur is not None:
                seqs.append(b"".join(cur))
            cur = []
        elif cur is not None:
            cur.append(line.strip())
    if cur is not None:
        seqs.append(b"".join(cur))
    return seqs
