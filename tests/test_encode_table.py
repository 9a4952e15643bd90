"""The device's branchless DNA encode (csrc/boss_kernels.hpp encode_dna) against the alphabet of
kmer/alphabets.hpp:127-143: A/a 0, C/c 1, G/g 2, T/t/U/u 3, every other byte invalid (4).
The table constant is read from the header and evaluated for all 256 byte values."""
import os
import re

HDR = os.path.join(os.path.dirname(__file__), "..", "projects2014-metagenome_amd", "csrc", "boss_kernels.hpp")


def _table():
    src = open(HDR).read()
    m = re.search(r"TAB\s*=\s*(0x[0-9a-fA-F]+)ull", src)
    assert m, "encode_dna table constant not found"
    return int(m.group(1), 16)


def test_encode_table_matches_alphabet():
    tab = _table()
    want = {ord(c): v for c, v in zip("AaCcGgTtUu", [0, 0, 1, 1, 2, 2, 3, 3, 3, 3])}
    for c in range(256):
        idx = ((c | 0x20) - 0x61) & 0xFFFFFFFF
        got = 4 if idx > 20 else (tab >> (3 * idx)) & 7
        assert got == want.get(c, 4), (c, got)
