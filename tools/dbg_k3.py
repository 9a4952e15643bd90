import sys, importlib
sys.path[:0] = ['.', 'oracle', 'tests']
boss = importlib.import_module("projects2014-metagenome_amd.boss")
from test_oracle_goldens import CONSTRUCT_SEQS
import oracle_ctypes as O
for k in (2, 3, 4):
    ctor = boss.IBOSSChunkConstructor.initialize(k)
    ctor.add_sequences(CONSTRUCT_SEQS)
    c = ctor.build_chunk()
    w = O.build_chunk(k, CONSTRUCT_SEQS)
    print("k", k, "match", (c.W == w.W).all(), flush=True)
    d = O.dummy_kmers(k, CONSTRUCT_SEQS)
    print(" oracle dummies", [hex(x) for x in d[:8, 0]], flush=True)
