import importlib, os, sys, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo")); sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import numpy as np, bench
boss = importlib.import_module("projects2014-metagenome_amd.boss")
asc = bench.make_reads_host_codes(2_000_000, 150, 12345, "genome", 10.0)
data = asc.reshape(-1); off = np.arange(len(asc) + 1, dtype=np.uint64) * asc.shape[1]
for rep in range(2):
    ctor = boss.IBOSSChunkConstructor.initialize(30, both_strands=True, num_threads=8)
    ctor.add_packed(data, off)
    ch = ctor.build_chunk()
    t = ctor.timings()
    print(os.environ.get("MTG_KSPEC"), rep, "levels", t.spec_levels, "fallbacks", t.spec_fallbacks, "rows", ch.n if hasattr(ch, "n") else len(ch.W), flush=True)
