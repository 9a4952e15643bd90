"""One configs[3] share (125 M reads) through the single build and the P = 1 distributed build, with
MTG_TRACE / MTG_DEBUG on (stderr): the rounds' plan and every step's sizes.
    python tools/gpu/cfg4_dist_debug.py [reads] [single|dist|both]"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

boss = importlib.import_module("projects2014-metagenome_amd.boss")
dev = torch.device("cuda", 0)
seq = bench.make_reads_device(torch, int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000, 150, 1000,
                              "genome", 10.0, dev)
torch.cuda.synchronize()
torch.cuda.empty_cache()
mode = sys.argv[2] if len(sys.argv) > 2 else "both"
for dist in ((False, True) if mode == "both" else (mode == "dist",)):
    ctor = boss.IBOSSChunkConstructor.initialize(30, both_strands=True)
    comm = boss.Comm.local_group(1)[0] if dist else None
    dc = ctor.build_device(seq.data_ptr(), seq.numel(), comm=comm)
    t = ctor.timings()
    print("dist" if dist else "single", "rows", dc.n, "batches", t.n_batches, "mode", t.collect_mode,
          "total_ms", t.total_ms, "peak_GB", t.peak_bytes / 1e9, flush=True)
    del dc, ctor, comm
