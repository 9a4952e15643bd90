"""Workspace allocations of one configs[1] build (MTG_TRACE=1 lists every new block >= 256 MiB) and the
held bytes after each of three builds.  Usage: python tools/ws_trace.py"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["MTG_TRACE"] = "1"
import bench  # noqa: E402


def main():
    import torch
    boss = importlib.import_module("projects2014-metagenome_amd.boss")
    dev = torch.device("cuda", 0)
    seq = bench.make_reads_device(torch, 10_000_000, 150, 1000, "genome", 10.0, dev)
    torch.cuda.synchronize()
    ctor = boss.IBOSSChunkConstructor.initialize(30, both_strands=True)
    for i in range(3):
        ctor.build_device(seq.data_ptr(), seq.numel())
        t = ctor.timings()
        print("build %d: peak_bytes %.2f GB, cached %.2f GB" % (i, t.peak_bytes / 1e9, t.cached_bytes / 1e9), flush=True)


if __name__ == "__main__":
    main()
