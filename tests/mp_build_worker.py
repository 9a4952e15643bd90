"""One rank of the two-process GPU exchange test (tests/test_gpu_multiproc.py): a separate process
on the box's one GPU, exchanging with its peer through torch.distributed over gloo via the
library's host-staged callbacks (mtg_comm_create_callbacks).  Builds its share of the reads and
saves its rank chunk.  Usage: mp_build_worker.py RANK WORLD PORT READS.npz OUT.npz K CANONICAL BITS"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    reads_path, out_path = sys.argv[4], sys.argv[5]
    k, canonical, bits = int(sys.argv[6]), sys.argv[7] == "1", int(sys.argv[8])
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    boss = importlib.import_module("projects2014-metagenome_amd.boss")
    z = np.load(reads_path)
    data, off = z["data"], z["offsets"]
    n = len(off) - 1
    mine = list(range(rank, n, world))
    ctor = boss.IBOSSChunkConstructor.initialize(k, both_strands=canonical, bits_per_count=bits)
    if mine:
        ctor.add_sequences([data[off[i]:off[i + 1]].tobytes() for i in mine])
    comm = boss.Comm.torch_distributed()
    ch = ctor.build_chunk(comm=comm)
    t = ctor.timings()
    np.savez(out_path, W=ch.W, last=ch.last, F=ch.F,
             weights=ch.weights if ch.weights is not None else np.zeros(0, dtype=np.uint32),
             n_real=ch.n_real, n_dummy=ch.n_dummy, world=t.world, n_sent=t.n_sent, batches=t.n_batches,
             coresident=t.coresident, hidden_ms=t.exchange_hidden_ms)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
