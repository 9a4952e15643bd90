"""Benchmark: k-mers/s ingested into BOSS (MetaGraph `build` hot path) on MI355X.

One step = the whole device path on one batch of synthetic reads already resident in HBM:
extract -> canonicalise -> sort -> unique -> reverse-complement augment -> dummy sinks/sources
-> lift+merge -> W/last/F (BASELINE.json configs[1]: k = 31, 10 M synthetic 150 bp reads,
KMerBOSS<uint64_t> keys, canonical mode).  value = k-mer positions offered to the extractor
(reads * (150 - k + 1)) / seconds, summed over ranks.

Multi-GPU (torchrun, one rank per GPU): ONE build of all ranks' reads.  Every rank holds its
own 10 M reads (weak scaling: "scaling": "weak"), all sampled from one shared genome, and
returns the chunk of one range of BOSS order; the exchange steps (k-mers, sink / in-edge
queries, dummy sources) run over RCCL on xGMI inside the timed step (libmtg_boss.so's own RCCL
communicator; torch.distributed only bootstraps it and times the job).

Synthetic data: a seeded random ACGT genome of (all ranks' reads)*150/10 bases (10x coverage);
reads start uniformly, strand 50/50, 0.1 % substitutions; each read is followed by a '$'
separator.
"""
import argparse
import ctypes
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--k", type=int, default=31, help="DBG k (BOSS k = k - 1)")
    ap.add_argument("--mode", default="canonical", choices=["canonical", "basic"])
    ap.add_argument("--count-width", type=int, default=0)
    ap.add_argument("--data", default="genome", choices=["genome", "uniform"])
    ap.add_argument("--coverage", type=float, default=10.0)
    ap.add_argument("--cpu-sample-reads", type=int, default=2_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args()


def make_reads_device(torch, n_reads, read_len, seed, data, coverage, device, world=1,
                      genome_seed=999):
    """Reads + '$' separators as one uint8 tensor on `device` (ASCII ACGT).  The genome is
    shared by all `world` ranks (same seed, sized for all their reads); the reads are the
    rank's own (`seed`)."""
    g = torch.Generator(device=device)
    lut = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=device)
    stride = read_len + 1
    out = torch.empty(n_reads * stride, dtype=torch.uint8, device=device)
    view = out.view(n_reads, stride)
    view[:, read_len] = ord("$")
    chunk = 1 << 20
    if data == "genome":
        glen = max(int(world * n_reads * read_len / coverage), read_len + 1)
        g.manual_seed(genome_seed)
        genome = torch.randint(0, 4, (glen,), dtype=torch.uint8, device=device, generator=g)
    g.manual_seed(seed)
    ar = torch.arange(read_len, device=device)
    for r0 in range(0, n_reads, chunk):
        r1 = min(n_reads, r0 + chunk)
        m = r1 - r0
        if data == "genome":
            st = torch.randint(0, glen - read_len + 1, (m, 1), device=device, generator=g)
            codes = genome[st + ar]
            rev = torch.rand((m, 1), device=device, generator=g) < 0.5
            codes = torch.where(rev, 3 - codes.flip(1), codes)
            sub = torch.rand((m, read_len), device=device, generator=g) < 0.001
            alt = (codes + torch.randint(1, 4, (m, read_len), dtype=torch.uint8, device=device,
                                         generator=g)) % 4
            codes = torch.where(sub, alt, codes)
        else:
            codes = torch.randint(0, 4, (m, read_len), dtype=torch.uint8, device=device,
                                  generator=g)
        view[r0:r1, :read_len] = lut[codes.long()]
    return out


def make_reads_host(n_reads, read_len, seed, data, coverage):
    """The same generator family on the host (numpy), for the CPU baseline sample."""
    import numpy as np
    rng = np.random.default_rng(seed)
    lut = np.frombuffer(b"ACGT", dtype=np.uint8)
    if data == "genome":
        glen = max(int(n_reads * read_len / coverage), read_len + 1)
        genome = rng.integers(0, 4, size=glen, dtype=np.uint8)
        st = rng.integers(0, glen - read_len + 1, size=(n_reads, 1))
        codes = genome[st + np.arange(read_len)]
        rev = rng.random((n_reads, 1)) < 0.5
        codes = np.where(rev, 3 - codes[:, ::-1], codes)
        sub = rng.random((n_reads, read_len)) < 0.001
        alt = (codes + rng.integers(1, 4, size=(n_reads, read_len), dtype=np.uint8)) % 4
        codes = np.where(sub, alt, codes).astype(np.uint8)
    else:
        codes = rng.integers(0, 4, size=(n_reads, read_len), dtype=np.uint8)
    asc = lut[codes]
    return [asc[i].tobytes() for i in range(n_reads)]


def cpu_threads():
    """OpenMP threads the oracle runs on (OMP_NUM_THREADS, else this process's CPU set)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def cpu_baseline(args, kb):
    """Oracle (C restatement: OpenMP extraction + parallel LSD radix sort, serial dummy and
    emission passes) on a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ctypes
    reads = make_reads_host(args.cpu_sample_reads, args.read_len, 12345, args.data,
                            args.coverage)
    t0 = time.perf_counter()
    c = oracle_ctypes.build_chunk(kb, reads, canonical=args.mode == "canonical",
                                  bits_per_count=args.count_width)
    dt = time.perf_counter() - t0
    n = args.cpu_sample_reads * (args.read_len - args.k + 1)
    return {"value": n / dt, "unit": "k-mers/s", "cores": cpu_threads(), "kind": "port",
            "sample": "%d synthetic %d bp reads (%s, %gx coverage), k=%d %s, %.1f s, %d rows"
                      % (args.cpu_sample_reads, args.read_len, args.data, args.coverage,
                         args.k, args.mode, dt, len(c.W))}


def share_comm_id(rank, make_id):
    """Rank 0's 128-byte RCCL id, broadcast over the torch.distributed group."""
    import torch.distributed as dist
    obj = [make_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def max_over_ranks(elapsed, world, device):
    """The job's time is the slowest rank's (tests/test_distributed.py runs this over gloo)."""
    if world <= 1:
        return elapsed
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def job_throughput(kmers_per_rank, world, steps, elapsed):
    """Whole-job k-mers/s: every rank processes kmers_per_rank per step (weak scaling)."""
    return kmers_per_rank * world * steps / elapsed


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    boss = importlib.import_module("projects2014-metagenome_amd.boss")
    kb = args.k - 1
    seq = make_reads_device(torch, args.reads, args.read_len, 1000 + rank, args.data,
                            args.coverage, device, world)
    torch.cuda.synchronize()
    ctor = boss.IBOSSChunkConstructor.initialize(kb, both_strands=args.mode == "canonical",
                                                 bits_per_count=args.count_width,
                                                 device_id=local)
    stream = torch.cuda.current_stream(device).cuda_stream
    comm = None
    if world > 1:
        uid = share_comm_id(rank, boss.Comm.unique_id)
        comm = boss.Comm.rccl(uid, world, rank, local)

    def step():
        return ctor.build_device(seq.data_ptr(), seq.numel(), stream=stream, comm=comm)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    timings = []
    for _ in range(args.steps):
        dc = step()
        timings.append(ctor.timings().as_dict())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0, world, device)
    kmers_per_rank = args.reads * (args.read_len - args.k + 1)
    value = job_throughput(kmers_per_rank, world, args.steps, elapsed)
    last = timings[-1]
    # size-independent sanity of the result
    assert dc.n == last["n_rows"] and dc.n == 1 + dc.n_real + dc.n_dummy
    assert dc.F[4] <= dc.n - 1

    # roofline of the sort's partition pass (the radix-pass target is judged on
    # K2): the sort's first stand-alone MSD partition launch (level 2; level 1 is fused into K1)
    # reads and scatters every extracted k-mer once, 2 * N * 8 algorithmic bytes; its duration
    # comes from HIP events on the build stream
    pass_ms = sum(t["radix_pass_ms"] for t in timings) / len(timings)
    pass_bytes = last["radix_bytes"]
    achieved = pass_bytes / (pass_ms * 1e-3) / 1e9 if pass_ms > 0 else 0.0
    traffic = None
    prof = os.path.join(ROOT, "profiles", "r1_partition_traffic.json")
    if os.path.exists(prof):
        try:
            traffic = json.load(open(prof)).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    result = {
        "metric": "k-mers/s ingested into BOSS (k=31, 150 bp reads)",
        "value": value,
        "unit": "k-mers/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (%s-sampled %d bp reads, %gx coverage, seeded per rank)"
                % (args.data, args.read_len, args.coverage),
        "config": {"workload": "metagraph build -k %d --mode %s%s, %d synthetic %d bp reads per GPU"
                               % (args.k, args.mode,
                                  " --count-kmers --count-width %d" % args.count_width
                                  if args.count_width else "", args.reads, args.read_len),
                   "k": args.k, "reads_per_gpu": args.reads, "read_len": args.read_len,
                   "key": "KMerBOSS<uint64_t,2>" if 2 * args.k <= 64 else
                          "KMerBOSS<uint128_t,2>" if 2 * args.k <= 128 else "KMerBOSS<uint256_t,2>",
                   "parallelism": ("range-partitioned build over %d GPUs (RCCL all-to-all)"
                                   % world) if world > 1 else "single"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "msd_partition_kernel (K2 level-2 MSD partition pass; level 1 runs "
                               "inside the fused K1 extract_partition_kernel)",
                     "pass_ms": pass_ms, "bytes_per_launch": pass_bytes},
        "stages_ms": {k2: last[k2] for k2 in ("extract_ms", "sort_ms", "unique_ms", "rc_ms",
                                              "dummy_ms", "merge_ms", "emit_ms", "total_ms")},
        "counts": {k2: last[k2] for k2 in ("n_extracted", "n_unique", "n_real", "n_dummy",
                                           "n_rows", "radix_launches", "n_sent")},
        "exchange_ms": last["exchange_ms"],
    }
    if rank == 0 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, kb)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        del comm
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
