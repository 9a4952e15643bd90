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


# BASELINE.json configs this bench runs (configs[1] is the default line; configs[2] is the
# k=63 / 100 M-read u128 build that does not fit HBM in one pass and runs in key ranges)
CONFIGS = {
    "cfg2": {"k": 31, "reads": 10_000_000},
    "cfg3": {"k": 63, "reads": 100_000_000, "host_steps": 0, "cpu_sample_reads": 5_000_000,
             "steps": 2, "warmup": 1},
    # configs[3]: k=31, 1 B reads over 8 GPUs = 125 M reads per GPU on one shared genome (10x over
    # all ranks' reads); one share does not fit one pass, so every rank collects in key batches
    "cfg4": {"k": 31, "reads": 125_000_000, "host_steps": 0, "fasta_reads": 0,
             "cpu_sample_reads": 5_000_000, "steps": 2, "warmup": 1},
    # configs[4]: --count-kmers (SortedMultiset<uint8_t> saturating merge, 8-bit weights) on a KMC1
    # database of the canonical k=31 counts of every rank's reads (written by the builder's own GPU
    # counter, untimed), decoded into HBM before the timed region; across ranks the records of one
    # k-mer meet at its owner and their counts add (the count-aggregating merge)
    "cfg5": {"k": 31, "reads": 10_000_000, "count_width": 8, "fasta_reads": 0, "kmc": True},
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=sorted(CONFIGS), default=None,
                    help="a BASELINE config preset (explicit flags still override)")
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
    ap.add_argument("--host-steps", type=int, default=3,
                    help="steps of the host-buffer leg (0 = skip)")
    ap.add_argument("--fasta-reads", type=int, default=2_000_000,
                    help="reads of the FASTA-file leg (0 = skip)")
    ap.add_argument("--kmc", action="store_true",
                    help="build from a KMC1 database of the reads' canonical k-mer counts (configs[4])")
    ap.add_argument("--parity-full-max", type=int, default=10_000_000,
                    help="largest read count whose whole workload the bench checks against the oracle")
    ap.add_argument("--launch-timeout", type=float, default=None,
                    help="seconds the ranks started by --gpus N (no launcher) may run before they are killed "
                         "(default: 900 s + 10 s per step)")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check on the CPU: every rank joins a gloo group and rank 0 prints the "
                         "world it saw (no GPU, no build)")
    args = ap.parse_args()
    if args.config:
        given = {a.split("=")[0].lstrip("-").replace("-", "_") for a in sys.argv[1:] if a.startswith("--")}
        for key, val in CONFIGS[args.config].items():
            if key not in given:
                setattr(args, key, val)
    return args


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


def make_reads_host_codes(n_reads, read_len, seed, data, coverage):
    """The same generator family on the host (numpy): ASCII reads as an (n_reads, read_len) array."""
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
    return lut[codes]


def make_reads_host(n_reads, read_len, seed, data, coverage):
    asc = make_reads_host_codes(n_reads, read_len, seed, data, coverage)
    return [asc[i].tobytes() for i in range(n_reads)]


def cpu_threads():
    """OpenMP threads the oracle runs on (OMP_NUM_THREADS, else this process's CPU set)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def cpu_baseline(args, kb, boss):
    """Oracle (C restatement: OpenMP extraction + parallel LSD radix sort, serial dummy and
    emission passes) on a bounded sample of the same workload.  The same sample is then built on
    the GPU through the host C ABI and compared with the oracle's chunk bit for bit (W, last, F,
    weights): the `parity` field of the bench line."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle_ctypes
    asc = make_reads_host_codes(args.cpu_sample_reads, args.read_len, 12345, args.data,
                                args.coverage)
    reads = [asc[i].tobytes() for i in range(len(asc))]
    canonical = args.mode == "canonical"
    t0 = time.perf_counter()
    c = oracle_ctypes.build_chunk(kb, reads, canonical=canonical, bits_per_count=args.count_width)
    dt = time.perf_counter() - t0
    n = args.cpu_sample_reads * (args.read_len - args.k + 1)
    base = {"value": n / dt, "unit": "k-mers/s", "cores": cpu_threads(), "kind": "port",
            "sample": "%d synthetic %d bp reads (%s, %gx coverage), k=%d %s, %.1f s, %d rows"
                      % (args.cpu_sample_reads, args.read_len, args.data, args.coverage,
                         args.k, args.mode, dt, len(c.W))}
    ctor = boss.IBOSSChunkConstructor.initialize(kb, both_strands=canonical,
                                                 bits_per_count=args.count_width,
                                                 num_threads=cpu_threads())
    ctor.add_packed(asc.reshape(-1), np.arange(len(asc) + 1, dtype=np.uint64) * args.read_len)
    g = ctor.build_chunk()
    same = (len(g.W) == len(c.W) and np.array_equal(g.W, c.W) and np.array_equal(g.last, c.last)
            and np.array_equal(g.F, c.F) and
            (c.weights is None if g.weights is None else np.array_equal(g.weights, c.weights)))
    parity = {"ok": bool(same), "rows": int(len(c.W)),
              "what": "GPU build (host C ABI) of the cpu_baseline sample vs the oracle: W, last, F, "
                      "weights bit for bit"}
    return base, parity


def full_parity(args, kb, boss, dc, seq):
    """The bench's own workload, whole: the device chunk of the last timed step against the oracle
    built from all of this rank's reads (W, last, F, weights bit for bit).  Single-GPU lines only."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle_ctypes
    L = boss.lib()
    W = np.empty(dc.n, dtype=np.uint8)
    last = np.empty(dc.n, dtype=np.uint8)
    L.mtg_memcpy_d2h(W.ctypes.data, dc.W, dc.n)
    L.mtg_memcpy_d2h(last.ctypes.data, dc.last, dc.n)
    wt = None
    if args.count_width:
        wt = np.empty(dc.n, dtype=np.uint32)
        L.mtg_memcpy_d2h(wt.ctypes.data, dc.weights, dc.n * 4)
    F = np.array([int(f) for f in dc.F], dtype=np.uint64)
    host = seq.cpu().numpy()  # the reads with their '$' separators
    stride = args.read_len + 1
    t0 = time.perf_counter()
    c = oracle_ctypes.build_chunk_packed(kb, host, np.arange(args.reads + 1, dtype=np.uint64) * stride,
                                         canonical=args.mode == "canonical", bits_per_count=args.count_width)
    dt = time.perf_counter() - t0
    same = (len(W) == len(c.W) and np.array_equal(W, c.W) and np.array_equal(last, c.last)
            and np.array_equal(F, c.F) and (wt is None or np.array_equal(wt, c.weights)))
    return {"ok": bool(same), "rows": int(len(c.W)), "oracle_s": dt,
            "what": "the timed step's device chunk (all %d reads of the workload) vs the oracle on the same "
                    "reads: W, last, F, weights bit for bit" % args.reads}


def cpu_baseline_kmc(args, kb, boss, kmc_base, n_records):
    """configs[4]'s CPU baseline: the oracle on a bounded sample of the KMC database's records (the
    first `cpu_sample_reads`, each one k-mer with its count, as the reference's KMC branch feeds
    them, cli/parse_sequences.hpp:50-101); the same sample through the GPU's host C ABI is the
    parity check."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import kmc_oracle
    import oracle_ctypes
    canonical = args.mode == "canonical"
    recs = kmc_oracle.read_kmers(kmc_base, not canonical)[:args.cpu_sample_reads]
    seqs = [r for r, _ in recs]
    counts = [c for _, c in recs]
    t0 = time.perf_counter()
    c = oracle_ctypes.build_chunk(kb, seqs, canonical=canonical, bits_per_count=args.count_width,
                                  counts=counts)
    dt = time.perf_counter() - t0
    base = {"value": len(seqs) / dt, "unit": "k-mers/s", "cores": cpu_threads(), "kind": "port",
            "sample": "the first %d of %d KMC records (k=%d counts of %d reads), %s, %.1f s, %d rows"
                      % (len(seqs), n_records, args.k, args.reads, args.mode, dt, len(c.W))}
    ctor = boss.IBOSSChunkConstructor.initialize(kb, both_strands=canonical,
                                                 bits_per_count=args.count_width,
                                                 num_threads=cpu_threads())
    ctor.add_sequences(seqs, counts)
    g = ctor.build_chunk()
    same = (len(g.W) == len(c.W) and np.array_equal(g.W, c.W) and np.array_equal(g.last, c.last)
            and np.array_equal(g.F, c.F) and np.array_equal(g.weights, c.weights))
    parity = {"ok": bool(same), "rows": int(len(c.W)),
              "what": "GPU build (host C ABI) of the cpu_baseline record sample vs the oracle: W, last, "
                      "F, weights bit for bit"}
    return base, parity


def full_parity_kmc(args, kb, boss, dc, dreads):
    """configs[4]'s whole workload: the device chunk of the last timed step against the oracle built
    from every decoded KMC record of this rank's database (each record one k-mer with its count, as
    the reference's KMC branch feeds them: cli/parse_sequences.hpp:50-101, kmc_parser.cpp:27-62),
    W, last, F, weights bit for bit.  Single-GPU lines only."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle_ctypes
    L = boss.lib()
    W = np.empty(dc.n, dtype=np.uint8)
    last = np.empty(dc.n, dtype=np.uint8)
    wt = np.empty(dc.n, dtype=np.uint32)
    L.mtg_memcpy_d2h(W.ctypes.data, dc.W, dc.n)
    L.mtg_memcpy_d2h(last.ctypes.data, dc.last, dc.n)
    L.mtg_memcpy_d2h(wt.ctypes.data, dc.weights, dc.n * 4)
    F = np.array([int(f) for f in dc.F], dtype=np.uint64)
    n = dreads.n_reads
    seq = np.empty(dreads.seq_len, dtype=np.uint8)
    starts = np.empty(n + 1, dtype=np.uint64)
    counts = np.empty(n, dtype=np.uint32)
    L.mtg_memcpy_d2h(seq.ctypes.data, dreads.seq, dreads.seq_len)
    L.mtg_memcpy_d2h(starts.ctypes.data, dreads.read_starts, n * 8)
    L.mtg_memcpy_d2h(counts.ctypes.data, dreads.counts, n * 4)
    starts[n] = dreads.seq_len
    t0 = time.perf_counter()
    c = oracle_ctypes.build_chunk_packed(kb, seq, starts, canonical=args.mode == "canonical",
                                         bits_per_count=args.count_width, counts=counts)
    dt = time.perf_counter() - t0
    same = (len(W) == len(c.W) and np.array_equal(W, c.W) and np.array_equal(last, c.last)
            and np.array_equal(F, c.F) and np.array_equal(wt, c.weights))
    return {"ok": bool(same), "rows": int(len(c.W)), "records": int(n), "oracle_s": dt,
            "what": "the timed step's device chunk (all %d decoded KMC records of the workload) vs the oracle on "
                    "the same records and counts: W, last, F, weights bit for bit" % n}


def kmc_path(args, kb, boss, kmc_base, steps, n_records):
    """configs[4] from the database file: add_kmc (both files read into host memory) + build_chunk
    (records decoded on the device, the device path, host arrays out) -- the PCIe-inclusive rate."""
    canonical = args.mode == "canonical"
    ctor = boss.IBOSSChunkConstructor.initialize(kb, both_strands=canonical,
                                                 bits_per_count=args.count_width,
                                                 num_threads=cpu_threads())
    rows = []
    for it in range(steps + 1):  # the first build sizes the buffers (untimed)
        t0 = time.perf_counter()
        ctor.add_kmc(kmc_base)
        t1 = time.perf_counter()
        ch = ctor.build_chunk()
        dt = time.perf_counter() - t0
        t = ctor.timings()
        if it:
            rows.append((dt, t1 - t0, t.input_ms, t.total_ms, t.d2h_ms, t.host_total_ms))
        del ch
    m = [sum(r[i] for r in rows) / len(rows) for i in range(6)]
    return {"value": n_records / m[0], "unit": "k-mers/s", "ms_per_step": m[0] * 1e3,
            "stages_ms": {"read_files": m[1] * 1e3, "h2d_and_decode_on_device": m[2],
                          "device_path": m[3], "d2h_W_last_weights": m[4], "build_chunk_call": m[5]},
            "steps": steps, "what": "add_kmc + build_chunk through the C ABI, host arrays out"}


def host_path(args, kb, boss, seq, steps):
    """extract-start -> Chunk arrays on the HOST.  The bench's reads
    (copied to host memory once, outside the timing) go through the reference's interface:
    add_packed (staging into pinned memory, num_threads host threads), then build_chunk (one H2D
    of the reads, the device path, D2H of W / packed last / weights into pinned blocks)."""
    import numpy as np
    L = args.read_len
    host = seq.view(-1, L + 1)[:, :L].contiguous().cpu().numpy()
    n_reads = host.shape[0]
    offsets = np.arange(n_reads + 1, dtype=np.uint64) * L
    flat = host.reshape(-1)
    ctor = boss.IBOSSChunkConstructor.initialize(kb, both_strands=args.mode == "canonical",
                                                 bits_per_count=args.count_width,
                                                 num_threads=cpu_threads())
    rows = []
    for it in range(steps + 1):  # the first build sizes the pinned buffers (untimed)
        t0 = time.perf_counter()
        ctor.add_packed(flat, offsets)
        ch = ctor.build_chunk()
        dt = time.perf_counter() - t0
        t = ctor.timings()
        if it:
            rows.append((dt, t.stage_ms, t.h2d_ms, t.total_ms, t.d2h_ms, t.host_total_ms))
        del ch
    m = [sum(r[i] for r in rows) / len(rows) for i in range(6)]
    kmers = n_reads * (L - args.k + 1)
    return {"value": kmers / m[0], "unit": "k-mers/s", "ms_per_step": m[0] * 1e3,
            "stages_ms": {"stage_into_pinned": m[1], "h2d_reads": m[2], "device_path": m[3],
                          "d2h_W_last_weights": m[4], "build_chunk_call": m[5]},
            "steps": steps, "staging_threads": cpu_threads(),
            "what": "add_packed + build_chunk through the C ABI on the same reads, host arrays out"}


def fasta_path(args, kb, boss, steps, n_reads, files=8):
    """SURVEY.md section 8(d)(ii), end to end from FASTA files: a sample of the same generator
    written as `files` FASTA shards (60-column lines) to a temp dir (untimed), then per step
    add_fasta on one host thread per shard (read into pinned memory) + build_chunk (one H2D of
    the raw bytes, records split on the device, the device path, host arrays out)."""
    import shutil
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    asc = make_reads_host_codes(n_reads, args.read_len, 4321, args.data, args.coverage)
    tmp = tempfile.mkdtemp(prefix="mtg_fa_")
    paths, nbytes = [], 0
    try:
        for f in range(files):
            p = os.path.join(tmp, "reads_%03d.fa" % f)
            with open(p, "wb") as out:
                for i in range(f, n_reads, files):
                    r = asc[i].tobytes()
                    out.write(b">r%d\n" % i)
                    for j in range(0, len(r), 60):
                        out.write(r[j:j + 60] + b"\n")
            nbytes += os.path.getsize(p)
            paths.append(p)
        ctor = boss.IBOSSChunkConstructor.initialize(kb, both_strands=args.mode == "canonical",
                                                     bits_per_count=args.count_width)
        rows = []
        with ThreadPoolExecutor(max_workers=files) as ex:
            for it in range(steps + 1):  # the first build sizes the buffers (untimed)
                t0 = time.perf_counter()
                list(ex.map(ctor.add_fasta, paths))
                t1 = time.perf_counter()
                ch = ctor.build_chunk()
                dt = time.perf_counter() - t0
                t = ctor.timings()
                if it:
                    rows.append((dt, t1 - t0, t.input_ms, t.total_ms, t.d2h_ms, t.host_total_ms))
                del ch
        m = [sum(r[i] for r in rows) / len(rows) for i in range(6)]
        kmers = n_reads * (args.read_len - args.k + 1)
        return {"value": kmers / m[0], "unit": "k-mers/s", "ms_per_step": m[0] * 1e3,
                "fasta_gb_per_s": nbytes / m[0] / 1e9,
                "stages_ms": {"read_files_into_pinned": m[1] * 1e3, "h2d_and_split_on_device": m[2],
                              "device_path": m[3], "d2h_W_last_weights": m[4], "build_chunk_call": m[5]},
                "sample": "%d reads in %d FASTA files, %.0f MB" % (n_reads, files, nbytes / 1e6),
                "steps": steps}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def measured_copy_peak(torch, boss, device, nbytes=4 << 30, reps=10):
    """Achievable HBM bandwidth on this GPU: the library's copy kernel (mtg_device_copy: one 16-byte
    nontemporal load + store per thread, 6.44 TB/s on the MI355X in tools/copy_bench.hip, which compares
    copy shapes; profiles/r6_copy_bench.txt) over `nbytes` (read + write), timed with HIP events on
    torch's current stream; the second roofline denominator BASELINE.md asks for (the best of torch's
    copy_ and that kernel)."""
    src = torch.empty(nbytes, dtype=torch.uint8, device=device)
    dst = torch.empty_like(src)
    src.fill_(1)
    stream = torch.cuda.current_stream(device)
    best = 0.0
    for how in ("kernel", "torch"):
        def once():
            if how == "kernel":
                rc = boss.lib().mtg_device_copy(dst.data_ptr(), src.data_ptr(), nbytes, stream.cuda_stream)
                assert rc == 0
            else:
                dst.copy_(src)
        once()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            once()
        e1.record(stream)
        torch.cuda.synchronize()
        best = max(best, 2.0 * nbytes / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9)
    del src, dst
    torch.cuda.empty_cache()
    return best


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


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv=None, timeout=None):
    """`bench.py --gpus N` without a launcher: start N fresh child processes of this script, one
    per GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, before this process
    makes any GPU call (the parent never imports torch).  Rank 0's stdout is the bench line; the
    parent waits for all ranks and returns non-zero if any rank failed (the others are stopped)."""
    import subprocess
    argv = sys.argv[1:] if argv is None else argv
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    t0 = time.time()
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                sys.stderr.write("bench.py: rank %d exited with %d; stopping the others\n"
                                 % (procs.index(p), code))
                for q in pending:
                    q.terminate()
        if timeout is not None and time.time() - t0 > timeout and pending:
            sys.stderr.write("bench.py: rank(s) %s still running after %.0f s; killing them\n"
                             % (", ".join(str(procs.index(q)) for q in pending), timeout))
            for q in pending:
                q.kill()
            for q in pending:
                q.wait()
            pending = []
            rc = 124
        time.sleep(0.05)
    return rc


def dry_run(args, world, rank):
    """The launcher's CPU check: a gloo group of `world` ranks; rank 0 prints what every rank saw."""
    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    seen = [(rank, world)]
    if world > 1:
        seen = [None] * world
        dist.all_gather_object(seen, (rank, world))
    elapsed = max_over_ranks(0.001 * (rank + 1), world, torch.device("cpu"))
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks": seen, "max_elapsed_s": elapsed}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        limit = args.launch_timeout if args.launch_timeout else 900.0 + 10.0 * (args.steps + args.warmup)
        sys.exit(launch_ranks(args.gpus, timeout=limit))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.stderr.write("bench.py: --gpus %d but WORLD_SIZE=%d (one rank per GPU)\n" % (args.gpus, world))
        sys.exit(2)
    if args.dry_run:
        return dry_run(args, world, rank)
    import torch
    import torch.distributed as dist

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
    torch.cuda.empty_cache()  # the genome and the generator's temporaries (the library allocates itself)
    ctor = boss.IBOSSChunkConstructor.initialize(kb, both_strands=args.mode == "canonical",
                                                 bits_per_count=args.count_width,
                                                 device_id=local, num_threads=cpu_threads())
    stream = torch.cuda.current_stream(device).cuda_stream
    comm = None
    if world > 1:
        uid = share_comm_id(rank, boss.Comm.unique_id)
        comm = boss.Comm.rccl(uid, world, rank, local)

    kmers_per_rank = args.reads * (args.read_len - args.k + 1)
    kmc_dir = kmc_base = dreads = None
    if args.kmc:
        # configs[4]'s input: the canonical k-mer counts of this rank's reads as a KMC1 database
        # (GPU counter, untimed), decoded into HBM; one k-mer per record
        import tempfile
        kmc_dir = tempfile.mkdtemp(prefix="mtg_kmc_r%d_" % rank)
        kmc_base = os.path.join(kmc_dir, "reads")
        t0 = time.perf_counter()
        n_records = ctor.write_kmc(seq.data_ptr(), seq.numel(), kmc_base, args.k, canonical=True)
        kmc_write_s = time.perf_counter() - t0
        del seq
        torch.cuda.empty_cache()
        dreads = boss.DeviceReads(kmc_base, call_both_from_canonical=args.mode != "canonical",
                                  device_id=local)
        kmers_per_rank = dreads.n_reads

    # the achievable-copy denominator, measured before the builds fill HBM with the workspace
    copy_peak = measured_copy_peak(torch, boss, device) if rank == 0 else None

    def step():
        if dreads is not None:
            return ctor.build_device(*dreads.build_args(), stream=stream, comm=comm)
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
    ctor.trim()  # idle workspace blocks back to the device before the host legs build on their own
    value = job_throughput(kmers_per_rank, world, args.steps, elapsed)
    last = timings[-1]
    # size-independent sanity of the result
    assert dc.n == last["n_rows"] and dc.n == 1 + dc.n_real + dc.n_dummy
    assert dc.F[4] <= dc.n - 1
    # the rate counts offered windows; every one of them must have been extracted (no N here)
    assert last["n_extracted"] == kmers_per_rank, (last["n_extracted"], kmers_per_rank)

    # roofline of the sort's partition pass (the radix-pass target is judged on
    # K2): the sort's first stand-alone MSD partition launch (level 2; level 1 is fused into K1)
    # reads and scatters every extracted k-mer once, 2 * N * 8 algorithmic bytes; its duration
    # comes from HIP events on the build stream
    pass_ms = sum(t["radix_pass_ms"] for t in timings) / len(timings)
    pass_bytes = last["radix_bytes"]
    achieved = pass_bytes / (pass_ms * 1e-3) / 1e9 if pass_ms > 0 else 0.0
    # traffic: PMC HBM bytes of that launch from the committed rocprofv3 --pmc summary (a stored
    # profile of the same command, not measured in this process)
    traffic, traffic_src = None, None
    default_workload = args.config is None and args.k == 31 and args.reads == 10_000_000 and not args.count_width
    for tag in (("r6", "r5", "r4", "r3", "r2", "r1") if default_workload else ()):  # the stored profile is of the default workload
        prof = os.path.join(ROOT, "profiles", "%s_partition_traffic.json" % tag)
        if os.path.exists(prof):
            try:
                traffic = json.load(open(prof)).get("hbm_bytes_per_launch")
                traffic_src = "profiles/%s_partition_traffic.json (rocprofv3 --pmc, stored)" % tag
                break
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
        "dtype": "u64" if 2 * args.k <= 64 else "u128" if 2 * args.k <= 128 else "u256",
        "data": "synthetic (%s-sampled %d bp reads, %gx coverage, seeded per rank)"
                % (args.data, args.read_len, args.coverage),
        "config": {"workload": ("metagraph build -k %d --mode %s%s, %d synthetic %d bp reads per GPU"
                                % (args.k, args.mode,
                                   " --count-kmers --count-width %d" % args.count_width
                                   if args.count_width else "", args.reads, args.read_len))
                               + (" as a KMC1 database of their canonical %d-mer counts (%d records per GPU)"
                                  % (args.k, kmers_per_rank) if args.kmc else ""),
                   "preset": args.config,
                   "k": args.k, "reads_per_gpu": args.reads, "read_len": args.read_len,
                   "key": "KMerBOSS<uint64_t,2>" if 2 * args.k <= 64 else
                          "KMerBOSS<uint128_t,2>" if 2 * args.k <= 128 else "KMerBOSS<uint256_t,2>",
                   "parallelism": ("range-partitioned build over %d GPUs (RCCL all-to-all)"
                                   % world) if world > 1 else "single"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_src,
                     "peak_measured": copy_peak,
                     "frac_measured": achieved / copy_peak if copy_peak else None,
                     "peak_measured_how": "best of a copy kernel with one 16-byte nontemporal load + store per "
                                          "thread and torch copy_ over 4 GiB (read + write), HIP events",
                     "kernel": "msd_partition_kernel (K2 level-2 MSD partition pass; level 1 runs "
                               "inside the fused K1 extract_partition_kernel)",
                     "pass_ms": pass_ms, "bytes_per_launch": pass_bytes},
        "stages_ms": {k2: last[k2] for k2 in ("extract_ms", "sort_ms", "unique_ms", "rc_ms",
                                              "dummy_ms", "merge_ms", "emit_ms", "total_ms")},
        "counts": {k2: last[k2] for k2 in ("n_extracted", "n_unique", "n_real", "n_dummy",
                                           "n_rows", "radix_launches", "n_sent", "n_batches",
                                           "peak_bytes")},
        "exchange_ms": last["exchange_ms"],
        "sent_bytes": last["sent_bytes"],  # rank 0's bytes to the other ranks in the last step
        "collect_mode": last["collect_mode"],  # 0 one pass, 1 key ranges, 2 canonical rounds
    }
    if args.kmc:
        result["kmc_input"] = {"records_per_gpu": kmers_per_rank, "write_s": kmc_write_s,
                               "what": "GPU k-mer counter -> KMC1 files (untimed), mtg_kmc_load_device -> HBM"}
    if rank == 0 and args.host_steps > 0 and world == 1:
        if args.kmc:
            result["kmc_path"] = kmc_path(args, kb, boss, kmc_base, args.host_steps, kmers_per_rank)
        else:
            result["host_path"] = host_path(args, kb, boss, seq, args.host_steps)
            hp = result["host_path"]
            # SURVEY.md section 8(d)(i) as its own field: extract-start -> BOSS::Chunk arrays on the host,
            # through the reference's interface (add_packed + build_chunk); `value` stays the device-resident rate
            result["hot_path_host_arrays"] = {
                "value": hp["value"], "unit": "k-mers/s", "ms_per_step": hp["ms_per_step"],
                "device_path_ms": hp["stages_ms"]["device_path"],
                "host_legs_ms": hp["ms_per_step"] - hp["stages_ms"]["device_path"],
                "what": "SURVEY.md 8(d)(i): extract-start -> Chunk arrays (W, last, F, weights) on the host, the "
                        "same reads through add_packed + build_chunk (host_path)"}
        if args.fasta_reads > 0:
            result["fasta_path"] = fasta_path(args, kb, boss, args.host_steps, args.fasta_reads)
    if rank == 0 and not args.no_cpu_baseline:
        if args.kmc:
            result["cpu_baseline"], sample_parity = cpu_baseline_kmc(args, kb, boss, kmc_base, kmers_per_rank)
            if world == 1:
                result["parity"] = full_parity_kmc(args, kb, boss, dc, dreads)
                result["parity"]["sample"] = sample_parity
            else:
                result["parity"] = sample_parity
        else:
            result["cpu_baseline"], sample_parity = cpu_baseline(args, kb, boss)
            if world == 1 and args.reads <= args.parity_full_max:
                result["parity"] = full_parity(args, kb, boss, dc, seq)
                result["parity"]["sample"] = sample_parity
            else:
                result["parity"] = sample_parity
    if kmc_dir:
        import shutil
        del dreads
        shutil.rmtree(kmc_dir, ignore_errors=True)
    assert result["n_gpus"] == args.gpus, (result["n_gpus"], args.gpus)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        del comm
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
