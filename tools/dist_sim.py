"""Multi-rank build on ONE GPU (in-process rank group) vs the single build of the same reads.

    python tools/dist_sim.py --ranks 2 --reads 5000000

Each of P ranks holds --reads reads sampled from one shared genome (10x over all P ranks), as in
bench.py --gpus P.  The P ranks share the device, so the wall time is roughly the SUM of their
work; comparing it with one single-GPU build of all P * reads reads gives the work the
distributed algorithm adds (exchanges here are device copies, not xGMI).
"""
import argparse
import importlib
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--reads", type=int, default=5_000_000)
    ap.add_argument("--k", type=int, default=31)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--no-single", action="store_true", help="skip the single build (profiling the ranks only)")
    ap.add_argument("--serial", action="store_true",
                    help="one rank owns the device at a time (MTG_LOCAL_SERIAL): the step is the SUM of the "
                         "ranks' work, and each rank's device time is measured alone")
    ap.add_argument("--only-single", action="store_true", help="the single build only (its kernel profile)")
    ap.add_argument("--pieces", type=int, default=None,
                    help="exchange-1 pieces of the routed collect (MTG_DIST_PIECES; default: the library's)")
    ap.add_argument("--collect", default=None, choices=["routed", "superkmer", "local"],
                    help="the multi-GPU collect (MTG_DIST_COLLECT; default: the library's)")
    args = ap.parse_args()
    import torch
    boss = importlib.import_module("projects2014-metagenome_amd.boss")
    dev = torch.device("cuda", 0)
    P = args.ranks
    seqs = [bench.make_reads_device(torch, args.reads, 150, 1000 + r, "genome", 10.0, dev, P)
            for r in range(P)]
    whole = torch.cat(seqs)
    torch.cuda.synchronize()
    kb = args.k - 1
    t_single, ts, rows_single = 0.0, {}, None
    if not args.no_single:
        single = boss.IBOSSChunkConstructor.initialize(kb, both_strands=True)
        for _ in range(2):
            single.build_device(whole.data_ptr(), whole.numel())
        t0 = time.perf_counter()
        for _ in range(args.steps):
            dc = single.build_device(whole.data_ptr(), whole.numel())
        t_single = (time.perf_counter() - t0) / args.steps
        ts = single.timings().as_dict()
        rows_single = dc.n
    if args.only_single:
        print(json.dumps({"single_ms": t_single * 1e3, "rows": rows_single}))
        return

    if args.serial:
        os.environ["MTG_LOCAL_SERIAL"] = "1"
    if args.pieces:
        os.environ["MTG_DIST_PIECES"] = str(args.pieces)
    if args.collect and args.collect != "routed":
        os.environ["MTG_DIST_COLLECT"] = args.collect
    comms = boss.Comm.local_group(P)
    ctors = [boss.IBOSSChunkConstructor.initialize(kb, both_strands=True) for _ in range(P)]
    res = [None] * P

    def run(r):
        res[r] = ctors[r].build_device(seqs[r].data_ptr(), seqs[r].numel(), comm=comms[r])

    def step():
        th = [threading.Thread(target=run, args=(r,)) for r in range(P)]
        for t in th:
            t.start()
        for t in th:
            t.join()

    step()
    step()
    for cm in comms:
        cm.held_ms(reset=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t_dist = (time.perf_counter() - t0) / args.steps
    rows_dist = sum(c.n for c in res) - (P - 1)
    assert rows_single is None or rows_dist == rows_single, (rows_dist, rows_single)
    per_rank = [c.timings().as_dict() for c in ctors]
    held = [cm.held_ms() / args.steps for cm in comms]
    keys = ("extract_ms", "sort_ms", "unique_ms", "rc_ms", "dummy_ms", "merge_ms", "emit_ms",
            "total_ms", "exchange_ms", "exchange_hidden_ms")
    print(json.dumps({
        "ranks": P, "reads_per_rank": args.reads, "rows": rows_single,
        "single_ms": t_single * 1e3, "dist_wall_ms": t_dist * 1e3, "serial": args.serial,
        # serial mode: each rank's device time alone; work ratio = their sum / the single build, and
        # the weak-scaling estimate P * single(P reads) / (P * max rank) = P / (P * max / single)
        "rank_held_ms": [round(h, 2) for h in held] if args.serial else None,
        "work_ratio": round(sum(held) / (t_single * 1e3), 3) if args.serial and t_single else None,
        "max_rank_ratio": round(P * max(held) / (t_single * 1e3), 3) if args.serial and t_single else None,
        "single_stages": {k: round(ts[k], 2) for k in keys if k in ts},
        "rank_stages": [{k: round(t[k], 2) for k in keys} for t in per_rank],
        "pieces": os.environ.get("MTG_DIST_PIECES", "default"),
        "n_sent": [t["n_sent"] for t in per_rank],
        "sent_bytes": [t["sent_bytes"] for t in per_rank],
        "n_real": [t["n_real"] for t in per_rank],
    }, indent=1))


if __name__ == "__main__":
    main()
