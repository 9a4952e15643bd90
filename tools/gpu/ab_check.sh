#!/bin/bash
# A/B of prebuilt library variants with a parity gate: each ab/<variant>/libmtg_boss.so first runs
# the 2 M-read bench-generator parity tests (default MSD plan vs the oracle), then the default bench
# twice, interleaved with the other variants.  Usage: tools/gpu/ab_check.sh <tag> <variant>...
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
LIB=projects2014-metagenome_amd/libmtg_boss.so
for v in "$@"; do
  cp ab/$v/libmtg_boss.so $LIB || exit 1
  timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "bench_generator" > $OUT/$v.pytest.log 2>&1
  rc=$?; echo "$v parity rc=$rc $(tail -1 $OUT/$v.pytest.log)"; [ $rc -ne 0 ] && exit $rc
done
for rep in 1 2; do
  for v in "$@"; do
    cp ab/$v/libmtg_boss.so $LIB || exit 1
    timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-steps 0 > $OUT/$v.$rep.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/$v.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.2f ms' % d['ms_per_step'], {k: round(v, 2) for k, v in d['stages_ms'].items()}, 'pass %.3f' % d['roofline']['pass_ms'])" $OUT/$v.$rep.log $v
  done
done
