#!/bin/bash
# first GPU session: parity tests, smoke, small + default bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --reads 1000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_1m.log 2>&1
rc=$?; echo "bench1m rc=$rc"; tail -5 gpurun_out/bench_1m.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench_default.log
exit $rc
