set -e
mkdir -p gpurun_out/fb
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "alternate or fused" > gpurun_out/fb/pytest.log 2>&1
for b in 1024 512 256; do
  MTG_FUSED_BLOCK=$b timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/fb/bench_$b.log 2>&1
done
