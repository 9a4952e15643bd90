set -e
mkdir -p gpurun_out/pw
MTG_PART_WIDE_BLOCK=512 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "large or transcripts_k20" > gpurun_out/pw/pytest.log 2>&1
for b in 1024 512; do
  MTG_PART_WIDE_BLOCK=$b timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pw/bench_$b.log 2>&1
done
