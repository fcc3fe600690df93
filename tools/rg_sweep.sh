set -e
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
for g in 1 2 4; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline 0 --row-groups $g > gpurun_out/bench_g$g.log 2>&1
done
