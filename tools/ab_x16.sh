#!/bin/bash
# A/B of the bf16 residual shadow (QT_X16) on one box: bench (no CPU baseline) + rocprof kernel stats of each arm
set -e
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
for v in 1 0 1 0; do
  QT_X16=$v timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline 0 --steps 3 > gpurun_out/ab_x16_$v.log 2>&1
  echo "x16=$v $(tail -1 gpurun_out/ab_x16_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/ab_x16.txt
done
for v in 1 0; do
  QT_X16=$v timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_x16_$v -o run -- python3 bench.py --cpu-baseline 0 --roofline 0 --steps 2 --warmup 1 > gpurun_out/prof_x16_$v.log 2>&1
  tr=$(find gpurun_out/prof_x16_$v -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_summary.py "$tr" gpurun_out/prof_x16_$v/summary.txt
  find gpurun_out/prof_x16_$v -name "*kernel_trace*" -delete
done
