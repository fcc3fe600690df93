# GPU parity suite then a short bench (no CPU baseline / roofline); used while iterating
set -e
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
timeout -k 10 400 python bench.py --cpu-baseline 0 --roofline 0 "$@" > gpurun_out/bench.log 2>&1
