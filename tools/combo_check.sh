set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cc_t.log 2>&1
timeout -k 10 600 python bench.py --workload vd64 --cpu-baseline 0 --roofline 0 > gpurun_out/cc_vd64.log 2>&1
bash tools/dp_rehearsal.sh
