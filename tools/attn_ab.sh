set -e
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
QT_ATTN_SHORT=0 timeout -k 10 300 python tools/microbench.py 2>&1 | grep attention > gpurun_out/attn.log
QT_ATTN_SHORT=1 timeout -k 10 300 python tools/microbench.py 2>&1 | grep "L=17" | sed 's/^/short4 /' >> gpurun_out/attn.log
timeout -k 10 400 python bench.py --cpu-baseline 0 --roofline 0 > gpurun_out/bench.log 2>&1
