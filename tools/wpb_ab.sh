set -e
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
timeout -k 10 300 python tools/microbench.py > gpurun_out/mb_auto.log 2>&1
QT_GEMV_WPB=16 timeout -k 10 300 python tools/microbench.py > gpurun_out/mb_16.log 2>&1
QT_GEMV_WPB=4 timeout -k 10 300 python tools/microbench.py > gpurun_out/mb_4.log 2>&1
timeout -k 10 400 python bench.py --cpu-baseline 0 --roofline 0 > gpurun_out/bench.log 2>&1
