set -e
timeout -k 10 500 python bench.py --cpu-baseline 0 --roofline 0 > gpurun_out/fpb_1.log 2>&1
timeout -k 10 500 python bench.py --cpu-baseline 0 --roofline 0 > gpurun_out/fpb_2.log 2>&1
QT_IM2COL_MAX_M=256 timeout -k 10 500 python bench.py --cpu-baseline 0 --roofline 0 > gpurun_out/fpb_3.log 2>&1
