# gemv_lds (A staged in LDS) vs gemv_wt: kernel tests under the switch, then hot/cold GEMV timings for both
set -e
QT_GEMV_LDS=1 timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "gemm or gemv or swiglu" > gpurun_out/tl.log 2>&1
QT_GEMV_LDS=0 timeout -k 10 300 python tools/gemv_hot_cold.py > gpurun_out/hc0.log 2>&1
QT_GEMV_LDS=1 timeout -k 10 300 python tools/gemv_hot_cold.py > gpurun_out/hc1.log 2>&1
