# HALF (paired k tiles share the activation fetch) vs the plain decode GEMV: kernel tests, then cold timings
set -e
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "gemm or gemv or swiglu or oproj" > gpurun_out/tl.log 2>&1
for h in 0 1; do
  echo "== QT_GEMV_HALF=$h" >> gpurun_out/half.log
  QT_GEMV_HALF=$h QT_HC_COLD_ONLY=1 timeout -k 10 200 python tools/gemv_hot_cold.py 2>&1 | grep "us/launch" >> gpurun_out/half.log
done
