# decode GEMV split-K auto vs off (cold weights), after kernel tests
set -e
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "gemm or gemv or swiglu" > gpurun_out/tl.log 2>&1
for sk in 0 1 2 4; do
  echo "== QT_HC_SPLITK=$sk" >> gpurun_out/split.log
  QT_HC_SPLITK=$sk QT_HC_COLD_ONLY=1 timeout -k 10 200 python tools/gemv_hot_cold.py 2>&1 | grep "us/launch" >> gpurun_out/split.log
done
