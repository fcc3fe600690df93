# decode GEMV fold / row groups: kernel tests under each setting, then cold timings
set -e
for cfg in "QT_GEMV_RG=0" "QT_GEMV_RG=2" "QT_GEMV_FOLD=2"; do
  env $cfg timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "gemm or gemv or swiglu" > gpurun_out/tl.log 2>&1
  echo "== $cfg $(tail -1 gpurun_out/tl.log)" >> gpurun_out/rg.log
  env $cfg QT_HC_COLD_ONLY=1 timeout -k 10 200 python tools/gemv_hot_cold.py 2>&1 | grep "us/launch" >> gpurun_out/rg.log
done
QT_GEMV_RG=2 QT_HC_SPLITK=1 QT_HC_COLD_ONLY=1 timeout -k 10 200 python tools/gemv_hot_cold.py 2>&1 | grep "us/launch" | sed 's/^/RG2-nosplit /' >> gpurun_out/rg.log
