# decode-GEMV overhead attribution: QT_GEMV_DBG 1 = no A loads, 2 = no MFMA; split-K auto vs off
set -e
for cfg in "QT_GEMV_DBG=0" "QT_GEMV_DBG=1" "QT_GEMV_DBG=3" "QT_GEMV_DBG=0 QT_HC_SPLITK=1" "QT_GEMV_DBG=1 QT_HC_SPLITK=1"; do
  echo "== $cfg" >> gpurun_out/dbg.log
  env $cfg QT_HC_COLD_ONLY=1 timeout -k 10 200 python tools/gemv_hot_cold.py 2>&1 | grep "us/launch" >> gpurun_out/dbg.log
done
