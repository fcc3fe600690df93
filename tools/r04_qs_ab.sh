# head-split attn_oproj: one wave per q head (QT_AO_QS=2) vs both q heads in a wave (QT_AO_QS=1):
# parity tests on the default, phase timings and the layer microbench for both, every GPU step time-limited, chained.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "attn_oproj" > gpurun_out/qs_tests.txt 2>&1
for q in 1 2; do
  QT_AO_QS=$q AOPH_OUT=aoph_qs$q.txt bash tools/ao_phases.sh
  QT_AO_QS=$q QT_CPL_KEYS=10 timeout -k 10 240 python tools/cp_layer_bench.py > gpurun_out/cpl10_qs$q.txt 2>&1
  QT_AO_QS=$q timeout -k 10 240 python tools/cp_layer_bench.py > gpurun_out/cpl17_qs$q.txt 2>&1
done
