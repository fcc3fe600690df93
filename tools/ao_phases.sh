# qt_decode_attn_oproj phase timing (QT_AO_STOP = end after phase n) on the code-predictor layer microbench
set -e
for st in 1 2 3 4 0; do
  QT_AO_STOP=$st timeout -k 10 120 python tools/cp_layer_bench.py 2>&1 | grep "fused attention" | sed "s/^/stop=$st /" >> gpurun_out/${AOPH_OUT:-aoph.txt}
done
