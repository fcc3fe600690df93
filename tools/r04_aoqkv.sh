# fused q/k/v + head-split attention + o_proj: parity tests, layer microbench (10 / 17 keys), phase timing, bench A/B
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "attn_oproj" > gpurun_out/aoqkv_tests.txt 2>&1
QT_CPL_KEYS=10 timeout -k 10 240 python tools/cp_layer_bench.py > gpurun_out/aoqkv_cpl10.txt 2>&1
timeout -k 10 240 python tools/cp_layer_bench.py > gpurun_out/aoqkv_cpl17.txt 2>&1
if [ -n "$AOQKV_FULL" ]; then
  QT_AO_QKV=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py -x -q -s -m gpu --timeout 300 --timeout-method thread -k "bf16_teacher_forced and (cv17_b8 or cv06)" > gpurun_out/aoqkv_full.txt 2>&1
  QT_AO_QKV=0 timeout -k 10 600 python bench.py > gpurun_out/aoqkv_bench0.json 2>/dev/null
  QT_AO_QKV=1 timeout -k 10 600 python bench.py > gpurun_out/aoqkv_bench1.json 2>/dev/null
fi
