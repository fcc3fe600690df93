# head-split attn_oproj with v_dot2 attention: parity tests, phase timing, layer microbench (10 / 17 keys)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "attn_oproj or full_dims or sample_full or talker" > gpurun_out/dot2_tests.txt 2>&1
AOPH_OUT=aoph_dot2.txt bash tools/ao_phases.sh
QT_CPL_KEYS=10 timeout -k 10 240 python tools/cp_layer_bench.py > gpurun_out/cpl10_dot2.txt 2>&1
timeout -k 10 240 python tools/cp_layer_bench.py > gpurun_out/cpl17_dot2.txt 2>&1
if [ -n "$QT_DOT2_BENCH" ]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench_dot2.json 2> gpurun_out/bench_dot2.err
fi
