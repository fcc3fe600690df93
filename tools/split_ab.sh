# gemm_pf2_k split-K: parity, then narrow-output routes at 24..256 rows (row-group GEMV vs gemm_pf2_k with / without split)
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "pf2 or skinny or gemm" > gpurun_out/split_t.log 2>&1
export QT_PB_M=24,48,80,112,160,200,256,680
for d in 1.7b 0.6b; do
QT_PB_DIMS=$d QT_SKINNY=1 timeout -k 10 300 python tools/prefill_gemm_bench.py > gpurun_out/spl_rule_$d.log 2>&1
QT_PB_DIMS=$d QT_GEMV_MAX_M=16 QT_IGEMM_MIN_M=17 QT_SK=0 QT_SKINNY=0 timeout -k 10 300 python tools/prefill_gemm_bench.py > gpurun_out/spl_pf2_$d.log 2>&1
QT_PB_DIMS=$d QT_GEMV_MAX_M=16 QT_IGEMM_MIN_M=17 QT_SK=0 QT_SKINNY=0 QT_PF2_SPLIT=0 timeout -k 10 300 python tools/prefill_gemm_bench.py > gpurun_out/spl_pf2ns_$d.log 2>&1
done
