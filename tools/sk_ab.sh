# skinny GEMM routes at 17..256 rows: row-group GEMV (default before gemm_sk), gemm_sk_k, gemm_pf2_k forced
set -e
export QT_PB_M=24,48,80,112,160,200,256
for d in 1.7b 0.6b; do
QT_PB_DIMS=$d QT_SK=0 timeout -k 10 300 python tools/prefill_gemm_bench.py > gpurun_out/skr_gemv_$d.log 2>&1
QT_PB_DIMS=$d QT_SK=1 timeout -k 10 300 python tools/prefill_gemm_bench.py > gpurun_out/skr_sk_$d.log 2>&1
QT_PB_DIMS=$d QT_SK=0 QT_GEMV_MAX_M=16 QT_IGEMM_MIN_M=17 timeout -k 10 300 python tools/prefill_gemm_bench.py > gpurun_out/skr_pf2_$d.log 2>&1
done
