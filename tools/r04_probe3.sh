# Round-4 A/B probe: the prefill GEMM's deep-pipeline variants (QT_PF2_DEEP), then the bench line with the (column
# group, row) and the head-split fused code-predictor attention + o_proj (QT_AO_HS).  set -e: a failing step ends it.
set -e
mkdir -p gpurun_out
QT_PB_M=24,48,96,160,256,680 QT_PF2_DEEP=0 timeout -k 10 300 python tools/prefill_gemm_bench.py > gpurun_out/r04_pf2_deep0.txt 2>&1
QT_PB_M=24,48,96,160,256,680 QT_PF2_DEEP=1 timeout -k 10 300 python tools/prefill_gemm_bench.py > gpurun_out/r04_pf2_deep1.txt 2>&1
timeout -k 10 600 python bench.py --cpu-baseline 0 > gpurun_out/r04_bench_ao0.log 2>&1
QT_AO_HS=1 timeout -k 10 600 python bench.py --cpu-baseline 0 > gpurun_out/r04_bench_ao1.log 2>&1
QT_AO_HS=1 QT_PF2_DEEP=1 timeout -k 10 600 python bench.py --cpu-baseline 0 > gpurun_out/r04_bench_ao1_deep1.log 2>&1
