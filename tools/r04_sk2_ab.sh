# gemm_sk2_k (QT_SK2=1): numerics check, then the prefill shapes at 64..128 rows on both routes
set -e
mkdir -p gpurun_out
QT_SK2=1 timeout -k 10 120 python tools/sk2_check.py > gpurun_out/sk2_check.txt 2>&1
for v in 0 1; do
  QT_SK2=$v QT_PB_M=64,96,128 timeout -k 10 200 python tools/prefill_gemm_bench.py > gpurun_out/sk2_pb_$v.txt 2>&1
done
