set -e
for m in 8 16 32 1024; do
QT_ATTN_OPROJ_MAX=$m timeout -k 10 600 python bench.py --workload vd64 --slots 16 --cpu-baseline 0 --roofline 0 > gpurun_out/aomax_s16_$m.log 2>&1
QT_ATTN_OPROJ_MAX=$m timeout -k 10 600 python bench.py --workload vd64 --slots 32 --cpu-baseline 0 --roofline 0 > gpurun_out/aomax_s32_$m.log 2>&1
QT_ATTN_OPROJ_MAX=$m timeout -k 10 600 python bench.py --workload vd64 --cpu-baseline 0 --roofline 0 > gpurun_out/aomax_s64_$m.log 2>&1
done
