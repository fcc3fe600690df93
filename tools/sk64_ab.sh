set -e
for m in 48 64 48 64; do
QT_SK_MAX_M=$m timeout -k 10 600 python bench.py --workload vd64 --cpu-baseline 0 --roofline 0 > gpurun_out/sk64_$m.log 2>&1
grep -o '"value": [0-9.]*' gpurun_out/sk64_$m.log | sed "s/^/max $m /"
done
