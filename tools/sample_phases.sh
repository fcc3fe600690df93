set -e
for st in ${QT_STOPS:-1 2 3 4 5 0}; do QT_SAMPLE_STOP=$st timeout -k 10 120 python tools/sample_bench.py >> gpurun_out/sph.txt 2>&1; done
