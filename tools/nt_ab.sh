set -e
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
for m in auto 0 1; do
  if [ $m = auto ]; then timeout -k 10 400 python bench.py --cpu-baseline 0 --roofline 1 > gpurun_out/b_$m.log 2>&1;
  else QT_GEMV_NT=$m timeout -k 10 400 python bench.py --cpu-baseline 0 --roofline 1 > gpurun_out/b_$m.log 2>&1; fi
done
