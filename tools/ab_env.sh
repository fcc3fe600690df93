# GPU tests (optionally filtered), then the bench once per environment setting given as arguments
# usage: bash tools/ab_env.sh "<pytest -k expr or empty>" "VAR=a" "VAR=b" ...
set -e
k=$1; shift
if [ -n "$k" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$k" > gpurun_out/tk.log 2>&1
fi
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline 0 > gpurun_out/ab$i.log 2>&1
  echo "$e $(tail -1 gpurun_out/ab$i.log)" >> gpurun_out/ab.txt
done
