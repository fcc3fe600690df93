set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vd64prof -o run -- python3 bench.py --workload vd64 --steps 1 --warmup 1 --cpu-baseline 0 --roofline 0 > gpurun_out/vd64prof.log 2>&1
tr=$(find gpurun_out/vd64prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py "$tr" gpurun_out/vd64prof/summary.txt
find gpurun_out/vd64prof -name "*kernel_trace*" -delete
