#!/bin/bash
# rocprofv3 kernel trace + stats of bench.py; keeps the stats CSV and a per-(kernel, grid) summary.
# usage (on the GPU box, from the repo root): bash tools/prof.sh <tag> <bench args...>
tag=$1; shift
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag -o run -- python3 bench.py "$@" > gpurun_out/$tag.log 2>&1
rc=$?
echo rc=$rc >> gpurun_out/$tag.log
tr=$(find gpurun_out/$tag -name "*kernel_trace.csv" | head -1)
[ -n "$tr" ] && python3 tools/trace_summary.py "$tr" gpurun_out/$tag/summary.txt
[ -n "$tr" ] && python3 tools/trace_position.py "$tr" gpurun_out/$tag/position.txt
find gpurun_out/$tag -name "*kernel_trace*" -delete
exit $rc
