# rocprofv3 kernel stats of the codec decode alone
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pc -o run -- python3 tools/codec_bench.py > gpurun_out/pc.log 2>&1
rc=$?
tr=$(find gpurun_out/pc -name "*kernel_trace.csv" | head -1)
[ -n "$tr" ] && python3 tools/trace_summary.py "$tr" gpurun_out/pc/summary.txt
find gpurun_out/pc -name "*kernel_trace*" -delete
exit $rc
