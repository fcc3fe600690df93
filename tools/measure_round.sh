# Round measurement set (tag = $1): GPU tests, the default bench line (roofline + CPU baseline), rocprof
# kernel-trace stats of the same bench command, then two PMC passes (FETCH_SIZE, WRITE_SIZE) on the roofline kernel.
# Every GPU step has its own time limit and the steps are chained with && (a failed step ends the script).
set -e
tag=${1:-r03}
root=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_t.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/${tag}_bench.log 2>&1
tail -1 gpurun_out/${tag}_bench.log > gpurun_out/${tag}_bench_line.json
cd /tmp && export TMPDIR=/tmp && cd "$root"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc1 -o run -- python3 tools/pmc_gateup.py > gpurun_out/pmc1.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc2 -o run -- python3 tools/pmc_gateup.py > gpurun_out/pmc2.log 2>&1
python3 tools/pmc_reduce.py gpurun_out/pmc1 gpurun_out/pmc2 "$(cat gpurun_out/pmc_build_id.txt)" > gpurun_out/${tag}_pmc_gateup.json
bash tools/prof.sh ${tag}prof --cpu-baseline 0
