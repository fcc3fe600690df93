# Round-1 measurement set: GPU tests, rocprof kernel-trace stats of the full bench (same command as the bench
# line), then two PMC passes (FETCH_SIZE, WRITE_SIZE) on the roofline kernel, reduced to profiles/.
set -e
root=$(pwd)
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$root"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc1 -o run -- python3 tools/pmc_gateup.py > gpurun_out/pmc1.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc2 -o run -- python3 tools/pmc_gateup.py > gpurun_out/pmc2.log 2>&1
python3 tools/pmc_reduce.py gpurun_out/pmc1 gpurun_out/pmc2 > profiles/r01_pmc_gateup.json
cp profiles/r01_pmc_gateup.json gpurun_out/
bash tools/prof.sh r01bench
