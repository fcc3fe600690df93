# Round-6 closing pass on the final build: the GPU suite, then tools/r06_prof.sh (bench line, rocprof kernel stats,
# PMC passes for cp_step / talker_tail) and the BASELINE configs[1] / [4] config bench.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_gpu_tests_final.txt 2>&1
bash tools/r06_prof.sh
cd $R
timeout -k 10 400 python tools/config_bench.py --configs 1 4 > gpurun_out/r06_config_bench.jsonl 2>gpurun_out/r06_config_bench.err
echo done
