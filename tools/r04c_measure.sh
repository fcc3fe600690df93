# Round-4 end measurement (final build) on the current build: PMC passes (attn_oproj_hs_k: the bench's roofline kernel, and the
# talker gate-up GEMV), copied into profiles/ on the box so the bench line's traffic is this build's, then the bench
# line and the rocprofv3 kernel-trace stats of the same bench command.  Each GPU step time-limited, chained (set -e).
set -e
mkdir -p gpurun_out
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum"; do
  d=gpurun_out/pmc_ao_$(echo $pass | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $d -o run -- python3 tools/pmc_attn_oproj.py > $d.log 2>&1
done
python3 tools/pmc_kernel_reduce.py attn_oproj_hs_k gpurun_out/pmc_ao_meta.txt gpurun_out/pmc_ao_* > gpurun_out/r04c_pmc_attn_oproj_hs.json
python3 tools/pmc_kernel_reduce.py attn_oproj_k gpurun_out/pmc_ao_meta.txt gpurun_out/pmc_ao_* > gpurun_out/r04c_pmc_attn_oproj.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc1 -o run -- python3 tools/pmc_gateup.py > gpurun_out/pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc2 -o run -- python3 tools/pmc_gateup.py > gpurun_out/pmc2.log 2>&1
python3 tools/pmc_reduce.py gpurun_out/pmc1 gpurun_out/pmc2 "$(cat gpurun_out/pmc_build_id.txt)" > gpurun_out/r04c_pmc_gateup.json
cp gpurun_out/r04c_pmc_*.json profiles/
timeout -k 10 600 python bench.py > gpurun_out/r04c_bench.log 2>&1
tail -1 gpurun_out/r04c_bench.log > gpurun_out/r04c_bench_line.json
bash tools/prof.sh r04cprof --cpu-baseline 0
# the roofline kernels' average durations in that trace, labelled with the build (bench.py attaches them by build id)
bid=$(cat gpurun_out/pmc_build_id.txt)
python3 tools/rocprof_kernel_avg.py gpurun_out/r04cprof/run_kernel_stats.csv attn_oproj_hs_k $bid > gpurun_out/r04c_rocprof_attn_oproj_hs.json
python3 tools/rocprof_kernel_avg.py gpurun_out/r04cprof/run_kernel_stats.csv "gemv_wt<unsigned short, unsigned short, unsigned short, 4, 4, true, true" $bid > gpurun_out/r04c_rocprof_gateup.json
