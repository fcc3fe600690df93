# Round-6 profile pass (run through gpurun from the repo root): the default bench line, a rocprofv3 kernel-trace
# stats run of a short bench (only the stats CSV kept), and three PMC passes each over eager cp_step launches
# (tools/pmc_cp_step.py) and talker_tail launches (tools/pmc_talker_tail.py).  Reduced locally afterwards by
# tools/rocprof_kernel_avg.py and tools/pmc_kernel_reduce.py into profiles/r06_*.json.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python bench.py > gpurun_out/r06_bench.log 2>&1
tail -1 gpurun_out/r06_bench.log > gpurun_out/r06_bench_line.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_bench -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 > $R/gpurun_out/r06_prof_bench.log 2>&1
find /tmp/prof_bench -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/r06_rocprof_bench_kernel_stats.csv \;
for i in 1 2 3; do
  C=$(echo "FETCH_SIZE WRITE_SIZE TCP_TCC_READ_REQ_sum" | cut -d' ' -f$i)
  timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_cs$i -o run --output-format csv -- python3 $R/tools/pmc_cp_step.py > $R/gpurun_out/pmc$i.log 2>&1
done
for i in 1 2 3; do
  C=$(echo "FETCH_SIZE WRITE_SIZE TCP_TCC_READ_REQ_sum" | cut -d' ' -f$i)
  timeout -s KILL 180 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_tt$i -o run --output-format csv -- python3 $R/tools/pmc_talker_tail.py > $R/gpurun_out/pmct$i.log 2>&1
done
echo done
