# Round-4 first probe: code-predictor layer pieces, talker decode attention at long caches (split-KV crossover),
# PMC passes over the fused code-predictor attention + o_proj.  Every GPU step has its own time limit, chained by &&.
set -e
mkdir -p gpurun_out
timeout -k 10 240 python tools/cp_layer_bench.py > gpurun_out/r04_cpl17.txt 2>&1
QT_CPL_KEYS=10 timeout -k 10 240 python tools/cp_layer_bench.py > gpurun_out/r04_cpl10.txt 2>&1
ATTN_L=138,300,512,1024,2048,4000 ATTN_NS=1,2,4,8 timeout -k 10 300 python tools/talker_attn_bench.py > gpurun_out/r04_attn_long.txt 2>&1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum"; do
  d=gpurun_out/pmc_ao_$(echo $pass | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $d -o run -- python3 tools/pmc_attn_oproj.py > $d.log 2>&1
done
python3 tools/pmc_kernel_reduce.py attn_oproj_k gpurun_out/pmc_ao_meta.txt gpurun_out/pmc_ao_* > gpurun_out/r04_pmc_attn_oproj.json
python3 tools/pmc_kernel_reduce.py attn_oproj_hs_k gpurun_out/pmc_ao_meta.txt gpurun_out/pmc_ao_* > gpurun_out/r04_pmc_attn_oproj_hs.json
