root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmcg -o run -- python3 tools/pmc_gateup.py > gpurun_out/pmcg.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcg2 -o run -- python3 tools/pmc_gateup.py > gpurun_out/pmcg2.log 2>&1 || true
