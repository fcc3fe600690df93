# PMC passes over tools/pf_gemm_probe.py (prefill GEMM shapes at M = 680): L2 hit / miss, fabric fetch, SQ cycles,
# for gemm_pf2_k tile configs 3 and 4 next to hipBLASLt (Cijk kernels).  Raw rocprofv3 output is summarised on the
# box and deleted (it exceeds gpurun's copy-back limit).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_pf
mkdir -p $O
export QT_PROBE_SHAPES=${QT_PROBE_SHAPES:-gate-up,down}
M=${M:-680}
pass() {  # name counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmc_$n -o run -- python tools/pf_gemm_probe.py $M > $O/$n.log 2>&1
  python tools/pmc_summarize.py /tmp/pmc_$n gemm_pf2 Cijk > $O/$n.txt
  rm -rf /tmp/pmc_$n
}
for cfg in ${CFGS:-3 4}; do
  export QT_PF2_CFG=$cfg
  timeout -k 10 120 python tools/pf_gemm_probe.py $M > $O/time_$cfg.txt 2>&1
  pass hit$cfg TCC_HIT_sum TCC_MISS_sum
  pass fetch$cfg FETCH_SIZE
  pass sq$cfg SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY
done
