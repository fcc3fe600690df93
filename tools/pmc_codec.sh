# SQ counters for the codec decode (separate --pmc pass, no tracing domains)
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d gpurun_out/pmcc -o run -- python3 tools/codec_bench.py 2 64 > gpurun_out/pmcc.log 2>&1
