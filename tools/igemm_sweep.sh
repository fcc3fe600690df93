timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "igemm or codec" > gpurun_out/t.log 2>&1
for c in default 4,2 4,1 6,1 8,1 8,2; do
  if [ "$c" = default ]; then timeout -k 10 120 python tools/codec_bench.py; else QT_IGEMM_CFG=$c timeout -k 10 120 python tools/codec_bench.py; fi 2>&1 | grep codec | sed "s/^/$c  /"
done > gpurun_out/sweep.log
