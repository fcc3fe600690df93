# Round-4 GPU probe: parity of the new kernels first, then microbenchmarks + PMC (r04_probe1.sh), then the other new
# GPU tests.  Steps chained under set -e: a failing step ends the script.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "attn_oproj or split_kv" > gpurun_out/r04_t_kernels.txt 2>&1
bash tools/r04_probe1.sh
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "full_processor_chain or releases_codec_slot or continuous_batching or stream_voice_clone or greedy_codes" \
  > gpurun_out/r04_t_new.txt 2>&1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -s tests/test_gpu_full.py \
  -k "refill or bf16_teacher" > gpurun_out/r04_t_full.txt 2>&1
