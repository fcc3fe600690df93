# Round-4 probe 4: the one-wave-per-row sampler (sample_w_k) -- parity tests, latency A/B (QT_SAMPLE_WAVE), bench A/B.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "sample or greedy_codes or continuous_batching or stream_matches or eos_ragged or bf16" > gpurun_out/r04_t_sampler.txt 2>&1
QT_SAMPLE_WAVE=0 timeout -k 10 200 python tools/sample_bench.py > gpurun_out/r04_sample_bench_w0.txt 2>&1
QT_SAMPLE_WAVE=1 timeout -k 10 200 python tools/sample_bench.py > gpurun_out/r04_sample_bench_w1.txt 2>&1
timeout -k 10 600 python bench.py --cpu-baseline 0 > gpurun_out/r04_bench_w1.log 2>&1
QT_SAMPLE_WAVE=0 timeout -k 10 600 python bench.py --cpu-baseline 0 --roofline 0 > gpurun_out/r04_bench_w0.log 2>&1
