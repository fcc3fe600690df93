set -e
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
timeout -k 10 300 python tools/codec_bench.py > gpurun_out/codec.log 2>&1
