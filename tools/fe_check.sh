# voice-clone front end: frontend parity tests, then the configs[4] check set
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontend.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fe_t.log 2>&1
bash tools/vc_check.sh
