# short-window conv im2col route: parity (conv + codec stream tests), then first-window feed time and first packets
set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/i2c_t.log 2>&1
QT_IM2COL=0 timeout -k 10 300 python tools/codec_feed_prof.py > gpurun_out/i2c_feed0.log 2>&1
QT_IM2COL=1 timeout -k 10 300 python tools/codec_feed_prof.py > gpurun_out/i2c_feed1.log 2>&1
QT_IM2COL=0 QT_CF_B=1 timeout -k 10 300 python tools/codec_feed_prof.py > gpurun_out/i2c_feed0_b1.log 2>&1
QT_IM2COL=1 QT_CF_B=1 timeout -k 10 300 python tools/codec_feed_prof.py > gpurun_out/i2c_feed1_b1.log 2>&1
timeout -k 10 500 python bench.py --cpu-baseline 0 --roofline 0 > gpurun_out/i2c_bench.log 2>&1
