set -e
for m in 256 512 1024 2048; do
QT_IM2COL_MAX_M=$m timeout -k 10 300 python tools/codec_feed_prof.py > gpurun_out/i2cab_$m.log 2>&1
QT_IM2COL_MAX_M=$m QT_CF_B=1 timeout -k 10 300 python tools/codec_feed_prof.py > gpurun_out/i2cab_b1_$m.log 2>&1
done
