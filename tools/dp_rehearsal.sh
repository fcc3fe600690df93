# 2-rank rehearsal of bench.py's data-parallel path on a single GPU (gloo collectives, both ranks on cuda:0):
# the default configs[2] weak-scaling workload and the configs[3] vd64 strong-scaling workload.
set -e
QT_BENCH_BACKEND=gloo QT_BENCH_SAME_DEVICE=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 \
  --cpu-baseline 0 --roofline 0 > gpurun_out/dp2.log 2>&1
tail -1 gpurun_out/dp2.log
QT_BENCH_BACKEND=gloo QT_BENCH_SAME_DEVICE=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 1 --warmup 1 \
  --workload vd64 > gpurun_out/dp2_vd64.log 2>&1
tail -1 gpurun_out/dp2_vd64.log
