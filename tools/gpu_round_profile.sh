#!/bin/bash
# Round-end evidence on one GPU box, every step under its own time limit and chained so
# that a failing step ends the run:
#   bash tools/gpu_round_profile.sh TAG
# -> gpurun_out/TAG/: rocprofv3 kernel stats + FETCH_SIZE/WRITE_SIZE passes (gpu_profile.sh),
#    the default bench line (c4, with the CPU baseline), c3 and the c5 workload on 1 GPU,
#    and the N=2 path rehearsed with two gloo ranks on this one card.
set -euo pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash tools/gpu_profile.sh $TAG
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 python bench.py --scene refl --resolution 1080 --samples 4 --cpu-seconds 0 > $OUT/bench_c3_refl.json 2> $OUT/c3.err
timeout -k 10 400 python bench.py --resolution 4096 --samples 16 --steps 2 --warmup 1 --cpu-seconds 0 > $OUT/bench_c5_1gpu.json 2> $OUT/c5.err
YRT_BENCH_DEVICES=1 YRT_BENCH_BACKEND=gloo YRT_BENCH_OVERLAP=1 timeout -k 10 400 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 3 --warmup 1 --cpu-seconds 0 > $OUT/bench_n2_rehearsal_gloo_1gpu.json 2> $OUT/n2.err
ls $OUT
