#!/bin/bash
# One round's evidence set on one GPU box, in parts (each well under gpurun's 20-minute
# limit), collected once at the round's final build (ROUND=r6 by default):
#   bash tools/gpu/evidence.sh A TAG   -m gpu suite, smoke, c4 counters + kernel stats, the
#                                    default bench line (the three CPU legs), N=2 rehearsal
#   bash tools/gpu/evidence.sh B TAG   c3 and c5 counters + bench lines
#   bash tools/gpu/evidence.sh C TAG   counters of rank 0 of 2, 4 and 8 at c4 (bench.py
#                                    --profile-rank): the N-rank lines' roofline
#   bash tools/gpu/evidence.sh E TAG   the same at c5 (4096x4096, 16x16 spp)
#   bash tools/gpu/evidence.sh D TAG   instance1k / instance100k at c4 settings: counters
#                                    + bench lines
# Every GPU step has its own time limit; a failing step ends the script. The counter
# summaries (stamped with libyrt.so's code identity) go to this copy's profiles/ and to
# gpurun_out/TAG/, so the bench lines that follow carry the issue roofline.
set -u
PART=$1; TAG=$2; ROUND=${ROUND:-r6}
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() { "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED (rc=$rc): $*"; exit $rc; fi; }
summ() {  # key, pmc dir
  run python tools/pmc_summary.py --key $1 --csv $2/p*/p*_counter_collection.csv --source profiles/$ROUND/${2#gpurun_out/} \
      --traffic profiles/pmc_traffic.json --issue profiles/issue_counters.json > $2/summary.json
  cp profiles/pmc_traffic.json profiles/issue_counters.json $OUT/
}
pmc() {  # tag-suffix, timeout, bench args...
  local sub=$1 tmo=$2; shift 2
  PMC_TIMEOUT=$tmo run bash tools/gpu/issue_pmc.sh $TAG/$sub "$@" > $OUT/$sub.log 2>&1
}
if [ "$PART" = A ]; then
  run timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  tail -n 2 $OUT/pytest.log
  run timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  pmc pmc_c4 150
  summ instance10000-1920x1080-s8-n1-wavefront $OUT/pmc_c4
  run timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
  cut -c1-300 $OUT/bench.json
  YRT_BENCH_DEVICES=1 YRT_BENCH_BACKEND=gloo YRT_BENCH_OVERLAP=1 run timeout -k 10 400 \
    python bench.py --gpus 2 --steps 3 --warmup 1 --cpu-seconds 0 > $OUT/bench_n2_rehearsal_gloo_1gpu.json 2> $OUT/n2.err
  grep -h '^{' $OUT/bench_n2_rehearsal_gloo_1gpu.json | cut -c1-300
elif [ "$PART" = B ]; then
  pmc pmc_c3 200 --scene refl --resolution 1080 --samples 4
  summ refl-1920x1080-s4-n1-wavefront $OUT/pmc_c3
  pmc pmc_c5 300 --resolution 4096 --width 4096 --samples 16
  summ instance10000-4096x4096-s16-n1-wavefront $OUT/pmc_c5
  run timeout -k 10 300 python bench.py --scene refl --resolution 1080 --samples 4 --cpu-seconds 0 > $OUT/bench_c3_refl.json 2> $OUT/c3.err
  run timeout -k 10 400 python bench.py --resolution 4096 --width 4096 --samples 16 --steps 2 --warmup 1 --cpu-seconds 6 > $OUT/bench_c5_1gpu.json 2> $OUT/c5.err
  cut -c1-300 $OUT/bench_c3_refl.json $OUT/bench_c5_1gpu.json
elif [ "$PART" = C ]; then
  run timeout -k 10 300 python tools/rank_share.py > $OUT/rank_share_c4.json 2> $OUT/rank_share.err
  for n in 2 4 8; do
    pmc pmc_c4_r0of$n 150 --profile-rank 0/$n
    summ instance10000-1920x1080-s8-n$n-wavefront $OUT/pmc_c4_r0of$n
  done
elif [ "$PART" = E ]; then
  for n in 2 4 8; do
    pmc pmc_c5_r0of$n 200 --profile-rank 0/$n --resolution 4096 --width 4096 --samples 16
    summ instance10000-4096x4096-s16-n$n-wavefront $OUT/pmc_c5_r0of$n
  done
else
  for s in instance1k instance100k; do
    pmc pmc_$s 200 --scene $s
    summ $s-1920x1080-s8-n1-wavefront $OUT/pmc_$s
    run timeout -k 10 300 python bench.py --scene $s --cpu-seconds 0 > $OUT/bench_$s.json 2> $OUT/$s.err
    cut -c1-300 $OUT/bench_$s.json
  done
fi
