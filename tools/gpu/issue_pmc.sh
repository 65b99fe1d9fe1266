#!/bin/bash
# Counter passes for the roofline on the GPU box, one rocprofv3 run per group (kernel
# trace only, never combined with sys/runtime traces; each group within the per-block
# limits: <= 8 SQ, <= 2 GRBM, FETCH_SIZE and WRITE_SIZE alone), then the kernel-trace
# stats of the same command. A pass that times out ends the script.
#   bash tools/gpu/issue_pmc.sh TAG [bench args...]
set -u
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
B="bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-count-pass $*"
groups=(
  "SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
  "SQC_DCACHE_HITS SQC_DCACHE_MISSES"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for g in "${groups[@]}"; do
  i=$((i+1))
  timeout -s KILL ${PMC_TIMEOUT:-150} rocprofv3 --pmc $g --output-format csv -d $OUT/p$i -o p$i -- python3 $B > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($g): rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o ks -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 "$@" > $OUT/ks.log 2>&1
echo "kernel stats: rc=$?"
find $OUT -name '*.csv' | sort
