#!/bin/bash
# GPU box: two counter passes (issue/wait, scalar cache) of one c4 frame for each library
# variant (bench.py loads YRT_LIB), one rocprofv3 --pmc run per pass and variant.
#   bash tools/gpu_pmc_variants.sh TAG lib.so ...
set -u
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
groups=("SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
        "SQC_DCACHE_HITS SQC_DCACHE_MISSES")
for lib in "$@"; do
  name=$(basename $lib .so)
  i=0
  for g in "${groups[@]}"; do
    i=$((i+1))
    YRT_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d $OUT/$name/p$i -o p$i -- \
      python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 > $OUT/$name.p$i.log 2>&1
    rc=$?
    echo "$name pass $i: rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
