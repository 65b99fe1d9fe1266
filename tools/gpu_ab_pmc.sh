#!/bin/bash
# GPU box: in-process A/B of library variants (tools/ab_variants.py) at c4 and at
# instance100k, then the scalar-cache and wait counters of selected variants (bench.py
# with YRT_LIB pointing at the variant; one rocprofv3 pass per group).
#   AB_LIBS="a b c" PMC_LIBS="a c" bash tools/gpu_ab_pmc.sh TAG [scene ...]
set -u
TAG=$1; shift
SCENES=${*:-instance10000}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
V=yocto_raytracing_amd/variants
run() { "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED (rc=$rc): $*"; exit $rc; fi; }
for s in $SCENES; do
  libs=""; for l in $AB_LIBS; do libs="$libs $V/libyrt_$l.so"; done
  run timeout -k 10 500 python tools/ab_variants.py --rounds ${AB_ROUNDS:-7} --scene $s $libs > $OUT/ab_$s.txt 2>&1
  grep -v '^{' $OUT/ab_$s.txt | grep -v amdgpu.ids
done
for s in $SCENES; do
  for l in ${PMC_LIBS:-}; do
    i=0
    for g in "SQC_DCACHE_HITS SQC_DCACHE_MISSES" "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
      i=$((i+1))
      YRT_LIB=$V/libyrt_$l.so timeout -s KILL 150 rocprofv3 --pmc $g --output-format csv -d $OUT/pmc_${s}_$l/p$i -o p$i -- \
        python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-count-pass --scene $s > $OUT/pmc_${s}_$l.p$i.log 2>&1
      rc=$?; echo "pmc $s $l pass $i rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
    done
  done
done
