set -u
OUT=gpurun_out/a9
mkdir -p $OUT
export TMPDIR=/tmp
V=yocto_raytracing_amd/variants
timeout -k 10 250 python tools/ab_variants.py --rounds 7 $V/libyrt_bunonly.so $V/libyrt_both.so $V/libyrt_both2.so > $OUT/ab_c4.txt 2>&1
rc=$?; grep -v '^{' $OUT/ab_c4.txt | grep -v amdgpu.ids; if [ $rc -ne 0 ]; then exit $rc; fi
for l in bunonly both2; do
  i=0
  for g in "SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE" "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_INSTS_LDS SQ_WAVES"; do
    i=$((i+1))
    YRT_LIB=$V/libyrt_$l.so timeout -s KILL 150 rocprofv3 --pmc $g --output-format csv -d $OUT/pmc_$l/p$i -o p$i -- \
      python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-count-pass > $OUT/pmc_$l.p$i.log 2>&1
    rc=$?; echo "pmc $l pass $i rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
