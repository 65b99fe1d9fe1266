set -u
OUT=gpurun_out/a3
mkdir -p $OUT
export TMPDIR=/tmp
V=yocto_raytracing_amd/variants
timeout -k 10 300 python tools/ab_variants.py --rounds 9 --scene refl --resolution 1080 --samples 4 \
  $V/libyrt_cur.so $V/libyrt_sw6.so $V/libyrt_lw6.so $V/libyrt_lw5.so $V/libyrt_fp1lw6.so $V/libyrt_fp1lw5.so > $OUT/ab_c3.txt 2>&1
rc=$?; grep -v '^{' $OUT/ab_c3.txt | grep -v amdgpu.ids; if [ $rc -ne 0 ]; then exit $rc; fi
for l in cur lw6 fp1lw6; do
  YRT_LIB=$V/libyrt_$l.so timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/pmc_c3_$l -o p -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-count-pass \
    --scene refl --resolution 1080 --samples 4 > $OUT/pmc_c3_$l.log 2>&1
  rc=$?; echo "pmc c3 $l rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 300 python tools/ab_variants.py --rounds 9 $V/libyrt_cur.so $V/libyrt_sv0.so > $OUT/ab_c4_v.txt 2>&1
rc=$?; grep -v '^{' $OUT/ab_c4_v.txt | grep -v amdgpu.ids; if [ $rc -ne 0 ]; then exit $rc; fi
for l in cur h16; do
  for c in FETCH_SIZE WRITE_SIZE; do
    YRT_LIB=$V/libyrt_$l.so timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_c4_${l}_$c -o p -- \
      python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --no-count-pass > $OUT/pmc_c4_${l}_$c.log 2>&1
    rc=$?; echo "pmc c4 $l $c rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
