set -u
OUT=gpurun_out/a4
mkdir -p $OUT
V=yocto_raytracing_amd/variants
timeout -k 10 300 python tools/ab_variants.py --rounds 9 $V/libyrt_cur.so $V/libyrt_sw6.so $V/libyrt_sw5.so $V/libyrt_sw8.so > $OUT/ab_c4.txt 2>&1
rc=$?; grep -v '^{' $OUT/ab_c4.txt | grep -v amdgpu.ids; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/ab_variants.py --rounds 9 --scene refl --resolution 1080 --samples 4 $V/libyrt_base.so $V/libyrt_cur.so $V/libyrt_lw6.so > $OUT/ab_c3.txt 2>&1
rc=$?; grep -v '^{' $OUT/ab_c3.txt | grep -v amdgpu.ids; exit $rc
