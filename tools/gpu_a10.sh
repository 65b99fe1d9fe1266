set -u
OUT=gpurun_out/a10
mkdir -p $OUT
V=yocto_raytracing_amd/variants
for s in instance10000 instance100k instance1k; do
timeout -k 10 250 python tools/ab_variants.py --rounds 7 --scene $s $V/libyrt_none.so $V/libyrt_bunonly.so $V/libyrt_both.so $V/libyrt_both12.so > $OUT/ab_$s.txt 2>&1
rc=$?; grep -v '^{' $OUT/ab_$s.txt | grep -v amdgpu.ids; if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 200 python tools/ab_variants.py --rounds 7 --scene refl --resolution 1080 --samples 4 $V/libyrt_none.so $V/libyrt_both.so > $OUT/ab_c3.txt 2>&1
rc=$?; grep -v '^{' $OUT/ab_c3.txt | grep -v amdgpu.ids; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python tools/ab_variants.py --rounds 7 --scene basic --resolution 720 --samples 1 $V/libyrt_none.so $V/libyrt_both.so > $OUT/ab_c2.txt 2>&1
rc=$?; grep -v '^{' $OUT/ab_c2.txt | grep -v amdgpu.ids; exit $rc
