set -u
OUT=gpurun_out/a13
mkdir -p $OUT
V=yocto_raytracing_amd/variants
for s in instance10000 instance100k instance1k; do
timeout -k 10 250 python tools/ab_variants.py --rounds 7 --scene $s $V/libyrt_base.so $V/libyrt_none.so $V/libyrt_adapt.so > $OUT/ab_$s.txt 2>&1
rc=$?; grep -v '^{' $OUT/ab_$s.txt | grep -v amdgpu.ids; if [ $rc -ne 0 ]; then exit $rc; fi
done
for a in "--scene refl --resolution 1080 --samples 4" "--resolution 4096 --samples 16 --share 0/8"; do
timeout -k 10 250 python tools/ab_variants.py --rounds 3 $a $V/libyrt_base.so $V/libyrt_adapt.so > $OUT/ab_x.txt 2>&1
rc=$?; grep -v '^{' $OUT/ab_x.txt | grep -v amdgpu.ids; if [ $rc -ne 0 ]; then exit $rc; fi
done
