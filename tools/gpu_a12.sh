set -u
OUT=gpurun_out/a12
mkdir -p $OUT
V=yocto_raytracing_amd/variants
for s in instance100k instance10000; do
YRT_LIST_DEBUG=1 timeout -k 10 250 python tools/ab_variants.py --rounds 5 --scene $s $V/libyrt_adapt.so > $OUT/dbg_$s.txt 2>&1
rc=$?; grep -v '^{' $OUT/dbg_$s.txt | grep -v amdgpu.ids | sort | uniq -c | head; if [ $rc -ne 0 ]; then exit $rc; fi
done
for s in instance10000 instance100k; do
timeout -k 10 250 python tools/ab_variants.py --rounds 7 --scene $s $V/libyrt_none.so $V/libyrt_adapt.so > $OUT/ab_$s.txt 2>&1
rc=$?; grep -v '^{' $OUT/ab_$s.txt | grep -v amdgpu.ids; if [ $rc -ne 0 ]; then exit $rc; fi
done
