set -u
OUT=gpurun_out/a21
mkdir -p $OUT
V=yocto_raytracing_amd/variants
run() { tag=$1; shift; timeout -k 10 200 python tools/ab_variants.py --rounds 7 "$@" $V/libyrt_p0.so $V/libyrt_nt.so $V/libyrt_p0.so > $OUT/ab_$tag.txt 2>&1; rc=$?; grep -v '^{' $OUT/ab_$tag.txt | grep -v amdgpu.ids | sed "s/^/$tag /"; return $rc; }
run c4 && run c4_r0of8 --share 0/8 && run c4_r0of4 --share 0/4 && run c3 --scene refl --samples 4
