set -u
OUT=gpurun_out/a17
mkdir -p $OUT
V=yocto_raytracing_amd/variants
run() { tag=$1; shift; timeout -k 10 200 python tools/ab_variants.py --rounds 7 "$@" $V/libyrt_cur.so $V/libyrt_pall.so > $OUT/ab_$tag.txt 2>&1; rc=$?; grep -v '^{' $OUT/ab_$tag.txt | grep -v amdgpu.ids | sed "s/^/$tag /"; return $rc; }
run c3 --scene refl --samples 4 && run c2 --scene basic --resolution 720 --samples 1 && run c1 --scene simple --resolution 720 --samples 1 && run c4_360 --resolution 360 --samples 2 && run c4 && run i100k_r0of8 --scene instance100k --share 0/8 && run c5_r0of8 --resolution 4096 --width 4096 --samples 16 --share 0/8
