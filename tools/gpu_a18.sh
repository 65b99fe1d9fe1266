set -u
OUT=gpurun_out/a18
mkdir -p $OUT
V=yocto_raytracing_amd/variants
run() { tag=$1; shift; timeout -k 10 200 python tools/ab_variants.py --rounds 7 "$@" $V/libyrt_pall.so $V/libyrt_ps.so > $OUT/ab_$tag.txt 2>&1; rc=$?; grep -v '^{' $OUT/ab_$tag.txt | grep -v amdgpu.ids | sed "s/^/$tag /"; return $rc; }
run c3 --scene refl --samples 4 && run c1 --scene simple --resolution 720 --samples 1 && run c4_360 --resolution 360 --samples 2 && run c4_180 --resolution 180 --samples 1 && run i1k_360 --scene instance1k --resolution 360 --samples 4 && run c2_4 --scene basic --resolution 720 --samples 4
