set -u
mkdir -p gpurun_out/a2
V=yocto_raytracing_amd/variants
timeout -k 10 300 python tools/ab_variants.py --rounds 9 --scene refl --resolution 1080 --samples 4 $V/libyrt_cur.so $V/libyrt_fp1.so $V/libyrt_fp1w6.so $V/libyrt_h16.so > gpurun_out/a2/ab_c3.txt 2>&1
rc=$?; grep -v '^{' gpurun_out/a2/ab_c3.txt | grep -v amdgpu.ids; exit $rc
