set -u
OUT=gpurun_out/a11
mkdir -p $OUT
V=yocto_raytracing_amd/variants
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 2 $OUT/pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
for s in instance10000 instance100k instance1k; do
timeout -k 10 250 python tools/ab_variants.py --rounds 7 --scene $s $V/libyrt_base.so $V/libyrt_none.so $V/libyrt_adapt.so > $OUT/ab_$s.txt 2>&1
rc=$?; grep -v '^{' $OUT/ab_$s.txt | grep -v amdgpu.ids; if [ $rc -ne 0 ]; then exit $rc; fi
done
