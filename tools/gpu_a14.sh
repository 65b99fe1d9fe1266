set -u
OUT=gpurun_out/a14
mkdir -p $OUT
V=yocto_raytracing_amd/variants
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 2 $OUT/pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
for s in instance10000 instance100k instance1k; do
YRT_LIST_DEBUG=1 timeout -k 10 250 python tools/ab_variants.py --rounds 5 --scene $s $V/libyrt_base.so $V/libyrt_probe.so > $OUT/ab_$s.txt 2>&1
rc=$?; grep -v '^{' $OUT/ab_$s.txt | grep -v amdgpu.ids | sort | uniq -c; if [ $rc -ne 0 ]; then exit $rc; fi
done
