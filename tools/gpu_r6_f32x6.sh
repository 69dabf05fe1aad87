# round 6: precision "f32x6" (the LN + QKV / LN + MLP forwards on the three-way
# split kernels, G / GELU' saved by the x6 MLP forward, the backward exact f32):
# encoder parity tests in the mode, the guided and joint CDM curves against the
# reference at the f32 bounds, then guided CDM / joint CDM / guided CLIP benches
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6_f32x6}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "f32x6" \
  "tests/test_gpu_cdm_guided.py::test_guided_default_config_curve_vs_reference" \
  "tests/test_gpu_cdm_joint.py::test_joint_cdm_default_config_curve_vs_reference" > $OUT/tests.log 2>&1
rc=$?
grep -E "CDM curve|guided curve|PASSED|FAILED|passed|failed" $OUT/tests.log | tail -30
[ $rc -le 1 ] || exit 2
if grep -qiE "hip error|illegal|memory access fault|core dumped" $OUT/tests.log; then exit 2; fi
for i in 1 2; do
  for w in cdm_guided cdm_joint; do
    for pr in f32 f32fwd f32x6; do
      timeout -k 10 300 python bench.py --workload $w --precision $pr --steps 100 --warmup 10 --no-cpu-baseline \
        > $OUT/b_${w}_$pr.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 3; }
      echo "$w $pr $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_${w}_$pr.json)"
    done
  done
done | tee $OUT/ab.txt
echo done
