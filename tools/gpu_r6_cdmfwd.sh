# round 6: the joint CDM (T = 162) and the guided joint CDM (lr 1e-2) in precision
# "f32fwd" (f32-accurate x6 forward, split-bf16 backward) against the reference
# curves at the f32 bounds, then their bench steps in f32 / f32fwd, alternating
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6_cdmfwd}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  "tests/test_gpu_cdm_guided.py::test_guided_default_config_curve_vs_reference" \
  "tests/test_gpu_cdm_joint.py::test_joint_cdm_default_config_curve_vs_reference" > $OUT/tests.log 2>&1
rc=$?
grep -E "CDM curve|passed|failed" $OUT/tests.log
[ $rc -le 1 ] || exit 2
if grep -qiE "hip error|illegal|memory access fault|core dumped" $OUT/tests.log; then exit 2; fi
for i in 1 2; do
  for w in cdm_joint cdm_guided; do
    for pr in f32 f32fwd; do
      timeout -k 10 300 python bench.py --workload $w --precision $pr --steps 100 --warmup 10 --no-cpu-baseline \
        > $OUT/b_${w}_$pr.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 3; }
      echo "$w $pr $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_${w}_$pr.json)"
    done
  done
done | tee $OUT/ab.txt
echo done
