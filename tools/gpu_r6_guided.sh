# round 6: guided CLIP at its new default (precision "f32fwd": LN1 + QKV and LN2 +
# MLP forwards exact f32, attention and the backward split-bf16) -- the guided
# parity tests (both 3001-step runs: the default and exact f32), the guided CLI,
# the f32 kernels alone (the MLP forward with and without saving G / GELU'), and
# guided bench steps in f32 / default / x3
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6_guided}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
  tests/test_gpu_parity.py -k "guided or f32fwd" tests/test_gpu_cli.py::test_guided_sequential_cdm_cli \
  > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 2; }
grep -E "guided 3001|guided curve|passed|failed" $OUT/tests.log
timeout -k 10 200 python tools/kbench.py --reps 20 --precision f32 > $OUT/kbench_f32.txt 2>&1 || exit 4
grep -E "ln_mlp_fwd|ln_qkv_fwd" $OUT/kbench_f32.txt
for i in 1 2; do
  for pr in f32 default x3; do
    case "$pr" in default) arg="";; *) arg="--precision $pr";; esac
    timeout -k 10 300 python bench.py --guide $arg --steps 200 --warmup 10 --no-cpu-baseline --no-final-risk \
      > $OUT/b_$pr.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 3; }
    echo "$pr $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_$pr.json)"
  done
done | tee $OUT/ab.txt
echo done
