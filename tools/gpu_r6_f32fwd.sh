# round 6: the CLIP plan's mixed mode (precision "f32fwd": exact-f32 forward,
# split-bf16 backward).  usage: bash tools/gpu_r6_f32fwd.sh TAG [PARTS...]
# (PARTS: $GHM_F32FWD values, the forward stages kept on the f32 kernels; default
# "qkv,attn,mlp").  Per PARTS: the whole guided 3001-step run against the
# reference's CPU run and spread (its ratio line; a numerical failure goes on),
# then guided bench steps per PARTS beside f32 and x3, alternating
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6_f32fwd}
shift
[ $# -gt 0 ] || set -- qkv,attn,mlp
mkdir -p $OUT
for v in "$@"; do
  GHM_F32FWD=$v timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    "tests/test_gpu_parity.py::test_guided_full_run_final_risk_vs_reference_cpu_run[None]" -s > $OUT/tests_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(grep -o 'worst ratio[^;]*' $OUT/tests_$v.log) $(grep -o 'final risk [0-9.]* vs reference CPU run [0-9.]* (rel [0-9.e-]*)' $OUT/tests_$v.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 2
  # a numerical failure goes on; a device error ends the call
  if grep -qiE "hip error|illegal|memory access fault|core dumped" $OUT/tests_$v.log; then exit 2; fi
done | tee $OUT/curves.txt
[ ${PIPESTATUS[0]} -eq 0 ] || exit 2
for i in 1 2; do
  for v in f32 x3 "$@"; do
    case "$v" in f32|x3) pr=$v;; *) pr=f32fwd;; esac
    GHM_F32FWD=$v timeout -k 10 300 python bench.py --guide --precision $pr --steps 200 --warmup 10 --no-cpu-baseline \
      --no-final-risk > $OUT/b_$v.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 3; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_$v.json)"
  done
done | tee $OUT/ab.txt
echo done
