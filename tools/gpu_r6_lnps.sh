# round 6: the weight gradients on pre-split operands (ghm_wgrad_x3p): the LN1 / LN2
# rows the forward kernels split (GHM_LN_PRESPLIT, default on) and G from the MLP
# backward (GHM_G_PRESPLIT, split_out 2): parity tests, isolated kernel times,
# alternating 200-step benches
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6_lnps}
mkdir -p $OUT
if [ "$SKIP_TESTS" != "1" ]; then
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_cdm.py tests/test_gpu_cli.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit 2
fi
timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 --only wgrad_w1_x3,wgrad_w1_x3p,wgrad_qkv_x3,wgrad_qkv_x3p,ln_qkv_fwd_x3,ln_qkv_fwd_x3s,ln_mlp_fwd_x3b,ln_mlp_fwd_x3bs,wgrad_w2_x3,wgrad_w2_x3p,mlp_bwd_rc_x3,mlp_bwd_rc_x3g > $OUT/kbench.txt 2>&1 || exit 3
cat $OUT/kbench.txt
for i in 1 2 3; do
  for v in "GHM_LN_PRESPLIT=1" "GHM_LN_PRESPLIT=0" "GHM_G_PRESPLIT=1"; do
    env $v timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-final-risk > $OUT/b.json 2> $OUT/b.err || { tail -3 $OUT/b.err; exit 4; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/b.json)"
  done
done > $OUT/ab.txt || exit 4
cat $OUT/ab.txt
echo done
