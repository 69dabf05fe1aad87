# round 6: the x6 MLP forward's accumulation (GHM_X6_CHAIN=1: products chained from
# zero, the residual added at the end; default: zero-started six-product groups added
# on the VALU into the residual-seeded sum) -- accuracy against float64, kernel time,
# the guided 3001-step run and alternating guided benches
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6_x6chain}
mkdir -p $OUT
for v in 0 1; do
  GHM_X6_CHAIN=$v timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py -k "mlp6" > $OUT/unit_$v.log 2>&1
  echo "chain=$v $(grep -c PASSED $OUT/unit_$v.log) passed; $(grep -o "vs float64: {[^}]*}" $OUT/unit_$v.log | head -2 | tr '\n' ' ')"
  if grep -qiE "hip error|illegal|memory access fault|core dumped" $OUT/unit_$v.log; then exit 2; fi
  GHM_X6_CHAIN=$v timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 --only ln_mlp_fwd_x6 > $OUT/kbench_$v.txt 2>&1 || exit 3
  grep ln_mlp_fwd_x6 $OUT/kbench_$v.txt
done
GHM_X6_CHAIN=1 timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_guided_full_run_final_risk_vs_reference_cpu_run[None]" > $OUT/curve_1.log 2>&1
echo "curve chain=1 rc=$? $(grep -o 'worst ratio[^;]*' $OUT/curve_1.log) $(grep -o 'final risk [0-9.]* vs reference CPU run [0-9.]* (rel [0-9.e-]*)' $OUT/curve_1.log)"
if grep -qiE "hip error|illegal|memory access fault|core dumped" $OUT/curve_1.log; then exit 2; fi
for i in 1 2 3; do
  for v in 0 1; do
    GHM_X6_CHAIN=$v timeout -k 10 300 python bench.py --guide --steps 200 --warmup 10 --no-cpu-baseline --no-final-risk \
      > $OUT/b_$v.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 4; }
    echo "chain=$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_$v.json)"
  done
done | tee $OUT/ab.txt
echo done
