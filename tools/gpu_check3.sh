# usage: bash tools/gpu_check3.sh TAG : whole GPU suite, smoke, kbench, wgrad-stream A/B bench, determinism digests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
tail -3 $OUT/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 3
timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 --json $OUT/kbench.json > $OUT/kbench.txt 2>&1 || exit 4
grep -E "wgrad|mlp_bwd_rc|readout" $OUT/kbench.txt
for v in 0 1 0 1; do
  GHM_WGRAD_STREAM=$v timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-final-risk > $OUT/bench_ws$v.json 2> $OUT/bench_ws$v.err
  echo "ws=$v rc=$? $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_ws$v.json)"
done
for r in a b; do GHM_WGRAD_STREAM=1 timeout -k 10 120 python tools/det_check.py 30 > $OUT/det_ws_$r.txt 2>&1; echo "det ws rc=$? $(head -1 $OUT/det_ws_$r.txt)"; done
echo done
