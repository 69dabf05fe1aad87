# usage: bash tools/gpu_quick.sh TAG [KBENCH_ONLY] : fast GPU check — parity tests, kbench subset, x3 bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-q1}
ONLY=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
if [ -n "$ONLY" ]; then
  timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 --only $ONLY > $OUT/kbench.txt 2>&1 || exit 3
else
  timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 > $OUT/kbench.txt 2>&1 || exit 3
fi
grep " us" $OUT/kbench.txt
timeout -k 10 200 python bench.py --precision x3 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 4
grep -o '"ms_per_step": [0-9.]*' $OUT/bench.json
