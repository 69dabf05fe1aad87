# usage: bash tools/gpu_r3_check.sh TAG [pytest args] : GPU tests (all, or the given files), smoke, bench line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
T=${@:-tests}
timeout -k 10 900 python -u -m pytest $T -m gpu -v -rA --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
grep -E "^FAILED|^ERROR|passed|failed" $OUT/gpu_tests.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 3
timeout -k 10 400 python bench.py --no-final-risk > $OUT/bench.json 2> $OUT/bench.err || exit 4
cat $OUT/bench.json
echo done
