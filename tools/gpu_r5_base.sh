cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r5_base
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
grep -E "^FAILED|^ERROR|passed|failed" $OUT/gpu_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 3
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 4
cat $OUT/bench.json
