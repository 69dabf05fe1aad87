# usage: bash tools/gpu_r3_base.sh TAG : GPU tests, smoke, bench (full), rocprof kernel stats of the bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
ok() { r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
grep -E "^FAILED|^ERROR|passed|failed" $OUT/gpu_tests.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 3
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 4
grep -o '"ms_per_step": [0-9.]*' $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_clip -o run -- \
   python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-final-risk > $OUT/prof_clip.json 2> $OUT/prof_clip.err
ok $? || exit 6
find $OUT -name '*kernel_trace.csv' -size +4M -delete
echo done
