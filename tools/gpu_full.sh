# usage: bash tools/gpu_full.sh TAG : parity tests, bench, rocprof kernel trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -rA > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
   python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err
echo "prof rc=$?" >> $OUT/prof_bench.err
