# usage: bash tools/gpu_x3.sh TAG : parity tests (both precisions) + bench both precisions + kbench + rocprof
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-x1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --precision f32 --no-cpu-baseline > $OUT/bench_f32.json 2> $OUT/bench_f32.err || exit $?
timeout -k 10 300 python bench.py --precision x3 --no-cpu-baseline > $OUT/bench_x3.json 2> $OUT/bench_x3.err || exit $?
timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 --json $OUT/kbench.json > $OUT/kbench.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
   python bench.py --steps 20 --warmup 3 --no-cpu-baseline --precision x3 > $OUT/prof_bench.json 2> $OUT/prof_bench.err
echo "prof rc=$?" >> $OUT/prof_bench.err
