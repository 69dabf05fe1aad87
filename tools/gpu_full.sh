# usage: bash tools/gpu_full.sh TAG : parity tests, default bench (with CPU baseline), f32 bench,
# kbench, rocprof kernel trace + stats, HBM traffic PMC passes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ok() { r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 3
timeout -k 10 300 python bench.py --precision f32 --no-cpu-baseline > $OUT/bench_f32.json 2> $OUT/bench_f32.err || exit 4
timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 --json $OUT/kbench.json > $OUT/kbench.txt 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
   python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err
ok $? || exit 6
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python tools/kbench.py --reps 3 --precision x3 > $OUT/fetch.log 2>&1
ok $? || exit 7
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python tools/kbench.py --reps 3 --precision x3 > $OUT/write.log 2>&1
ok $? || exit 8
echo done
