# usage: bash tools/gpu_cdm.sh TAG : all GPU tests (CLIP + CDM + CLI), CLIP bench, CDM bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-cdm}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
grep -E "PASSED|FAILED|curve|passed|failed" $OUT/gpu_tests.log | tail -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_clip.json 2> $OUT/bench_clip.err || exit 3
cat $OUT/bench_clip.json
timeout -k 10 300 python bench.py --workload cdm > $OUT/bench_cdm.json 2> $OUT/bench_cdm.err || exit 4
cat $OUT/bench_cdm.json
