# usage: bash tools/gpu_vlm_x3.sh TAG : GEMM / x3 attention / VLM parity tests, VLM bench + kernel stats
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-vlmx3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_vlm.py -x -v -s --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "rc=$rc" >> $OUT/tests.log
grep -E "PASSED|FAILED|curve|passed|failed|Error|error|assert" $OUT/tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload vlm --no-cpu-baseline > $OUT/bench_vlm.json 2> $OUT/bench_vlm.err || exit 4
cat $OUT/bench_vlm.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_vlm -o run -- \
   python bench.py --workload vlm --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof_vlm.json 2> $OUT/prof_vlm.err
r=$?; [ $r -le 1 ] || exit 5
echo done
