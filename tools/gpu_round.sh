# usage: bash tools/gpu_round.sh TAG : all GPU tests, smoke, the five workload benches,
# rocprof kernel stats of the CLIP (headline) and VLM benches
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ok() { r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
if [ "$SKIP_TESTS" != "1" ]; then  # SKIP_TESTS=1: the benches and profiles only
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
grep -E "^FAILED|^ERROR|passed|failed" $OUT/gpu_tests.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 3
fi
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 4
cat $OUT/bench.json
timeout -k 10 400 python bench.py --guide > $OUT/bench_clip_guided.json 2> $OUT/bench_clip_guided.err || exit 4
echo "clip_guided $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_clip_guided.json)"
for w in vlm cdm cdm_joint cdm_guided vlm_joint; do
  timeout -k 10 400 python bench.py --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit 5
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$w.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_clip -o run -- \
   python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-final-risk > $OUT/prof_clip.json 2> $OUT/prof_clip.err
ok $? || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_vlm -o run -- \
   python bench.py --workload vlm --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof_vlm.json 2> $OUT/prof_vlm.err
ok $? || exit 7
# keep the stats, drop the per-dispatch traces (gpurun merges back at most 64 MiB)
find $OUT -name '*kernel_trace.csv' -size +4M -delete
du -sh $OUT
echo done
