# usage: bash tools/gpu_ab_cdm.sh TAG : CDM + CLIP GPU tests, then CDM bench at two wgrad split settings
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-abcdm}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
tail -3 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for mt in 32 256 512; do
  GHM_WGRAD_MIN_TOKENS=$mt timeout -k 10 200 python bench.py --workload cdm --no-cpu-baseline > $OUT/bench_cdm_$mt.json 2> $OUT/bench_cdm_$mt.err || exit 3
  echo "min_tokens=$mt $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_cdm_$mt.json) $(grep -o '"kernel_ms": [0-9.]*' $OUT/bench_cdm_$mt.json)"
done
timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/bench_clip.json 2> $OUT/bench_clip.err || exit 4
echo "clip $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_clip.json) $(grep -o '"kernel_ms": [0-9.]*' $OUT/bench_clip.json)"
