# VLM data-gradient split-k A/B (GHM_VLM_DSPLIT; round 4 "r4_ab25"): GEMM + VLM GPU
# tests with the split on, then alternating VLM benches per setting.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r4_ab25 && mkdir -p $O
GHM_VLM_DSPLIT=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gemm.py tests/test_gpu_vlm.py tests/test_gpu_vlm_joint.py tests/test_gpu_vlm_guided.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
for i in 1 2; do for v in 1 2 3; do
  GHM_VLM_DSPLIT=$v timeout -k 10 200 python bench.py --workload vlm --no-cpu-baseline > $O/b.json 2> $O/b.err || exit 3
  echo "dsplit=$v $(grep -o '"ms_per_step": [0-9.]*' $O/b.json)"
done; done | tee $O/ab.txt
for v in 1 2; do
  GHM_VLM_DSPLIT=$v timeout -k 10 200 python bench.py --workload vlm_joint --no-cpu-baseline > $O/bj.json 2> $O/bj.err || exit 3
  echo "vlm_joint dsplit=$v $(grep -o '"ms_per_step": [0-9.]*' $O/bj.json)"
done | tee -a $O/ab.txt
