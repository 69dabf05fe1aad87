# VLM fused bias-gradient row sums: GEMM + VLM GPU tests, then the VLM bench line and
# its rocprof stats (round 4 "r4_ab24").  Every GPU step under its own time limit.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r4_ab24 && mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gemm.py tests/test_gpu_vlm.py tests/test_gpu_vlm_joint.py tests/test_gpu_vlm_guided.py \
  tests/test_gpu_dp_cdm_vlm.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -3 $O/tests.log
timeout -k 10 200 python bench.py --workload vlm --no-cpu-baseline > $O/b.json 2> $O/b.err || exit 3
cat $O/b.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python bench.py --workload vlm --steps 20 --warmup 3 --no-cpu-baseline > $O/p.json 2> $O/p.err || exit 3
find $O -name '*kernel_trace.csv' -size +4M -delete
echo done
