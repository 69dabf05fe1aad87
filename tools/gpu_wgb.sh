cd $GRAFT_REPO_ROOT
bash tools/gpu_counters.sh c_r2 || exit 1
for b in 256 1024; do GHM_WGRAD_BLOCKS=$b timeout -k 10 200 python bench.py --no-cpu-baseline --no-final-risk > gpurun_out/c_r2/bench_wg$b.json 2>/dev/null || exit 2; done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-final-risk > gpurun_out/c_r2/bench_wg512.json 2>/dev/null
