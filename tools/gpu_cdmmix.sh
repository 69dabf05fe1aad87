cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
K="default_config_curve_vs_reference and f32"
GHM_LONG_ATTN=x3 timeout -k 10 300 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gpu_cdm_joint.py tests/test_gpu_cdm_guided.py -k "$K" > gpurun_out/r2_cdmmix.log 2>&1
GHM_LONG_ATTN=x3 timeout -k 10 150 python bench.py --workload cdm_joint --precision f32 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2_cdmmix_bench.json 2>/dev/null
exit 0
