# round 6 item 1: the VLM suite once with the pre-split weight images on
# (GHM_VLM_PACK=1, job table now a fixed device buffer), then the CDM module
# cases at their default precision and the module-API AdamW / DP paths
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6_pack}
mkdir -p $OUT
GHM_VLM_PACK=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_gemm.py tests/test_gpu_vlm.py tests/test_gpu_vlm_sguided.py tests/test_gpu_vlm_guided.py \
  tests/test_gpu_vlm_joint.py > $OUT/tests_pack.log 2>&1
rc=$?; tail -3 $OUT/tests_pack.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_cdm.py tests/test_gpu_parity.py tests/test_gpu_dp.py > $OUT/tests_misc.log 2>&1
rc=$?; tail -3 $OUT/tests_misc.log; [ $rc -eq 0 ] || exit 3
echo done
