# round 6 item 5: the GEMM-path encoder at n_embd = 64 / 256, then the suites its
# kernel changes touch (GEMM 64-column tiles, D = 64 attention, LN rows)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6_width}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v -rA --timeout 200 --timeout-method thread tests/test_gpu_width.py \
  > $OUT/tests_width.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/tests_width.log | tail -3; [ $rc -le 1 ] || exit 2
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm.py \
  tests/test_gpu_vlm.py tests/test_gpu_parity.py tests/test_gpu_cdm.py tests/test_gpu_cli.py > $OUT/tests_reg.log 2>&1
rc=$?; tail -3 $OUT/tests_reg.log; [ $rc -eq 0 ] || exit 3
echo done
