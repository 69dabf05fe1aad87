# usage: bash tools/gpu_tests_probe.sh : the GPU suite, then the LN-statistics probes (qkv_xcc, qkv_dbg beside k_wgrad_x3<0>) -> gpurun_out/r4_t1
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r4_t1 && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log; grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/race_probe.py qkv_xcc wgrad0 40 > $O/probe_xcc.txt 2>&1 || exit 3
tail -4 $O/probe_xcc.txt
timeout -k 10 300 python tools/race_probe.py qkv_dbg wgrad0 20 > $O/probe_dbg.txt 2>&1 || exit 4
tail -3 $O/probe_dbg.txt
