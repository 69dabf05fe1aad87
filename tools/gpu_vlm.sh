# usage: bash tools/gpu_vlm.sh TAG : VLM GPU parity tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-vlm}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_vlm.py -x -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "rc=$rc" >> $OUT/tests.log
grep -E "PASSED|FAILED|curve|passed|failed|Error|error" $OUT/tests.log | tail -30
exit $rc
