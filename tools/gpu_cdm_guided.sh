# usage: bash tools/gpu_cdm_guided.sh TAG : guided + joint CDM parity tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-cdmg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_cdm_guided.py tests/test_gpu_cdm_joint.py tests/test_gpu_cdm.py -x -v -s --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "rc=$rc" >> $OUT/tests.log
grep -E "PASSED|FAILED|curve|passed|failed|Error|error|assert" $OUT/tests.log | tail -40
exit $rc
