# usage: bash tools/gpu_variant_check.sh TAG LIB... : the encoder parity tests run on each variant library
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for lib in "$@"; do
  n=$(basename $(dirname $lib))
  GHM_HIP_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py -k "forward_stages or encoder_backward or bit_identical or vs_reference_fixture or curve_vs_reference" \
    > gpurun_out/$TAG/tests_$n.log 2>&1 || { tail -20 gpurun_out/$TAG/tests_$n.log; exit 2; }
  echo "$n $(tail -1 gpurun_out/$TAG/tests_$n.log)"
done
