# usage: bash tools/gpu_ab2.sh TAG VARIANT_DIR... : parity tests (in-tree lib), then kbench + bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_cli.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 2; }
tail -2 $OUT/tests.log
bash tools/gpu_ab.sh $TAG "$@"
