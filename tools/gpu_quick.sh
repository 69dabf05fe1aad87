# usage: bash tools/gpu_quick.sh TAG "TESTS" [kbench --only list] : GPU tests then isolated kernel times
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; TESTS=$2; ONLY=$3
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 2; }
  tail -2 $OUT/tests.log
fi
if [ -n "$ONLY" ]; then
  timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 --only $ONLY > $OUT/kbench.txt 2>&1 || { tail $OUT/kbench.txt; exit 5; }
  cat $OUT/kbench.txt
fi
echo done
