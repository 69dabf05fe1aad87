# usage: bash tools/gpu_abn.sh TAG "TESTS" VARIANT_DIR... : parity tests on the in-tree lib, then per-kernel
#        timings (kbench) and alternating 200-step CLIP benches of every variant lib and the in-tree lib ("tree")
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; TESTS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 2; }
  tail -2 $OUT/tests.log
fi
for v in "$@" tree; do
  if [ $v = tree ]; then L=""; else L=$PWD/$v/libghm_hip.so; fi
  GHM_HIP_LIB=$L timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 > $OUT/kbench_$(basename $v).txt 2>&1 || exit 3
done
for i in 1 2 3; do
  for v in "$@" tree; do
    if [ $v = tree ]; then L=""; else L=$PWD/$v/libghm_hip.so; fi
    GHM_HIP_LIB=$L timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-final-risk 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | sed "s|^|$(basename $v) |" || exit 4
  done
done | tee $OUT/ab.txt
for v in "$@" tree; do echo "== $v"; grep -E "mlp|wgrad|qkv|attn" $OUT/kbench_$(basename $v).txt; done
echo done
