# usage: bash tools/gpu_r3_ab3.sh TAG VARIANT... : CLIP parity/DP/CLI GPU tests, alternating 200-step
#        benches of the variant libs vs the in-tree build, then a rocprofv3 kernel trace of the in-tree bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dp.py tests/test_gpu_cli.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 2; }
tail -2 $OUT/tests.log
for i in 1 2 3; do
  for v in "$@" tree; do
    if [ $v = tree ]; then L=""; else L=$PWD/$v/libghm_hip.so; fi
    GHM_HIP_LIB=$L timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-final-risk 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | sed "s|^|$(basename $v) |" || exit 4
  done
done | tee $OUT/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_clip -o run -- \
   python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-final-risk > $OUT/prof_clip.json 2> $OUT/prof_clip.err
r=$?; [ $r -le 1 ] || exit 6
find $OUT -name '*kernel_trace.csv' -size +6M -delete
echo done
