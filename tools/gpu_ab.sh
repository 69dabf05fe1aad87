# usage: bash tools/gpu_ab.sh TAG VARIANT_DIR... : kbench + x3 bench for the in-tree lib and each variant lib
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 > $OUT/kb_base.txt 2>&1 || exit 3
timeout -k 10 200 python bench.py --precision x3 --no-cpu-baseline --no-final-risk > $OUT/bench_base.json 2>&1 || exit 4
for v in "$@"; do
  n=$(basename $v)
  GHM_HIP_LIB=$PWD/$v/libghm_hip.so timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 > $OUT/kb_$n.txt 2>&1 || exit 5
  GHM_HIP_LIB=$PWD/$v/libghm_hip.so timeout -k 10 200 python bench.py --precision x3 --no-cpu-baseline --no-final-risk > $OUT/bench_$n.json 2>&1 || exit 6
done
echo done
