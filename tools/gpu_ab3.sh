# usage: bash tools/gpu_ab3.sh TAG VARIANT_DIR : kbench/bench A/B plus wgrad split sweeps on the in-tree lib
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash tools/gpu_ab.sh $TAG "$@" || exit 1
for b in 128 256; do
  GHM_WGRAD_BLOCKS=$b timeout -k 10 200 python bench.py --no-cpu-baseline --no-final-risk > $OUT/bench_wg$b.json 2>/dev/null || exit 2
done
echo done
