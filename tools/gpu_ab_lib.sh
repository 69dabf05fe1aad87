# usage: bash tools/gpu_ab_lib.sh LIB_A [reps] : alternate 200-step benches, LIB_A (GHM_HIP_LIB) vs the in-tree build
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
A=$1; R=${2:-3}
for i in $(seq 1 $R); do
  GHM_HIP_LIB=$PWD/$A timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-final-risk 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | sed 's/^/base /'
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-final-risk 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | sed 's/^/new  /'
done
