# usage: bash tools/gpu_kb_libs.sh TAG KERNELS LIB... : isolated kbench times of KERNELS (comma list) for the
#        in-tree library and each variant library (paths relative to the repo), three alternating rounds
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; K=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 120 python tools/kbench.py --reps 50 --precision x3 --only $K > $OUT/tree_$i.txt 2>&1 || exit 2
  echo "tree: $(grep -v amdgpu $OUT/tree_$i.txt | tr '\n' ' ')"
  for v in "$@"; do
    GHM_HIP_LIB=$v timeout -k 10 120 python tools/kbench.py --reps 50 --precision x3 --only $K > $OUT/v_$i.txt 2>&1 || exit 3
    echo "$v: $(grep -v amdgpu $OUT/v_$i.txt | tr '\n' ' ')"
  done
done | tee $OUT/kb.txt
