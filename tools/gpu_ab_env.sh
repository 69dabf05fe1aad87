# usage: bash tools/gpu_ab_env.sh VAR VAL_A VAL_B [reps] : alternate bench runs with VAR=VAL_A / VAL_B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
VAR=$1; A=$2; B=$3; R=${4:-3}
mkdir -p gpurun_out/ab
for i in $(seq 1 $R); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-final-risk > gpurun_out/ab/b_$v_$i.json 2> gpurun_out/ab/err || exit 3
    echo "$VAR=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/b_$v_$i.json)"
  done
done
