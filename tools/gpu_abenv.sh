# usage: bash tools/gpu_abenv.sh TAG "TESTS" SETTING... : GPU tests (in-tree lib), kbench (in-tree lib and every
#        GHM_HIP_LIB= setting), then alternating 200-step CLIP benches, one per SETTING ("-" = defaults, else
#        VAR=VAL[,VAR=VAL...]; GHM_HIP_LIB=<relative path> selects a variant library; DIR=<dir> runs
#        <dir>/bench.py, a checkout made by tools/make_abbase.sh)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; TESTS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 2; }
  tail -2 $OUT/tests.log
fi
timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 > $OUT/kbench_tree.txt 2>&1 || exit 5
for v in "$@"; do
  case "$v" in GHM_HIP_LIB=*) env $(echo $v | tr ',' ' ') timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 > $OUT/kbench_$(echo $v | md5sum | cut -c1-6).txt 2>&1 || exit 5; echo "kbench $v -> $(echo $v | md5sum | cut -c1-6)";; esac
done
for i in 1 2 3; do
  for v in "$@"; do
    B=bench.py
    case "$v" in DIR=*) B=${v#DIR=}/bench.py; E="";; -) E="";; *) E=$(echo $v | tr ',' ' ');; esac
    env $E timeout -k 10 200 python $B --steps 200 --warmup 10 --no-cpu-baseline --no-final-risk > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 3; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/b.json)"
  done
done | tee $OUT/ab.txt
echo done
