# usage: bash tools/gpu_quick.sh TAG : GPU parity tests + kernel microbench + bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -rA > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/kbench.py --reps 10 --json $OUT/kbench.json > $OUT/kbench.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
