# usage: bash tools/gpu_quick2.sh TAG [pytest files...] : selected GPU tests, isolated kbench, a short bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-q}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
FILES=${@:-tests/test_gpu_parity.py}
timeout -k 10 400 python -u -m pytest $FILES -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 --json $OUT/kbench.json > $OUT/kbench.txt 2>&1 || exit 4
cat $OUT/kbench.txt | grep -v amdgpu.ids
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-final-risk > $OUT/bench.json 2> $OUT/bench.err || exit 5
grep -o '"ms_per_step": [0-9.]*' $OUT/bench.json
