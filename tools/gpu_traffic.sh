# usage: bash tools/gpu_traffic.sh TAG : HBM traffic per kernel (two PMC passes over kbench)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-t1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ok() { r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python tools/kbench.py --reps 3 --precision x3 > $OUT/fetch.log 2>&1
ok $? || exit 2
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python tools/kbench.py --reps 3 --precision x3 > $OUT/write.log 2>&1
ok $? || exit 3
echo done
timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 --json $OUT/kbench.json > $OUT/kbench.txt 2>&1 || exit 4
