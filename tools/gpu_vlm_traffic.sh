# usage: bash tools/gpu_vlm_traffic.sh TAG : HBM traffic per kernel of the sequential-VLM bench (two PMC passes,
#        FETCH_SIZE and WRITE_SIZE, each its own run) -> gpurun_out/TAG/traffic_vlm.json (tools/traffic.py)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-vt1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ok() { r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python bench.py --workload vlm --steps 3 --warmup 1 --no-cpu-baseline > $OUT/fetch.log 2>&1
ok $? || exit 2
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python bench.py --workload vlm --steps 3 --warmup 1 --no-cpu-baseline > $OUT/write.log 2>&1
ok $? || exit 3
python tools/traffic.py $OUT/fetch $OUT/write --json $OUT/traffic_vlm.json --over "bench.py --workload vlm --steps 3 --warmup 1" > $OUT/traffic_vlm.txt || exit 4
find $OUT -name '*counter_collection.csv' -size +4M -delete
echo done
