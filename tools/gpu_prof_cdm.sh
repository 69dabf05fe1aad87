# usage: bash tools/gpu_prof_cdm.sh TAG : rocprofv3 kernel stats of the CDM bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-cdmprof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
   python bench.py --workload cdm --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
python tools/kstats.py $OUT/prof/run_kernel_stats.csv 23 30
