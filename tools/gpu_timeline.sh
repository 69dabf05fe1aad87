# usage: bash tools/gpu_timeline.sh TAG [bench args...] -> gpurun_out/tl_TAG/ (kernel trace + stats + timeline)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-x}
shift
mkdir -p gpurun_out/tl_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tl_$TAG -o run -- \
   python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-final-risk "$@" > gpurun_out/tl_$TAG/bench.json 2> gpurun_out/tl_$TAG/bench.err
rc=$?
echo "prof rc=$rc" >> gpurun_out/tl_$TAG/bench.err
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/tl_$TAG -name '*kernel_trace.csv' | head -1)
# step -26: a timed step (bench.py then replays 10 serial + 10 concurrent stamped-twin steps and 3 eager ones)
python tools/timeline.py "$f" k_adamw -26 -v > gpurun_out/tl_$TAG/timeline.txt
s=$(find gpurun_out/tl_$TAG -name '*kernel_stats.csv' | head -1)
python tools/kstats.py "$s" 26 30 > gpurun_out/tl_$TAG/kstats.txt
# keep the derived timeline / stats, drop the per-dispatch trace (gpurun merges back at most 64 MiB)
find gpurun_out/tl_$TAG -name '*kernel_trace.csv' -size +4M -delete
