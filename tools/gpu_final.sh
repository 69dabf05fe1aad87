# usage: bash tools/gpu_final.sh TAG : GPU suite, smoke, all benches, rocprof stats + timeline, PMC traffic, kbench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-f}
bash tools/gpu_round.sh $TAG || exit $?
bash tools/gpu_traffic.sh ${TAG}_t || exit $?
bash tools/gpu_timeline.sh $TAG || exit $?
python tools/traffic.py gpurun_out/${TAG}_t/fetch gpurun_out/${TAG}_t/write --json gpurun_out/${TAG}_t/traffic.json > gpurun_out/${TAG}_t/traffic.txt
find gpurun_out -name '*kernel_trace.csv' -size +4M -delete
echo final-done
