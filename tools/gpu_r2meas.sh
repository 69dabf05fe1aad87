# usage: bash tools/gpu_r2meas.sh TAG : PMC traffic passes + isolated kbench + a CLIP step timeline
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-m1}
bash tools/gpu_traffic.sh $TAG || exit $?
bash tools/gpu_timeline.sh $TAG || exit $?
f=$(find gpurun_out/$TAG/fetch -name '*counter_collection.csv' | head -1)
python tools/traffic.py gpurun_out/$TAG/fetch gpurun_out/$TAG/write --json gpurun_out/$TAG/traffic.json > gpurun_out/$TAG/traffic.txt
find gpurun_out -name '*kernel_trace.csv' -size +4M -delete
echo done
