# usage: bash tools/gpu_prof.sh TAG  -> gpurun_out/prof_TAG/ (kernel trace + stats)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r1}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -k "adamw" > gpurun_out/prof_$TAG/adamw_test.log 2>&1
echo "adamw rc=$?" >> gpurun_out/prof_$TAG/adamw_test.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
   python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$TAG/bench.json 2> gpurun_out/prof_$TAG/bench.err
echo "prof rc=$?" >> gpurun_out/prof_$TAG/bench.err
