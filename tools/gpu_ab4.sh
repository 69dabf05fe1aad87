# usage: bash tools/gpu_ab4.sh TAG VARIANT_DIR : CLIP + VLM + CDM parity tests (in-tree lib), then kbench/bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_vlm.py tests/test_gpu_vlm_joint.py tests/test_gpu_vlm_guided.py tests/test_gpu_cdm.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 2; }
tail -2 $OUT/tests.log
bash tools/gpu_ab.sh $TAG "$@"
for w in vlm vlm_joint; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > $OUT/bench_${w}_base.json 2>/dev/null || exit 3
  GHM_HIP_LIB=$PWD/$1/libghm_hip.so timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > $OUT/bench_${w}_prev.json 2>/dev/null || exit 4
done
echo done
