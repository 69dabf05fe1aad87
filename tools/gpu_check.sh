cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m2 -E "gfx950|Marketing" > gpurun_out/devinfo.txt
timeout -k 10 600 python -m pytest tests -m gpu -q -v -rA > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
  echo "bench rc=$?" >> gpurun_out/bench1.err
fi
