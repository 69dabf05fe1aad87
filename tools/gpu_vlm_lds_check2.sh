# permuted rows for the k-contiguous GEMM tiles (round 4 "r4_ab27"): GEMM + VLM
# + joint CDM GPU tests, the VLM / joint VLM / joint CDM bench lines, one LDS PMC pass.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r4_ab27 && mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gemm.py tests/test_gpu_vlm.py tests/test_gpu_vlm_joint.py tests/test_gpu_vlm_guided.py \
  tests/test_gpu_cdm_joint.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
for w in vlm vlm vlm_joint cdm_joint; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > $O/b_$w.json 2> $O/b_$w.err || exit 3
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $O/b_$w.json)"
done | tee $O/ab.txt
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --output-format csv \
  -d $O/pmc -o run -- python bench.py --workload vlm --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc.log 2>&1 || exit 4
echo done
