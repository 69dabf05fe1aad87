# usage: bash tools/gpu_check2.sh TAG : whole GPU suite, smoke, kbench, 200-step bench, LDS counters of the wgrad kernels
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
tail -3 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 3
timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 --json $OUT/kbench.json > $OUT/kbench.txt 2>&1 || exit 4
grep -E "wgrad|mlp_bwd_rc" $OUT/kbench.txt
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-final-risk > $OUT/bench.json 2> $OUT/bench.err || exit 5
echo "ws: $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench.json)"
GHM_WGRAD_STREAM=0 timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-final-risk > $OUT/bench_nows.json 2> $OUT/bench_nows.err || exit 6
echo "no ws: $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_nows.json)"
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d $OUT/pmc -o run -- python tools/kbench.py --reps 2 --only wgrad_w2_x3,wgrad_w1_x3,wgrad_qkv_x3,qkv_bwd_x3,ln_qkv_fwd_x3,attn_fwd_x3,attn_bwd_x3 > $OUT/pmc.log 2>&1
echo done
