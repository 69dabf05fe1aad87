# usage: bash tools/gpu_r3_v3.sh TAG : parity check, tower-order x deferred-reduce A/B + timelines, stats probes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_gemm.py -m gpu -k "forward_stages or encoder_backward or train_steps or default_config_curve or attention_x3 or bit_identical or unperturbed" > $OUT/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -n 2 $OUT/parity.log; [ $rc -eq 0 ] || exit 2
for i in 1 2; do
  for cfg in "sequential 0 split" "sequential 1 split" "interleave 1 split" "interleave 1 fused"; do
    set -- $cfg
    GHM_TOWER_ORDER=$1 GHM_DEFER_REDUCE=$2 GHM_ATTN_BWD=$3 timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-final-risk 2>/dev/null > $OUT/bench_$1_$2_$3.json || exit 4
    echo "$1 defer=$2 attn=$3 $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$1_$2_$3.json)"
  done
done
for cfg in "sequential 0 split" "interleave 1 fused"; do
  set -- $cfg
  GHM_TOWER_ORDER=$1 GHM_DEFER_REDUCE=$2 GHM_ATTN_BWD=$3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tl_$1 -o run -- \
     python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-final-risk > /dev/null 2>&1 || exit 5
  python tools/timeline.py $OUT/tl_$1/run_kernel_trace.csv k_adamw -5 -v > $OUT/timeline_$1.txt 2>&1
  head -2 $OUT/timeline_$1.txt
  find $OUT/tl_$1 -name '*kernel_trace.csv' -size +4M -delete
done
bash tools/gpu_r3_probe2.sh $TAG
