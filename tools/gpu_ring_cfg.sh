# usage: bash tools/gpu_ring_cfg.sh TAG ["VARIANTS"] ["CFGS"] : ring weight-gradient tests, then isolated times of the
# weight-gradient kernels under each GHM_WGRAD_RING_CFG, then alternating step benches
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wgrad_ring.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 2; }
tail -1 $OUT/tests.log
VARIANTS=${2:-"GHM_WGRAD_RING_CFG=1 GHM_WGRAD_RING_CFG=2 GHM_WGRAD_RING_CFG=3 GHM_WGRAD_RING=0"}
CFGS=${3:-"1 2 3"}
K=mlp_bwd_rc_x3,wgrad_w2_x3,wgrad_w1_x3,wgrad_qkv_x3,wgrad_ring_w2,wgrad_ring_w1,wgrad_ring_qkv
for c in $CFGS; do
  GHM_WGRAD_RING_CFG=$c timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 --only $K > $OUT/kbench_cfg$c.txt 2>&1 || { tail $OUT/kbench_cfg$c.txt; exit 5; }
  echo "cfg $c"; grep -E "wgrad|mlp" $OUT/kbench_cfg$c.txt
done
for i in 1 2; do
  for v in $VARIANTS; do
    env $v timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-final-risk > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 3; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/b.json)"
  done
done | tee $OUT/ab.txt
