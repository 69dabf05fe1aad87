# usage: bash tools/gpu_proto.sh TAG : review item 2 — isolated times of the fused-dW MLP backward prototype
# (abvar/proto, built by tools/build_variant.sh WORKTREE abvar/proto -DGHM_ABLATION_BUILD -DGHM_FUSED_DW_PROTO)
# against the product's MLP backward + dW2 / dW1 kernels, then its HBM traffic (FETCH_SIZE / WRITE_SIZE pass)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
K=mlp_bwd_rc_x3,wgrad_w2_x3,wgrad_w1_x3,reduce_w2,wgrad_ring_w2,wgrad_ring_w1,mlp_bwd_fused_proto,fused_proto_reduce
[ -n "$SKIP_KBENCH" ] || GHM_HIP_LIB=abvar/proto/libghm_hip.so timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 --only $K > $OUT/kbench.txt 2>&1 || { tail $OUT/kbench.txt; exit 5; }
cat $OUT/kbench.txt
for c in FETCH_SIZE WRITE_SIZE; do
  GHM_HIP_LIB=abvar/proto/libghm_hip.so timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- python tools/kbench.py --reps 2 --only $K > $OUT/pmc_$c.log 2>&1
  r=$?; [ $r -eq 0 ] || [ $r -eq 1 ] || exit 6
done
echo done
