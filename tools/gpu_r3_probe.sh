# usage: bash tools/gpu_r3_probe.sh TAG : determinism probes + wait-fix A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
for va in "qkv_load wgrad0" "qkv_dev wgrad0" "qkv_load fwd_mlp" "qkv_dev fwd_mlp" "qkv_bwd wgrad0" \
          "mlp_bwd wgrad0" "mlp_bwd fwd_mlp" "wgrad wgrad0" "wgrad fwd_mlp" "mlp_bwd mlp_bwd"; do
  set -- $va
  timeout -k 10 120 python tools/race_probe.py $1 $2 15 > $OUT/probe_$1_$2.txt 2>&1 || exit 3
  echo "$(tail -n 1 $OUT/probe_$1_$2.txt)"
done
for va in "mlp_bwd wgrad0" "mlp_bwd fwd_mlp" "mlp_bwd mlp_bwd"; do
  set -- $va
  GHM_HIP_LIB=$PWD/ablib/base/libghm_hip.so timeout -k 10 120 python tools/race_probe.py $1 $2 15 > $OUT/probe_legacy_$1_$2.txt 2>&1 || exit 4
  echo "legacy vmcnt(4): $(tail -n 1 $OUT/probe_legacy_$1_$2.txt)"
done
bash tools/gpu_ab_lib.sh ablib/base/libghm_hip.so 2
echo done
