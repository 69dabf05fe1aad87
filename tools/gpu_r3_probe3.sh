# usage: bash tools/gpu_r3_probe3.sh TAG : which statistics the QKV backward's late plain load returns
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
for va in "qkv_dbgu wgrad0" "qkv_dbgu none" "qkv_load none" "qkv_dbg wgrad0" "qkv_dev wgrad0" "mlp_bwd wgrad0"; do
  set -- $va
  timeout -k 10 150 python tools/race_probe.py $1 $2 40 > $OUT/probe_$1_$2.txt 2>&1 || exit 3
  echo "$(tail -n 1 $OUT/probe_$1_$2.txt)"
done
echo done
