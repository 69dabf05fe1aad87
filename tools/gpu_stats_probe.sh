# usage: bash tools/gpu_stats_probe.sh TAG : LN-statistics load characterisation (DESIGN.md §4 "Determinism")
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
for va in "qkv_dbg wgrad0" "qkv_load wgrad0" "qkv_dev wgrad0" "qkv_sc1 wgrad0" "qkv_bwd wgrad0" "qkv_dbg none"; do
  set -- $va
  timeout -k 10 150 python tools/race_probe.py $1 $2 40 > $OUT/probe_$1_$2.txt 2>&1 || exit 3
  echo "$(tail -n 1 $OUT/probe_$1_$2.txt)"
done
echo done
