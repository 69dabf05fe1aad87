# VLM split-k settings rechecked after the LDS-conflict fixes (round 4 "r4_ab29"):
# weight-gradient slabs (GHM_VLM_NSPLIT) and data-gradient slabs (GHM_VLM_DSPLIT), alternating.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r4_ab29 && mkdir -p $O
for i in 1 2; do for v in "16 1" "12 1" "24 1" "16 3"; do
  set -- $v
  GHM_VLM_NSPLIT=$1 GHM_VLM_DSPLIT=$2 timeout -k 10 200 python bench.py --workload vlm --no-cpu-baseline > $O/b.json 2> $O/b.err || exit 3
  echo "nsplit=$1 dsplit=$2 $(grep -o '"ms_per_step": [0-9.]*' $O/b.json)"
done; done | tee $O/ab.txt
