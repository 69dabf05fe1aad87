cd $GRAFT_REPO_ROOT
for i in 1 2; do for v in 256 512 384; do
  GHM_WGRAD_BLOCKS=$v timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-final-risk 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/blocks=$v /"
done; done
