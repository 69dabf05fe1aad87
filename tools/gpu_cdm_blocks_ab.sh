# usage: bash tools/gpu_cdm_blocks_ab.sh : CDM / joint-CDM step vs the weight-gradient split target (GHM_WGRAD_BLOCKS)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r4_ab23
for w in cdm cdm_joint; do for v in 256 128 192 384; do
  GHM_WGRAD_BLOCKS=$v timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/r4_ab23/b.json 2> gpurun_out/r4_ab23/b.err || exit 3
  echo "$w blocks=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4_ab23/b.json)"
done; done | tee gpurun_out/r4_ab23/ab.txt
