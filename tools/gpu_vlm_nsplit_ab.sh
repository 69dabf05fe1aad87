cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r4_ab22
for i in 1; do for v in 16 12 20 24; do
  GHM_VLM_NSPLIT=$v timeout -k 10 200 python bench.py --workload vlm --no-cpu-baseline > gpurun_out/r4_ab22/b.json 2> gpurun_out/r4_ab22/b.err || exit 3
  echo "nsplit=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4_ab22/b.json)"
done; done | tee gpurun_out/r4_ab22/ab.txt
