# GEMM tile-height cut A/B (GHM_GEMM_TM2_MIN_N: 128-row tiles for N >= the cut, 64-row
# below; round 4 "r4_ab28"), alternating VLM benches after the LDS-conflict fixes.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r4_ab28 && mkdir -p $O
for i in 1 2; do for v in 768 256 100000; do
  GHM_GEMM_TM2_MIN_N=$v timeout -k 10 200 python bench.py --workload vlm --no-cpu-baseline > $O/b.json 2> $O/b.err || exit 3
  echo "tm2_min_n=$v $(grep -o '"ms_per_step": [0-9.]*' $O/b.json)"
done; done | tee $O/ab.txt
