# One SQ counter pass (LDS conflicts, waits) over short sequential and joint CDM benches
# (round 4 "r4_m4"), each under its own KILL timeout.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r4_m4 && mkdir -p $O
for w in cdm cdm_joint; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES \
    --output-format csv -d $O/$w -o run -- python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $O/$w.log 2>&1 || exit 3
  echo "$w ok"
done
