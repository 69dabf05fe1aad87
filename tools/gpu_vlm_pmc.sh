# usage: bash tools/gpu_vlm_pmc.sh [TAG]   SQ counter passes over a short VLM bench (round 4 "r4_m3"): where the split-bf16
# GEMM's wave cycles go (waits, LDS conflicts, MFMA busy).  One pass per run, each
# under its own KILL timeout; summarise with tools/pmc_summary.py.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${1:-r4_m3} && mkdir -p $O
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_FLAT SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $O/pmc$i -o run -- \
    python bench.py --workload vlm --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc$i.log 2>&1 || exit $((10+i))
  echo "pass $i ok"
done
echo done
