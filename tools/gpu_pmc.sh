# usage: bash tools/gpu_pmc.sh TAG KERNELS : SQ counter passes over kbench --only KERNELS
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-p1}
ONLY=${2:-ln_mlp_fwd_x3,mlp_bwd_x3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ok() { r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_FLAT SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o run -- python tools/kbench.py --reps 2 --only $ONLY > $OUT/pmc$i.log 2>&1
  ok $? || exit $((10+i))
done
echo done
