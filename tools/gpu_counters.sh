# usage: bash tools/gpu_counters.sh TAG : kernel microbench + SQ/TCC counter passes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-c1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1
timeout -k 10 300 python tools/kbench.py --reps 10 --json $OUT/kbench.json > $OUT/kbench.txt 2>&1 || exit $?
ok() { r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc1 -o run -- python tools/kbench.py --reps 2 > $OUT/pmc1.log 2>&1
ok $? || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc2 -o run -- python tools/kbench.py --reps 2 > $OUT/pmc2.log 2>&1
ok $? || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc3 -o run -- python tools/kbench.py --reps 2 > $OUT/pmc3.log 2>&1
ok $? || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --output-format csv -d $OUT/pmc4 -o run -- python tools/kbench.py --reps 2 > $OUT/pmc4.log 2>&1
echo "done $?" >> $OUT/pmc4.log
