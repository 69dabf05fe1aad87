# usage: bash tools/gpu_r3_round.sh TAG : GPU tests, smoke, bench (full), rocprof kernel stats of the bench,
#        MFMA-utilisation and HBM-traffic PMC passes over kbench (x3 kernels)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
ok() { r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/gpu_tests.log
grep -E "^FAILED|^ERROR|passed|failed" $OUT/gpu_tests.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 3
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 4
grep -o '"ms_per_step": [0-9.]*' $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_clip -o run -- \
   python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-final-risk > $OUT/prof_clip.json 2> $OUT/prof_clip.err
ok $? || exit 6
find $OUT -name '*kernel_trace.csv' -size +4M -delete
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o run -- python tools/kbench.py --reps 2 --precision x3 > $OUT/pmc$i.log 2>&1
  ok $? || exit $((10+i))
done
python tools/mfma_util.py $OUT $OUT/mfma_util.txt > /dev/null
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python tools/kbench.py --reps 3 --precision x3 > $OUT/fetch.log 2>&1
ok $? || exit 20
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python tools/kbench.py --reps 3 --precision x3 > $OUT/write.log 2>&1
ok $? || exit 21
python tools/traffic.py $OUT/fetch $OUT/write --json $OUT/traffic.json > $OUT/traffic.txt
timeout -k 10 200 python tools/kbench.py --reps 20 --precision x3 --json $OUT/kbench.json > $OUT/kbench.txt 2>&1 || exit 22
echo done
