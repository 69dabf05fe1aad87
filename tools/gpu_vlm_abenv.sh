# usage: [WL=workload] bash tools/gpu_vlm_abenv.sh TAG "TESTS" SETTING... : GPU tests, then alternating benches of WL (default vlm)
#        (3 rounds), one per SETTING ("-" = defaults, else VAR=VAL[,VAR=VAL...]), then one rocprofv3 kernel-stats
#        run per SETTING (gpurun_out/TAG/stats_<n>.txt: the k_gemm_x3 kernels' average durations)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; TESTS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 2; }
  tail -2 $OUT/tests.log
fi
for i in 1 2 3; do
  for v in "$@"; do
    case "$v" in -) E="";; *) E=$(echo $v | tr ',' ' ');; esac
    env $E timeout -k 10 200 python bench.py --workload ${WL:-vlm} --steps 100 --warmup 10 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 3; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/b.json)"
  done
done | tee $OUT/ab.txt
n=0
for v in "$@"; do
  n=$((n + 1))
  case "$v" in -) E="";; *) E=$(echo $v | tr ',' ' ');; esac
  # env before rocprofv3: the profiler's preload must not exec through env
  [ -z "$E" ] || export $E
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$n -o run -- \
     python bench.py --workload ${WL:-vlm} --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof_$n.json 2> $OUT/prof_$n.err || exit 4
  for x in $E; do unset ${x%%=*}; done
  s=$(find $OUT/prof_$n -name '*kernel_stats.csv' | head -1)
  { echo "# $v"; python -c "
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:16]:
    print(f\"{float(r['AverageNs']) / 1e3:8.1f} us  x{r['Calls']:>5}  {r['Name'].replace('(anonymous namespace)::', '')[:90]}\")
" "$s"; } > $OUT/stats_$n.txt
  find $OUT/prof_$n -name '*kernel_trace.csv' -delete
done
echo done
