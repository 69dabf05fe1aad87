export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k "wcolsum or colsum or rows_linear" > $O/t.log 2>&1 || exit 2
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/kbench.py --reps 20 --precision x3 --only embed_bwd_tok,embed_bwd_pos,embed_bwd_old > $O/kb.txt 2>&1 || exit 3
