# usage: bash tools/gpu_measure.sh TAG : per-kernel HBM traffic (FETCH_SIZE / WRITE_SIZE passes), the SQ counter
#        passes of the big x3 kernels (MFMA busy, VALU / LDS instruction mix, LDS bank conflicts) and a step timeline
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-m1}
mkdir -p gpurun_out/$TAG
bash tools/gpu_traffic.sh ${TAG}_traffic || exit 2
python tools/traffic.py gpurun_out/${TAG}_traffic/fetch gpurun_out/${TAG}_traffic/write --json gpurun_out/${TAG}_traffic/traffic.json > gpurun_out/${TAG}_traffic/traffic.txt 2>&1 || exit 3
bash tools/gpu_pmc.sh ${TAG}_pmc ln_mlp_fwd_x3b,mlp_bwd_rc_x3,attn_bwd_x3,wgrad_w2_x3,wgrad_w1_x3,wgrad_qkv_x3,qkv_bwd_x3,ln_qkv_fwd_x3,attn_fwd_x3,ln_mlp_fwd_x6,ln_qkv_fwd_x6 || exit 4
python tools/mfma_util.py gpurun_out/${TAG}_pmc gpurun_out/${TAG}_pmc/mfma_util.txt > /dev/null 2>&1
python tools/pmc_summary.py gpurun_out/${TAG}_pmc/pmc1 gpurun_out/${TAG}_pmc/pmc2 gpurun_out/${TAG}_pmc/pmc3 > gpurun_out/${TAG}_pmc/summary.txt 2>&1
bash tools/gpu_timeline.sh ${TAG} || exit 5
echo done
