# round 6: (1) review item 2 -- the two towers serialized on one stream (each layer
# kernel then runs alone on the chip, as one merged two-tower grid would run its
# halves) against the concurrent two-stream step, alternating 200-step benches;
# (2) the VLM step's FETCH / WRITE passes for the VLM line's traffic field
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_abenv.sh ${1:-r6_serial} "" - GHM_SERIAL_TOWERS=1 || exit 2
bash tools/gpu_vlm_traffic.sh ${1:-r6_serial}_vt || exit 3
echo done
