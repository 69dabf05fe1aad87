# usage: bash tools/make_abbase.sh GIT_REV [OUT=abbase] : a runnable checkout of GIT_REV's bench.py,
#        Python package and native libraries (built here) for same-call A/B against the working tree
#        (tools/gpu_abenv.sh setting DIR=abbase); the Python side travels with the library, so the
#        two builds may differ in their C ABI
set -e
REV=$1; OUT=${2:-abbase}
rm -rf $OUT && mkdir -p $OUT
git archive $REV bench.py multimodal-ghm_amd include Makefile | tar -x -C $OUT
(cd $OUT && make -j8 > /dev/null)
rm -rf $OUT/build
echo built $OUT from $(git rev-parse --short $REV)
