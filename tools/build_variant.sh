# usage: bash tools/build_variant.sh GIT_REV|WORKTREE OUT_DIR [extra hipcc flags] : build libghm_hip.so of the
#        csrc at GIT_REV (or of the working tree) into OUT_DIR
# (A/B timing: GHM_HIP_LIB=OUT_DIR/libghm_hip.so selects it at run time)
set -e
REV=$1; OUT=$2; shift 2; EXTRA="$@"
SRC=$(mktemp -d)
mkdir -p $SRC/csrc $SRC/include $OUT
if [ "$REV" = WORKTREE ]; then
  mkdir -p $SRC/multimodal-ghm_amd && cp -r multimodal-ghm_amd/csrc $SRC/multimodal-ghm_amd/ && cp -r include $SRC/
else
  git archive $REV multimodal-ghm_amd/csrc include | tar -x -C $SRC
fi
objs=""
for f in $SRC/multimodal-ghm_amd/csrc/*.hip; do
  o=$SRC/$(basename $f .hip).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $EXTRA -c -o $o $f &
  objs="$objs $o"
done
wait
# a variant id: the variant's sources hashed (flags appended), so check_build_id reports it
printf '// variant build (tools/build_variant.sh)\nextern "C" const char* ghm_build_id(void) { return "variant-%s"; }\n' \
  "$(cat $SRC/multimodal-ghm_amd/csrc/* $SRC/include/*.h | sha256sum | cut -c1-12)$(echo $EXTRA | tr -d ' ')" > $SRC/bid.cpp
g++ -O2 -fPIC -c -o $SRC/bid.o $SRC/bid.cpp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libghm_hip.so $objs $SRC/bid.o
rm -rf $SRC
echo built $OUT/libghm_hip.so
