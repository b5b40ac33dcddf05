#!/bin/bash
# Build a library variant from the kernel sources of a commit (default: the working tree), optionally
# patched by a python script run in the copy's csrc -- A/B of code-path alternatives that do not stay
# in the tree.  Output: code-nerf_amd/codenerf/lib/variants/lib_<name>.so (load it with
# CODENERF_ALLOW_STALE=1 CODENERF_LIB=...).      tools/build_patched.sh <name> [<commit>|tree] [patch.py]
set -e
NAME=$1; REV=${2:-tree}; PATCH=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/cn_variant_$NAME
rm -rf $W && mkdir -p $W
if [ "$REV" = tree ]; then
  mkdir -p $W/code-nerf_amd/codenerf $W/include
  cp -r $ROOT/code-nerf_amd/csrc $W/code-nerf_amd/ && rm -rf $W/code-nerf_amd/csrc/build*
  cp $ROOT/code-nerf_amd/codenerf/provenance.py $W/code-nerf_amd/codenerf/
  cp $ROOT/include/*.h $W/include/
else
  (cd $ROOT && git archive $REV code-nerf_amd/csrc code-nerf_amd/codenerf/provenance.py include) | tar -x -C $W
fi
[ -n "$PATCH" ] && (cd $W/code-nerf_amd/csrc && python3 $(cd "$(dirname "$PATCH")" && pwd)/$(basename "$PATCH"))
mkdir -p $ROOT/code-nerf_amd/codenerf/lib/variants
make -s -C $W/code-nerf_amd/csrc -j8 OUT=$ROOT/code-nerf_amd/codenerf/lib/variants/lib_$NAME.so >/dev/null
echo "built $NAME ($REV ${PATCH:-})"
