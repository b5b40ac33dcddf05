#!/bin/bash
# Build ablation variants of libcodenerf_hip.so into code-nerf_amd/codenerf/lib/ablate/
set -e
cd "$(dirname "$0")/../code-nerf_amd/csrc"
mkdir -p ../codenerf/lib/ablate
for v in "$@"; do
  flags=""
  for f in $(echo $v | tr '+' ' '); do [ "$f" != "base" ] && flags="$flags -DCN_ABLATE_$f"; done
  make -s BUILD=build_$v OUT=../codenerf/lib/ablate/lib_$v.so CXXFLAGS_EXTRA="$flags" -j8 >/dev/null
  echo "built $v ($flags)"
done
