#!/bin/bash
# Build variants of libcodenerf_hip.so into code-nerf_amd/codenerf/lib/variants/lib_<name>.so for A/B
# runs (CODENERF_LIB=... selects one).  A name is '+'-joined parts: base (no flag) or D<MACRO>[=<v>] for
# an experiment's own -D flag.   tools/build_variants.sh base DCN_FOO=2
# (the round-3..5 clock probes were removed from the kernels in round 6; their records stay in profiles/)
set -e
cd "$(dirname "$0")/../code-nerf_amd/csrc"
mkdir -p ../codenerf/lib/variants
for v in "$@"; do
  flags=""
  for f in $(echo $v | tr '+' ' '); do
    case $f in base) ;; D*) flags="$flags -${f}";;
      *) echo "unknown variant part $f"; exit 1;; esac
  done
  make -s BUILD=build_$v OUT=../codenerf/lib/variants/lib_$v.so CXXFLAGS_EXTRA="$flags" -j8 >/dev/null
  echo "built $v ($flags)"
done
