#!/bin/bash
# Build variants of libcodenerf_hip.so into code-nerf_amd/codenerf/lib/variants/lib_<name>.so for A/B
# and probe runs (CODENERF_LIB=... selects one).  A name is '+'-joined parts: base (no flag), a probe
# of csrc/cn_instrument.h (PROLOGUE, WGTIME, TN_WAITPROF -> -DCN_PROBE_<part>), or D<MACRO>[=<v>]
# for an experiment's own -D flag.   tools/build_variants.sh base PROLOGUE DCN_FOO=2
set -e
cd "$(dirname "$0")/../code-nerf_amd/csrc"
mkdir -p ../codenerf/lib/variants
for v in "$@"; do
  flags=""
  for f in $(echo $v | tr '+' ' '); do
    case $f in base) ;; PROLOGUE|WGTIME|TN_WAITPROF) flags="$flags -DCN_PROBE_$f";; D*) flags="$flags -${f}";;
      *) echo "unknown variant part $f"; exit 1;; esac
  done
  make -s BUILD=build_$v OUT=../codenerf/lib/variants/lib_$v.so CXXFLAGS_EXTRA="$flags" -j8 >/dev/null
  echo "built $v ($flags)"
done
