// Instrumentation probes of the field and dW kernels: OFF in every product build.
//
// Each probe is compiled in only when its macro is defined on the hipcc line
// (tools/build_variants.sh PROLOGUE | WGTIME | TN_WAITPROF writes such a library to
// code-nerf_amd/codenerf/lib/variants/); the product library defines none of them, so the
// kernels' code is the same as with the probe sites absent.
//
//   CN_PROBE_PROLOGUE    field_w16 forward / backward: per (workgroup, wave) shader clocks from a
//                        tile's start to its first weight chunk, the tile loop's clocks and the
//                        tile count of the last launch (read by cn_debug_prologue; tools/prologue.py)
//   CN_PROBE_WGTIME      field_w16 forward: each workgroup's start / end wall clock (100 MHz)
//                        (read by cn_debug_wgtime; tools/wgtime.py)
//   CN_PROBE_TN_WAITPROF whole-tile dW GEMM: per (workgroup, wave) clocks at the stage barrier, in
//                        the DMA issue, in the whole loop, and the stage count (read by
//                        cn_debug_tnprof; tools/tnprof.py)
//
// The probes write their records with ordinary (vector) global stores from one lane.
#pragma once

#if defined(CN_PROBE_PROLOGUE) || defined(CN_PROBE_WGTIME) || defined(CN_PROBE_TN_WAITPROF)
#define CN_INSTRUMENTED 1
#endif
