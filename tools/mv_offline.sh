#!/bin/bash
# Compile a dumped Move-block signature (WSMC_JIT_DUMP=<dir> writes mv_<n>.sig) offline with hipcc,
# the run-time compile's options, and print the kernels' register use. Usage:
#   tools/mv_offline.sh gpurun_out/r05_jd/mv_4.sig [out.s]
set -euo pipefail
sig="$1"
out="${2:-/tmp/mv_offline.s}"
root="$(cd "$(dirname "$0")/.." && pwd)"
tu=/tmp/mv_offline_tu.hip
python3 - "$sig" "$tu" <<'EOF'
import sys
sig = open(sys.argv[1]).read().strip()
if sig.startswith("mv:"):
    sig = sig[3:]
src = ('#define WSMC_TABLES_LDS 1\n#include "wsmc_mv_body.h"\n'
       'struct WsmcMvSig { static constexpr wsmc::MvSig sig = ' + sig + '; };\n'
       'constexpr unsigned kMvArgsAt = (sizeof(wsmc::ProgInlineBlk) + alignof(wsmc::MvArgs) - 1) & '
       '~(unsigned)(alignof(wsmc::MvArgs) - 1);\n'
       'extern "C" __global__ __launch_bounds__(256) void wsmc_mv_i(wsmc::ProgInlineBlk, wsmc::MvArgs) {\n'
       '  const char* ka = (const char*)__builtin_amdgcn_kernarg_segment_ptr();\n'
       '  wsmc::mv_body<WsmcMvSig>(ka + __builtin_offsetof(wsmc::ProgInlineBlk, w), '
       '*reinterpret_cast<const wsmc::MvArgs*>(ka + kMvArgsAt));\n}\n'
       'extern "C" __global__ __launch_bounds__(256) void wsmc_mv_g(wsmc::ProgInlineBlk, wsmc::MvArgs) {\n'
       '  const char* ka = (const char*)__builtin_amdgcn_kernarg_segment_ptr();\n'
       '  const wsmc::MvArgs& a = *reinterpret_cast<const wsmc::MvArgs*>(ka + kMvArgsAt);\n'
       '  wsmc::mv_body<WsmcMvSig>(a.prog, a);\n}\n')
open(sys.argv[2], "w").write(src)
EOF
/opt/rocm/bin/hipcc -x hip --cuda-device-only --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
    -fno-fast-math -munsafe-fp-atomics -Wno-unused-result -I"$root/include" \
    -I"$root/weightedsampling.jl_amd/csrc" -S -o "$out" "$tu"
grep -E '^\s+\.(vgpr_count|sgpr_count|vgpr_spill_count|name):' "$out" | grep -B0 -A0 -E 'name: +wsmc|count' || true
