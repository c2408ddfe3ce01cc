#!/bin/bash
# Build libwsmc with extra -D flags into tools/variants/libwsmc_<name>.so (experiments only;
# select with WSMC_LIB=...). Usage: tools/build_variant.sh NAME -DWSMC_SCAN_BLOCK=512 ...
set -e
name=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/tools/variants/obj_$name
mkdir -p "$O"
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math --offload-arch=gfx950 -I$R/include -I$R/weightedsampling.jl_amd/csrc -I$R/weightedsampling.jl_amd/build -Wno-unused-result -munsafe-fp-atomics $*"
/opt/rocm/bin/hipcc $F -c "$R/weightedsampling.jl_amd/csrc/wsmc_kernels.hip" -o "$O/k.o" &
/opt/rocm/bin/hipcc $F -c "$R/weightedsampling.jl_amd/csrc/wsmc_api.hip" -o "$O/a.o" &
/opt/rocm/bin/hipcc $F -c "$R/weightedsampling.jl_amd/csrc/wsmc_multi.hip" -o "$O/m.o" &
/opt/rocm/bin/hipcc $F -c "$R/weightedsampling.jl_amd/csrc/wsmc_jit.hip" -o "$O/j.o" &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$O/k.o" "$O/a.o" "$O/m.o" "$O/j.o" -o "$R/tools/variants/libwsmc_$name.so" -L/opt/rocm/lib -lrccl -lhiprtc -Wl,-rpath,/opt/rocm/lib
rm -rf "$O"
echo "$R/tools/variants/libwsmc_$name.so"
