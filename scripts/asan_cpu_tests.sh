#!/bin/bash
# Host-side AddressSanitizer run of the CPU test suite (type map, plan compiler, raw
# export, external32 signature: everything that runs without a GPU).  The device code is
# compiled normally; only host objects are instrumented (-Xarch_host -fsanitize=address).
set -e
cd "$(dirname "$0")/../ompi_amd/csrc"
mkdir -p build_asan
for f in ddt_typemap ddt_optimize ddt_plan ddt_convertor ddt_external ddt_pool; do
  /opt/rocm/bin/hipcc -std=c++17 -O1 -g -fPIC -I../../include --offload-arch=gfx950 \
    -Xarch_host -fsanitize=address -fno-omit-frame-pointer -c $f.cpp -o build_asan/$f.o
done
# the opal bridge (plain C, gcc in the product build) with the same instrumentation
/opt/rocm/llvm/bin/clang -std=gnu11 -O1 -g -fPIC -pthread -I../../include -fsanitize=address \
  -fno-omit-frame-pointer -c ../../bridge/opal_datatype_hip_bridge.c -o build_asan/opal_datatype_hip_bridge.o
for f in ddt_kernels ddt_sorted ddt_move_p0 ddt_move_p1 ddt_move_u0 ddt_move_u1; do
  /opt/rocm/bin/hipcc -std=c++17 -O1 -fPIC -I../../include --offload-arch=gfx950 -x hip \
    -c $f.hip -o build_asan/$f.o &
done
wait
printf 'extern "C" const char *ddt_build_id(void) { return "%s"; }\n' "$(python3 ../../scripts/srcsha.py)" > build_asan/ddt_build_id.cpp
g++ -O1 -fPIC -c build_asan/ddt_build_id.cpp -o build_asan/ddt_build_id.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Xarch_host -fsanitize=address \
  -o build_asan/libddt_hip_asan.so build_asan/*.o
cd ../..
ASAN_RT=$(/opt/rocm/bin/hipcc -print-file-name=libclang_rt.asan-x86_64.so)
# the ASan runtime goes first; whatever the environment already preloads stays in the list
DDT_LIB_PATH=$PWD/ompi_amd/csrc/build_asan/libddt_hip_asan.so LD_PRELOAD=$ASAN_RT${LD_PRELOAD:+:$LD_PRELOAD} \
  ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 python -m pytest tests -q -x -m "not gpu" -p no:cacheprovider "$@"
