#!/bin/bash
# Address-sanitized HOST code on the GPU (device code uninstrumented; GPU
# ASan / xnack are not used): the engine's host side (-Xarch_host
# -fsanitize=address), libopenr_decision and the oracle built with clang's
# shared ASan runtime into build/asan/, and tests/native/link_events_driver
# (the instrumented executable, so the runtime loads first) run the link-event
# sequences of tests/link_events.py against the oracle.
#   bash scripts/asan_gpu.sh build        (here, CPU: compiles everything)
#   bash scripts/asan_gpu.sh run [seeds] [host]   (on the GPU box)
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build/asan
CLANGRT=$(dirname "$(/opt/rocm/lib/llvm/bin/clang++ -print-file-name=libclang_rt.asan-x86_64.so)")
[ -f "$CLANGRT/libclang_rt.asan-x86_64.so" ] || CLANGRT=$(ls -d /opt/rocm/lib/llvm/lib/clang/*/lib/linux | head -1)
SAN="-fsanitize=address -fno-omit-frame-pointer -shared-libsan"
case ${1:-build} in
build)
  mkdir -p "$OUT/obj"
  E=$ROOT/openr_amd/csrc/engine
  pids=()
  for f in spf_kernels spf_bfs spf_msbfs spf_ksp2 spf_dial spf_wdial spf_wderive spf_levels \
           spf_cover spf_msdist spf_update spf_leaf spf_twin spf_small spf_engine spf_sweep; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -Wno-unused-result \
      -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer \
      -c -o "$OUT/obj/$f.o" "$E/$f.hip" &
    pids+=($!)
    if [ ${#pids[@]} -ge 8 ]; then wait "${pids[0]}"; pids=("${pids[@]:1}"); fi
  done
  for p in "${pids[@]}"; do wait "$p"; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $SAN -o "$OUT/libopenr_spf_hip.so" "$OUT"/obj/*.o \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -Wl,-rpath,"$CLANGRT"
  D=$ROOT/openr_amd/csrc/decision
  CXX=/opt/rocm/lib/llvm/bin/clang++
  $CXX -O1 -g -std=c++17 -fPIC -shared $SAN -o "$OUT/libopenr_decision.so" \
    $D/link_state.cpp $D/spf_solver.cpp $D/adjdb_thrift.cpp $D/decision_capi.cpp \
    -L"$OUT" -lopenr_spf_hip -Wl,-rpath,'$ORIGIN' -Wl,-rpath,"$CLANGRT"
  $CXX -O1 -g -std=c++17 -fPIC -shared -pthread $SAN -o "$OUT/liboracle.so" "$ROOT/oracle/linkstate_oracle.cpp" \
    -Wl,-rpath,"$CLANGRT"
  $CXX -O1 -g -std=c++17 $SAN -o "$OUT/link_events_driver" "$ROOT/tests/native/link_events_driver.cpp" \
    -L"$OUT" -lopenr_decision -lopenr_spf_hip -loracle -Wl,-rpath,'$ORIGIN' -Wl,-rpath,"$CLANGRT"
  echo "built $OUT";;
run)
  export ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:verify_asan_link_order=0:protect_shadow_gap=0"
  "$OUT/link_events_driver" "${2:-6}" 0 "${3:-0}";;
esac
