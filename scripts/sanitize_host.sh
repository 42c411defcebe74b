#!/bin/bash
# Host-side sanitizer run (CPU only, no GPU): libopenr_decision.so and the
# oracle rebuilt with -fsanitize=address,undefined (or thread with
# SAN=thread) into /tmp/openr_san/, then the CPU tests that drive them --
# incl. the link-event sequences with every SPF on the host
# (tests/test_host_link_events.py) -- with the sanitizer runtime preloaded
# into the (uninstrumented) Python interpreter.
#   bash scripts/sanitize_host.sh [pytest args...]
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SAN=${SAN:-address,undefined}
OUT=/tmp/openr_san/${SAN//,/_}
mkdir -p "$OUT"
D=$ROOT/openr_amd/csrc/decision
FL="-O1 -g -fno-omit-frame-pointer -std=c++17 -fPIC -shared -fsanitize=$SAN"
g++ $FL -o "$OUT/libopenr_decision.so" $D/link_state.cpp $D/spf_solver.cpp $D/adjdb_thrift.cpp $D/decision_capi.cpp \
  -L"$ROOT/openr_amd/lib" -lopenr_spf_hip -Wl,-rpath,"$ROOT/openr_amd/lib"
g++ $FL -pthread -o "$OUT/liboracle.so" "$ROOT/oracle/linkstate_oracle.cpp"
case $SAN in
  thread) RT=$(g++ -print-file-name=libtsan.so); export TSAN_OPTIONS="halt_on_error=1 report_signal_unsafe=0";;
  *) RT="$(g++ -print-file-name=libasan.so) $(g++ -print-file-name=libubsan.so)"
     export ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1"
     export UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1";;
esac
cd "$ROOT"
TESTS=${*:-tests/test_host_link_events.py tests/test_host_link_patch.py tests/test_host_linkstate.py}
OPENR_DECISION_SO="$OUT/libopenr_decision.so" OPENR_ORACLE_SO="$OUT/liboracle.so" \
  LD_PRELOAD="$RT" python -m pytest -x -q -p no:cacheprovider -m "not gpu" $TESTS
