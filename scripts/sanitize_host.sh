#!/bin/bash
# Build the native host runtime + csrc/selftest/host_selftest.cc under
# AddressSanitizer+UBSan and under ThreadSanitizer, and run the self-test
# (CPU only; GPU sanitizers are not used).  usage: scripts/sanitize_host.sh [asan|tsan|all]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${SANITIZE_OUT:-/tmp/pbx_sanitize}"
mode="${1:-all}"
mkdir -p "$OUT"
SRC=("$ROOT/csrc/selftest/host_selftest.cc" "$ROOT"/csrc/host/{slot_dataset,key_agent,side_tables,cpu_ps,async_dense,dump,metrics,flags,msg_service,file_mgr}.cc)
g++ -O1 -g -shared -fPIC -I"$ROOT/csrc/host" "$ROOT/csrc/plugins/criteo_tsv_parser.cc" -o "$OUT/criteo_tsv_parser.so"
run() {  # name flags...
  local name=$1; shift
  g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fopenmp "$@" -I"$ROOT/csrc" "${SRC[@]}" -o "$OUT/selftest_$name" -ldl -lpthread
  rm -rf "$OUT/work_$name" && mkdir -p "$OUT/work_$name"
  echo "== $name"
  "$OUT/selftest_$name" "$OUT/work_$name" "$OUT/criteo_tsv_parser.so"
}
if [[ $mode == asan || $mode == all ]]; then
  ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
    run asan -fsanitize=address,undefined -fno-sanitize-recover=undefined
fi
if [[ $mode == tsan || $mode == all ]]; then
  # OpenMP runtime internals are not TSan-instrumented: run its regions on one thread
  OMP_NUM_THREADS=1 TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 run tsan -fsanitize=thread
fi
