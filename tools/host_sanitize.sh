#!/bin/bash
# Host-side sanitizer build of the native launch planners: AddressSanitizer +
# UndefinedBehaviorSanitizer over tools/host_checks.cpp, which sweeps the planners of
# csrc/include/apex_amd/launch_plan.h (the header the .hip launchers call) over ResNet /
# transformer / edge shapes and asserts their coverage invariants.  CPU only -- GPU ASan and
# xnack+ code objects are not available on this pool.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-/tmp/apex_host_checks}
${CXX:-g++} -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
  -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I"$ROOT/rocm-apex_amd/csrc/include" \
  "$ROOT/tools/host_checks.cpp" -o "$OUT"
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 "$OUT"
