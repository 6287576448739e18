#!/usr/bin/env bash
# ASan + UBSan run of the C++ host runtime (block manager, scheduler, pybind bindings) under
# its CPU test suites: tests/test_runtime.py (scheduler/block-manager semantics), the
# hypothesis property tests (randomised op sequences) and the CPU engine tests (the runtime
# driven by real engine steps).  Host code only -- nothing here touches a GPU.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${1:-/tmp/akap_asan}
python3 -m aws_k8s_ansible_provisioner_amd.build_ext --sanitize-runtime "$OUT"
export AKAP_RUNTIME_DIR="$OUT"
export LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
# python itself is not instrumented: leak reports would list interpreter allocations
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:strict_string_checks=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
python3 -m pytest -x -q -p no:cacheprovider tests/test_runtime.py tests/test_properties.py \
    tests/test_engine_cpu.py -m "not gpu"
