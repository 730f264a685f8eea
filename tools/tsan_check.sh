#!/bin/bash
# Race detection for the native control-plane core (survey §5.2): build it with
# -fsanitize=thread and run a multi-threaded producer/consumer stress under libtsan.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${TMPDIR:-/tmp}/ai4e_tsan
mkdir -p "$OUT"
EXT=$(python -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
g++ -O1 -g -fsanitize=thread -std=c++17 -shared -fPIC -I"$(python -c 'import sysconfig;print(sysconfig.get_paths()["include"])')" \
    -I"$(python -c 'import pybind11;print(pybind11.get_include())')" "$ROOT/csrc/core/ai4e_core.cpp" -o "$OUT/_ai4e_core$EXT" -lpthread
TSAN_OPTIONS="halt_on_error=1 report_signal_unsafe=0" LD_PRELOAD=$(gcc -print-file-name=libtsan.so) \
    python "$ROOT/tools/tsan_stress.py" "$OUT" 2>&1 | tee "$OUT/tsan.log" | tail -3
! grep -q "WARNING: ThreadSanitizer" "$OUT/tsan.log"
