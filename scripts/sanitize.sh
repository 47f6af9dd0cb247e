#!/bin/bash
# AddressSanitizer + UndefinedBehaviorSanitizer builds of the host C libraries -- the plugin
# (killerbeez_amd/csrc/kbz_plugin.c: JSON, hex, state files, worker threads) and the oracle
# restatement (oracle/kbz_oracle.c) -- and the CPU tests that exercise them, run against those
# builds (SURVEY.md §5 "Race detection / sanitizers").  Host code only: no GPU sanitizer.
# usage: scripts/sanitize.sh [extra pytest args]      (CPU; a few minutes)
set -e
cd "$(dirname "$0")/.."
python -c "from killerbeez_amd import build; build.build_all()"
OUT=build/asan
mkdir -p $OUT
SAN="-fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer -g -O1"
gcc $SAN -fPIC -shared -Wall -std=gnu11 -pthread -I include killerbeez_amd/csrc/kbz_plugin.c \
  -L killerbeez_amd -lkbz_hip -Wl,-rpath,$PWD/killerbeez_amd -o $OUT/libkbz_plugin.so
gcc $SAN -fPIC -shared -Wall -Wno-unused-function -Wno-unused-variable -fopenmp \
  oracle/kbz_oracle.c -o $OUT/libkbz_oracle.so
PRE="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
# leaks: the Python interpreter's own allocations are not ours to report
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:alloc_dealloc_mismatch=0:detect_odr_violation=0
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
KBZ_PLUGIN_LIB=$PWD/$OUT/libkbz_plugin.so KBZ_ORACLE_LIB=$PWD/$OUT/libkbz_oracle.so \
  LD_PRELOAD="$PRE${LD_PRELOAD:+ $LD_PRELOAD}" python -m pytest -q -p no:cacheprovider -m "not gpu" \
  tests/test_plugin.py tests/test_plugin_fuzz.py tests/test_golden.py tests/test_oracle_pin.py "$@"
echo "sanitizer suite clean"
