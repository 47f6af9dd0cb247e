#!/bin/bash
# Round-4 GPU call: parity suite, smoke, then the legs named in LEGS (bench.py args per leg),
# then optional diagnostics (DIAG: tail = k_scan per-wave records from the KBZ_TAIL_STAMPS
# variant).  Each GPU step has its own time limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04}; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
# heartbeat: the first import torch on a fresh box plus collection can be silent for minutes
( while sleep 30; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -z "$SKIP_TESTS" ]; then
  step pytest
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
  tail -2 $O/pytest_gpu.txt
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
  tail -1 $O/smoke.txt
fi
IFS=';' read -ra LEGS <<< "${LEGS:-config2|--no-cpu}"
for leg in "${LEGS[@]}"; do
  [ -z "$leg" ] && continue
  name=${leg%%|*}; args=${leg#*|}
  step "bench $name ($args)"
  KBZ_BENCH_KTRACE_OUT=$O/ktrace_$name.json timeout -k 10 400 python -u bench.py $args > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  tail -c 400 $O/bench_$name.json; echo
done
for d in $DIAG; do
  case $d in
    tail)
      step "tail stamps"
      KBZ_HIP_LIB=$PWD/build_variants/tailst/libkbz_hip.so timeout -k 10 200 python -u tools/tail_stamps.py > $O/tail_stamps.txt 2>&1 || { tail $O/tail_stamps.txt; exit 1; }
      cat $O/tail_stamps.txt | cut -c1-600 ;;
    pass1d)
      step "k_pass1d per-wave stamps (config 3)"
      KBZ_STAMP_NAMES=d KBZ_HIP_LIB=$PWD/build_variants/stamps/libkbz_hip.so timeout -k 10 200 python -u tools/stamps_wide.py > $O/stamps_pass1d.txt 2>&1 || { tail $O/stamps_pass1d.txt; exit 1; }
      cat $O/stamps_pass1d.txt ;;
  esac
done
step done
