#!/bin/bash
# round-3 GPU call: full parity on the in-tree build, wide-kernel parity of the CN variants,
# config-3 A/B (base / cn6 / cn7), stamps of k_pass1d, config-2 and config-3 bench lines.
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_v5}; mkdir -p $O
echo "== pytest (in-tree)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for v in $PARITY_VARIANTS; do
  echo "== pytest wide ($v)"
  KBZ_HIP_LIB=$PWD/build_variants/$v/libkbz_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "wide" > $O/pytest_$v.txt 2>&1 || { tail -30 $O/pytest_$v.txt; exit 1; }
  tail -1 $O/pytest_$v.txt
done
echo "== ab"
VARIANTS="$VARIANTS" BENCH_ARGS="--workload config3" STEPS=8 bash scripts/ab_variants.sh || exit 1
for v in $STAMP_VARIANTS; do
  echo "== stamps $v"; KBZ_STAMP_NAMES=d KBZ_HIP_LIB=$PWD/build_variants/$v/libkbz_hip.so timeout -k 10 200 python -u tools/stamps_wide.py > $O/stamps_$v.txt 2>&1 || { tail $O/stamps_$v.txt; exit 1; }
  cat $O/stamps_$v.txt
done
for w in $BENCH_WL; do
  echo "== bench $w"; timeout -k 10 300 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail $O/bench_$w.err; exit 1; }
  tail -c 400 $O/bench_$w.json
done
exit 0
