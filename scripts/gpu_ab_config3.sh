#!/bin/bash
# Config-3 session: VALU probe, pass-1 parity tests, k_pass1w variant A/B (timing only).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== valuprobe"; timeout -k 10 60 ./tools/valuprobe > gpurun_out/valuprobe.txt 2>&1; rc=$?; cat gpurun_out/valuprobe.txt; [ $rc -eq 0 ] || exit $rc
echo "== parity"; timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_wide.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_wide.log; [ $rc -eq 0 ] || exit $rc
echo "== ab"; VARIANTS="${VARIANTS:-v4 lp0 nl2 nl8 d3}" BENCH_ARGS="--workload config3" STEPS=6 bash scripts/ab_variants.sh
if [ -d build_variants/st_v4 ]; then
  echo "== stamps"; KBZ_HIP_LIB=$PWD/build_variants/st_v4/libkbz_hip.so timeout -k 10 200 python tools/stamps_wide.py 2>&1 | grep -v amdgpu.ids
fi
