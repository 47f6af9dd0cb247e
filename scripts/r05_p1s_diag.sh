#!/bin/bash
# Config-2 pass-1 diagnosis: timing-only ablations of k_pass1s (KBZ_AB_P1S variants), per-wave
# stamps of the current k_pass1s, and one SQ-counter pass (VALU issue floor) on the product.
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_diag}; mkdir -p $O
( while sleep 30; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
echo "== ab $(date +%T)"
STEPS=10 VARIANTS="${VARIANTS:-base ab1 ab2 ab4 ab8 ab3 ab16 ab32 ab48 base2}" timeout -k 10 900 bash scripts/ab_variants.sh > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
echo "== stamps $(date +%T)"
KBZ_HIP_LIB=$PWD/build_variants/stamps/libkbz_hip.so timeout -k 10 200 python tools/stamps.py > $O/stamps_k_pass1s.txt 2>&1 || { tail $O/stamps_k_pass1s.txt; exit 1; }
cat $O/stamps_k_pass1s.txt
echo "== sq $(date +%T)"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O/sq -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-pmc --no-ktrace --no-variants > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
f=$(find $O/sq -name '*counter_collection.csv' | head -1); grep k_pass1 "$f" > $O/sq_k_pass1s_config2.csv; rm -rf $O/sq
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O/sq2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-pmc --no-ktrace --no-variants > $O/sq2.log 2>&1 && { f=$(find $O/sq2 -name '*counter_collection.csv' | head -1); grep k_pass1 "$f" > $O/sq2_k_pass1s_config2.csv; rm -rf $O/sq2; }
echo "== done $(date +%T)"
