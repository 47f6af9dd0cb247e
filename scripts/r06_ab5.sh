#!/bin/bash
# Round 6: the AFL plugin's small windows from C (tools/plugin_loop): k_small with one-wave
# workgroups (small64) and sub-batched windows (KBZ_PLUGIN_SUBBATCH), alternating with the
# product; then the plugin parity tests.
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${TAG:-r06_ab5}; mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_plugin.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
P=/tmp/kbz_pool
python3 - <<PY || exit 1
import numpy as np
from killerbeez_amd import synth
t, oc = synth.sparse_np(2048, 65536, seed=0x5EED)
t.tofile("$P.bin"); oc.astype(np.int8).tofile("$P.oc")
PY
for rep in 1 2; do
  for v in base small64 sub4 sub8 sub8_small64; do
    lp=""; sk=0
    case $v in *small64*) lp=$PWD/build_variants/small64;; esac
    case $v in sub4*) sk=4;; sub8*) sk=8;; esac
    for b in 1 16 64; do
      e=4096; [ $b = 1 ] && e=2048
      r=$(LD_LIBRARY_PATH=$lp KBZ_PLUGIN_SUBBATCH=$sk timeout -k 10 120 ./tools/plugin_loop afl $P.bin $P.oc 65536 2048 $e $b) || { echo "$v $b failed"; exit 1; }
      echo "$v B=$b $r" | tee -a $O/ab_small.txt
    done
  done
done
rm -f $P.bin $P.oc
