#!/bin/bash
# Round 6: k_small with one-wave workgroups (4x the workgroups reading the window over PCIe) on the
# AFL plugin's small windows, from C (tools/plugin_loop), alternating with the product.
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/r06_ab5; mkdir -p $O
P=/tmp/kbz_pool
python3 - <<PY || exit 1
import numpy as np
from killerbeez_amd import synth
t, oc = synth.sparse_np(2048, 65536, seed=0x5EED)
t.tofile("$P.bin"); oc.astype(np.int8).tofile("$P.oc")
PY
for rep in 1 2 3; do
  for v in base small64; do
    lp=""; [ $v != base ] && lp=$PWD/build_variants/$v
    for b in 1 16 64; do
      e=4096; [ $b = 1 ] && e=2048
      r=$(LD_LIBRARY_PATH=$lp timeout -k 10 120 ./tools/plugin_loop afl $P.bin $P.oc 65536 2048 $e $b) || { echo "$v $b failed"; exit 1; }
      echo "$v B=$b $r" | tee -a $O/ab_small.txt
    done
  done
done
rm -f $P.bin $P.oc
