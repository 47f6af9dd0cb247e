#!/bin/bash
# Round-6 plugin-path evidence: tools/plugin_loop (the plugins driven from C in the fuzz loop's
# shape) with and without the early host-to-device copy of large windows (A/B, alternating), and
# kernel + HIP API traces of the batch-16 AFL and batch-256 DynamoRIO loops.
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_plugin}; mkdir -p $O
( while sleep 30; do date +%T >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
P=/tmp/kbz_pool
python3 - <<EOF || exit 1
import numpy as np
from killerbeez_amd import synth
t, oc = synth.sparse_np(2048, 65536, seed=0x5EED)
t.tofile("$P.bin"); oc.astype(np.int8).tofile("$P.oc")
np.zeros(2048, np.int8).tofile("$P.oc0")
EOF
loop() {  # mode batch execs [env...]
  local m=$1 b=$2 e=$3; shift 3
  local oc=$P.oc; [ $m = dynamorio ] && oc=$P.oc0
  env "$@" timeout -k 10 120 ./tools/plugin_loop $m $P.bin $oc 65536 2048 $e $b
}
if [ -z "$SKIP_AB" ]; then
  echo "== A/B early copy $(date +%T)"
  for rep in 1 2; do
    for ec in 0 1; do
      for spec in "afl 256 8192" "afl 4096 16384" "dynamorio 256 8192" "dynamorio 4096 16384"; do
        set -- $spec
        r=$(loop $1 $2 $3 KBZ_PLUGIN_EARLY_COPY=$ec) || { echo "loop failed"; exit 1; }
        echo "early_copy=$ec $1 B=$2 $r" | tee -a $O/ab_early_copy.txt
      done
    done
  done
fi
if [ -n "$TRACE" ]; then
  for spec in "afl 16 2048" "dynamorio 256 2048"; do
    set -- $spec
    echo "== trace $1 B=$2 $(date +%T)"
    oc=$P.oc; [ $1 = dynamorio ] && oc=$P.oc0
    timeout -k 10 180 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $O/tr_$1_$2 -o run -- ./tools/plugin_loop $1 $P.bin $oc 65536 2048 $3 $2 > $O/tr_$1_$2.json 2> $O/tr_$1_$2.err || { tail $O/tr_$1_$2.err; exit 1; }
    cat $O/tr_$1_$2.json
    for f in $(find $O/tr_$1_$2 -name '*_stats.csv'); do cp $f $O/$(basename $f .csv)_$1_$2.csv; done
    rm -f $(find $O/tr_$1_$2 -name '*_trace.csv' -size +20M)
  done
fi
rm -f $P.bin $P.oc $P.oc0
echo "== done $(date +%T)"
