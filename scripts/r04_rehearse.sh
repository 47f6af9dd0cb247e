#!/bin/bash
# The multi-rank bench path on one GPU (KBZ_BENCH_REHEARSE=1: 2 ranks on cuda:0, gloo
# collectives): triage, merge and stream legs; timings meaningless, the path is what is checked.
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04_rehearse}; mkdir -p $O
for w in config2 merge stream; do
  echo "== $w $(date +%T)"
  KBZ_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --workload $w --steps 3 --warmup 2 --no-cpu --no-pmc --no-ktrace --no-variants > $O/rehearse_$w.json 2> $O/rehearse_$w.err || { tail -20 $O/rehearse_$w.err; exit 1; }
  tail -c 300 $O/rehearse_$w.json; echo
done
