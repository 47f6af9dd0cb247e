#!/bin/bash
# The multi-rank bench path on one GPU: 2 ranks on cuda:0, gloo collectives (KBZ_BENCH_REHEARSE);
# timings are meaningless, completion and the line's fields are what is checked.
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${TAG:-r05_final}/rehearsal_2ranks_1gpu; mkdir -p $O
for w in config2 merge stream; do
  echo "== rehearsal $w $(date +%T)"
  KBZ_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 2 --no-cpu --workload $w > $O/$w.json 2> $O/$w.err || { tail -20 $O/$w.err; exit 1; }
  tail -c 300 $O/$w.json; echo
done
