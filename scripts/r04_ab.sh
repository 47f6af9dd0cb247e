#!/bin/bash
# Same-box A/B of environment settings on one bench workload (AB: "name=ENV=V name2=ENV=V",
# ARGS: bench.py arguments), alternated ROUNDS times; one line per run with ms_per_step and
# the pass-1 HIP-event time.  Timing only: the numbers that count come from bench.py itself.
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04_ab}; mkdir -p $O
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in $AB; do
    name=${spec%%=*}; env=${spec#*=}
    [ "$env" = none ] && env=""
    env $env timeout -k 10 200 python -u bench.py ${ARGS:---no-cpu --no-pmc --no-ktrace --no-variants --steps 30} > $O/ab_${name}_$r.json 2> $O/ab_${name}_$r.err || { tail -5 $O/ab_${name}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/ab_${name}_$r.json').read().strip().splitlines()[-1]); print('$name', $r, d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('pass1_share_of_step'))"
  done
done
