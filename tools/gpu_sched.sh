#!/bin/bash
# GPU box: C3 bench under batch-scheduling variants (env settings per line of SCHED_CFGS,
# separated by ';'). One JSON summary line per variant under gpurun_out/sched/.
set -o pipefail
O=gpurun_out/sched; mkdir -p $O
IFS=';' read -ra CFGS <<< "${SCHED_CFGS:-ICX_STAGGER=0;ICX_STAGGER=1}"
k=0
for cfg in "${CFGS[@]}"; do
  k=$((k+1))
  env $cfg timeout -k 10 200 python bench.py --no-cpu --no-pcie --steps ${STEPS:-5} ${BENCH_ARGS:-} > $O/v$k.json 2> $O/v$k.err || { echo "variant $cfg failed"; tail -5 $O/v$k.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$O/v$k.json'));print('$cfg |', d['value'], d['ms_per_step'], d['roofline']['stage_ms'], d['parity'])"
done
