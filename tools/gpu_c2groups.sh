cd "$GRAFT_REPO_ROOT"
for g in 2 4 8; do ICX_GROUPS=$g timeout -k 10 300 python3 bench.py --workload c2 --steps 10 --warmup 3 --no-cpu --no-pcie > gpurun_out/c2g$g.json 2>gpurun_out/c2g$g.err || exit 1; python3 -c "import json,sys; d=json.loads(open(\"gpurun_out/c2g$g.json\").read().splitlines()[-1]); print(\"groups $g\", d[\"value\"]/1000, d[\"ms_per_step\"])"; done
