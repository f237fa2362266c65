# A/B of k_back420 builds (ICX_FUSE420=3) against the plane path (mode 2) on one box.
set -e
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
ARGS="${BENCH_ARGS:---steps 10 --warmup 2 --no-cpu --no-pcie}"
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py $ARGS > "gpurun_out/bab_$lab.json"
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'], {k:round(v,2) for k,v in d['roofline']['stage_ms'].items()}, d['parity'].get('all_status_ok'), d['parity'])" "gpurun_out/bab_$lab.json" "$lab"
}
for rep in 1 ${REPS2:-}; do
  run base2 ICX_FUSE420=2
  for v in ${VARIANTS:-pp0w4}; do run "$v" ICX_FUSE420=3 ICX_LIB=imagecodecs_amd/exp/libicx_$v.so; done
done
