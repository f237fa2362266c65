set -e
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_png.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03r_png.log 2>&1 || { tail -40 gpurun_out/r03r_png.log; exit 1; }
tail -1 gpurun_out/r03r_png.log
for k in 2 3 4 6; do
  ICX_PNG_INFLIGHT=$k timeout -k 10 300 python3 bench.py --workload c5 --steps 5 --warmup 1 --no-cpu > gpurun_out/r_c5_k$k.json
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('inflight', sys.argv[2], d['value'], d['ms_per_step'], d['parity'])" gpurun_out/r_c5_k$k.json $k
done
