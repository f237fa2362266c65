set -e
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_png.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03q_png.log 2>&1 || { tail -40 gpurun_out/r03q_png.log; exit 1; }
tail -1 gpurun_out/r03q_png.log
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --workload c5 --steps 5 --warmup 1 --no-cpu > gpurun_out/q_c5_batch.json
  timeout -k 10 300 python3 bench.py --workload c5 --steps 5 --warmup 1 --no-cpu --png-single > gpurun_out/q_c5_single.json
  for f in batch single; do python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['stage_ms'], d['parity'])" gpurun_out/q_c5_$f.json $f; done
done
