set -e
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fallback.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03p_fb.log 2>&1 || { tail -40 gpurun_out/r03p_fb.log; exit 1; }
grep -E "PASS|FAIL|clean" gpurun_out/r03p_fb.log | cut -c1-160
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_foreign.py tests/test_gpu_multi.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03p_tests.log 2>&1 || { tail -40 gpurun_out/r03p_tests.log; exit 1; }
tail -1 gpurun_out/r03p_tests.log
run() { local lab=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-pcie > gpurun_out/p_$lab.json; python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'], {k:round(v,2) for k,v in d['roofline']['stage_ms'].items()})" gpurun_out/p_$lab.json $lab; }
for rep in 1 2; do run r2 ICX_X=0; run r1 ICX_ROUNDS=1; done

