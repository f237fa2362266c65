set -e
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
run() { local lab=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-pcie > gpurun_out/s_$lab.json; python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/s_$lab.json $lab; }
for rep in 1 2; do run base ICX_X=0; run w5 ICX_LIB=imagecodecs_amd/exp/libicx_w5.so; run w4 ICX_LIB=imagecodecs_amd/exp/libicx_w4.so; done
for rep in 1 2; do for k in 3 6 8; do
  ICX_PNG_INFLIGHT=$k timeout -k 10 300 python3 bench.py --workload c5 --steps 5 --warmup 1 --no-cpu > gpurun_out/s_c5_k$k.json
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('c5 inflight', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/s_c5_k$k.json $k
done; done
