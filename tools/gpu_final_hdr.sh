set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/fin
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/fin/gpu_tests.log 2>&1 && tail -2 gpurun_out/fin/gpu_tests.log &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fin/smoke.log 2>&1 && cat gpurun_out/fin/smoke.log | tail -2 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin/trace_hdr -o run -- python3 bench.py --workload hdr --steps 3 --no-cpu > gpurun_out/fin/rocprof_hdr.json 2> gpurun_out/fin/rocprof_hdr.err && cat gpurun_out/fin/rocprof_hdr.json
