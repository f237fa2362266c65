set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hdr.py tests/test_cxx_dropin.py > gpurun_out/gpu_hdr_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_hdr_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload hdr --steps 5 > gpurun_out/bench_hdr.json 2> gpurun_out/bench_hdr.err && cat gpurun_out/bench_hdr.json &&
timeout -k 10 300 python -u bench.py --workload hdrflat --steps 5 --no-cpu > gpurun_out/bench_hdrflat.json 2> gpurun_out/bench_hdrflat.err && cat gpurun_out/bench_hdrflat.json
