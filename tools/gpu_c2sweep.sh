#!/bin/bash
# C2 decode-lane size / guess lead sweep (tuning aid): GPU decode tests, then C2 bench lines for
# each "SUB LEAD" pair (LEAD -1: the library default), then one C3 line.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_dec4.log 2>&1
tail -1 gpurun_out/gpu_dec4.log
SWEEP=${SWEEP:-"2048,-1 512,-1 512,0 512,2048 1024,-1 256,-1 512,-1"}
for cfg in $SWEEP; do
    S=${cfg%,*}; L=${cfg#*,}
    if [ "$L" -ge 0 ]; then export ICX_GUESS_LEAD=$L; else unset ICX_GUESS_LEAD; fi
    ICX_SUB_BYTES=$S timeout -k 10 200 python bench.py --workload c2 --no-cpu --no-pcie --steps 10 > gpurun_out/c2s.json 2>/dev/null || exit 1
    echo "c2 sub $S lead $L $(cut -c60-130 gpurun_out/c2s.json)"
done
unset ICX_GUESS_LEAD
timeout -k 10 200 python bench.py --no-cpu --no-pcie --steps 8 > gpurun_out/c3s.json 2>/dev/null || exit 1
echo "c3 $(cut -c60-130 gpurun_out/c3s.json)"
