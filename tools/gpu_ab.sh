#!/bin/bash
# GPU box: decode parity tests, then the C3 bench under pipeline/group variants, then the C5 bench.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_decode.py > gpurun_out/ab/tests.log 2>&1 || { tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -2 gpurun_out/ab/tests.log
for cfg in ${AB_CFGS:-"1,0" "2,0" "2,256" "2,128"}; do
  p=${cfg%,*}; g=${cfg#*,}
  ICX_PIPES=$p timeout -k 10 200 python bench.py --no-cpu --steps 5 --group $g > gpurun_out/ab/c3_p${p}_g${g}.json 2> gpurun_out/ab/err_${p}_${g}.log || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab/c3_p${p}_g${g}.json'));print('pipes=$p group=$g',d['value'],d['ms_per_step'],d['roofline']['stage_ms'],d['parity'])"
done
if [ -z "$AB_NO_C5" ]; then
  timeout -k 10 400 python bench.py --workload c5 --steps 2 > gpurun_out/ab/c5.json 2> gpurun_out/ab/c5.err || { tail gpurun_out/ab/c5.err; exit 1; }
  cat gpurun_out/ab/c5.json
fi
