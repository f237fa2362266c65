#!/bin/bash
# A/B bench on one GPU box: the same bench.py command under each library build, interleaved
# REPS times (box-to-box spread is larger than most single changes, so compare on one box).
#   LABEL=r05a LIBS="exp/libicx_r04.so lib/libicx.so" BENCH_ARGS="--workload c3 --steps 20 --warmup 5" \
#     tools/gpu_ab.sh
# Optional: TESTS="tests/test_gpu_decode.py ..." runs those GPU tests first (new library), and
# PROF=1 adds one rocprofv3 --kernel-trace --stats pass per library after the benches (PROF_ARGS:
# its bench arguments, default BENCH_ARGS; PROF_PIPES=1 runs it on one pipeline, kernels alone), and
# prints each library's kernel summary (tools/prof_db.py).
# Output: gpurun_out/<LABEL>_ab.txt (one JSON line per run, tagged with its library).
set -o pipefail
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R" || exit 1
L="${LABEL:-ab}"; REPS="${REPS:-2}"
mkdir -p gpurun_out
OUT="gpurun_out/${L}_ab.txt"; : > "$OUT"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > "gpurun_out/${L}_tests.log" 2>&1
  rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/${L}_tests.log)"
  [ $rc -eq 0 ] || { tail -30 "gpurun_out/${L}_tests.log"; exit $rc; }
fi
for rep in $(seq 1 "$REPS"); do
  for lib in ${LIBS:-lib/libicx.so}; do
    ICX_LIB="$R/imagecodecs_amd/$lib" timeout -k 10 300 python3 bench.py --no-cpu --no-pcie ${BENCH_ARGS:-} \
      > gpurun_out/${L}_one.json 2> gpurun_out/${L}_one.err
    rc=$?
    echo "{\"lib\": \"$lib\", \"rep\": $rep, \"rc\": $rc, \"line\": $(cat gpurun_out/${L}_one.json | tail -1 || echo null)}" >> "$OUT"
    python3 - "$lib" gpurun_out/${L}_one.json <<'EOF'
import json, sys
try:
    d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    print(sys.argv[1], round(d["value"] / 1000, 2), "GP/s", d["ms_per_step"], "ms/step", "frac", d.get("roofline", {}).get("frac"))
except Exception as e:
    print(sys.argv[1], "no result", e)
EOF
    case $rc in 0) ;; *) tail -20 gpurun_out/${L}_one.err; exit $rc;; esac
  done
done
if [ -n "${PROF:-}" ]; then
  export TMPDIR=/tmp
  for lib in ${LIBS:-lib/libicx.so}; do
    tag=$(basename "$lib" .so)
    ICX_PIPES="${PROF_PIPES:-2}" ICX_LIB="$R/imagecodecs_amd/$lib" timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      -d "gpurun_out/${L}_prof_${tag}" -o run -- python3 bench.py --no-cpu --no-pcie ${PROF_ARGS:-${BENCH_ARGS:-}} \
      > "gpurun_out/${L}_prof_${tag}.log" 2>&1
    rc=$?; echo "prof $tag rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    python3 tools/prof_db.py "gpurun_out/${L}_prof_${tag}/run_results.db" --top 12
  done
fi
