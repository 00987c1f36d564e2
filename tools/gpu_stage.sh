#!/bin/bash
# GPU steps of a round, one named stage per gpurun call (each step under its
# own time limit; the first failure ends the call):
#   gpurun -- bash tools/gpu_stage.sh <tag> <stage>...
# stages: dump (dump-launch + parity tests), suite (the whole -m gpu suite),
# c3 | c3cl | c2 | c4 | c5 (bench lines), ab (tools/ab_dump.sh),
# prof_c3 | prof_c3cl (rocprofv3 kernel stats + PMC passes, tools/profile.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
BENCH="python3 -u bench.py"
for st in "$@"; do
  echo "== $st $(date +%T)"
  case $st in
    dump) timeout -k 10 700 $PYT tests/test_gpu_dump.py tests/test_gpu_parity.py > "$OUT/dump_tests.log" 2>&1 ;;
    suite) timeout -k 10 1000 $PYT -m gpu tests > "$OUT/gpu_tests.log" 2>&1 ;;
    c3) timeout -k 10 400 $BENCH > "$OUT/bench_c3.json.log" 2>&1 ;;
    c3cl) timeout -k 10 400 $BENCH --data clustered --batch1-steps 0 --no-cpu-baseline > "$OUT/bench_c3cl.json.log" 2>&1 ;;
    c2) timeout -k 10 300 $BENCH --workload c2 --no-cpu-baseline > "$OUT/bench_c2.json.log" 2>&1 ;;
    c4) timeout -k 10 400 $BENCH --workload c4 > "$OUT/bench_c4.json.log" 2>&1 ;;
    c5) timeout -k 10 900 $BENCH --workload c5 > "$OUT/bench_c5.json.log" 2>&1 ;;
    ab) timeout -k 10 1000 bash tools/ab_dump.sh > "$OUT/ab_dump.txt" 2>&1 ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
  rc=$?
  echo "== $st rc=$rc $(date +%T)"
  for f in "$OUT"/*"$st"*.log; do [ -f "$f" ] && tail -3 "$f"; done
  [ $rc -eq 0 ] || exit $rc
done
