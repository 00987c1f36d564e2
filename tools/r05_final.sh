#!/bin/bash
# Round-5 evidence (through gpurun), in parts that each fit one call:
#   tools/r05_final.sh tests <tag>    GPU suite, smoke(), the MFMA ceiling probe, C5
#   tools/r05_final.sh bench <tag>    bench.py lines: C3 (default, with the CPU
#                                     baseline, batch-1 and wide-k legs), C3 L2,
#                                     clustered C3 (IP, L2), C2, C4
# Every GPU step runs under its own time limit; the script stops at the first
# step that does not finish cleanly (pytest's exit 1 still lets the rest run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PART=$1; TAG=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # run <name> <seconds> <cmd...>: stdout -> $OUT/<name>, stderr -> $OUT/<name>.err
  local name=$1 lim=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$lim" "$@" > "$OUT/$name" 2> "$OUT/$name.err"
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 "$OUT/$name.err"; exit $rc; }
  tail -c 400 "$OUT/$name"; echo
}
case $PART in
  tests)
    echo "[$(date +%T)] gpu tests"
    timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
      > "$OUT/gpu_tests.log" 2>&1
    rc=$?; tail -4 "$OUT/gpu_tests.log"
    { [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || { echo "tests rc=$rc: stop"; exit $rc; }
    run smoke.txt 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
    run mfma_ceiling.json 120 tools/mfma_ceiling
    run bench_c5.json 600 python3 -u bench.py --workload c5 --no-cpu-baseline
    ;;
  bench)
    run bench_c3.json 600 python3 -u bench.py
    run bench_c3l2.json 400 python3 -u bench.py --metric l2 --no-cpu-baseline --batch1-steps 0 --wide-k-steps 0
    run bench_c3cl.json 400 python3 -u bench.py --data clustered --no-cpu-baseline --batch1-steps 0 --wide-k-steps 0
    run bench_c3cll2.json 400 python3 -u bench.py --data clustered --metric l2 --no-cpu-baseline --batch1-steps 0 --wide-k-steps 0
    run bench_c2.json 300 python3 -u bench.py --workload c2 --no-cpu-baseline
    run bench_c4.json 400 python3 -u bench.py --workload c4 --no-cpu-baseline
    ;;
  *) echo "unknown part $PART"; exit 2 ;;
esac
echo "part $PART ok"
