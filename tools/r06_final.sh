#!/bin/bash
# Round-6 final evidence (through gpurun), in two parts that each fit a call:
#   tools/r06_final.sh tests <tag>   GPU suite, smoke(), the default bench line
#   tools/r06_final.sh prof <tag>    C2 bench + rocprofv3 trace/PMC (C2, C3)
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
  tail -c 300 "$OUT/$name"; echo
}
case $PART in
  tests)
    echo "[$(date +%T)] gpu tests"
    timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
      > "$OUT/gpu_tests.log" 2>&1
    rc=$?; tail -4 "$OUT/gpu_tests.log"
    { [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || { echo "tests rc=$rc: stop"; exit $rc; }
    run smoke.txt 300 python3 -c "import __graft_entry__ as g; g.smoke()"
    run bench_c3.json 600 python3 -u bench.py
    ;;
  prof)
    run bench_c2.json 300 python3 -u bench.py --workload c2 --no-cpu-baseline
    run prof_c2.txt 900 bash tools/profile.sh ${TAG}c2 --workload c2
    run prof_c3.txt 900 bash tools/profile.sh ${TAG}c3
    ;;
  *) echo "unknown part $PART"; exit 2 ;;
esac
echo "part $PART ok"
