set -u
OUT=gpurun_out/r06j; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -4 $OUT/gpu_tests.log
{ [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || { echo "tests rc=$rc"; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit $?
cat $OUT/smoke.txt
timeout -k 10 600 python3 -u bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit $?
tail -c 1500 $OUT/bench_c3.json
