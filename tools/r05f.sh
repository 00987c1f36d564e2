set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r05f
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py -m gpu -q --timeout 240 --timeout-method thread -k "selfjoin or l2_int8 or tombstone" > gpurun_out/r05f/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05f/tests.log; { [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || exit $rc
timeout -k 10 400 python3 -u bench.py --workload c5 --no-cpu-baseline > gpurun_out/r05f/c5.json 2> gpurun_out/r05f/c5.err || { echo c5 failed; tail -3 gpurun_out/r05f/c5.err; exit 1; }
tail -c 600 gpurun_out/r05f/c5.json
for w in "l2cl:--metric l2 --data clustered" "cl:--data clustered"; do
  t=${w%%:*}; a=${w#*:}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05f/prof_$t -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --batch1-steps 0 --wide-k-steps 0 $a > gpurun_out/r05f/$t.log 2>&1 || { echo "$t failed"; exit 1; }
done
echo done
