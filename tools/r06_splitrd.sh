#!/bin/bash
# Split fragment reads in the dump launches' segmented schedule: dump / parity /
# C3 tests on the new default, then interleaved A/B against the no-split build
# (tools/build_variant.sh nosplit -DVS_X1_SPLITRD=0) on C3 and clustered C3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-srd}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  -k "test_gpu_dump or test_gpu_parity or test_gpu_c3" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { echo "tests rc=$rc: stop"; exit $rc; }
bash tools/ab_x1.sh ${TAG}_c3 base nosplit -- --any-k 0 --clustered-steps 0 || exit $?
bash tools/ab_x1.sh ${TAG}_cl base nosplit -- --any-k 0 --clustered-steps 0 --data clustered || exit $?
