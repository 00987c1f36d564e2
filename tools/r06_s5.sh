#!/bin/bash
# Round 6: the 320-row int8 dump launch (gemm_dump_s5): dump tests,
# then C3 A/B against gemm_topk_x1's dump form (VS_X1_S5=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-w1}; K=${2:-test_gpu_dump}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1
rc=$?; tail -4 $OUT/tests.log
[ $rc -eq 0 ] || { echo "tests rc=$rc: stop"; exit $rc; }
bash tools/ab_env.sh $TAG "s5a:" "s0a:VS_X1_S5=0" "s5b:" "s0b:VS_X1_S5=0" "s5c:"
