#!/bin/bash
# Round-5 profiler evidence (through gpurun): kernel traces + FETCH/WRITE passes
# for C2, C4, C3 L2 and C3 IP (tools/profile.sh), then the SQ counters of C3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for spec in "r05c2:--workload c2" "r05c4:--workload c4" "r05l2:--metric l2" "r05c3:" \
            "r05cl:--data clustered" "r05c5:--workload c5"; do
  tag=${spec%%:*}; args=${spec#*:}
  bash tools/profile.sh "$tag" $args || { echo "profile $tag failed"; exit 1; }
done
# where a k = 60 search (B = 4096) spends its time beyond the filter pass
mkdir -p gpurun_out/prof_r05wk
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r05wk/trace -o run \
  -- python3 bench.py --steps 1 --warmup 1 --batch1-steps 0 --wide-k 60 --wide-k-steps 3 --no-cpu-baseline \
  > gpurun_out/prof_r05wk/bench.log 2>&1 || { echo "wide-k trace failed"; exit 1; }
PMC_GROUPS="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" \
  bash tools/pmc_passes.sh r05c3sq || exit 1
echo "profiles ok"
