#!/bin/bash
# Round-5 profiler evidence (through gpurun): kernel traces + FETCH/WRITE passes
# for C2, C4, C3 L2 and C3 IP (tools/profile.sh), then the SQ counters of C3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for spec in "r05c2:--workload c2" "r05c4:--workload c4" "r05l2:--metric l2" "r05c3:"; do
  tag=${spec%%:*}; args=${spec#*:}
  bash tools/profile.sh "$tag" $args || { echo "profile $tag failed"; exit 1; }
done
PMC_GROUPS="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" \
  bash tools/pmc_passes.sh r05c3sq || exit 1
echo "profiles ok"
