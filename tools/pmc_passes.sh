#!/bin/bash
# Counter passes for one bench.py workload (one rocprofv3 --pmc pass per group,
# nothing else traced in the same pass).  Run through gpurun.
#   tools/pmc_passes.sh <tag> [bench args...]
# Output: gpurun_out/pmc_<tag>/<group>/run_counter_collection.csv
set -u
TAG=${1:-x}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
GROUPS_=(
  "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
  "TCC_HIT_sum TCC_MISS_sum"
  "FETCH_SIZE"
)
i=0
for g in "${GROUPS_[@]}"; do
  timeout -k 10 400 rocprofv3 --pmc $g --output-format csv -d "$OUT/g$i" -o run \
    -- python3 bench.py --steps 1 --warmup 0 --batch1-steps 0 --no-cpu-baseline "$@" \
    > "$OUT/g$i.log" 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_table.py "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
