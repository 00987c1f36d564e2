#!/bin/bash
# Counter passes for one bench.py workload (one rocprofv3 --pmc pass per group,
# nothing else traced in the same pass).  Run through gpurun.
#   tools/pmc_passes.sh <tag> [bench args...]
#   PMC_GROUPS="A B;C D" tools/pmc_passes.sh <tag> ...   (groups separated by ';')
# Output: gpurun_out/pmc_<tag>/g<i>/run_counter_collection.csv + summary.txt
set -u
TAG=${1:-x}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
DEFAULT="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS;TCC_HIT_sum TCC_MISS_sum;FETCH_SIZE"
IFS=';' read -ra GROUPS_ <<< "${PMC_GROUPS:-$DEFAULT}"
i=0
for g in "${GROUPS_[@]}"; do
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $g --output-format csv -d "$OUT/g$i" -o run \
    -- python3 bench.py --steps 1 --warmup 0 --batch1-steps 0 --wide-k-steps 0 --any-k 0 --clustered-steps 0 --no-cpu-baseline "$@" \
    > "$OUT/g$i.log" 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_table.py "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
