#!/bin/bash
# SQ counters of the int8 dump launches, gemm_dump_s5 vs gemm_topk_x1's dump
# form (VS_X1_S5=0): clock (GRBM_GUI_ACTIVE per XCD / dispatch time), MFMA
# busy and wave stall buckets.  One --pmc pass each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-pmcab}
OUT=gpurun_out/$TAG; mkdir -p $OUT
C="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for v in 1 0; do
  VS_X1_S5=$v timeout -k 10 -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/s$v -o run \
    -- python3 bench.py --steps 1 --warmup 0 --batch1-steps 0 --wide-k-steps 0 --any-k 0 --clustered-steps 0 --no-cpu-baseline \
    > $OUT/s$v.log 2>&1 || { echo "pass $v failed rc=$?"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
root = sys.argv[1]
for v in ("s1", "s0"):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in glob.glob(os.path.join(root, v, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            n = r["Kernel_Name"]
            if "gemm_dump_s5" in n or "gemm_topk_x1<8, 0, true" in n:
                vals[n[:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for n, c in vals.items():
        m = {k: sum(x) / len(x) for k, x in c.items()}
        g = m["GRBM_GUI_ACTIVE"] / 8
        print(v, n, "n=%d" % len(c["GRBM_GUI_ACTIVE"]), "cycles/XCD %.4g" % g,
              "mfma_busy %.3f" % (m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * g)),
              "wait_any/wave %.3f" % (m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]),
              "wait_inst/wave %.3f" % (m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"]),
              "active/wave %.3f" % (m["SQ_ACTIVE_INST_ANY"] / m["SQ_WAVE_CYCLES"]))
PY
