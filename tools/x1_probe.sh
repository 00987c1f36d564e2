#!/bin/bash
# Ablation probes of the x1 filter kernel (run through gpurun after building
# the variants here with tools/build_variant.sh <name> -DVS_X1_PROBE=<mask>):
#   tools/x1_probe.sh <variant>...   (variant "base" = the default library)
# Mean x1e dispatch time per variant from rocprofv3 --kernel-trace --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/probe
mkdir -p "$OUT"
for v in "$@"; do
  lib=book-recommendation-engine_amd/vsearch/libvsearch_$v.so
  [ "$v" = base ] && lib=book-recommendation-engine_amd/vsearch/libvsearch.so
  VSEARCH_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/$v" -o run -- python3 tools/x1_probe.py > "$OUT/$v.log" 2>&1 || { echo "$v failed"; exit 1; }
  python3 - "$OUT/$v" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "gemm_topk_x1" in r["Name"]:
        print(f"{sys.argv[2]:8s} calls={r['Calls']} mean_ms={float(r['AverageNs'])/1e6:.4f}")
PY
done
