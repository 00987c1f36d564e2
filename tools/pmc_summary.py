"""Summarise rocprofv3 PMC passes into profiles/<tag>_pmc_<workload>.json.

    python tools/pmc_summary.py <prof_dir> <tag> <workload>

<prof_dir> is a tools/profile.sh output (gpurun_out/prof_<tag>) with pmc_fetch/ and
pmc_write/ CSVs.  Per kernel: mean FETCH_SIZE / WRITE_SIZE (KB) per dispatch and
the HBM bytes per launch, with the gfx950 correction of MI355X_MICROARCH.md §HBM:
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming read
(both `global_load_dwordx4` and LDS-DMA), so it is doubled; WRITE_SIZE is exact
for 16-B streaming stores.  The correction was checked on gemv_topk, whose
doubled FETCH_SIZE equals the corpus bytes exactly (61.44 GB at 10M x 1536 fp32).
"""

import collections
import csv
import json
import os
import sys


def load(path):
    """Mean counter value per kernel name and per (name, grid size): one
    instantiation runs full-size passes and small gathered ones (the staged
    engine's later stages), whose bytes must not be averaged together."""
    agg = collections.defaultdict(list)
    grid = collections.defaultdict(list)
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
            grid[(r["Kernel_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return ({k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()},
            {k: (sum(v) / len(v), len(v)) for k, v in grid.items()})


def main():
    prof, tag, workload = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch, nf, fgrid = load(os.path.join(prof, "pmc_fetch", "run_counter_collection.csv"))
    write, _, wgrid = load(os.path.join(prof, "pmc_write", "run_counter_collection.csv"))
    out = {"source": prof, "correction": "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950)",
           "kernels": {}}
    for name in fetch:
        if name.startswith("__amd") or "at::native" in name:
            continue
        fk = fetch[name]
        wk = write.get(name, 0.0)
        out["kernels"][name] = {
            "dispatches": nf[name],
            "fetch_kb_per_launch": fk,
            "write_kb_per_launch": wk,
            "hbm_bytes_per_launch": 2.0 * fk * 1024 + wk * 1024,
            "by_grid": {
                str(g): {"dispatches": n, "fetch_kb_per_launch": f,
                         "write_kb_per_launch": wgrid.get((name, g), (0.0, 0))[0],
                         "hbm_bytes_per_launch": 2.0 * f * 1024
                         + wgrid.get((name, g), (0.0, 0))[0] * 1024}
                for (nm, g), (f, n) in sorted(fgrid.items()) if nm == name},
        }
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                       f"{tag}_pmc_{workload}.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", dst)


if __name__ == "__main__":
    main()
