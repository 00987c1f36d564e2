"""Per-kernel mean of every counter found under a tools/pmc_passes.sh output."""

import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sorted(glob.glob(os.path.join(root, "g*", "**", "*counter_collection.csv"),
                            recursive=True)):
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                name = r["Kernel_Name"]
                if name.startswith("__amd") or "at::native" in name:
                    continue
                vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, ctrs in vals.items():
        print(name[:90])
        for c, v in sorted(ctrs.items()):
            print(f"  {c:28s} {sum(v) / len(v):.6g}   (n={len(v)})")


if __name__ == "__main__":
    main()
