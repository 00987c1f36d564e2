"""Build-time guard (csrc/Makefile): the x1 filter kernels issue LDS-DMA loads
from inline asm, which hipcc's vmcnt bookkeeping does not see, so they must not
use scratch (no spill reloads beside uncounted loads).  Reads hipcc's
-Rpass-analysis=kernel-resource-usage remarks and fails on any kernel whose
mangled name contains the given substring and has ScratchSize > 0."""
import re
import sys


def main(path, needle):
    cur, bad, seen = None, [], 0
    for line in open(path, encoding="utf-8", errors="replace"):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            continue
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and cur and needle in cur:
            seen += 1
            if int(m.group(1)) > 0:
                bad.append((cur, int(m.group(1))))
    if not seen:
        sys.exit(f"check_no_spill: no kernel matching {needle!r} in {path}")
    if bad:
        sys.exit("check_no_spill: scratch in " + ", ".join(f"{n} ({b} B/lane)" for n, b in bad))
    print(f"check_no_spill: {seen} {needle} kernels, no scratch")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
