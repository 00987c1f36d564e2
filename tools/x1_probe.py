"""Diagnostic driver for tools/x1_probe.sh: one 2.56M x 1536 IP index, three
batch-4096 top-10 searches on the filter engine (the kernel durations are read
from rocprofv3's kernel trace; probe builds return wrong lists by design)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "book-recommendation-engine_amd"))

from vsearch import faiss as vf  # noqa: E402
from vsearch.synth import synthetic_rows  # noqa: E402

n = int(os.environ.get("PROBE_N", "2560000"))
index = vf.IndexFlatIP(1536)
index.reserve(n)
index.add_synthetic(n, seed=1234)
xq = synthetic_rows(50_000_000, 4096, 1536, 5678)
for _ in range(3):
    index.search(xq, 10)
print("probe ok", os.environ.get("VSEARCH_LIB", "default"))
