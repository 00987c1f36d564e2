"""Host-side cost of one device-resident search (C2 shape: 1M x 1536 IP,
batch 1024, top-10): per-call host time of search_device without a sync
against the GPU time per search, to tell a launch-bound loop from a
kernel-bound one."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "book-recommendation-engine_amd"))

import torch  # noqa: E402

from vsearch import faiss as vf  # noqa: E402
from vsearch.synth import synthetic_rows  # noqa: E402

n, nq, k = int(os.environ.get("PROBE_N", "1000000")), 1024, 10
index = vf.IndexFlatIP(1536)
index.add_synthetic(n, seed=1234)
xq = torch.from_numpy(synthetic_rows(50_000_000, nq, 1536, 5678)).cuda()
D = torch.empty((nq, k), dtype=torch.float32, device="cuda")
I = torch.empty((nq, k), dtype=torch.int64, device="cuda")
st = torch.cuda.current_stream().cuda_stream
for _ in range(5):
    index.search_device(xq.data_ptr(), nq, k, D.data_ptr(), I.data_ptr(), stream=st)
torch.cuda.synchronize()
host = []
t0 = time.perf_counter()
for _ in range(30):
    a = time.perf_counter()
    index.search_device(xq.data_ptr(), nq, k, D.data_ptr(), I.data_ptr(), stream=st)
    host.append(time.perf_counter() - a)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
host.sort()
print(f"host per call: median {host[15]*1e3:.3f} ms, max {host[-1]*1e3:.3f} ms; "
      f"enqueue 30 calls {(t1-t0)*1e3:.1f} ms; wall incl. drain {(t2-t0)*1e3/30:.3f} ms per search")
