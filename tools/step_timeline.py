"""One search's kernel timeline (run under rocprofv3 --kernel-trace through
gpurun, then `--report <kernel_trace.csv>` here): builds a synthetic index,
runs WARM untimed searches, sleeps 0.2 s (the gap the report splits on), then
one search.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- \
        python3 tools/step_timeline.py --n 1000000 --b 1024
    python3 tools/step_timeline.py --report OUT/.../run_kernel_trace.csv
"""
import argparse
import csv
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "book-recommendation-engine_amd"))


def report(path, gap_ms=100.0):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    cut = 0
    for i in range(1, len(ev)):
        if ev[i][0] - ev[i - 1][1] > gap_ms * 1e6:
            cut = i
    ev = ev[cut:]
    t0 = ev[0][0]
    busy = 0
    for s, e, name in ev:
        busy += e - s
        print(f"{(s - t0) / 1e3:9.1f} us {(e - s) / 1e3:8.1f} us  {name[:100]}")
    print(f"span {(ev[-1][1] - t0) / 1e3:.1f} us, kernels {len(ev)}, busy {busy / 1e3:.1f} us")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--report")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--b", type=int, default=1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--l2", action="store_true")
    ap.add_argument("--warm", type=int, default=3)
    a = ap.parse_args()
    if a.report:
        report(a.report)
        return
    import torch
    from vsearch import faiss as vf
    from vsearch.synth import synthetic_rows
    d = 1536
    index = vf.IndexFlat(d, vf.METRIC_L2 if a.l2 else vf.METRIC_INNER_PRODUCT)
    index.reserve(a.n)
    index.add_synthetic(a.n, seed=1234)
    xq = torch.from_numpy(synthetic_rows(50_000_000, a.b, d, 5678)).cuda()
    st = torch.cuda.current_stream().cuda_stream
    D = torch.empty(a.b, a.k, device="cuda")
    I = torch.empty(a.b, a.k, dtype=torch.int64, device="cuda")

    def one():
        index.search_device(xq.data_ptr(), a.b, a.k, D.data_ptr(), I.data_ptr(), stream=st)

    for _ in range(a.warm):
        one()
    torch.cuda.synchronize()
    time.sleep(0.2)
    t0 = time.perf_counter()
    one()
    torch.cuda.synchronize()
    print(f"one search {1e3 * (time.perf_counter() - t0):.3f} ms (n={a.n}, b={a.b}, k={a.k})", flush=True)


if __name__ == "__main__":
    main()
