"""Where a C5 mutation round's time goes (host vs device), on a reduced corpus.

Prints host timestamps around: 10 asynchronous searches, torch.cuda.synchronize(),
the HIP runtime's own hipDeviceSynchronize(), remove_ids, append_synthetic_ids.
Used to check that bench.py's synchronisation brackets the library's work.

    python tools/c5_timeline.py [--ntotal 10000000]
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "book-recommendation-engine_amd"))
from vsearch.sharded import ShardedIndexFlat  # noqa: E402
import vsearch.faiss as vfaiss  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ntotal", type=int, default=10_000_000)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.distributed.init_process_group("gloo", rank=0, world_size=1)
    hip = ctypes.CDLL("libamdhip64.so.7")
    N, d, B, k = a.ntotal, 1536, 8, 10
    idx = ShardedIndexFlat(d, vfaiss.METRIC_INNER_PRODUCT, device=0, dtype="bf16")
    idx.add_synthetic(N, seed=1234)
    xq = torch.randn(64, d, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    idx.search_device(xq[:B], k, stream=st)
    torch.cuda.synchronize()
    rng = np.random.default_rng(1)
    for rnd in range(3):
        t = [time.perf_counter()]
        for i in range(10):
            idx.search_device(xq[:B], k, stream=st)
        t.append(time.perf_counter())
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        hip.hipDeviceSynchronize()
        t.append(time.perf_counter())
        rm = np.sort(rng.choice(N, N // 100, replace=False)).astype(np.int64)
        t.append(time.perf_counter())
        idx.remove_ids(rm)
        t.append(time.perf_counter())
        torch.cuda.synchronize()
        hip.hipDeviceSynchronize()
        t.append(time.perf_counter())
        idx.append_synthetic_ids(np.arange(N + rnd * (N // 100), N + (rnd + 1) * (N // 100)), seed=1234)
        t.append(time.perf_counter())
        hip.hipDeviceSynchronize()
        t.append(time.perf_counter())
        ms = [round((t[i + 1] - t[i]) * 1e3, 2) for i in range(len(t) - 1)]
        print(f"round {rnd}: enqueue10 {ms[0]} torch_sync {ms[1]} hip_sync {ms[2]} draw {ms[3]} "
              f"remove {ms[4]} remove_sync {ms[5]} append {ms[6]} append_sync {ms[7]} ms",
              flush=True)
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
