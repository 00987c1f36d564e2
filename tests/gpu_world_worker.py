"""One rank of tests/test_gpu_world2.py (run as its own process, never
collected): a real HIP shard of ShardedIndexFlat on GPU 0 beside its peers,
torch.distributed over gloo (RCCL refuses two ranks on one GPU), so the N > 1
path of the row-sharded search runs on a one-GPU box: raw per-shard 2k-1
lists (VS_RAW_ORDER, the paged search past k = 32: any k), the all-gather, and
vs_merge_topk over `world` parts on the GPU (sharded.py search /
search_device), plus removals and appends across shards.  Each check compares
with the fp64 oracle over the whole corpus; rank 0 prints one JSON line of
named results (True = equal)."""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "book-recommendation-engine_amd"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import flat
    from vsearch import faiss as vf
    from vsearch.sharded import ShardedIndexFlat, shard_bounds

    res = {}

    def check(name, D, I, x, xq, k, metric, exact_scores):
        """Rank 0 compares with the oracle (every rank holds the merged lists)."""
        if rank != 0:
            return
        Dr, Ir = flat.knn_exact(x, xq, k, metric)
        if exact_scores:  # integer rows: labels and scores bit for bit
            res[name] = bool(np.array_equal(I, Ir) and np.array_equal(D, Dr))
        else:  # float rows: labels exact up to the fp32 tie window, scores 1e-5
            res[name] = not flat.mismatches(D, I, Dr, Ir, metric, x, xq)

    for metric in (vf.METRIC_INNER_PRODUCT, vf.METRIC_L2):
        mn = "ip" if metric == vf.METRIC_INNER_PRODUCT else "l2"
        # the round-1 counterexample (d = 1): faiss's IP tie rule across shards
        xc = np.array([2, 0, 1, 0, 0, 0, 1, 1, 1, 2, 2], dtype=np.float32)[:, None]
        idc = ShardedIndexFlat(1, metric, device=0)
        idc.add_global(xc)
        q1 = np.ones((1, 1), np.float32)
        D, I = idc.search(q1, 4)
        check(f"{mn}_counterexample", D, I, xc, q1, 4, metric, True)

        # tie-heavy integer rows (exact scores): labels and scores bit for bit,
        # k past 32 (raw 2k-1 entries: several pages on every shard; k = 100
        # and 300 past one page's 64 and the merge past 128 entries)
        rng = np.random.default_rng(11 + metric)
        x = rng.integers(-2, 3, size=(3001, 8)).astype(np.float32)
        xq = rng.integers(-2, 3, size=(37, 8)).astype(np.float32)
        idx = ShardedIndexFlat(8, metric, device=0)
        idx.add_global(x)
        lo, hi = shard_bounds(3001, world, rank)
        res[f"{mn}_layout"] = bool(idx.ntotal == 3001 and idx.shard.ntotal == hi - lo)
        for k in (1, 4, 10, 33, 64, 100, 300):
            D, I = idx.search(xq, k)
            check(f"{mn}_ties_k{k}", D, I, x, xq, k, metric, True)
            # the device path: the same lists through search_device
            Dd, Id = idx.search_device(torch.from_numpy(xq).cuda(), k)
            torch.cuda.synchronize()
            check(f"{mn}_ties_device_k{k}", Dd.cpu().numpy(), Id.cpu().numpy(), x, xq, k,
                  metric, True)
        # removals compact inside shards and shift later bases; appends land on
        # the last shard
        rm = np.array([0, 5, 1500, 1501, 3000, 99999], dtype=np.int64)
        n = idx.remove_ids(rm)
        xr, nr = flat.remove_ids(x, rm)
        res[f"{mn}_remove_count"] = bool(n == nr and idx.ntotal == xr.shape[0])
        idx.add_global(x[:17])
        x2 = np.concatenate([xr, x[:17]])
        for k in (10, 60, 150):
            D, I = idx.search(xq, k)
            check(f"{mn}_mutated_k{k}", D, I, x2, xq, k, metric, True)

        # float rows at 1536-d, batch 512: the staged filter engine on every
        # shard (fp32 key window of the oracle)
        xf = rng.standard_normal((20000, 1536)).astype(np.float32)
        qf = rng.standard_normal((512, 1536)).astype(np.float32)
        idf = ShardedIndexFlat(1536, metric, device=0)
        idf.add_global(xf)
        for k in (10, 50, 100):
            Dd, Id = idf.search_device(torch.from_numpy(qf).cuda(), k)
            torch.cuda.synchronize()
            check(f"{mn}_float_device_k{k}", Dd.cpu().numpy(), Id.cpu().numpy(), xf, qf, k,
                  metric, False)
        # a caller's stream other than torch's current one (sharded.py runs the
        # search, the gather and the merge in that stream's order): the queries
        # are written on the current stream, the lists read back after a sync of
        # the side stream alone
        side = torch.cuda.Stream()
        qd = torch.from_numpy(qf).cuda()
        side.wait_stream(torch.cuda.current_stream())
        Dd, Id = idf.search_device(qd, 10, stream=side.cuda_stream)
        side.synchronize()
        check(f"{mn}_float_side_stream_k10", Dd.cpu().numpy(), Id.cpu().numpy(), xf, qf, 10,
              metric, False)
    if rank == 0:
        print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
