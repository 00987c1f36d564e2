"""Row-sharded flat index across the GPUs of one node (one process per GPU).

Global labels 0..N-1 are split into contiguous blocks; rank g owns
[off_g, off_g + n_g) and its shard reports global labels (vs_set_id_base).
A search runs the local fused top-k on every rank, all-gathers the per-shard
lists over RCCL (torch.distributed backend "nccl" = RCCL on ROCm, over xGMI),
and merges them on the GPU — so the result equals the single-index result,
ties included:
  * L2: each shard returns its k best by (distance, label); the k best of the
    union are among them, in the same lexicographic order faiss's CMax heap uses.
  * inner product: faiss's CMin heap tie rule is a function of the 2k-1
    lexicographically best (-score, label) pairs of the whole corpus
    (oracle/flat.py faiss_order), so each shard returns its RAW best
    m = 2k-1 pairs (VS_RAW_ORDER, no tie rule applied; any k: the shard's
    paged search, vs_api.hip run_paged) and the merge (vs_merge_topk, any
    k_in) applies the rule once to the union of those lists.
The exchange is B*m*12 bytes per rank: latency-bound, not link-bound.

Appends go to the last shard; removals compact inside each shard and shift the
later shards' id bases, so global labels stay faiss positions.
"""

from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _lib
from . import faiss as vfaiss


def shard_bounds(ntotal: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block of rows owned by `rank`."""
    lo = ntotal * rank // world
    hi = ntotal * (rank + 1) // world
    return lo, hi


class ShardedIndexFlat:
    """One shard per rank; collective search.  Requires torch.distributed to be
    initialised (any backend for host tensors; "nccl" for device tensors)."""

    def __init__(self, d: int, metric: int = vfaiss.METRIC_L2, *, device: Optional[int] = None,
                 group=None, shard=None, merge=None, dtype: str = "f32"):
        """`shard` / `merge` let tests substitute the per-rank index and the list
        merge (e.g. the CPU oracle under gloo); production uses the GPU ones."""
        import torch.distributed as dist

        self._dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.shard = (shard if shard is not None
                      else vfaiss.IndexFlat(d, metric, device=device, dtype=dtype))
        self._merge = merge
        self.d = d
        self.metric_type = metric
        self._counts = np.zeros(self.world, dtype=np.int64)

    # -- layout ---------------------------------------------------------------------
    def _sync_counts(self) -> None:
        import torch

        mine = torch.tensor([self.shard.ntotal], dtype=torch.int64)
        dev = self._coll_device()
        mine = mine.to(dev)
        allc = [torch.zeros_like(mine) for _ in range(self.world)]
        self._dist.all_gather(allc, mine, group=self.group)
        self._counts = np.array([int(c.item()) for c in allc], dtype=np.int64)
        base = int(self._counts[: self.rank].sum())
        self.shard.set_id_base(base)

    def _coll_device(self):
        import torch

        backend = self._dist.get_backend(self.group)
        if backend == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    @property
    def ntotal(self) -> int:
        return int(self._counts.sum())

    def add_synthetic(self, ntotal: int, seed: int) -> None:
        """Each rank generates its own block of the global synthetic corpus."""
        lo, hi = shard_bounds(ntotal, self.world, self.rank)
        if hi > lo:
            self.shard.reserve(hi - lo)
            self.shard.add_synthetic(hi - lo, seed, row0=lo)
        self._sync_counts()

    def append_synthetic_ids(self, gen_ids, seed: int) -> None:
        """Append synthetic rows (by generator row number) at the end of the
        global label space, i.e. on the last shard."""
        if self.rank == self.world - 1:
            self.shard.add_synthetic_ids(gen_ids, seed)
        self._sync_counts()

    def add_global(self, x: np.ndarray) -> None:
        """Every rank passes the same rows; each keeps its block (initial load)."""
        x = np.ascontiguousarray(x, dtype=np.float32)
        lo, hi = shard_bounds(x.shape[0], self.world, self.rank)
        if self.ntotal:
            # appends go to the last shard (labels continue at ntotal)
            if self.rank == self.world - 1:
                self.shard.add(x)
        elif hi > lo:
            self.shard.add(x[lo:hi])
        self._sync_counts()

    def remove_ids(self, ids) -> int:
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        n = self.shard.remove_ids(ids)  # shard ignores labels outside its block
        self._sync_counts()
        return int(n) if self.world == 1 else self._allreduce_int(n)

    def _allreduce_int(self, n: int) -> int:
        import torch

        t = torch.tensor([n], dtype=torch.int64, device=self._coll_device())
        self._dist.all_reduce(t, group=self.group)
        return int(t.item())

    # -- search ---------------------------------------------------------------------
    def shard_k(self, k: int) -> int:
        """Entries each shard contributes to the merge (see the module docstring)."""
        if self.metric_type == vfaiss.METRIC_INNER_PRODUCT:
            return 2 * int(k) - 1  # raw searches page past 64 entries (any k)
        return int(k)

    def search(self, x, k: int):
        """Host-array convenience wrapper: same contract as IndexFlat.search."""
        import torch

        x = np.ascontiguousarray(x, dtype=np.float32)
        kin = self.shard_k(k)
        D, I = self.shard.search(x, kin, raw=True)
        dev = self._coll_device()
        Dt = torch.from_numpy(D).to(dev)
        It = torch.from_numpy(I).to(dev)
        Dall, Iall = self._gather(Dt, It)
        if self._merge is not None:
            return self._merge(Dall.cpu().numpy(), Iall.cpu().numpy(), self.metric_type, k)
        if dev.type != "cuda":
            # gloo gathered host tensors: the merge itself still runs on the GPU
            gpu = torch.device("cuda", self.shard.device)
            Dall, Iall = Dall.to(gpu), Iall.to(gpu)
        Dm, Im = self.merge_device(Dall, Iall, x.shape[0], kin, k)
        return Dm.cpu().numpy(), Im.cpu().numpy()

    def _gather(self, Dt, It):
        import torch

        if Dt.device.type == "cuda" and self._dist.get_backend(self.group) != "nccl":
            # gloo gathers host tensors only (its GPU support is broadcast and
            # all-reduce): stage through the host, hand device tensors back
            Dh, Ih = self._gather(Dt.cpu(), It.cpu())
            return Dh.to(Dt.device), Ih.to(It.device)
        # flat (world*nq, k) outputs: the layout every backend accepts
        Dall = torch.empty((self.world * Dt.shape[0],) + tuple(Dt.shape[1:]), dtype=Dt.dtype,
                           device=Dt.device)
        Iall = torch.empty((self.world * It.shape[0],) + tuple(It.shape[1:]), dtype=It.dtype,
                           device=It.device)
        self._dist.all_gather_into_tensor(Dall, Dt.contiguous(), group=self.group)
        self._dist.all_gather_into_tensor(Iall, It.contiguous(), group=self.group)
        return (Dall.view((self.world,) + tuple(Dt.shape)),
                Iall.view((self.world,) + tuple(It.shape)))

    def merge_device(self, Dall, Iall, nq: int, k_in: int, k: int, stream: int = 0):
        import torch

        Dm = torch.empty((nq, k), dtype=torch.float32, device=Dall.device)
        Im = torch.empty((nq, k), dtype=torch.int64, device=Dall.device)
        _lib.check(_lib.load().vs_merge_topk(
            ctypes.c_void_p(Dall.data_ptr()), ctypes.c_void_p(Iall.data_ptr()), self.world, nq,
            k_in, k, self.metric_type, ctypes.c_void_p(Dm.data_ptr()),
            ctypes.c_void_p(Im.data_ptr()), ctypes.c_void_p(stream)), "vs_merge_topk")
        return Dm, Im

    def search_device(self, xq, k: int, stream: int = 0):
        """Device tensors end to end: xq (nq, d) float32 cuda tensor on this rank's
        GPU (replicated on every rank) -> merged (D, I) cuda tensors.

        Every step runs in the order of `stream`: the shard search writes its
        lists there, and the output allocations, the collective (RCCL runs it on
        its own stream after waiting for the current one, and makes the current
        one wait for it) and the merge all see `stream` as torch's current stream,
        so a caller's stream other than torch's current one orders the gather
        after the search and the merge after the gather (no race either way)."""
        import torch

        cur = torch.cuda.current_stream(xq.device)
        if stream and stream != cur.cuda_stream:
            ext = torch.cuda.ExternalStream(stream, device=xq.device)
            with torch.cuda.stream(ext):
                return self._search_device(xq, k, stream)
        return self._search_device(xq, k, stream)

    def _search_device(self, xq, k: int, stream: int):
        import torch

        nq = xq.shape[0]
        if self.world == 1:  # the shard is the whole index: faiss order directly
            Dl = torch.empty((nq, k), dtype=torch.float32, device=xq.device)
            Il = torch.empty((nq, k), dtype=torch.int64, device=xq.device)
            self.shard.search_device(xq.data_ptr(), nq, k, Dl.data_ptr(), Il.data_ptr(), stream)
            return Dl, Il
        kin = self.shard_k(k)
        Dl = torch.empty((nq, kin), dtype=torch.float32, device=xq.device)
        Il = torch.empty((nq, kin), dtype=torch.int64, device=xq.device)
        self.shard.search_device(xq.data_ptr(), nq, kin, Dl.data_ptr(), Il.data_ptr(), stream,
                                 raw=True)
        Dall, Iall = self._gather(Dl, Il)
        return self.merge_device(Dall, Iall, nq, kin, k, stream)
