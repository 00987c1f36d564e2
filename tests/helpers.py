"""Test doubles built on the CPU oracle (test infrastructure only).

OracleIndex implements the faiss-index surface that the host logic (LangChain
store, persistence, sharding) uses, with the oracle as its arithmetic, so the
host logic is testable on CPU.  It is never used by product code."""

from __future__ import annotations

import numpy as np

from oracle import flat


class OracleIndex:
    is_trained = True

    def __init__(self, d: int, metric: int = flat.METRIC_L2):
        self.d = int(d)
        self.metric_type = int(metric)
        self._x = np.zeros((0, self.d), dtype=np.float32)
        self._base = 0
        self.device = 0

    @property
    def ntotal(self) -> int:
        return self._x.shape[0]

    def add(self, x):
        x = np.ascontiguousarray(x, dtype=np.float32)
        assert x.shape[1] == self.d
        self._x = np.concatenate([self._x, x])

    def search(self, x, k, raw=False):
        x = np.ascontiguousarray(x, dtype=np.float32)
        assert x.shape[1] == self.d
        assert k > 0
        if raw:  # VS_RAW_ORDER: lexicographic (key, label), no IP tie rule
            D, I = flat.knn_lex(self._x, x, k, self.metric_type)
        else:
            D, I = flat.knn_exact(self._x, x, k, self.metric_type)
        I = np.where(I >= 0, I + self._base, -1)
        return D, I

    def reconstruct(self, i):
        if not 0 <= i < self.ntotal:
            raise RuntimeError("key out of range")
        return self._x[i].copy()

    def reconstruct_n(self, n0=0, ni=-1):
        if ni == -1:
            ni = self.ntotal - n0
        return self._x[n0:n0 + ni].copy()

    def remove_ids(self, ids):
        ids = np.asarray(ids, dtype=np.int64) - self._base
        self._x, n = flat.remove_ids(self._x, ids)
        return n

    def set_id_base(self, base):
        self._base = int(base)

    def reset(self):
        self._x = np.zeros((0, self.d), dtype=np.float32)


def oracle_merge(Dall, Iall, metric, k):
    """Merge gathered shard lists [G][nq][k_in] with the oracle's tie rule."""
    G, nq, kin = Dall.shape
    D = np.full((nq, k), flat.neutral(metric), dtype=np.float32)
    I = np.full((nq, k), -1, dtype=np.int64)
    for q in range(nq):
        s = Dall[:, q, :].ravel()
        ids = Iall[:, q, :].ravel()
        keep = ids >= 0
        s, ids = s[keep], ids[keep]
        if ids.size == 0:
            continue
        key = s if metric == flat.METRIC_L2 else -s
        sel = flat.faiss_order(ids, key, k, metric)
        pos = {int(i): j for j, i in enumerate(ids)}
        D[q, :sel.size] = [s[pos[int(i)]] for i in sel]
        I[q, :sel.size] = sel
    return D, I
