"""Student-neighbour self-join on the MI355X engine.

Replaces the per-student pgvector loop of the graph refresher
(src/graph_refresher/main.py:299-354) and the single-student query of the
similarity worker (src/incremental_workers/similarity/main.py:80-94):

    vectors -> "[%.6f,...]" pgvector literals (main.py:301)
    for each student s:  SELECT student_id, 1-(vec <=> src.vec) AS sim ...
                         WHERE student_id <> s ORDER BY vec <=> src.vec LIMIT 15
    keep rows with sim >= S.similarity_threshold (0.75; main.py:350-354, settings.py:139)

Here all students are one ``vs_selfjoin`` launch (cosine, exclude self by row,
top-k), with the %.6f quantisation applied on the host exactly as the text
round-trip does.  Output rows are the ``student_similarity(a, b, sim)`` tuples
(sql/00_init_schema.sql:105-111) the refresher would insert.

Semantics notes: ties (equal similarity) are ordered by lower row; SQL leaves
them unspecified.  Zero-norm vectors never match; pgvector returns NaN for them
and the refresher's ``sim >= threshold`` test drops NaN too.
"""

from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import faiss as vfaiss

DEFAULT_K = 15  # LIMIT 15 (graph_refresher/main.py:346, similarity/main.py:86)
DEFAULT_THRESHOLD = 0.75  # S.similarity_threshold (src/common/settings.py:139)


def pgvector_quantize(vectors) -> np.ndarray:
    """The f"{x:.6f}" text literal (graph_refresher/main.py:301) parsed back to float32."""
    v = np.asarray(vectors, dtype=np.float64)
    txt = np.char.mod("%.6f", v)
    return txt.astype(np.float64).astype(np.float32)


def build_student_index(vectors, *, quantize: bool = True, device: Optional[int] = None):
    x = pgvector_quantize(vectors) if quantize else np.ascontiguousarray(vectors, np.float32)
    index = vfaiss.IndexFlatIP(x.shape[1], device=device)
    index.add(x)
    return index


def student_neighbours(keys: Sequence[str], vectors, *, k: int = DEFAULT_K,
                       threshold: Optional[float] = DEFAULT_THRESHOLD, quantize: bool = True,
                       device: Optional[int] = None) -> List[Tuple[str, str, float]]:
    """All-students top-k cosine neighbours as (a, b, sim) rows.

    ``threshold=None`` keeps all k (the similarity worker's behaviour,
    similarity/main.py:89-94); a number applies the refresher's filter.
    """
    keys = list(keys)
    if len(keys) == 0:
        return []
    index = build_student_index(vectors, quantize=quantize, device=device)
    min_sim = -np.inf if threshold is None else float(threshold)
    S, I = index.selfjoin(k, exclude_self=True, min_sim=min_sim)
    rows = []
    for a in range(len(keys)):
        for j in range(S.shape[1]):
            b = int(I[a, j])
            if b < 0:
                continue
            rows.append((keys[a], keys[b], float(S[a, j])))
    return rows


class StudentIndex:
    """Resident student vectors for per-event similarity (the similarity worker,
    src/incremental_workers/similarity/main.py:57-102, runs one student's query
    per STUDENT_EMBEDDING event).  The matrix is uploaded once; each event is one
    single-row self-join on the kept index (an HBM-bound scan, no re-upload), and
    a re-embedded student replaces its own row (the student_embeddings upsert of
    student_embedding/main.py:120-146)."""

    def __init__(self, keys: Sequence[str], vectors, *, quantize: bool = True,
                 device: Optional[int] = None):
        self.keys: List[str] = list(keys)
        if len(set(self.keys)) != len(self.keys):
            raise ValueError("StudentIndex: duplicate student keys")
        self.quantize = quantize
        self.index = build_student_index(vectors, quantize=quantize, device=device)
        self._row = {key: i for i, key in enumerate(self.keys)}

    def __len__(self) -> int:
        return len(self.keys)

    def neighbours_of(self, student: str, k: int = DEFAULT_K) -> List[Tuple[str, str, float]]:
        q = self._row[student]
        S, I = self.index.selfjoin(k, q0=q, nq=1, exclude_self=True)
        return [(student, self.keys[int(b)], float(s)) for s, b in zip(S[0], I[0]) if b >= 0]

    def neighbours(self, k: int = DEFAULT_K,
                   threshold: Optional[float] = DEFAULT_THRESHOLD) -> List[Tuple[str, str, float]]:
        min_sim = -np.inf if threshold is None else float(threshold)
        S, I = self.index.selfjoin(k, exclude_self=True, min_sim=min_sim)
        return [(self.keys[a], self.keys[int(b)], float(S[a, j]))
                for a in range(S.shape[0]) for j, b in enumerate(I[a]) if b >= 0]

    def upsert(self, student: str, vector) -> None:
        """Insert or replace one student's vector (a removed row compacts the
        later rows, faiss remove_ids semantics; the key list follows)."""
        v = np.asarray(vector, dtype=np.float32).reshape(1, -1)
        v = pgvector_quantize(v) if self.quantize else v
        if student in self._row:
            r = self._row.pop(student)
            self.index.remove_ids(np.array([r], dtype=np.int64))
            del self.keys[r]
            self._row = {key: i for i, key in enumerate(self.keys)}
        self.index.add(v)
        self._row[student] = len(self.keys)
        self.keys.append(student)


def student_neighbours_of(student: str, keys: Sequence[str], vectors, *, k: int = DEFAULT_K,
                          quantize: bool = True, device: Optional[int] = None,
                          index: Optional[StudentIndex] = None):
    """One student's rows (the similarity worker's compute_similarity).  Pass a
    resident ``StudentIndex`` to avoid uploading the matrix on every event."""
    if index is None:
        index = StudentIndex(keys, vectors, quantize=quantize, device=device)
    return index.neighbours_of(student, k)
