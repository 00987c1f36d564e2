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


def student_neighbours_of(student: str, keys: Sequence[str], vectors, *, k: int = DEFAULT_K,
                          quantize: bool = True, device: Optional[int] = None):
    """One student's rows (the similarity worker's compute_similarity)."""
    keys = list(keys)
    q = keys.index(student)
    index = build_student_index(vectors, quantize=quantize, device=device)
    S, I = index.selfjoin(k, q0=q, nq=1, exclude_self=True)
    return [(student, keys[int(b)], float(s)) for s, b in zip(S[0], I[0]) if b >= 0]
