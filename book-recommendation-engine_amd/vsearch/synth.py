"""Deterministic synthetic inputs (the reference's embeddings come from OpenAI over
the network, which does not exist here; the reference's own tests stub them too,
tests/test_integration_ingestion_graph.py:40-48).

* ``synth_embed(text)`` — text -> unit-norm 1536-d float32:
  seed = first 8 bytes (little-endian) of SHA-256(text),
  ``np.random.Generator(PCG64(seed)).standard_normal(dim)``, L2-normalised in
  float64, cast to float32 (mimics text-embedding-3-small's unit-norm output;
  model/dim from src/common/settings.py:16-18).
* ``SynthEmbeddings`` — an ``Embeddings``-like object (embed_documents /
  embed_query) for the drop-in store.
* ``book_text`` / ``student_text`` — the reference's text templates
  (book_vector/main.py:449-460 full-rebuild template; embedding/student.py:15-41
  StudentFlattener).
* ``synthetic_rows`` — numpy restatement of the counter-based corpus generator
  that libvsearch's ``vs_fill_synthetic`` runs on the GPU:
  x[i, j] = ((splitmix64(seed ^ (i*d + j)) >> 40) * 2^-23) - 1.
"""

from __future__ import annotations

import csv
import hashlib
import json
from typing import Dict, List, Sequence

import numpy as np

EMBED_DIM = 1536  # text-embedding-3-small (src/common/settings.py:16-18, sql/00_init_schema.sql:92)


def synth_embed(text: str, dim: int = EMBED_DIM) -> np.ndarray:
    seed = int.from_bytes(hashlib.sha256(text.encode("utf-8")).digest()[:8], "little")
    v = np.random.Generator(np.random.PCG64(seed)).standard_normal(dim)
    v /= np.sqrt(np.dot(v, v))
    return v.astype(np.float32)


class SynthEmbeddings:
    """Stand-in for ``OpenAIEmbeddings`` with deterministic unit-norm vectors."""

    def __init__(self, dim: int = EMBED_DIM):
        self.dim = dim

    def embed_documents(self, texts: Sequence[str]) -> List[List[float]]:
        return [synth_embed(t, self.dim).tolist() for t in texts]

    def embed_query(self, text: str) -> List[float]:
        return synth_embed(text, self.dim).tolist()


def book_text(row: Dict[str, str]) -> str:
    """Full-rebuild text template of src/incremental_workers/book_vector/main.py:449-460."""
    try:
        genre_list = json.loads(row.get("genre") or "[]")
    except Exception:
        genre_list = []
    genres_str = ", ".join(genre_list)
    desc = row.get("description") or ""
    return (
        f"{row['title']} by {row['author']}. "
        f"Genre: {genres_str}. "
        f"Reading level: {row['reading_level']} ({row['difficulty_band']}). "
        f"Published {row['publication_year']}. "
        f"{desc}"
    )


def book_metadata(row: Dict[str, str]) -> Dict[str, str]:
    """Metadata dict of book_vector/main.py:462-466."""
    try:
        genre_list = json.loads(row.get("genre") or "[]")
    except Exception:
        genre_list = []
    return {"book_id": row["book_id"], "genre": ", ".join(genre_list),
            "level": row["reading_level"]}


def student_text(row: Dict[str, str]) -> str:
    """StudentFlattener text (src/embedding/student.py:15-41)."""
    parts = [f"Grade {row.get('grade_level', 4)} student with id {row.get('student_id')}"]
    homeroom = row.get("homeroom_teacher")
    if homeroom:
        tok = homeroom.lower().replace("ms. ", "").replace("mr. ", "").replace(" ", "-")
        parts.append(f"teacher-{tok}")
    lunch = row.get("lunch_period")
    if lunch:
        parts.append(f"lunch-{lunch}")
    prior = row.get("prior_year_reading_score")
    if prior:
        # the DB column is numeric: ints stay ints (round(3, 1) == 3), floats round
        try:
            prior = int(prior)
        except ValueError:
            try:
                prior = round(float(prior), 1)
            except ValueError:
                pass
        parts.append(f"reading-level-{prior}")
    return " ".join(parts)


def read_csv(path: str) -> List[Dict[str, str]]:
    with open(path, newline="", encoding="utf-8") as f:
        return list(csv.DictReader(f))


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def synthetic_rows(row0: int, n: int, d: int, seed: int) -> np.ndarray:
    """Rows [row0, row0+n) of the counter-based corpus (float32 in [-1, 1))."""
    i = np.arange(row0, row0 + n, dtype=np.uint64)[:, None]
    j = np.arange(d, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        ctr = i * np.uint64(d) + j
    z = _splitmix64(np.uint64(seed) ^ ctr)
    return ((z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 8388608.0)
            - np.float32(1.0)).astype(np.float32)
