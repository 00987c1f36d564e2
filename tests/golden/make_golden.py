"""Generate the committed golden fixtures for BASELINE config 1 (CSV samples).

Run in the build container (needs /root/reference/data, which does not exist on
the GPU box):   python tests/golden/make_golden.py

Inputs (data, not source): the reference's sample CSVs
  /root/reference/data/catalog_sample.csv   (341 books; CSV order = label order)
  /root/reference/data/students_sample.csv  (25 students)
are reduced to the texts the reference would embed — the full-rebuild template
of src/incremental_workers/book_vector/main.py:449-460 and the StudentFlattener
text of src/embedding/student.py:15-41 — plus the book metadata dict of
book_vector/main.py:462-466.  Embeddings are deterministic (vsearch.synth.synth_embed;
SURVEY.md §8d), so the fixture stores texts, and tests regenerate the vectors.

Expected outputs come from the fp64 oracle (oracle/flat.py), cross-checked here
against the C faiss-heap restatement (oracle/faiss_flat.c):
  * books: queries = all 341 book vectors + 64 keyword queries, k = 30, metric L2 and IP
  * students: cosine self-join (pgvector semantics), k = 15 and k = 50, no threshold
  * the reference's own 3-d tie stub ([i%3]*3, query [0,0,0]; tests/test_integration_ingestion_graph.py:40-48)
"""

from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "book-recommendation-engine_amd"))

from oracle import cfaiss, flat  # noqa: E402
from vsearch import synth  # noqa: E402

REF_DATA = "/root/reference/data"

KEYWORDS = [
    "space adventure", "friendship animals", "dragons and magic", "mystery at school",
    "funny family stories", "ocean exploration", "dinosaurs", "princess fairy tale",
    "sports teamwork", "robots and technology", "historical war story", "graphic novel humor",
    "detective puzzle", "survival in the wilderness", "time travel", "ghost story",
    "horses and ranch life", "superheroes", "cooking and food", "music and dance",
    "immigrant family", "civil rights history", "science experiments", "poetry for kids",
    "pirates treasure", "camping trip", "new sibling", "moving to a new town",
    "bullying and kindness", "a dog's journey", "cats", "wizards school",
    "fantasy quest", "middle school drama", "diary of a kid", "chapter book series",
    "picture book bedtime", "nature and seasons", "weather and storms", "planets and stars",
    "ancient egypt", "knights and castles", "myths and legends", "fairy tales retold",
    "comic adventure", "mystery detective kids", "animal rescue", "farm life",
    "city life", "basketball", "soccer", "baseball", "art and painting",
    "friendship breakup", "grief and loss", "courage", "family road trip", "holiday story",
    "winter snow", "summer camp", "zombies", "aliens", "inventors", "biography of a scientist",
]
assert len(KEYWORDS) == 64


def main() -> None:
    books = synth.read_csv(os.path.join(REF_DATA, "catalog_sample.csv"))
    students = synth.read_csv(os.path.join(REF_DATA, "students_sample.csv"))
    book_texts = [synth.book_text(r) for r in books]
    book_meta = [synth.book_metadata(r) for r in books]
    student_keys = [r["student_id"] for r in students]
    student_texts = [synth.student_text(r) for r in students]

    xb = np.stack([synth.synth_embed(t) for t in book_texts])
    xq = np.concatenate([xb, np.stack([synth.synth_embed(t) for t in KEYWORDS])])
    xs = np.stack([synth.synth_embed(t) for t in student_texts])

    out = {}
    for metric, name in ((flat.METRIC_L2, "l2"), (flat.METRIC_INNER_PRODUCT, "ip")):
        D, I = flat.knn_exact(xb, xq, 30, metric)
        Dc, Ic = cfaiss.knn_seq(xb, xq, 30, metric)
        assert not flat.mismatches(Dc, Ic, D, I, metric, xb, xq), name
        out[f"books_{name}_D"] = D
        out[f"books_{name}_I"] = I
    for k in (15, 50):
        S, I = flat.pgvector_cosine_topk(xs, k)
        out[f"students_k{k}_S"] = S
        out[f"students_k{k}_I"] = I
    tie_b = np.array([[float(i % 3)] * 3 for i in range(len(books))], dtype=np.float32)
    tie_q = np.zeros((1, 3), dtype=np.float32)
    for metric, name in ((flat.METRIC_L2, "l2"), (flat.METRIC_INNER_PRODUCT, "ip")):
        for k in (1, 4, 5, 10):
            D, I = cfaiss.knn_seq(tie_b, tie_q, k, metric)
            Dn, In = flat.knn_exact(tie_b, tie_q, k, metric)
            assert np.array_equal(I, In) and np.array_equal(D, Dn)
            out[f"tie_{name}_k{k}_I"] = I
            out[f"tie_{name}_k{k}_D"] = D
    np.savez_compressed(os.path.join(HERE, "csv_sample_expected.npz"), **out)
    with open(os.path.join(HERE, "csv_sample_inputs.json"), "w", encoding="utf-8") as f:
        json.dump({
            "source": "reference data/catalog_sample.csv + data/students_sample.csv "
                      "(texts per book_vector/main.py:449-460 and embedding/student.py:15-41)",
            "embedding": "vsearch.synth.synth_embed (sha256 -> PCG64 -> normal -> unit norm)",
            "book_texts": book_texts,
            "book_metadata": book_meta,
            "keywords": KEYWORDS,
            "student_keys": student_keys,
            "student_texts": student_texts,
        }, f, indent=0)
    print("wrote", sorted(out))


if __name__ == "__main__":
    main()
