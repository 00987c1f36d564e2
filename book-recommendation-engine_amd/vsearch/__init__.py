"""vsearch — MI355X-native exact vector search for the book-recommendation engine.

Layers (bottom-up):
  libvsearch.so   HIP kernels for gfx950 + the C-ABI of include/vsearch.h
  vsearch._lib    ctypes binding (fails loudly if the library is not built)
  vsearch.faiss   faiss-compatible IndexFlatL2 / IndexFlatIP / read_index / write_index
  vsearch.langchain  drop-in for langchain_community.vectorstores.FAISS
  vsearch.students   pgvector cosine self-join replacement (graph refresher)
  vsearch.sharded    row-sharded multi-GPU index (RCCL all-gather top-k merge)
  vsearch.synth      deterministic synthetic embeddings / corpus generator
"""

from ._lib import METRIC_INNER_PRODUCT, METRIC_L2, VSearchError  # noqa: F401

__version__ = "0.1.0"
