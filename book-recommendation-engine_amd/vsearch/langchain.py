"""Drop-in for ``langchain_community.vectorstores.FAISS`` on the MI355X engine.

The reference hard-imports ``from langchain_community.vectorstores import FAISS``
(src/ingestion_service/pipeline.py:15, ingestion_service/main.py:51,
incremental_workers/book_vector/main.py:53,432, recommendation_api/candidate_builder.py:31,
service.py:31, mcp_book_server.py:24).  langchain-community 0.3.26
(/root/reference/poetry.lock:1577-1578) is not vendored; this module restates the
method surface those call sites use, with the same argument meaning, return
types and error behaviour:

* ``FAISS.from_texts`` / ``from_embeddings`` — IndexFlatIP for
  ``DistanceStrategy.MAX_INNER_PRODUCT``, IndexFlatL2 otherwise (the reference
  never passes a strategy, so its stores are L2: SURVEY.md §0.2).
* ``add_texts`` / ``add_embeddings`` — uuid4 ids by default, ``ValueError`` on
  duplicate ids, labels continue at ``len(index_to_docstore_id)``.
* ``similarity_search[_with_score][_by_vector]`` — ``index.search(vec, k or
  fetch_k)``, skip label -1, docstore lookup, optional metadata filter and
  ``score_threshold`` (``<=`` for L2, ``>=`` for inner product), ``docs[:k]``;
  the score is faiss's D value (squared L2 / inner product) as ``np.float32``.
* ``delete`` — ``ValueError`` for unknown ids, then ``index.remove_ids`` and
  contiguous renumbering of ``index_to_docstore_id``.
* ``save_local`` / ``load_local`` — ``index.faiss`` in faiss's flat binary
  format plus a JSON docstore sidecar (``index.docstore.json``; LangChain's
  ``index.pkl`` needs LangChain's classes to unpickle and is not read);
  ``load_local`` still demands ``allow_dangerous_deserialization=True``.
"""

from __future__ import annotations

import enum
import json
import logging
import math
import operator
import uuid
import warnings
from pathlib import Path
from typing import Any, Callable, Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import faiss as vfaiss

logger = logging.getLogger(__name__)

__all__ = ["Document", "InMemoryDocstore", "DistanceStrategy", "FAISS",
           "migrate_reference_store", "full_faiss_rebuild"]


class Document:
    """langchain_core.documents.Document (page_content, metadata, id)."""

    __slots__ = ("page_content", "metadata", "id")

    def __init__(self, page_content: str, metadata: Optional[dict] = None,
                 id: Optional[str] = None, **_ignored):
        if not isinstance(page_content, str):
            raise TypeError("page_content must be a str")
        self.page_content = page_content
        self.metadata = {} if metadata is None else metadata
        self.id = id

    @property
    def type(self) -> str:
        return "Document"

    def __eq__(self, other):
        return (isinstance(other, Document) and self.page_content == other.page_content
                and self.metadata == other.metadata and self.id == other.id)

    def __repr__(self):
        idp = f"id='{self.id}', " if self.id is not None else ""
        return f"Document({idp}metadata={self.metadata!r}, page_content={self.page_content!r})"

    def to_json(self) -> dict:
        return {"page_content": self.page_content, "metadata": self.metadata, "id": self.id}

    @classmethod
    def from_json(cls, obj: dict) -> "Document":
        return cls(page_content=obj["page_content"], metadata=obj.get("metadata") or {},
                   id=obj.get("id"))


class InMemoryDocstore:
    """langchain_community.docstore.in_memory.InMemoryDocstore."""

    def __init__(self, _dict: Optional[Dict[str, Document]] = None):
        self._dict = _dict if _dict is not None else {}

    def add(self, texts: Dict[str, Document]) -> None:
        overlapping = set(texts).intersection(self._dict)
        if overlapping:
            raise ValueError(f"Tried to add ids that already exist: {overlapping}")
        self._dict = {**self._dict, **texts}

    def delete(self, ids: List) -> None:
        overlapping = set(ids).intersection(self._dict)
        if not overlapping:
            raise ValueError(f"Tried to delete ids that does not  exist: {ids}")
        for _id in ids:
            self._dict.pop(_id)

    def search(self, search: str):
        if search not in self._dict:
            return f"ID {search} not found."
        return self._dict[search]


class DistanceStrategy(str, enum.Enum):
    """langchain_community.vectorstores.utils.DistanceStrategy."""

    EUCLIDEAN_DISTANCE = "EUCLIDEAN_DISTANCE"
    MAX_INNER_PRODUCT = "MAX_INNER_PRODUCT"
    DOT_PRODUCT = "DOT_PRODUCT"
    JACCARD = "JACCARD"
    COSINE = "COSINE"


def _len_check_if_sized(x: Any, y: Any, x_name: str, y_name: str) -> None:
    if hasattr(x, "__len__") and hasattr(y, "__len__") and len(x) != len(y):
        raise ValueError(
            f"{x_name} and {y_name} expected to be equal length but "
            f"len({x_name})={len(x)} and len({y_name})={len(y)}"
        )


_FILTER_OPS: Dict[str, Callable[[Any, Any], bool]] = {
    "$eq": operator.eq,
    "$neq": operator.ne,
    "$gt": operator.gt,
    "$lt": operator.lt,
    "$gte": operator.ge,
    "$lte": operator.le,
    "$in": lambda a, b: a in b,
    "$nin": lambda a, b: a not in b,
}


def _create_filter_func(filter: Any) -> Callable[[Dict[str, Any]], bool]:
    """Metadata filter: callable, or MongoDB-style dict ($eq/$neq/$gt/$lt/$gte/$lte/
    $in/$nin/$and/$or/$not; a bare list value means membership)."""
    if callable(filter):
        return filter
    if not isinstance(filter, dict):
        raise ValueError(f"filter must be a dict of metadata or a callable, not {type(filter)}")

    def filter_func_cond(field: str, condition: Any) -> Callable[[Dict[str, Any]], bool]:
        if isinstance(condition, dict):
            ops = []
            for op, value in condition.items():
                if op not in _FILTER_OPS:
                    raise ValueError(f"filter contains unsupported operator: {op}")
                ops.append((_FILTER_OPS[op], value))

            def cond(doc, ops=ops):
                try:
                    return all(fn(doc.get(field), value) for fn, value in ops)
                except TypeError:  # e.g. None > 3
                    return False

            return cond
        if isinstance(condition, list):
            return lambda doc: doc.get(field) in condition
        return lambda doc: doc.get(field) == condition

    def build(f: Dict[str, Any]) -> Callable[[Dict[str, Any]], bool]:
        parts = []
        for key, value in f.items():
            if key == "$and":
                subs = [build(x) for x in value]
                parts.append(lambda doc, subs=subs: all(s(doc) for s in subs))
            elif key == "$or":
                subs = [build(x) for x in value]
                parts.append(lambda doc, subs=subs: any(s(doc) for s in subs))
            elif key == "$not":
                sub = build(value)
                parts.append(lambda doc, sub=sub: not sub(doc))
            else:
                parts.append(filter_func_cond(key, value))
        return lambda doc: all(p(doc) for p in parts)

    return build(filter)


class FAISS:
    """Vector store over a vsearch flat index (LangChain ``FAISS`` API)."""

    def __init__(self, embedding_function, index, docstore, index_to_docstore_id: Dict[int, str],
                 relevance_score_fn: Optional[Callable[[float], float]] = None,
                 normalize_L2: bool = False,
                 distance_strategy: DistanceStrategy = DistanceStrategy.EUCLIDEAN_DISTANCE):
        if not (hasattr(embedding_function, "embed_query") or callable(embedding_function)):
            logger.warning("`embedding_function` is expected to be an Embeddings object")
        self.embedding_function = embedding_function
        self.index = index
        self.docstore = docstore
        self.index_to_docstore_id = index_to_docstore_id
        self.distance_strategy = DistanceStrategy(distance_strategy)
        self.override_relevance_score_fn = relevance_score_fn
        self._normalize_L2 = normalize_L2
        self._keymap_field: Optional[str] = None  # metadata field indexed by _key_index
        self._keymap: Dict[Any, List[str]] = {}
        if (self.distance_strategy != DistanceStrategy.EUCLIDEAN_DISTANCE
                and self._normalize_L2):
            warnings.warn(
                f"Normalizing L2 is not applicable for metric type: {self.distance_strategy}")

    # -- embeddings --------------------------------------------------------------------
    @property
    def embeddings(self):
        return self.embedding_function if hasattr(self.embedding_function, "embed_query") else None

    def _embed_documents(self, texts: List[str]) -> List[List[float]]:
        if hasattr(self.embedding_function, "embed_documents"):
            return self.embedding_function.embed_documents(texts)
        return [self.embedding_function(t) for t in texts]

    def _embed_query(self, text: str) -> List[float]:
        if hasattr(self.embedding_function, "embed_query"):
            return self.embedding_function.embed_query(text)
        return self.embedding_function(text)

    # -- writes ---------------------------------------------------------------------------
    def __add(self, texts: Iterable[str], embeddings: Iterable[List[float]],
              metadatas: Optional[Iterable[dict]] = None,
              ids: Optional[List[str]] = None) -> List[str]:
        if not hasattr(self.docstore, "add"):
            raise ValueError("If trying to add texts, the underlying docstore should support "
                             f"adding items, which {self.docstore} does not")
        _len_check_if_sized(texts, metadatas, "texts", "metadatas")
        ids = ids or [str(uuid.uuid4()) for _ in texts]
        _len_check_if_sized(texts, ids, "texts", "ids")
        _metadatas = metadatas or ({} for _ in texts)
        documents = [Document(id=id_, page_content=t, metadata=m)
                     for id_, t, m in zip(ids, texts, _metadatas)]
        _len_check_if_sized(documents, embeddings, "documents", "embeddings")
        if ids and len(ids) != len(set(ids)):
            raise ValueError("Duplicate ids found in the ids list.")
        vector = np.array(embeddings, dtype=np.float32)
        if vector.ndim == 1:
            vector = vector.reshape(len(documents), -1)
        if self._normalize_L2:
            vfaiss.normalize_L2(vector)
        self.index.add(vector)
        self.docstore.add({id_: doc for id_, doc in zip(ids, documents)})
        starting_len = len(self.index_to_docstore_id)
        self.index_to_docstore_id.update({starting_len + j: id_ for j, id_ in enumerate(ids)})
        if self._keymap_field is not None:
            for doc in documents:
                key = doc.metadata.get(self._keymap_field)
                if key is not None:
                    self._keymap.setdefault(key, []).append(doc.id)
        return ids

    def add_texts(self, texts: Iterable[str], metadatas: Optional[List[dict]] = None,
                  ids: Optional[List[str]] = None, **kwargs: Any) -> List[str]:
        texts = list(texts)
        embeddings = self._embed_documents(texts)
        return self.__add(texts, embeddings, metadatas=metadatas, ids=ids)

    def add_embeddings(self, text_embeddings: Iterable[Tuple[str, List[float]]],
                       metadatas: Optional[List[dict]] = None, ids: Optional[List[str]] = None,
                       **kwargs: Any) -> List[str]:
        texts, embeddings = zip(*text_embeddings)
        return self.__add(texts, embeddings, metadatas=metadatas, ids=ids)

    def add_documents(self, documents: List[Document], **kwargs: Any) -> List[str]:
        texts = [d.page_content for d in documents]
        metadatas = [d.metadata for d in documents]
        if "ids" not in kwargs:
            ids = [d.id for d in documents]
            if any(ids):
                kwargs["ids"] = [i if i else str(uuid.uuid4()) for i in ids]
        return self.add_texts(texts, metadatas, **kwargs)

    def _key_index(self, field: str) -> Dict[Any, List[str]]:
        """metadata[field] -> docstore ids holding it.  Built by one scan on first use
        for `field`, then maintained by every add / delete (O(changed rows))."""
        if self._keymap_field != field:
            keymap: Dict[Any, List[str]] = {}
            for i in sorted(self.index_to_docstore_id):
                _id = self.index_to_docstore_id[i]
                doc = self.docstore.search(_id)
                if isinstance(doc, Document) and doc.metadata.get(field) is not None:
                    keymap.setdefault(doc.metadata[field], []).append(_id)
            self._keymap_field, self._keymap = field, keymap
        return self._keymap

    def ids_for_key(self, value: Any, field: str = "book_id") -> List[str]:
        """Docstore ids whose metadata[field] == value, in label order."""
        return list(self._key_index(field).get(value, ()))

    def upsert_embeddings(self, texts: Sequence[str], embeddings: Sequence[List[float]],
                          metadatas: Sequence[dict], key: str = "book_id",
                          ids: Optional[List[str]] = None) -> List[str]:
        """Delete-then-add.  The reference appends a second row when a
        book is re-embedded (incremental_workers/book_vector/main.py:148,
        ingestion_service/pipeline.py:363), so searches return the stale copy too.
        Here every existing row whose metadata[key] matches an incoming row is
        removed first (one remove_ids compaction on the device), and within the
        batch the last row for a key wins.  Rows without the key are plain appends."""
        texts, embeddings, metadatas = list(texts), list(embeddings), list(metadatas)
        _len_check_if_sized(texts, metadatas, "texts", "metadatas")
        _len_check_if_sized(texts, embeddings, "texts", "embeddings")
        if ids is not None:
            _len_check_if_sized(texts, ids, "texts", "ids")
        last = {m.get(key): j for j, m in enumerate(metadatas) if m.get(key) is not None}
        keep = [j for j, m in enumerate(metadatas)
                if m.get(key) is None or last[m.get(key)] == j]
        keymap = self._key_index(key)
        stale = [sid for j in keep if metadatas[j].get(key) is not None
                 for sid in keymap.get(metadatas[j][key], ())]
        if ids is not None:
            clash = set(ids[j] for j in keep).intersection(self.index_to_docstore_id.values())
            clash.difference_update(stale)
            if clash:
                raise ValueError(f"Tried to add ids that already exist: {clash}")
        if stale:
            self.delete(stale)
        return self.__add([texts[j] for j in keep], [embeddings[j] for j in keep],
                          metadatas=[metadatas[j] for j in keep],
                          ids=None if ids is None else [ids[j] for j in keep])

    def upsert_texts(self, texts: Iterable[str], metadatas: List[dict], key: str = "book_id",
                     ids: Optional[List[str]] = None, **kwargs: Any) -> List[str]:
        """`add_texts` with delete-then-add on metadata[key]; embeds before mutating,
        so an embedding failure leaves the store unchanged."""
        texts = list(texts)
        embeddings = self._embed_documents(texts)
        return self.upsert_embeddings(texts, embeddings, metadatas, key=key, ids=ids)

    def delete(self, ids: Optional[List[str]] = None, **kwargs: Any) -> Optional[bool]:
        if ids is None:
            raise ValueError("No ids provided to delete.")
        missing_ids = set(ids).difference(self.index_to_docstore_id.values())
        if missing_ids:
            raise ValueError(
                f"Some specified ids do not exist in the current store. Ids not found: "
                f"{missing_ids}")
        reversed_index = {id_: idx for idx, id_ in self.index_to_docstore_id.items()}
        index_to_delete = {reversed_index[id_] for id_ in ids}
        self.index.remove_ids(np.fromiter(index_to_delete, dtype=np.int64))
        if self._keymap_field is not None:
            for id_ in ids:
                doc = self.docstore.search(id_)
                key = doc.metadata.get(self._keymap_field) if isinstance(doc, Document) else None
                lst = self._keymap.get(key)
                if lst is not None and id_ in lst:
                    lst.remove(id_)
                    if not lst:
                        del self._keymap[key]
        self.docstore.delete(ids)
        remaining_ids = [id_ for i, id_ in sorted(self.index_to_docstore_id.items())
                         if i not in index_to_delete]
        self.index_to_docstore_id = {i: id_ for i, id_ in enumerate(remaining_ids)}
        return True

    def get_by_ids(self, ids: Sequence[str], /) -> List[Document]:
        docs = [self.docstore.search(id_) for id_ in ids]
        return [d for d in docs if isinstance(d, Document)]

    def merge_from(self, target: "FAISS") -> None:
        if not hasattr(self.docstore, "add"):
            raise ValueError("Cannot merge with this type of docstore")
        index_offset = len(self.index_to_docstore_id)
        if target.index.ntotal:
            self.index.add(target.index.reconstruct_n(0, target.index.ntotal))
        full_info = []
        for i, target_id in target.index_to_docstore_id.items():
            doc = target.docstore.search(target_id)
            if not isinstance(doc, Document):
                raise ValueError("Document should be returned")
            full_info.append((index_offset + i, target_id, doc))
        self.docstore.add({_id: doc for _, _id, doc in full_info})
        self.index_to_docstore_id.update({index: _id for index, _id, _ in full_info})

    # -- reads ------------------------------------------------------------------------------
    def similarity_search_with_score_by_vector(self, embedding: List[float], k: int = 4,
                                               filter: Optional[Any] = None, fetch_k: int = 20,
                                               **kwargs: Any) -> List[Tuple[Document, float]]:
        vector = np.array([embedding], dtype=np.float32)
        if self._normalize_L2:
            vfaiss.normalize_L2(vector)
        scores, indices = self.index.search(vector, k if filter is None else fetch_k)
        docs = []
        filter_func = _create_filter_func(filter) if filter is not None else None
        for j, i in enumerate(indices[0]):
            if i == -1:
                continue
            _id = self.index_to_docstore_id[int(i)]
            doc = self.docstore.search(_id)
            if not isinstance(doc, Document):
                raise ValueError(f"Could not find document for id {_id}, got {doc}")
            if filter_func is None or filter_func(doc.metadata):
                docs.append((doc, scores[0][j]))
        score_threshold = kwargs.get("score_threshold")
        if score_threshold is not None:
            cmp = (operator.ge if self.distance_strategy in
                   (DistanceStrategy.MAX_INNER_PRODUCT, DistanceStrategy.JACCARD) else operator.le)
            docs = [(doc, s) for doc, s in docs if cmp(s, score_threshold)]
        return docs[:k]

    def similarity_search_with_score(self, query: str, k: int = 4, filter: Optional[Any] = None,
                                     fetch_k: int = 20, **kwargs: Any):
        embedding = self._embed_query(query)
        return self.similarity_search_with_score_by_vector(embedding, k, filter=filter,
                                                           fetch_k=fetch_k, **kwargs)

    def similarity_search_by_vector(self, embedding: List[float], k: int = 4,
                                    filter: Optional[Any] = None, fetch_k: int = 20,
                                    **kwargs: Any) -> List[Document]:
        return [d for d, _ in self.similarity_search_with_score_by_vector(
            embedding, k, filter=filter, fetch_k=fetch_k, **kwargs)]

    def similarity_search(self, query: str, k: int = 4, filter: Optional[Any] = None,
                          fetch_k: int = 20, **kwargs: Any) -> List[Document]:
        return [d for d, _ in self.similarity_search_with_score(
            query, k, filter=filter, fetch_k=fetch_k, **kwargs)]

    def similarity_search_batch_by_vector(self, embeddings, k: int = 4):
        """Batched variant (one engine call for many queries): list of
        [(Document, score)] per query, label -1 skipped."""
        vec = np.array(embeddings, dtype=np.float32)
        if self._normalize_L2:
            vfaiss.normalize_L2(vec)
        scores, indices = self.index.search(vec, k)
        out = []
        for qi in range(vec.shape[0]):
            row = []
            for j, i in enumerate(indices[qi]):
                if i == -1:
                    continue
                doc = self.docstore.search(self.index_to_docstore_id[int(i)])
                row.append((doc, scores[qi][j]))
            out.append(row)
        return out

    def _select_relevance_score_fn(self) -> Callable[[float], float]:
        if self.override_relevance_score_fn is not None:
            return self.override_relevance_score_fn
        if self.distance_strategy == DistanceStrategy.MAX_INNER_PRODUCT:
            return lambda s: 1.0 - s if s > 0 else -1.0 * s
        if self.distance_strategy == DistanceStrategy.EUCLIDEAN_DISTANCE:
            return lambda d: 1.0 - d / math.sqrt(2)
        if self.distance_strategy == DistanceStrategy.COSINE:
            return lambda d: 1.0 - d
        raise ValueError("Unknown distance strategy, must be cosine, max_inner_product,"
                         " or euclidean")

    def similarity_search_with_relevance_scores(self, query: str, k: int = 4,
                                                filter: Optional[Any] = None, fetch_k: int = 20,
                                                **kwargs: Any):
        fn = self._select_relevance_score_fn()
        score_threshold = kwargs.pop("score_threshold", None)
        docs = self.similarity_search_with_score(query, k=k, filter=filter, fetch_k=fetch_k,
                                                 **kwargs)
        out = [(doc, fn(score)) for doc, score in docs]
        if score_threshold is not None:
            out = [(d, s) for d, s in out if s >= score_threshold]
        return out

    # -- construction -------------------------------------------------------------------------
    @classmethod
    def __from(cls, texts, embeddings, embedding, metadatas=None, ids=None,
               normalize_L2: bool = False,
               distance_strategy: DistanceStrategy = DistanceStrategy.EUCLIDEAN_DISTANCE,
               **kwargs: Any) -> "FAISS":
        device = kwargs.pop("device", None)
        dim = len(embeddings[0])
        if distance_strategy == DistanceStrategy.MAX_INNER_PRODUCT:
            index = vfaiss.IndexFlatIP(dim, device=device)
        else:
            index = vfaiss.IndexFlatL2(dim, device=device)
        docstore = kwargs.pop("docstore", InMemoryDocstore())
        index_to_docstore_id = kwargs.pop("index_to_docstore_id", {})
        vecstore = cls(embedding, index, docstore, index_to_docstore_id,
                       normalize_L2=normalize_L2, distance_strategy=distance_strategy, **kwargs)
        vecstore.__add(texts, embeddings, metadatas=metadatas, ids=ids)
        return vecstore

    @classmethod
    def from_texts(cls, texts: List[str], embedding, metadatas: Optional[List[dict]] = None,
                   ids: Optional[List[str]] = None, **kwargs: Any) -> "FAISS":
        embeddings = embedding.embed_documents(texts)
        return cls.__from(texts, embeddings, embedding, metadatas=metadatas, ids=ids, **kwargs)

    @classmethod
    def from_embeddings(cls, text_embeddings: Iterable[Tuple[str, List[float]]], embedding,
                        metadatas: Optional[List[dict]] = None, ids: Optional[List[str]] = None,
                        **kwargs: Any) -> "FAISS":
        texts, embeddings = zip(*text_embeddings)
        return cls.__from(list(texts), list(embeddings), embedding, metadatas=metadatas, ids=ids,
                          **kwargs)

    # -- persistence ----------------------------------------------------------------------------
    def save_local(self, folder_path: str, index_name: str = "index") -> None:
        path = Path(folder_path)
        path.mkdir(exist_ok=True, parents=True)
        vfaiss.write_index(self.index, str(path / f"{index_name}.faiss"))
        store = getattr(self.docstore, "_dict", None)
        if store is None:
            raise ValueError("save_local: only InMemoryDocstore-like docstores are supported")
        payload = {
            "format": "vsearch-docstore-v1",
            "index_to_docstore_id": [[int(i), _id] for i, _id in self.index_to_docstore_id.items()],
            "docstore": {k: v.to_json() for k, v in store.items()},
        }
        tmp = path / f"{index_name}.docstore.json.tmp"
        with open(tmp, "w", encoding="utf-8") as f:
            json.dump(payload, f)
        tmp.replace(path / f"{index_name}.docstore.json")

    @classmethod
    def load_local(cls, folder_path: str, embeddings, index_name: str = "index", *,
                   allow_dangerous_deserialization: bool = False, **kwargs: Any) -> "FAISS":
        if not allow_dangerous_deserialization:
            raise ValueError(
                "The de-serialization relies loading a pickle file. Pickle files can be modified "
                "to deliver a malicious payload that results in execution of arbitrary code on "
                "your machine.You will need to set `allow_dangerous_deserialization` to `True` "
                "to enable deserialization. If you do this, make sure that you trust the source "
                "of the data. For example, if you are loading a file that you created, and know "
                "that no one else has modified the file, then this is safe to do. Do not set "
                "this to `True` if you are loading a file from an untrusted source (e.g., some "
                "random site on the internet.)."
            )
        path = Path(folder_path)
        if not (path / f"{index_name}.docstore.json").exists() and \
                (path / f"{index_name}.pkl").exists():
            # a store written by LangChain itself: its docstore is a pickle of
            # LangChain classes, which this loader never unpickles
            raise ReferenceStoreError(
                f"{path}: found {index_name}.pkl (a LangChain pickle) but no "
                f"{index_name}.docstore.json. Migrate it once with "
                "vsearch.langchain.migrate_reference_store (the vectors of "
                f"{index_name}.faiss kept, the docstore rebuilt from the catalog rows in "
                "label order, no re-embedding), or rebuild it with "
                "vsearch.langchain.full_faiss_rebuild (the reference's own book_vector "
                "full_faiss_rebuild, main.py:428-471); the pickle is not loaded.")
        index = vfaiss.read_index(str(path / f"{index_name}.faiss"),
                                  device=kwargs.pop("device", None),
                                  index_factory=kwargs.pop("index_factory", None))
        with open(path / f"{index_name}.docstore.json", "r", encoding="utf-8") as f:
            payload = json.load(f)
        docstore = InMemoryDocstore({k: Document.from_json(v)
                                     for k, v in payload["docstore"].items()})
        index_to_docstore_id = {int(i): _id for i, _id in payload["index_to_docstore_id"]}
        return cls(embeddings, index, docstore, index_to_docstore_id, **kwargs)


class ReferenceStoreError(ValueError):
    """load_local found a LangChain-written store (index.pkl docstore) that this
    drop-in does not unpickle; see full_faiss_rebuild."""


def migrate_reference_store(folder_path: str, texts: List[str], metadatas: List[dict],
                            embeddings=None, ids: Optional[List[str]] = None,
                            index_name: str = "index", *, verify_sample: int = 8,
                            verify_min_cosine: float = 0.999,
                            **kwargs: Any) -> "FAISS":
    """Migrates a store the reference wrote (``index.faiss`` + LangChain's pickled
    ``index.pkl``) WITHOUT re-embedding the catalogue: the vectors are read from
    ``index.faiss`` (faiss's flat format, vsearch.faiss.read_index) onto the GPU,
    and the docstore — which lives only in the pickle, never opened here — is
    rebuilt from the caller's catalogue rows.

    ``texts`` / ``metadatas`` must be the rows in the order the store was built,
    i.e. label order: the reference's full rebuild embeds
    ``SELECT ... FROM catalog`` row by row with the main.py:449-460 text and the
    main.py:461-465 metadata (vsearch.synth.book_text / book_metadata restate
    both) and appends incremental books with ``add_texts`` (main.py:148).  A row
    count that differs from ``index.faiss``'s ntotal is refused.  ``ids``
    default to fresh uuid4 strings, as ``FAISS.from_texts`` assigns them
    (docstore ids are internal to the store: the reference's readers use
    ``metadata["book_id"]``).

    The label order is checked by default: ``verify_sample`` (8) evenly spaced
    texts are embedded with ``embeddings`` and each must point the same way as
    its stored row (cosine >= ``verify_min_cosine``; a remote embedding API is
    not bit-reproducible, so no element-wise comparison), at that many
    embedding calls instead of the whole catalogue.  The reference's rebuild
    query has no ORDER BY (book_vector/main.py:439), so the caller must give
    the rows in the order that query returned them when the store was built;
    a store that ``ensure_store`` seeded (main.py:121: ``from_texts(["dummy"],
    metadatas=[{"book_id": "dummy"}])`` before the first ``add_texts``) holds
    that row at label 0, and it must be passed too.  ``verify_sample=0`` skips
    the check (only when the order is known by construction).
    Writes ``index.docstore.json`` beside the untouched ``index.faiss`` /
    ``index.pkl``; afterwards ``FAISS.load_local`` opens the directory."""
    path = Path(folder_path)
    index = vfaiss.read_index(str(path / f"{index_name}.faiss"),
                              device=kwargs.pop("device", None),
                              index_factory=kwargs.pop("index_factory", None))
    texts = list(texts)
    metadatas = list(metadatas)
    n = int(index.ntotal)
    if len(texts) != n or len(metadatas) != n:
        raise ValueError(f"migrate_reference_store: {index_name}.faiss holds {n} rows but "
                         f"{len(texts)} texts / {len(metadatas)} metadatas were given (the rows "
                         "must be the catalogue in the store's label order)")
    ids = list(ids) if ids is not None else [str(uuid.uuid4()) for _ in texts]
    if len(ids) != n or len(set(ids)) != n:
        raise ValueError("migrate_reference_store: ids must be n distinct strings")
    if verify_sample > 0 and n:
        if embeddings is None:
            raise ValueError("migrate_reference_store: the label-order check needs embeddings "
                             "(or verify_sample=0 when the row order is known)")
        pick = sorted({int(i) for i in np.linspace(0, n - 1, min(verify_sample, n))})
        got = np.asarray(embeddings.embed_documents([texts[i] for i in pick]), dtype=np.float64)
        for j, i in enumerate(pick):
            row = np.asarray(index.reconstruct(i), dtype=np.float64)
            den = float(np.linalg.norm(row) * np.linalg.norm(got[j]))
            cos = float(row @ got[j]) / den if den > 0 else (1.0 if not row.any() and
                                                             not got[j].any() else 0.0)
            if not cos >= verify_min_cosine:
                raise ValueError(f"migrate_reference_store: row {i} of {index_name}.faiss is "
                                 f"not the embedding of texts[{i}] (cosine {cos:.6f} < "
                                 f"{verify_min_cosine}): the rows are not in the store's "
                                 "label order (a store seeded by ensure_store holds its "
                                 "'dummy' row at label 0)")
    docstore = InMemoryDocstore({_id: Document(page_content=t, metadata=m, id=_id)
                                 for t, m, _id in zip(texts, metadatas, ids)})
    store = FAISS(embeddings, index, docstore, dict(enumerate(ids)), **kwargs)
    payload = {
        "format": "vsearch-docstore-v1",
        "index_to_docstore_id": [[i, _id] for i, _id in enumerate(ids)],
        "docstore": {k: v.to_json() for k, v in docstore._dict.items()},
    }
    tmp = path / f"{index_name}.docstore.json.tmp"
    with open(tmp, "w", encoding="utf-8") as f:
        json.dump(payload, f)
    tmp.replace(path / f"{index_name}.docstore.json")
    return store


def full_faiss_rebuild(texts: List[str], embeddings, metadatas: List[dict], folder_path: str,
                       ids: Optional[List[str]] = None, index_name: str = "index",
                       **kwargs: Any) -> "FAISS":
    """The migration path from a reference-written store: the reference's own
    full rebuild (src/incremental_workers/book_vector/main.py:428-471: one
    ``FAISS.from_texts`` over every catalog row with the main.py:449-466 text
    and metadata, then ``save_local(vec_dir)``), writing this drop-in's format
    (index.faiss + index.docstore.json) into the same directory.  Files the
    reference wrote there (index.pkl) are left untouched and no longer read."""
    store = FAISS.from_texts(list(texts), embeddings, metadatas=list(metadatas), ids=ids,
                             **kwargs)
    store.save_local(folder_path, index_name=index_name)
    return store

