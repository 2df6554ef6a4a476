"""Retrieve helpers on the MI355X core (mirror of reference ``retriever/utils.py``).

``get_index`` and ``get_feature_vector`` are the ingest helpers (the reference
duplicates them verbatim, ``retriever/utils.py:23-56``); ``search`` keeps the
reference's contract (``:59-66``): ``ValueError("Input embedding is empty")`` on a
falsy input, otherwise ``index.query(vector, top_k, include_values=True)``
→ ids, best first.  The query itself is the HIP exact cosine scan + top-k.
"""
from __future__ import annotations

from ..ingesting.utils import embed_locally, get_feature_vector, get_index  # noqa: F401


def search(index, input_emb, top_k):
    if input_emb is None or len(input_emb) == 0:
        raise ValueError("Input embedding is empty")
    matching = index.query(vector=input_emb, top_k=top_k, include_values=True)["matches"]
    match_ids = [match_id["id"] for match_id in matching]
    return match_ids
