"""Oracle (test infrastructure): exact cosine top-k standing in for Pinecone ``query``.

Reference call sites: ``retriever/utils.py:59-66`` (``search`` →
``index.query(vector, top_k, include_values=True)["matches"]`` → ids best
first) over an index created with ``metric="cosine"`` (``ingesting/utils.py:29-36``);
upsert at ``ingesting/main.py:156-158``.  Pinecone (``pinecone==5.4.0`` SDK,
remote closed server) is not available, so the published semantics are
restated: score = (q/‖q‖)·(x/‖x‖), matches ordered by score descending; the
build fixes the tie rule as score desc, then row asc.

``cosine_topk`` scores in float64 on the rows it is given (for a quantised
index, pass the stored rows fetched back from the device, so the oracle runs
on the same quantised values).  ``cosine_topk_f32`` is the plain numpy fp32
path (normalise, ``X @ q``, ``argpartition``) used as the timed CPU baseline.
"""
from __future__ import annotations

import numpy as np


def normalize_rows(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.float64)
    n = np.linalg.norm(x, axis=-1, keepdims=True)
    return x / n


def _select(scores: np.ndarray, k: int):
    n = scores.shape[0]
    k = min(k, n)
    if k == 0:
        return np.zeros(0, np.int64), np.zeros(0, scores.dtype)
    if k < n:
        kth = np.partition(scores, n - k)[n - k]
        cand = np.nonzero(scores >= kth)[0]
    else:
        cand = np.arange(n)
    order = np.lexsort((cand, -scores[cand]))[:k]  # score desc, then row asc
    rows = cand[order]
    return rows.astype(np.int64), scores[rows]


def cosine_topk(rows: np.ndarray, queries: np.ndarray, k: int, rows_normalized: bool = False):
    """Exact cosine top-k in float64. Returns (rows [Q,k] int64, scores [Q,k] float64)."""
    X = np.asarray(rows, dtype=np.float64)
    if not rows_normalized:
        X = normalize_rows(X)
    Qn = normalize_rows(np.atleast_2d(queries))
    S = Qn @ X.T
    out_r, out_s = [], []
    for q in range(S.shape[0]):
        r, s = _select(S[q], k)
        out_r.append(r)
        out_s.append(s)
    return np.stack(out_r), np.stack(out_s)


def cosine_topk_f32(rows_normalized_f32: np.ndarray, query: np.ndarray, k: int):
    """The CPU baseline path: fp32 normalise-query, X @ q, argpartition, stable sort."""
    q = np.asarray(query, dtype=np.float32)
    q = q / np.linalg.norm(q)
    s = rows_normalized_f32 @ q
    return _select(s, k)


def topk_equal_modulo_ties(got_rows, got_scores, ref_rows, ref_scores, tol: float = 1e-5) -> bool:
    """North-star rule: identical top-k sets except for ties within ``tol`` score.

    Rows present in one list but not the other must have scores within ``tol``
    of the k-th (boundary) score of the reference.
    """
    got_rows = list(np.asarray(got_rows).tolist())
    ref_rows = list(np.asarray(ref_rows).tolist())
    if len(got_rows) != len(ref_rows):
        return False
    if set(got_rows) == set(ref_rows):
        return True
    kth = float(np.asarray(ref_scores)[-1])
    gs = dict(zip(got_rows, np.asarray(got_scores).tolist()))
    rs = dict(zip(ref_rows, np.asarray(ref_scores).tolist()))
    for r in set(got_rows) ^ set(ref_rows):
        s = gs.get(r, rs.get(r))
        if abs(s - kth) > tol:
            return False
    return True


def planted_index(query: np.ndarray, rows=10_000, dim=768, seed=0):
    """Seeded N(0,1) rows + 5 planted near-duplicates of the query at known rows."""
    rng = np.random.Generator(np.random.PCG64(seed))
    X = rng.standard_normal((rows, dim), dtype=np.float32)
    planted = [17, 4242, 9999, 123, 5000]
    for j, r in enumerate(planted):
        X[r] = query + np.float32(0.02 * (j + 1)) * rng.standard_normal(dim, dtype=np.float32) * np.abs(query).mean()
    return X, planted
