"""Index snapshot/restore (the reference's Pinecone index is durable
server-side, ingesting/utils.py:23-38; the in-HBM index is saved to disk instead).

Round-trip property: after save → load, query results are bit-identical, fetch
returns the same values and metadata, and upserts continue (overwrite by id, new
ids append)."""
import numpy as np
import pytest

from conftest import import_pkg

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", ["float32", "float16", "bfloat16"])
def test_index_save_load_round_trip(cuda, tmp_path, dtype):
    index = import_pkg("index")
    rng = np.random.default_rng(3)
    n, dim = 3000, 768
    X = rng.standard_normal((n, dim)).astype(np.float32)
    ix = index.Index("images", dimension=dim, dtype=dtype, capacity=4096, device=cuda)
    ix.upsert([(f"id{i}", X[i].tolist(), {"gcs_path": f"gs://b/{i}.jpg", "filename": f"{i}.jpg"}) for i in range(n)])
    Q = rng.standard_normal((3, dim)).astype(np.float32)
    before = [ix.query(vector=q.tolist(), top_k=10, include_metadata=True) for q in Q]
    ix.save(str(tmp_path / "snap"))
    ix2 = index.Index.load(str(tmp_path / "snap"), device=cuda)
    after = [ix2.query(vector=q.tolist(), top_k=10, include_metadata=True) for q in Q]
    assert before == after
    assert ix.fetch(["id5", "id2999"]) == ix2.fetch(["id5", "id2999"])
    assert ix2.describe_index_stats()["total_vector_count"] == n
    # upserts continue: overwrite an id, add a new one
    ix2.upsert([("id5", X[7].tolist(), {"filename": "x"}), ("new", X[9].tolist(), {})])
    m = ix2.query(vector=X[7].tolist(), top_k=2)["matches"]
    assert {mm["id"] for mm in m} == {"id5", "id7"}
    assert len(ix2) == n + 1


def test_sharded_save_load_single_rank(cuda, tmp_path):
    import torch

    sharded = import_pkg("sharded")
    sidx = sharded.ShardedIndex(512, dtype="float16", capacity_per_rank=100_000, device=cuda)
    sidx.fill_random(4, 70_000)
    q = torch.randn(16, 512, device=cuda)
    s1, r1 = sidx.search(q, 20)
    sidx.save(str(tmp_path / "s"))
    sidx2 = sharded.ShardedIndex(512, dtype="float16", capacity_per_rank=100_000, device=cuda)
    sidx2.load(str(tmp_path / "s"))
    s2, r2 = sidx2.search(q, 20)
    assert torch.equal(s1, s2) and torch.equal(r1, r2)
    sidx.close()
    sidx2.close()
