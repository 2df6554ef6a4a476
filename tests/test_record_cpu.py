"""``index.Record``: query matches / fetched vectors whose ``"values"`` list is built on first read.

The reference's ``search`` requests ``include_values=True`` and keeps only the ids
(``retriever/utils.py:62-65``); every way a caller can read the dict must still see the
list of floats a plain Pinecone-shaped dict holds (GPU-free: the rows are numpy arrays)."""
import copy
import json
import pickle

import numpy as np
import pytest

from conftest import import_pkg


def _rec():
    Record = import_pkg("index").Record
    row = np.array([0.5, -1.25, 3.0], np.float32)
    r = Record(row, id="a", score=0.75)
    dict.__setitem__(r, "metadata", {"gcs_path": "images/a.jpg"})
    return r, {"id": "a", "score": 0.75, "values": [0.5, -1.25, 3.0], "metadata": {"gcs_path": "images/a.jpg"}}


@pytest.mark.parametrize("read", [
    lambda r: r["values"],
    lambda r: r.get("values"),
    lambda r: dict(r)["values"],
    lambda r: {**r}["values"],
    lambda r: dict(r.items())["values"],
    lambda r: list(r.values())[2],
    lambda r: r.copy()["values"],
    lambda r: copy.deepcopy(r)["values"],
    lambda r: pickle.loads(pickle.dumps(r))["values"],
    lambda r: json.loads(json.dumps(r))["values"],
])
def test_every_read_path_sees_the_list(read):
    r, _ = _rec()
    v = read(r)
    assert v == [0.5, -1.25, 3.0] and all(type(x) is float for x in v)


def test_record_is_the_plain_dict():
    r, plain = _rec()
    assert list(r.keys()) == ["id", "score", "values", "metadata"] and len(r) == 4 and "values" in r
    assert r["id"] == "a" and r["score"] == 0.75  # other keys read without building the list
    assert r._row is not None
    assert r == plain and plain == r and not (r != plain)
    assert r._row is None and dict.__getitem__(r, "values") == plain["values"]
    r2, _ = _rec()
    assert repr(r2) == repr(plain)
    r3, _ = _rec()
    assert r3.pop("values") == plain["values"] and "values" not in r3


def test_record_without_values_is_a_plain_match():
    Record = import_pkg("index").Record
    r = Record(None, id="b", score=0.5)
    assert r == {"id": "b", "score": 0.5} and "values" not in r


def test_query_vector_rejects_nested_lists():
    """A nested query ([[v0..]]) is refused, as the per-element float() of the old parser did
    (no silent flattening); flat lists, tuples and arrays are accepted."""
    ix = import_pkg("index")
    v = [0.25] * 8
    assert ix._as_vector_np(v, 8).shape == (1, 8)
    assert ix._as_vector_np(tuple(v), 8).shape == (1, 8)
    assert ix._as_vector_np(np.asarray(v), 8).shape == (1, 8)
    for bad in ([v], np.asarray([v])):
        with pytest.raises(TypeError):
            ix._as_vector_np(bad, 8)


def test_f32list_carries_its_row_until_mutated():
    """An in-process embedding (index.F32List) is a plain list of floats for every reader, hands
    its float32 row to the query parser, and any mutation makes the parser read the list again."""
    ix = import_pkg("index")
    row = np.array([0.5, -2.0, 3.25, 1.0], np.float32)
    v = ix.F32List(row.tolist(), row)
    assert v == [0.5, -2.0, 3.25, 1.0] and isinstance(v, list) and json.loads(json.dumps(v)) == v
    assert ix._as_vector_np(v, 4)[0] is not None and np.array_equal(ix._as_vector_np(v, 4)[0], row)
    assert pickle.loads(pickle.dumps(v)) == v and type(pickle.loads(pickle.dumps(v))) is list
    for mutate in (lambda x: x.__setitem__(0, 9.0), lambda x: x.append(1.0), lambda x: x.pop(),
                   lambda x: x.reverse(), lambda x: x.sort(), lambda x: x.extend([1.0]), lambda x: x.insert(0, 7.0)):
        w = ix.F32List(row.tolist(), row)
        mutate(w)
        assert w.f32 is None
        if len(w) == 4:
            assert np.array_equal(ix._as_vector_np(w, 4)[0], np.asarray(w, np.float32))
    w = ix.F32List(row.tolist(), row)
    w += [1.0]
    assert w.f32 is None


def test_record_writes_drop_or_load_the_pending_row():
    """Writing or deleting "values" supersedes the pending row (it must not come back on the next
    read); update / |= / | see the loaded list, as on a plain dict."""
    r, plain = _rec()
    r["values"] = [1.0]
    assert r["values"] == [1.0] and r._row is None
    r, _ = _rec()
    r.update(values=[2.0])
    assert r["values"] == [2.0]
    r, _ = _rec()
    r.update({"score": 0.5})
    assert r["values"] == plain["values"] and r["score"] == 0.5
    r, _ = _rec()
    del r["values"]
    assert "values" not in r and r.get("values") is None and r == {k: v for k, v in plain.items() if k != "values"}
    r, _ = _rec()
    assert (r | {"score": 0.1})["values"] == plain["values"] and type(r | {}) is dict
    assert ({"x": 1} | r)["values"] == plain["values"]
    r, _ = _rec()
    r |= {"values": [3.0]}
    assert r["values"] == [3.0] and isinstance(r, import_pkg("index").Record)
    r, _ = _rec()
    r["metadata"] = {"gcs_path": "b"}
    assert r["values"] == plain["values"]
