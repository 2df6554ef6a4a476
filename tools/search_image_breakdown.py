"""Where POST /search_image's time goes (GPU; reference flow retriever/main.py:104-169): p50 of the
whole request through the FastAPI app (TestClient, in process, as bench.py's latency line) and of
each step timed alone on the same fixture JPEG over config 1's 10k x 768 index:

  request           the whole POST through one TestClient session (its event-loop thread kept)
  request_new_portal the same without the session: TestClient starts a thread + event loop per request
  testclient_floor  a POST of the same multipart body to a route that only reads it (one session:
                    TestClient + Starlette + the request/response plumbing every route pays)
  multipart_parse   parse_form of that body
  host_validation   PIL open + convert (the reference's validation decode; the route now skips it
                    when the in-process embed validates, see retriever/main.py)
  embed             embed_bytes (GPU decode + resize + ViT-MSN + 768 floats on the host)
  search            retriever.utils.search(index, feature, top_k=5)
  fetch             index.fetch(ids) of the 5 matches
  urls_json         the 5 URLs from metadata and their JSON encoding

    python tools/search_image_breakdown.py
"""
import importlib
import json
import os
import sys
import time
from io import BytesIO

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

PKG = "end-to-end-image-retrieval-service-with-k8s-jenkins_amd"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def p50(fn, reps=60, warm=5):
    for _ in range(warm):
        fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append((time.perf_counter() - t0) * 1e3)
    t.sort()
    return round(t[len(t) // 2], 4)


def main():
    from fastapi import FastAPI, Request
    from fastapi.testclient import TestClient
    from PIL import Image

    import bench

    emb = importlib.import_module(f"{PKG}.embedding.main")
    ing = importlib.import_module(f"{PKG}.ingesting.utils")
    ret = importlib.import_module(f"{PKG}.retriever.utils")
    retmain = importlib.import_module(f"{PKG}.retriever.main")
    mp = importlib.import_module(f"{PKG}.multipart")
    data = open(os.path.join(REPO, "tests", "golden", "test_image.jpeg"), "rb").read()
    vec = emb.embed_bytes(data)
    X, _ = bench.planted_index_rows(query=vec)
    ix = ing.get_index("breakdown-10k", dimension=768, dtype="float32", capacity=len(X))
    ix.upsert_tensor([f"r{i}" for i in range(len(X))], torch.from_numpy(X).to(torch.cuda.current_device()),
                     [{"gcs_path": f"images/r{i}.jpg"} for i in range(len(X))])
    out = {}
    client = TestClient(retmain.app)
    if "--profile" in sys.argv:  # where the request's host time goes, by function (cProfile)
        import cProfile
        import pstats

        retmain.index = lambda: ix
        client.__enter__()  # one session, as the bench line
        post_ = lambda: client.post("/search_image", files={"file": ("test_image.jpeg", data, "image/jpeg")})  # noqa: E731
        for _ in range(10):
            post_()
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(100):
            post_()
        pr.disable()
        pstats.Stats(pr).sort_stats("cumulative").print_stats(45)
        return
    old_index = retmain.index
    retmain.index = lambda: ix
    try:
        def post(c):
            r = c.post("/search_image", files={"file": ("test_image.jpeg", data, "image/jpeg")})
            assert r.status_code == 200 and len(r.json()) == 5
        with TestClient(retmain.app) as session:
            out["request"] = p50(lambda: post(session))
        out["request_new_portal"] = p50(lambda: post(client))
    finally:
        retmain.index = old_index

    floor_app = FastAPI()
    seen = {}

    @floor_app.post("/echo")
    async def echo(request: Request):
        seen["body"] = await request.body()
        seen["ctype"] = request.headers.get("content-type", "")
        return []

    with TestClient(floor_app) as fc:
        out["testclient_floor"] = p50(lambda: fc.post("/echo", files={"file": ("test_image.jpeg", data, "image/jpeg")}))
    body, ctype = seen["body"], seen["ctype"]
    out["multipart_parse"] = p50(lambda: mp.parse_form(body, ctype))
    out["host_validation"] = p50(lambda: Image.open(BytesIO(data)).convert("RGB"))
    out["embed"] = p50(lambda: emb.embed_bytes(data))
    out["search"] = p50(lambda: ret.search(ix, vec, top_k=5))
    ids = ret.search(ix, vec, top_k=5)
    out["fetch"] = p50(lambda: ix.fetch(ids=ids))
    resp = ix.fetch(ids=ids)

    def urls():
        u = [retmain.storage.signed_url(resp["vectors"][i]["metadata"]["gcs_path"], None) for i in ids]
        return json.dumps(u)
    out["urls_json"] = p50(urls)
    out["sum_of_steps_without_validation"] = round(sum(out[k] for k in ("testclient_floor", "multipart_parse", "embed",
                                                                         "search", "fetch", "urls_json")), 4)
    print(json.dumps({"search_image_breakdown_p50_ms": out}), flush=True)
    ix.close()


if __name__ == "__main__":
    main()
