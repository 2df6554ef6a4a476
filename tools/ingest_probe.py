"""Where the time of the batched ingest core goes (GPU): _prepare (validation + decode),
embed, ids/storage/upsert/responses, per batch of 256 JPEG uploads; then ingest_stream
at a few GIL switch intervals.

    python tools/ingest_probe.py
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from bench import synthetic_jpegs  # noqa: E402
from conftest import import_pkg  # noqa: E402


def main():
    core = import_pkg("ingesting.core")
    emb = import_pkg("embedding.main")
    index = import_pkg("index")
    import_pkg("config").Config.EMBED_MAX_BATCH = 256
    datas = synthetic_jpegs(256, 11)
    files = [(f"img{i}.jpg", d, "image/jpeg") for i, d in enumerate(datas)]
    ix = index.Index("probe", dimension=768, dtype="float16", capacity=256 * 40, device=0)
    if os.environ.get("PROBE_BENCH_MODEL"):  # the bench's own model + a JPEG stream first, as bench.py does
        vit = import_pkg("vit")
        bm = vit.VitMsnEmbedder(vit.random_state_dict(seed=0), device=0, max_batch=256)
        for _ in bm.embed_jpeg_stream([datas] * 4):
            pass
        torch.cuda.synchronize()
    core.ingest_many(files, ix)
    torch.cuda.synchronize()
    t = {"prepare": 0.0, "embed": 0.0, "finish_host": 0.0}
    reps = 4
    for _ in range(reps):
        t0 = time.perf_counter()
        prep = core._prepare(files)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        raw, _ = emb.get_embedder().embed_images(prep[4])
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        core._finish(prep, ix, core.StorageHook(), lambda: os.urandom(16).hex())
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        t["prepare"] += t1 - t0
        t["embed"] += t2 - t1
        t["finish_host"] += t3 - t2 - (t2 - t1)  # _finish embeds again
    print({k: round(v / reps * 1e3, 2) for k, v in t.items()}, "ms per batch of 256", flush=True)
    for sw in (0.005, 0.001, 0.0002):
        sys.setswitchinterval(sw)
        t0 = time.perf_counter()
        n = sum(len(r) for r in core.ingest_stream([files] * 8, ix))
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(f"ingest_stream switchinterval={sw}: {n / el:.0f} images/s", flush=True)
    sys.setswitchinterval(0.005)
    t0 = time.perf_counter()
    for _ in range(8):
        core.ingest_many(files, ix)
    torch.cuda.synchronize()
    print(f"ingest_many: {256 * 8 / (time.perf_counter() - t0):.0f} images/s", flush=True)


if __name__ == "__main__":
    main()
