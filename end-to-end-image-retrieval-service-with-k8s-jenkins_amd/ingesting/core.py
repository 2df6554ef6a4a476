"""Batched ingest core: N images → validate → GPU decode → ONE batched embed → ONE upsert.

Reference: ``push_image`` (``ingesting/main.py:101-168``) ingests one image per
request — extension check (``:111-115``), validation decode (``:116-119``),
``get_feature_vector`` over HTTP (``:124``), a uuid4 id (``:127-128``), GCS
upload + signed URL (``:130-151``), ``index.upsert([(file_id, feature,
{"gcs_path", "filename"})])`` (``:156-158``) and the 4-key response
(``:163-168``).  ``ingest_many`` keeps every one of those steps and their order
per image, but the arithmetic runs batched on the GPU: baseline JPEGs are
decoded on the device (bit-exact with the reference's PIL decode), every image
is embedded in ``rc_embed`` batches, and the raw CLS vectors go straight from
HBM into one ``Index.upsert_tensor`` call (normalised on the device, as
Pinecone's cosine index normalises server-side).  The result for image i equals
what a single ``/push_image`` of image i returns (modulo the random uuid).

Blob storage (GCS upload / signed URL) is out of scope: it is a hook
(``StorageHook``) whose default does nothing but name the object.  A real
deployment passes an object that uploads and signs.
"""
from __future__ import annotations

import sys
import threading
import uuid
from contextlib import contextmanager
from typing import Callable, Iterable, Iterator, Sequence

from fastapi import HTTPException

from ..config import Config

ALLOWED_EXTENSIONS = {"jpg", "jpeg", "png"}  # ingesting/main.py:112


class StorageHook:
    """No-op stand-in for the reference's GCS bucket (``ingesting/main.py:130-151``)."""

    def __init__(self, bucket: str = Config.GCS_BUCKET_NAME):
        self.bucket = bucket

    def upload(self, gcs_path: str, data: bytes, content_type: str | None) -> None:
        return None

    def signed_url(self, gcs_path: str, filename: str | None) -> str:
        return f"https://storage.googleapis.com/{self.bucket}/{gcs_path}"


def file_extension(filename: str | None) -> str:
    """``file.filename.split(".")[-1].lower()`` (ingesting/main.py:111)."""
    return (filename or "").split(".")[-1].lower()


def validate_extension(filename: str | None) -> str:
    ext = file_extension(filename)
    if ext not in ALLOWED_EXTENSIONS:
        raise HTTPException(status_code=400, detail="Only .jpg/.jpeg/.png allowed")
    return ext


def _prepare(files: Sequence[tuple]):
    """Extension checks, then the validation decode (ingesting/main.py:111-119) of every file:
    (names, blobs, content types, extensions, decoded images).  Raises the reference's 400s."""
    from ..embedding import main as emb

    names, blobs, ctypes_, exts = [], [], [], []
    for f in files:
        filename, data = f[0], f[1]
        exts.append(validate_extension(filename))
        names.append(filename)
        blobs.append(data)
        ctypes_.append(f[2] if len(f) > 2 else None)
    if not blobs:
        return names, blobs, ctypes_, exts, []
    try:  # validation decode (ingesting/main.py:116-119), on the GPU for baseline JPEGs
        images = emb.decode_many(blobs)
    except HTTPException as e:
        if e.status_code == 400:
            raise HTTPException(status_code=400, detail="Invalid image file")
        raise
    return names, blobs, ctypes_, exts, images


def _embed_for(embedder, images, index):
    """The batch's vectors in the form ``Index.upsert_tensor`` takes: one device tensor, or with
    an ``EmbedderPool`` the per-GPU slices.  A GPU-decoded image is embedded on the GPU that
    decoded it (no 150 KB image crosses GPUs); a host-decoded one on the GPU of the shard its
    new row will live on (rows are taken in order from len(index), global row g on shard g % S).
    A vector whose shard is on another GPU is copied there by the index (3 KB, counted in
    ``ShardSet.cross_device_rows``)."""
    import torch

    from ..vit import EmbedderPool

    if isinstance(embedder, EmbedderPool):
        plan = embedder.assign(len(images), base=len(index), shard_devices=getattr(index, "shard_devices", None))
        here = embedder.assign_by_location(images)
        assign = [h if isinstance(im, torch.Tensor) and im.is_cuda else p for im, h, p in zip(images, here, plan)]
        return [(pos, r) for pos, r, _ in embedder.embed_parts(images, normalized=False, assign=assign)]
    raw, _ = embedder.embed_images(images)
    return raw


def _finish(prep, index, storage: StorageHook, id_factory: Callable[[], str]) -> list[dict]:
    """Embed the decoded batch, then ids, storage hook and ONE upsert (ingesting/main.py:124-168)."""
    from ..embedding import main as emb

    names, blobs, ctypes_, exts, images = prep
    if not blobs:
        return []
    index = index() if callable(index) else index
    vecs = _embed_for(emb.get_embedder(), images, index)
    ids = [id_factory() for _ in blobs]
    paths = [f"images/{fid}.{ext}" for fid, ext in zip(ids, exts)]
    urls = []
    for p, data, ct, name in zip(paths, blobs, ctypes_, names):
        storage.upload(p, data, ct)
        urls.append(storage.signed_url(p, name))
    index.upsert_tensor(ids, vecs, [{"gcs_path": p, "filename": n} for p, n in zip(paths, names)])
    return [{"message": "Successfully!", "file_id": fid, "gcs_path": p, "signed_url": u}
            for fid, p, u in zip(ids, paths, urls)]


def ingest_many(files: Sequence[tuple], index, storage: StorageHook | None = None,
                id_factory: Callable[[], str] | None = None) -> list[dict]:
    """files: ``(filename, bytes[, content_type])`` per image → one response dict per image.

    Every image is validated before anything is embedded or stored (a bad file
    fails the whole call with the reference's 400, and nothing is ingested).
    ``index`` may be a zero-argument callable (opened only once the batch is valid)."""
    return _finish(_prepare(files), index, storage or StorageHook(), id_factory or (lambda: str(uuid.uuid4())))


def ingest_stream(batches: Iterable[Sequence[tuple]], index, storage: StorageHook | None = None,
                  id_factory: Callable[[], str] | None = None) -> Iterator[list[dict]]:
    """Bulk ingest: ``ingest_many`` over a stream of upload batches, pipelined.  Batch i+1 is
    validated and decoded (host Huffman on a worker thread, GPU reconstruction on a side
    stream) while the GPU embeds batch i and the host upserts it; yields each batch's
    responses in order, exactly what ``ingest_many`` returns for it.  A batch that fails
    validation raises its 400 when it is reached (the batches before it are ingested, the
    ones after it are not)."""
    import torch

    from ..embedding import main as emb

    storage = storage or StorageHook()
    id_factory = id_factory or (lambda: str(uuid.uuid4()))
    dev = emb.get_embedder().device
    side = torch.cuda.Stream(device=dev)
    main = torch.cuda.current_stream(dev)

    def prepare(files):
        with torch.cuda.device(dev), torch.cuda.stream(side):
            prep = _prepare(files)
            ev = torch.cuda.Event()
            ev.record(side)
        return prep, ev

    it = iter(batches)
    with _short_gil_switch():
        yield from _pipeline(it, prepare, main, index, storage, id_factory)


_switch_lock = threading.Lock()
_switch_users = 0
_switch_saved = None


@contextmanager
def _short_gil_switch():
    """GIL switch interval <= 1 ms while any ingest stream runs.  Both pipeline threads hold
    the GIL for short Python stretches between ctypes calls (which release it); at the
    default 5 ms each hand-off can stall the other thread that long (tools/ingest_probe.py:
    17.1k images/s at 5 ms, 18.4k at 1 ms).  Process-wide setting, so it is reference-
    counted: the first stream lowers it, the last one to finish (or be closed / collected)
    restores the value it found."""
    global _switch_users, _switch_saved
    with _switch_lock:
        if _switch_users == 0:
            _switch_saved = sys.getswitchinterval()
            sys.setswitchinterval(min(_switch_saved, 1e-3))
        _switch_users += 1
    try:
        yield
    finally:
        with _switch_lock:
            _switch_users -= 1
            if _switch_users == 0:
                sys.setswitchinterval(_switch_saved)


def _pipeline(it, prepare, main, index, storage, id_factory):
    """ingest_stream's loop: the worker prepares batch i+1 while this thread finishes batch i."""
    import concurrent.futures as cf

    import torch

    opened = None
    with cf.ThreadPoolExecutor(1) as ex:
        first = next(it, None)
        fut = ex.submit(prepare, first) if first is not None else None
        while fut is not None:
            prep, ev = fut.result()
            nxt = next(it, None)
            fut = ex.submit(prepare, nxt) if nxt is not None else None
            main.wait_event(ev)
            for im in prep[4]:
                if isinstance(im, torch.Tensor) and im.is_cuda:
                    im.record_stream(main)
            if opened is None:
                opened = index() if callable(index) else index
            yield _finish(prep, opened, storage, id_factory)


def push_one(filename: str, data: bytes, index, content_type: str | None = None, storage: StorageHook | None = None,
             feature_fn: Callable[[bytes], list] | None = None, id_factory: Callable[[], str] | None = None) -> dict:
    """The single-image ``/push_image`` flow (ingesting/main.py:101-168), step for step:
    ext check → validation decode → feature vector (``feature_fn``, default the in-process
    embed; the reference POSTs to /embed) → uuid → storage hook → ``index.upsert``.
    ``index`` may be a zero-argument callable (opened only once the image is valid)."""
    from io import BytesIO

    from PIL import Image, UnidentifiedImageError

    ext = validate_extension(filename)
    try:
        Image.open(BytesIO(data)).convert("RGB")
    except UnidentifiedImageError:
        raise HTTPException(status_code=400, detail="Invalid image file")
    if feature_fn is None:
        from ..embedding.main import embed_bytes as feature_fn
    feature = feature_fn(data)
    file_id = (id_factory or (lambda: str(uuid.uuid4())))()
    gcs_path = f"images/{file_id}.{ext}"
    storage = storage or StorageHook()
    storage.upload(gcs_path, data, content_type)
    signed_url = storage.signed_url(gcs_path, filename)
    index = index() if callable(index) else index
    index.upsert([(file_id, feature, {"gcs_path": gcs_path, "filename": filename})])
    return {"message": "Successfully!", "file_id": file_id, "gcs_path": gcs_path, "signed_url": signed_url}
