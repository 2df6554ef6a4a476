"""ViT-MSN image embedder on the HIP library (replaces ``extractor`` + ``model``).

Reference: ``embedding/main.py:33-39`` builds ``ViTImageProcessor`` and
``ViTMSNModel`` singletons; ``:97-114`` decodes with PIL, preprocesses, runs the
model under ``no_grad`` and returns ``last_hidden_state[:, 0, :]``.  Here the
decode stays on the host (PIL), the u8 HWC pixels go to HBM once, and
``rc_embed`` does resize → rescale/normalize → patch embed → 12 layers → final
LayerNorm of the CLS row on the GPU, returning the raw CLS vector (the /embed
body) and its L2-normalised copy (what the index stores).
"""
from __future__ import annotations

import json
import os
from typing import Iterable, Mapping, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_ptr
from .config import VIT_MSN_BASE, VIT_MSN_PREPROCESS

TIMER_IDS = {"gemm": 0, "fc1": 1, "attention": 2, "layernorm": 3, "preprocess": 4, "qkv": 5, "oproj": 6, "fc2": 7}


def _to_f32_numpy(t) -> np.ndarray:
    if isinstance(t, torch.Tensor):
        return t.detach().to("cpu", torch.float32).contiguous().numpy()
    return np.ascontiguousarray(np.asarray(t, dtype=np.float32))


def load_checkpoint_dir(path: str) -> tuple[dict, dict, dict]:
    """(state_dict, model_config, preprocess) from a local HF-style checkpoint directory.

    Loads only with loaders that execute nothing from the file: safetensors, or
    ``torch.load(weights_only=True)``.
    """
    cfg = dict(VIT_MSN_BASE)
    pre = dict(VIT_MSN_PREPROCESS)
    cj = os.path.join(path, "config.json")
    if os.path.exists(cj):
        with open(cj) as f:
            c = json.load(f)
        for k in cfg:
            if k in c:
                cfg[k] = c[k]
    pj = os.path.join(path, "preprocessor_config.json")
    if os.path.exists(pj):
        with open(pj) as f:
            p = json.load(f)
        if "resample" in p:
            pre["resample"] = int(p["resample"])
        if "rescale_factor" in p:
            pre["rescale_factor"] = float(p["rescale_factor"])
        if "image_mean" in p:
            pre["image_mean"] = tuple(p["image_mean"])
        if "image_std" in p:
            pre["image_std"] = tuple(p["image_std"])
        if isinstance(p.get("size"), dict) and "height" in p["size"]:
            pre["size"] = (p["size"]["height"], p["size"]["width"])
    st = os.path.join(path, "model.safetensors")
    if os.path.exists(st):
        from safetensors.numpy import load_file

        sd = load_file(st)
    else:
        sd = torch.load(os.path.join(path, "pytorch_model.bin"), map_location="cpu", weights_only=True)
    return dict(sd), cfg, pre


# transformers-5 module names → the checkpoint (legacy) layout rc_model_set_weight keys on
# (TR/conversion_mapping.py maps ViTMSNModel to the ViTModel rules); the same table as
# canonical_name() in csrc/vit.hip
_V5_RENAMES = (
    ("attention.q_proj", "attention.attention.query"), ("attention.k_proj", "attention.attention.key"),
    ("attention.v_proj", "attention.attention.value"), ("attention.o_proj", "attention.output.dense"),
    ("mlp.fc1", "intermediate.dense"), ("mlp.fc2", "output.dense"),
)
# checkpoint entries that are not part of the embedding model (ViTMSNForImageClassification's
# head, the masked-pretraining token)
_IGNORED_KEYS = ("classifier.", "vit.classifier.")
_IGNORED_SUFFIXES = ("mask_token",)


def canonical_key(name: str) -> str:
    n = name[4:] if name.startswith("vit.") else name
    if n.startswith("layers."):
        n = "encoder.layer." + n[len("layers."):]
    for a, b in _V5_RENAMES:
        if a in n:
            n = n.replace(a, b, 1)
            break
    return n


def expected_keys(num_layers: int) -> set[str]:
    """Every tensor ViTMSNModel's state dict holds (legacy layout, embedding/main.py:37-38)."""
    keys = {"embeddings.cls_token", "embeddings.position_embeddings", "embeddings.patch_embeddings.projection.weight",
            "embeddings.patch_embeddings.projection.bias", "layernorm.weight", "layernorm.bias"}
    for i in range(num_layers):
        p = f"encoder.layer.{i}."
        for nm in ("query", "key", "value"):
            keys |= {p + f"attention.attention.{nm}.weight", p + f"attention.attention.{nm}.bias"}
        for nm in ("attention.output.dense", "intermediate.dense", "output.dense"):
            keys |= {p + nm + ".weight", p + nm + ".bias"}
        for nm in ("layernorm_before", "layernorm_after"):
            keys |= {p + nm + ".weight", p + nm + ".bias"}
    return keys


def canonical_state_dict(state_dict: Mapping, num_layers: int | None = None) -> dict:
    """A checkpoint's tensors under the legacy key layout: accepts the legacy names, the
    transformers-5 names (``layers.N.attention.q_proj`` …) and a ``vit.`` prefix; drops the
    classifier head and mask token; raises ValueError on any other unknown key, on a
    missing key and on a key that two names map to."""
    out: dict = {}
    for name, t in state_dict.items():
        if name.startswith(_IGNORED_KEYS) or name.endswith(_IGNORED_SUFFIXES):
            continue
        k = canonical_key(name)
        if k in out:
            raise ValueError(f"checkpoint holds {k!r} twice (as {name!r} and another name)")
        out[k] = t
    if num_layers is None:
        num_layers = sum(1 for k in out if k.endswith("layernorm_before.weight"))
    want = expected_keys(num_layers)
    unknown = sorted(set(out) - want)
    missing = sorted(want - set(out))
    if unknown:
        raise ValueError(f"unknown checkpoint keys (not a ViT-MSN state dict?): {unknown[:8]}"
                         + (" …" if len(unknown) > 8 else ""))
    if missing:
        raise ValueError(f"checkpoint is missing {len(missing)} tensors, e.g. {missing[:8]}")
    return out


def _packed_view(ims: Sequence, device) -> "torch.Tensor | None":
    """[n, H, W, 3] view when ``ims`` are equal-size contiguous u8 device tensors lying back to
    back in one buffer (what JpegDecoder.decode returns for a chunk), else None."""
    first = ims[0]
    if not (isinstance(first, torch.Tensor) and first.is_cuda and first.device == torch.device(device)
            and first.dtype == torch.uint8 and first.is_contiguous()):
        return None
    n, z = len(ims), first.numel()
    base = first.data_ptr()
    for k, im in enumerate(ims):
        if not (isinstance(im, torch.Tensor) and im.shape == first.shape and im.is_cuda
                and im.data_ptr() == base + k * z and im.is_contiguous()
                and im.untyped_storage().data_ptr() == first.untyped_storage().data_ptr()):
            return None
    return first.as_strided((n,) + tuple(first.shape), (z,) + tuple(first.stride()))


class VitMsnEmbedder:
    """One ``rc_model`` on one GPU: fixed weights, workspace for ``max_batch`` images."""

    def __init__(self, state_dict: Mapping, device=None, max_batch: int = 32, model_config: dict | None = None,
                 preprocess: dict | None = None):
        self.lib = _lib.load()
        cfg = dict(VIT_MSN_BASE)
        cfg.update(model_config or {})
        if model_config is None:
            cfg["num_hidden_layers"] = sum(1 for k in state_dict if k.endswith("layernorm_before.weight"))
        state_dict = canonical_state_dict(state_dict, cfg["num_hidden_layers"])  # key errors before any GPU work
        self.config = cfg
        self.preprocess_params = dict(VIT_MSN_PREPROCESS)
        self.preprocess_params.update(preprocess or {})
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device if isinstance(device, int) else torch.device(device).index or 0)
        self.max_batch = int(max_batch)
        self.hidden = cfg["hidden_size"]
        self._jpeg = None  # GPU JPEG decoder, created on first embed_jpeg
        c = _lib.VitConfig(cfg["image_size"], cfg["patch_size"], cfg["hidden_size"], cfg["num_hidden_layers"],
                           cfg["num_attention_heads"], cfg["intermediate_size"], float(cfg["layer_norm_eps"]),
                           self.max_batch)
        h = _lib.C.c_void_p()
        check(self.lib.rc_model_create(self.device.index, _lib.C.byref(c), _lib.C.byref(h)))
        self._h = h
        try:
            for name, t in state_dict.items():
                a = _to_f32_numpy(t)
                check(self.lib.rc_model_set_weight(self._h, name.encode(), a.ctypes.data, a.size))
            p = self.preprocess_params
            mean = (_lib.C.c_float * 3)(*p["image_mean"])
            std = (_lib.C.c_float * 3)(*p["image_std"])
            check(self.lib.rc_model_set_preprocess(self._h, int(p["resample"]), float(p["rescale_factor"]), mean, std))
            check(self.lib.rc_model_finalize(self._h))
        except Exception:
            self.close()
            raise

    @classmethod
    def from_pretrained(cls, path: str, device=None, max_batch: int = 32) -> "VitMsnEmbedder":
        sd, cfg, pre = load_checkpoint_dir(path)
        return cls(sd, device=device, max_batch=max_batch, model_config=cfg, preprocess=pre)

    def close(self) -> None:
        if getattr(self, "_jpeg", None) is not None:
            self._jpeg.close()
            self._jpeg = None
        if getattr(self, "_h", None) is not None:
            check(self.lib.rc_model_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ compute --
    def _images(self, images_u8: torch.Tensor) -> torch.Tensor:
        if images_u8.dtype != torch.uint8 or images_u8.dim() != 4 or images_u8.shape[-1] != 3:
            raise ValueError("images must be uint8 [n, h, w, 3] (HWC RGB)")
        if images_u8.shape[0] > self.max_batch:
            raise ValueError(f"batch {images_u8.shape[0]} exceeds max_batch {self.max_batch}")
        return images_u8.to(self.device).contiguous()

    def embed(self, images_u8: torch.Tensor, normalized: bool = True, stream=None, out=None):
        """u8 [n,h,w,3] (any equal h,w) → (raw [n,H], normed [n,H] or None) f32 on the device."""
        x = self._images(images_u8)
        n, h, w = x.shape[:3]
        if out is None:
            raw = torch.empty((n, self.hidden), dtype=torch.float32, device=self.device)
            nrm = torch.empty((n, self.hidden), dtype=torch.float32, device=self.device) if normalized else None
        else:
            raw, nrm = out
        check(self.lib.rc_embed(self._h, ptr(x), n, h, w, ptr(raw), ptr(nrm), stream_ptr(stream)))
        return raw, nrm

    def preprocess(self, images_u8: torch.Tensor, stream=None) -> torch.Tensor:
        """u8 [n,h,w,3] → f32 pixel_values [n,3,S,S], exactly as ViTImageProcessor (parity hook)."""
        x = self._images(images_u8)
        n, h, w = x.shape[:3]
        S = self.config["image_size"]
        out = torch.empty((n, 3, S, S), dtype=torch.float32, device=self.device)
        check(self.lib.rc_preprocess(self._h, ptr(x), n, h, w, ptr(out), stream_ptr(stream)))
        return out

    def embed_images(self, images: Sequence, normalized: bool = False, out=None):
        """u8 HWC RGB images of any sizes (device tensors or host arrays) → (raw [n,H], normed [n,H]
        or None) f32 device tensors in input order; equal-size images share ``rc_embed`` batches.
        ``out``: caller-owned (raw, normed or None) — device tensors, or for a single image pinned
        host tensors the kernels write straight into (no D2H copy; the caller synchronises)."""
        n = len(images)
        if out is not None:
            raw, nrm = out
        else:
            raw = torch.empty((n, self.hidden), dtype=torch.float32, device=self.device)
            nrm = torch.empty((n, self.hidden), dtype=torch.float32, device=self.device) if normalized else None
        groups: dict[tuple[int, int], list[int]] = {}
        for i, im in enumerate(images):
            groups.setdefault((int(im.shape[0]), int(im.shape[1])), []).append(i)
        for idx in groups.values():
            for s0 in range(0, len(idx), self.max_batch):
                chunk = idx[s0:s0 + self.max_batch]
                x = _packed_view([images[i] for i in chunk], self.device)
                if x is not None:  # consecutive views of one decode buffer: no stack copy
                    pass
                elif all(isinstance(images[i], torch.Tensor) for i in chunk):
                    x = torch.stack([images[i].to(self.device) for i in chunk])
                elif not any(isinstance(images[i], torch.Tensor) for i in chunk):
                    x = torch.from_numpy(np.stack([np.asarray(images[i], dtype=np.uint8) for i in chunk]))
                else:  # GPU-decoded and host-decoded images of one size
                    x = torch.stack([torch.as_tensor(np.asarray(images[i], dtype=np.uint8)).to(self.device)
                                     if not isinstance(images[i], torch.Tensor) else images[i].to(self.device)
                                     for i in chunk])
                c0 = chunk[0]
                if chunk == list(range(c0, c0 + len(chunk))):  # in input order: embedded into its rows
                    sl = slice(c0, c0 + len(chunk))
                    self.embed(x, normalized=normalized, out=(raw[sl], nrm[sl] if normalized else None))
                    continue
                r, m = self.embed(x, normalized=normalized)
                sel = torch.tensor(chunk, dtype=torch.int64).pin_memory().to(self.device, non_blocking=True)
                raw.index_copy_(0, sel, r)
                if normalized:
                    nrm.index_copy_(0, sel, m)
        return raw, nrm

    def embed_pil(self, images: Sequence) -> list[list[float]]:
        """Host PIL RGB images (any sizes) → raw CLS vectors as Python lists (the /embed body)."""
        raw, _ = self.embed_images([np.asarray(im.convert("RGB"), dtype=np.uint8) for im in images])
        return raw.cpu().tolist()

    def _decoder(self):
        from .jpeg import JpegDecoder

        if self._jpeg is None:
            self._jpeg = JpegDecoder(self.device, max_images=max(self.max_batch, 32), max_pixels=1 << 24)
        return self._jpeg

    def decode_jpeg(self, datas: Sequence[bytes]) -> list[torch.Tensor]:
        """Baseline-JPEG byte strings → device HWC RGB u8 images at their own size (rc_jpeg_decode,
        bit-exact with the reference's PIL decode).  Raises jpeg.JpegUnsupported / ValueError."""
        return self._decoder().decode(datas)

    def decode_jpeg_for_embed(self, datas: Sequence[bytes]) -> torch.Tensor:
        """Baseline-JPEG byte strings (any sizes) → device u8 [n, S, S, 3], the model's input:
        decode fused with the processor's resize (rc_jpeg_decode_resized, bit-exact with PIL
        decode + Image.resize); rc_embed then runs no resize."""
        S = self.config["image_size"]
        return self._decoder().decode_resized(datas, S, int(self.preprocess_params["resample"]))

    def embed_jpeg(self, datas: Sequence[bytes]) -> list[list[float]]:
        """Baseline-JPEG byte strings → raw CLS vectors, decoded (and resized) on the GPU and
        embedded without a host RGB copy.  Raises jpeg.JpegUnsupported for streams the GPU
        decoder does not handle."""
        raw, _ = self.embed_images(list(self.decode_jpeg_for_embed(datas).unbind(0)))
        return raw.cpu().tolist()

    def embed_jpeg_stream(self, batches: Iterable[Sequence[bytes]], normalized: bool = True):
        """Pipelined JPEG bytes → embeddings for a stream of batches (bulk ingest; images of any
        sizes): batch i+1 is Huffman-decoded on a host worker thread and reconstructed +
        resized on a side stream (rc_jpeg_decode_resized) while the GPU embeds batch i.
        Yields (raw, normed) device tensors per batch (valid until the next iteration)."""
        import concurrent.futures as cf

        dec = self._decoder()
        S, resample = self.config["image_size"], int(self.preprocess_params["resample"])
        side = torch.cuda.Stream(device=self.device)
        main = torch.cuda.current_stream(self.device)

        def decode(datas):
            with torch.cuda.device(self.device), torch.cuda.stream(side):
                x = dec.decode_resized(datas, S, resample, stream=side)
                ev = torch.cuda.Event()
                ev.record(side)
            return x, ev

        it = iter(batches)
        with cf.ThreadPoolExecutor(1) as ex:
            first = next(it, None)
            fut = ex.submit(decode, first) if first is not None else None
            while fut is not None:
                x, ev = fut.result()
                nxt = next(it, None)
                fut = ex.submit(decode, nxt) if nxt is not None else None
                main.wait_event(ev)
                x.record_stream(main)
                yield self.embed(x, normalized=normalized)

    # ------------------------------------------------------------- timing --
    def timing(self, enable: bool | Iterable[str]) -> None:
        """Enable event timing for all kernels (True), none (False) or the named ones."""
        if isinstance(enable, bool):
            mask = -1 if enable else 0
        else:
            mask = 0
            for k in enable:
                mask |= 1 << TIMER_IDS[k]
        check(self.lib.rc_model_timing(self._h, mask))

    def set_parts(self, parts: int) -> None:
        """Encode batches as ``parts`` concurrent slices on separate streams (1 = one stream)."""
        check(self.lib.rc_model_set_parts(self._h, int(parts)))

    def set_ln_fold(self, on: bool) -> None:
        """Fold the LayerNorms into the GEMMs around them (default) or run the LN kernel."""
        check(self.lib.rc_model_set_ln_fold(self._h, int(bool(on))))

    def set_last_layer(self, cls_only: bool) -> None:
        """Run the last encoder layer on the CLS rows only (default) or on every row."""
        check(self.lib.rc_model_set_last_layer(self._h, int(bool(cls_only))))

    def set_graphs(self, on: bool) -> None:
        """Replay a one-image embed's launch chain as a captured HIP graph (default) or launch
        every kernel from the host (the same bits)."""
        check(self.lib.rc_model_set_graphs(self._h, int(bool(on))))

    def set_gemm_variant(self, variant: int) -> None:
        """Diagnostic builds only (tools/build_diag.sh, RC_LIB_PATH): the A/B kernel of the
        full-batch projections (0 auto, 4 ping-pong, 8 two-workgroup, 10 image-aligned, 100 + ABL).
        The product library picks one kernel per shape and has no such knob."""
        fn = getattr(self.lib, "rc_diag_set_gemm_variant", None)
        if fn is None:
            raise RuntimeError("GEMM variants are a diagnostic-build knob (tools/build_diag.sh)")
        check(fn(self._h, int(variant)))

    def timing_reset(self) -> None:
        check(self.lib.rc_model_timing_reset(self._h))

    def timing_read(self, kernel: str):
        ms = _lib.C.c_double()
        n = _lib.C.c_int64()
        w = _lib.C.c_double()
        check(self.lib.rc_model_timing_read(self._h, TIMER_IDS[kernel], _lib.C.byref(ms), _lib.C.byref(n), _lib.C.byref(w)))
        return ms.value, n.value, w.value


class EmbedderPool:
    """Data-parallel embedding over several GPUs in one process: one ``VitMsnEmbedder``
    (``rc_model``) per device, weights replicated, no collectives (image
    embedding is plain data parallel).  The reference scales its embedding pod by
    replicas behind one Service (``helm_charts/embedding/values.yaml:1``); here a
    batch is split over the pool's GPUs, which run their ``rc_embed`` calls concurrently
    (each call returns once its kernels are queued).

    ``embed_images`` returns the vectors gathered on the first device (the /embed body);
    ``embed_parts`` leaves each slice on the GPU that embedded it, so an ingest can hand
    the slices straight to the index shards on those GPUs (``Index.upsert_tensor`` with
    parts).  Devices may repeat (two models on one GPU: the parity test)."""

    def __init__(self, state_dict: Mapping, devices: Sequence, max_batch: int = 32, model_config: dict | None = None,
                 preprocess: dict | None = None):
        if not devices:
            raise ValueError("an embedder pool needs at least one device")
        self.members: list[VitMsnEmbedder] = []
        try:
            for d in devices:
                self.members.append(VitMsnEmbedder(state_dict, device=d, max_batch=max_batch,
                                                   model_config=model_config, preprocess=preprocess))
        except Exception:
            self.close()
            raise
        lead = self.members[0]
        self.device, self.hidden, self.max_batch, self.config = lead.device, lead.hidden, lead.max_batch, lead.config
        self.preprocess_params = lead.preprocess_params

    @classmethod
    def from_pretrained(cls, path: str, devices: Sequence, max_batch: int = 32) -> "EmbedderPool":
        sd, cfg, pre = load_checkpoint_dir(path)
        return cls(sd, devices, max_batch=max_batch, model_config=cfg, preprocess=pre)

    @property
    def devices(self) -> list[int]:
        return [m.device.index for m in self.members]

    def close(self) -> None:
        for m in getattr(self, "members", []):
            m.close()

    def assign(self, n: int, base: int = 0, shard_devices: Sequence[int] | None = None) -> list[int]:
        """Member of each of n images.  With ``shard_devices`` (an index's shard GPUs, global row
        g on shard g % S) image j, which will take row base + j, goes to a member on the GPU of
        its shard, so its vector never leaves that GPU; otherwise round-robin."""
        D = len(self.members)
        if not shard_devices:
            return [(base + j) % D for j in range(n)]
        if [int(d) for d in shard_devices] == self.devices:  # one member per shard, same GPUs
            return [(base + j) % D for j in range(n)]
        by_dev: dict[int, list[int]] = {}
        for i, m in enumerate(self.members):
            by_dev.setdefault(m.device.index, []).append(i)
        S = len(shard_devices)
        seen: dict[int, int] = {}
        out = []
        for j in range(n):
            s = (base + j) % S
            cands = by_dev.get(int(shard_devices[s]))
            if cands:  # several members on this GPU: take turns
                k = seen.get(s, 0)
                seen[s] = k + 1
                out.append(cands[k % len(cands)])
            else:
                out.append((base + j) % D)
        return out

    def assign_by_location(self, images: Sequence) -> list[int]:
        """Member of each image: a device tensor goes to a member on the GPU it lives on (several
        members there take turns), anything else round-robin — so a GPU-decoded image is embedded
        where it was decoded and never crosses GPUs."""
        by_dev: dict[int, list[int]] = {}
        for i, m in enumerate(self.members):
            by_dev.setdefault(m.device.index, []).append(i)
        D = len(self.members)
        turn: dict[int, int] = {}
        out = []
        for j, im in enumerate(images):
            cands = by_dev.get(im.device.index) if isinstance(im, torch.Tensor) and im.is_cuda else None
            if cands:
                k = turn.get(im.device.index, 0)
                turn[im.device.index] = k + 1
                out.append(cands[k % len(cands)])
            else:
                out.append(j % D)
        return out

    def embed_parts(self, images: Sequence, normalized: bool = True, assign: Sequence[int] | None = None):
        """[(positions, raw [m, H], normed [m, H] or None)] per member that got images, each on
        its member's GPU (queued on that GPU's current stream; no host synchronisation).  Default
        assignment round-robin; after ``decode_jpeg_for_embed`` pass ``assign_by_location``."""
        n = len(images)
        assign = list(assign) if assign is not None else self.assign(n)
        if len(assign) != n:
            raise ValueError("assign needs one member per image")
        out = []
        for mi, m in enumerate(self.members):
            pos = [j for j in range(n) if assign[j] == mi]
            if not pos:
                continue
            with torch.cuda.device(m.device):
                r, nr = m.embed_images([images[j] for j in pos], normalized=normalized)
            out.append((pos, r, nr))
        return out

    def embed_images(self, images: Sequence, normalized: bool = False, assign: Sequence[int] | None = None):
        """Same contract as ``VitMsnEmbedder.embed_images``: (raw, normed or None) on the first
        device, input order; the batch is embedded over every member concurrently."""
        n = len(images)
        raw = torch.empty((n, self.hidden), dtype=torch.float32, device=self.device)
        nrm = torch.empty((n, self.hidden), dtype=torch.float32, device=self.device) if normalized else None
        for pos, r, nr in self.embed_parts(images, normalized=normalized, assign=assign):
            sel = torch.tensor(pos, dtype=torch.int64, device=self.device)
            raw.index_copy_(0, sel, r.to(self.device))
            if normalized:
                nrm.index_copy_(0, sel, nr.to(self.device))
        return raw, nrm

    def embed(self, images_u8: torch.Tensor, normalized: bool = True, stream=None, out=None):
        """u8 [n,h,w,3] → (raw, normed) on the first device, slices embedded on every member."""
        if out is not None or stream is not None:
            raise ValueError("EmbedderPool.embed: out / stream are per-member; use embed_parts")
        return self.embed_images(list(images_u8.unbind(0)), normalized=normalized)

    def embed_pil(self, images: Sequence) -> list[list[float]]:
        raw, _ = self.embed_images([np.asarray(im.convert("RGB"), dtype=np.uint8) for im in images])
        return raw.cpu().tolist()

    def decode_jpeg(self, datas: Sequence[bytes]) -> list[torch.Tensor]:
        return self.members[0].decode_jpeg(datas)

    def decode_jpeg_for_embed(self, datas: Sequence[bytes], assign: Sequence[int] | None = None) -> list[torch.Tensor]:
        """Per-image device u8 [S, S, 3] inputs (input order).  Each member decodes its share
        (``assign``, default round-robin) on its own GPU — host Huffman, reconstruction and the
        fused resize — concurrently with the others (the library splits its host Huffman workers
        between concurrent calls), queued on the caller's current stream of that GPU.  An image
        stays on the GPU that decoded it and ``embed_parts`` embeds it there: only its 768-float
        vector ever crosses GPUs, not the 150 KB image."""
        n = len(datas)
        assign = list(assign) if assign is not None else self.assign(n)
        if len(assign) != n:
            raise ValueError("assign needs one member per image")
        groups: dict[int, list[int]] = {}
        for j, mi in enumerate(assign):
            groups.setdefault(mi, []).append(j)
        streams = {m.device.index: torch.cuda.current_stream(m.device) for m in self.members}

        def work(item):
            mi, pos = item
            m = self.members[mi]
            with torch.cuda.device(m.device), torch.cuda.stream(streams[m.device.index]):
                return pos, m.decode_jpeg_for_embed([datas[j] for j in pos])

        items = list(groups.items())
        if len(items) == 1:
            results = [work(items[0])]
        else:
            import concurrent.futures as cf

            with cf.ThreadPoolExecutor(len(items)) as ex:
                results = list(ex.map(work, items))
        out: list = [None] * n
        for pos, x in results:
            for j, im in zip(pos, x.unbind(0)):
                out[j] = im
        return out

    def embed_jpeg(self, datas: Sequence[bytes]) -> list[list[float]]:
        ims = self.decode_jpeg_for_embed(datas)
        raw, _ = self.embed_images(ims, assign=self.assign_by_location(ims))
        return raw.cpu().tolist()

    def preprocess(self, images_u8: torch.Tensor, stream=None) -> torch.Tensor:
        return self.members[0].preprocess(images_u8, stream=stream)

    def set_parts(self, parts: int) -> None:
        for m in self.members:
            m.set_parts(parts)

    def set_ln_fold(self, on: bool) -> None:
        for m in self.members:
            m.set_ln_fold(on)

    def set_last_layer(self, cls_only: bool) -> None:
        for m in self.members:
            m.set_last_layer(cls_only)

    def set_graphs(self, on: bool) -> None:
        for m in self.members:
            m.set_graphs(on)


def gflop_per_image(cfg: dict = VIT_MSN_BASE, cls_only_last: bool = False) -> float:
    """FLOPs (2 x MACs) of one ViT forward incl. attention (35.126 GFLOP).

    ``cls_only_last``: the FLOPs ``rc_embed`` executes when the last layer runs
    attention / O-proj / MLP for the CLS row only (rc_model_set_last_layer):
    LN1 + K/V stay on all T rows, Q and the rest shrink to one row (32.70 GFLOP).
    """
    H, F, L = cfg["hidden_size"], cfg["intermediate_size"], cfg["num_hidden_layers"]
    P = cfg["patch_size"]
    np_ = (cfg["image_size"] // P) ** 2
    T = np_ + 1
    patch = np_ * H * 3 * P * P
    per_layer = T * (3 * H * H + H * H + 2 * H * F) + 2 * T * T * H
    if not cls_only_last:
        return 2.0 * (patch + L * per_layer) / 1e9
    last = T * 2 * H * H + H * H + (H * H + 2 * H * F) + 2 * T * H
    return 2.0 * (patch + (L - 1) * per_layer + last) / 1e9


def random_state_dict(seed: int = 0, num_layers: int = 12, cfg: dict = VIT_MSN_BASE) -> dict[str, np.ndarray]:
    """Random-init ViT-MSN weights in the checkpoint's key layout (benchmarks: no checkpoint offline)."""
    g = torch.Generator().manual_seed(seed)
    H, F, P, T = cfg["hidden_size"], cfg["intermediate_size"], cfg["patch_size"], (cfg["image_size"] // cfg["patch_size"]) ** 2 + 1

    def rnd(*shape, std=0.02, mean=0.0):
        return (torch.randn(*shape, generator=g) * std + mean).numpy()

    sd = {
        "embeddings.cls_token": rnd(1, 1, H),
        "embeddings.position_embeddings": rnd(1, T, H),
        "embeddings.patch_embeddings.projection.weight": rnd(H, 3, P, P),
        "embeddings.patch_embeddings.projection.bias": rnd(H),
        "layernorm.weight": rnd(H, std=0.1, mean=1.0),
        "layernorm.bias": rnd(H),
    }
    for i in range(num_layers):
        p = f"encoder.layer.{i}."
        for nm in ("query", "key", "value"):
            sd[p + f"attention.attention.{nm}.weight"] = rnd(H, H)
            sd[p + f"attention.attention.{nm}.bias"] = rnd(H)
        sd[p + "attention.output.dense.weight"] = rnd(H, H)
        sd[p + "attention.output.dense.bias"] = rnd(H)
        sd[p + "intermediate.dense.weight"] = rnd(F, H)
        sd[p + "intermediate.dense.bias"] = rnd(F)
        sd[p + "output.dense.weight"] = rnd(H, F)
        sd[p + "output.dense.bias"] = rnd(H)
        for nm in ("layernorm_before", "layernorm_after"):
            sd[p + nm + ".weight"] = rnd(H, std=0.1, mean=1.0)
            sd[p + nm + ".bias"] = rnd(H)
    return sd
