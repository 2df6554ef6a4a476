"""GPU JPEG decode for the embedding path (replaces the PIL decode at
``embedding/main.py:97`` for baseline JPEGs).

``probe(data)`` reads the header (size, sampling, whether the GPU path handles
it); ``JpegDecoder.decode(list_of_bytes)`` Huffman-decodes on the host (one
thread per image inside the library) and reconstructs HWC RGB u8 on the GPU
(``rc_jpeg_decode``), bit-exact with ``Image.open(...).convert("RGB")``.
Streams the GPU path does not handle (progressive, arithmetic, 12-bit, CMYK /
RGB colour spaces, multi-scan) are reported by ``probe`` and by
``JpegUnsupported``; the caller keeps those on the reference's host decode.
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

import torch

from ._lib import JpegInfo, RC_ERR_UNSUPPORTED, RetrievalCoreError, check, load, stream_ptr


class JpegUnsupported(ValueError):
    """A valid image the GPU decoder does not reconstruct (decode it on the host)."""


def probe(data: bytes) -> JpegInfo:
    """Header of a JPEG stream; raises ValueError if ``data`` is not one."""
    info = JpegInfo()
    check(load().rc_jpeg_probe(data, len(data), C.byref(info)))
    return info


def is_gpu_decodable(data: bytes) -> bool:
    if len(data) < 4 or data[0] != 0xFF or data[1] != 0xD8:
        return False
    try:
        return bool(probe(data).supported)
    except ValueError:
        return False


def decode_coefficients(data: bytes):
    """Host entropy decode (test hook): (info, coef int16 [blocks, 64], qtab u16 [ncomp, 64])."""
    import numpy as np

    info = probe(data)
    if not info.supported:
        raise JpegUnsupported("JPEG stream outside the GPU decoder's scope")
    coef = np.zeros((info.blocks, 64), dtype=np.int16)
    qtab = np.zeros((3, 64), dtype=np.uint16)
    check(load().rc_jpeg_decode_coefficients(data, len(data), coef.ctypes.data, qtab.ctypes.data))
    return info, coef, qtab[: info.ncomp]


class JpegDecoder:
    """Batched GPU JPEG decoder with a fixed workspace (max_images, max_pixels)."""

    def __init__(self, device=None, max_images: int = 256, max_pixels: int = 1 << 22):
        self.lib = load()
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   (device.index if isinstance(device, torch.device) else int(device)))
        self.max_images = int(max_images)
        # worst case (4:4:4, MCU padding): 3 planes of ceil(w/8)*ceil(h/8) blocks;
        # pixels/64 per plane plus a padding margin per image
        self.max_blocks = int(3 * (max_pixels // 64) + 3 * 64 * max_images)
        h = C.c_void_p()
        check(self.lib.rc_jpeg_decoder_create(self.device.index, self.max_images, self.max_blocks, C.byref(h)))
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None):
            self.lib.rc_jpeg_decoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def decode(self, datas: Sequence[bytes], stream=None) -> list[torch.Tensor]:
        """JPEG byte strings -> device u8 HWC RGB tensors (views into one packed buffer)."""
        infos = [probe(d) for d in datas]
        for i, inf in enumerate(infos):
            if not inf.supported:
                raise JpegUnsupported(f"image {i}: JPEG stream outside the GPU decoder's scope")
        outs: list[torch.Tensor] = []
        for s in range(0, len(datas), self.max_images):
            chunk, cinf = datas[s:s + self.max_images], infos[s:s + self.max_images]
            sizes = [inf.width * inf.height * 3 for inf in cinf]
            offs = [0]
            for z in sizes[:-1]:
                offs.append(offs[-1] + z)
            buf = torch.empty(sum(sizes), dtype=torch.uint8, device=self.device)
            n = len(chunk)
            ptrs = (C.c_char_p * n)(*chunk)
            lens = (C.c_int64 * n)(*[len(d) for d in chunk])
            coffs = (C.c_int64 * n)(*offs)
            status = self.lib.rc_jpeg_decode(self._h, n, ptrs, lens, buf.data_ptr(), coffs, stream_ptr(stream))
            if status == RC_ERR_UNSUPPORTED:
                raise JpegUnsupported(self.lib.rc_last_error().decode())
            check(status)
            for inf, o, z in zip(cinf, offs, sizes):
                outs.append(buf[o:o + z].view(inf.height, inf.width, 3))
        return outs

    def decode_resized(self, datas: Sequence[bytes], size: int, resample: int, stream=None) -> torch.Tensor:
        """JPEG byte strings (any, mixed sizes) -> device u8 [n, size, size, 3]: the decode followed
        by Pillow's resample to size x size (ViTImageProcessor's resize), the colour pass fused
        with the horizontal resample (rc_jpeg_decode_resized); bit-exact with PIL decode +
        Image.resize."""
        infos = [probe(d) for d in datas]
        for i, inf in enumerate(infos):
            if not inf.supported:
                raise JpegUnsupported(f"image {i}: JPEG stream outside the GPU decoder's scope")
        out = torch.empty((len(datas), size, size, 3), dtype=torch.uint8, device=self.device)
        for s in range(0, len(datas), self.max_images):
            chunk = datas[s:s + self.max_images]
            n = len(chunk)
            ptrs = (C.c_char_p * n)(*chunk)
            lens = (C.c_int64 * n)(*[len(d) for d in chunk])
            status = self.lib.rc_jpeg_decode_resized(self._h, n, ptrs, lens, int(size), int(resample),
                                                     out[s:s + n].data_ptr(), stream_ptr(stream))
            if status == RC_ERR_UNSUPPORTED:
                raise JpegUnsupported(self.lib.rc_last_error().decode())
            check(status)
        return out

    def decode_batch(self, datas: Sequence[bytes], stream=None) -> torch.Tensor:
        """Equal-size JPEGs -> one device u8 [n, H, W, 3] tensor.  Within one chunk the
        images are packed back to back, so the batch is a view of the decode buffer
        (no stack copy); mixed sizes raise ValueError."""
        imgs = self.decode(datas, stream=stream)
        if not imgs:
            raise ValueError("empty batch")
        shape = imgs[0].shape
        if any(im.shape != shape for im in imgs):
            raise ValueError("decode_batch needs equal-size images")
        first = imgs[0]
        packed = (len(imgs) <= self.max_images
                  and all(im.data_ptr() == first.data_ptr() + i * first.numel() for i, im in enumerate(imgs)))
        if packed:
            return first.as_strided((len(imgs),) + tuple(shape), (first.numel(),) + tuple(first.stride()))
        return torch.stack(imgs)


__all__ = ["JpegDecoder", "JpegUnsupported", "probe", "is_gpu_decodable", "decode_coefficients", "RetrievalCoreError"]
