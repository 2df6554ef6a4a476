"""GPU JPEG decode (rc_jpeg_decode) against Pillow's decode of the same bytes —
the reference's own decode path, embedding/main.py:97.  Integer work: bit-exact."""
import numpy as np
import pytest

from conftest import import_pkg
from jpeg_cases import cases, pil_rgb, synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def J(cuda):
    return import_pkg("jpeg")


@pytest.fixture(scope="module")
def dec(J, cuda):
    d = J.JpegDecoder(device=0, max_images=128, max_pixels=1 << 21)
    yield d
    d.close()


def test_batch_of_mixed_streams_bit_exact(dec):
    cs = cases()
    outs = dec.decode([d for _, d in cs])
    for (name, data), got in zip(cs, outs):
        assert np.array_equal(got.cpu().numpy(), pil_rgb(data)), name


@pytest.mark.parametrize("name,data", cases()[::7], ids=[c[0] for c in cases()[::7]])
def test_single_image_calls_bit_exact(dec, name, data):
    (got,) = dec.decode([data])
    assert np.array_equal(got.cpu().numpy(), pil_rgb(data))


def test_repeated_calls_reuse_the_staging(dec):
    datas = [synthetic(224, 224, 100 + i, quality=85, subsampling=2) for i in range(24)]
    refs = [pil_rgb(d) for d in datas]
    for _ in range(3):
        outs = dec.decode(datas)  # no sync between calls: staging reuse must wait for the upload
        outs2 = dec.decode(datas[::-1])
        for o, r in zip(outs, refs):
            assert np.array_equal(o.cpu().numpy(), r)
        for o, r in zip(outs2, refs[::-1]):
            assert np.array_equal(o.cpu().numpy(), r)


def test_unsupported_stream_raises(J, dec):
    prog = synthetic(64, 64, 7, quality=80, progressive=True)
    with pytest.raises(J.JpegUnsupported):
        dec.decode([synthetic(32, 32, 1), prog])


def test_damaged_stream_raises_value_error(dec):
    data = synthetic(96, 96, 9, quality=90)
    with pytest.raises(ValueError):
        dec.decode([data[: len(data) // 2] + b"\xff\xd9"])


def test_gpu_decoded_embedding_equals_pil_decoded(dec, cuda):
    import torch

    vit = import_pkg("vit")
    from oracle.weights import seeded_vit_msn_weights

    m = vit.VitMsnEmbedder(seeded_vit_msn_weights(1907, num_layers=2), device=0, max_batch=4)
    data = dict(cases())["test_image"]
    (img,) = dec.decode([data])
    raw_gpu, _ = m.embed(img[None])
    raw_pil, _ = m.embed(torch.from_numpy(pil_rgb(data).copy())[None])
    assert torch.equal(raw_gpu, raw_pil)
    m.close()


def test_embed_jpeg_stream_matches_unpipelined(cuda):
    """Pipelined decode (worker thread + side stream) -> embed equals embedding PIL-decoded pixels."""
    import torch

    vit = import_pkg("vit")
    from oracle.weights import seeded_vit_msn_weights

    m = vit.VitMsnEmbedder(seeded_vit_msn_weights(1907, num_layers=2), device=0, max_batch=8)
    batches = [[synthetic(224, 224, 300 + 8 * b + i, quality=90, subsampling=2) for i in range(8)] for b in range(4)]
    got = [raw.clone() for raw, _ in m.embed_jpeg_stream(batches)]
    for b, datas in enumerate(batches):
        ref, _ = m.embed(torch.from_numpy(np.stack([pil_rgb(d) for d in datas])))
        assert torch.equal(got[b], ref)
    m.close()


def test_decode_batch_is_a_packed_view(dec):
    """decode_batch: one chunk of equal-size images is a view of the decode buffer (no stack
    copy) and bit-exact with PIL; a batch spanning chunks or mixed sizes is handled loudly."""
    datas = [synthetic(64, 48, 500 + i, quality=90, subsampling=2) for i in range(6)]
    x = dec.decode_batch(datas)
    assert tuple(x.shape) == (6, 48, 64, 3) and x.is_contiguous()
    assert np.array_equal(x.cpu().numpy(), np.stack([pil_rgb(d) for d in datas]))
    many = [datas[i % 6] for i in range(dec.max_images + 3)]  # two chunks -> stacked copy
    y = dec.decode_batch(many)
    assert np.array_equal(y[dec.max_images + 1].cpu().numpy(), pil_rgb(datas[(dec.max_images + 1) % 6]))
    with pytest.raises(ValueError):
        dec.decode_batch([datas[0], synthetic(32, 32, 1)])


def _pil_resized(data, size=224, resample=3):
    """PIL decode (embedding/main.py:97) + the processor's resize (ViTImageProcessorPil, :107)."""
    import io

    from PIL import Image

    im = Image.open(io.BytesIO(data)).convert("RGB")
    return np.asarray(im.resize((size, size), resample)) if im.size != (size, size) else np.asarray(im)


@pytest.mark.parametrize("resample", [3, 2])
def test_decode_resized_bit_exact_mixed_sizes(dec, resample):
    """rc_jpeg_decode_resized (colour pass fused with the horizontal resample, per-image vertical
    pass) == PIL decode + Image.resize, for every stream of the decode cases in ONE mixed batch
    (up- and downscale on either axis, one axis already 224, grayscale, 4:4:4 / 4:2:2 / 4:2:0)."""
    cs = cases()
    got = dec.decode_resized([d for _, d in cs], 224, resample)
    for (name, data), g in zip(cs, got):
        assert np.array_equal(g.cpu().numpy(), _pil_resized(data, 224, resample)), name


def test_decode_resized_wide_rows_and_reuse(J, cuda):
    """Rows wider than one LDS window (16384 px: several windows per row), a tall image, the
    reference fixture's 168 x 300, and repeated calls reusing the staging and the h-pass buffer."""
    d = J.JpegDecoder(device=0, max_images=8, max_pixels=1 << 22)
    datas = [synthetic(17000, 12, 41, quality=90, subsampling=2), synthetic(40, 3000, 42, quality=90, subsampling=1),
             dict(cases())["test_image"], synthetic(224, 224, 43, quality=95, subsampling=0)]
    for _ in range(2):
        got = d.decode_resized(datas, 224, 3)
        got2 = d.decode_resized(datas[::-1], 224, 3)
        for x, data in zip(got, datas):
            assert np.array_equal(x.cpu().numpy(), _pil_resized(data))
        for x, data in zip(got2, datas[::-1]):
            assert np.array_equal(x.cpu().numpy(), _pil_resized(data))
    d.close()


def test_fused_decode_embedding_equals_pil_path(cuda):
    """Embedding of the fused decode→resize equals the embedding of PIL-decoded pixels resized on
    the device (rc_embed's resize): the bulk stream and the per-request path use the fused one."""
    import torch

    vit = import_pkg("vit")
    from oracle.weights import seeded_vit_msn_weights

    m = vit.VitMsnEmbedder(seeded_vit_msn_weights(1907, num_layers=2), device=0, max_batch=8)
    batches = [[synthetic(168, 300, 700 + 8 * b + i, quality=90, subsampling=2) for i in range(8)] for b in range(3)]
    got = [raw.clone() for raw, _ in m.embed_jpeg_stream(batches)]
    for b, datas in enumerate(batches):
        ref, _ = m.embed(torch.from_numpy(np.stack([pil_rgb(d) for d in datas])))
        assert torch.equal(got[b], ref)
    mixed = [synthetic(168, 300, 800, quality=90), synthetic(224, 224, 801, quality=90), synthetic(640, 480, 802)]
    raw = torch.tensor(m.embed_jpeg(mixed))
    for i, data in enumerate(mixed):
        ref, _ = m.embed(torch.from_numpy(pil_rgb(data).copy())[None])
        assert torch.equal(raw[i], ref[0].cpu())
    m.close()


def test_decode_resized_band_and_two_pass_paths(J, cuda):
    """The band kernel (every image's band fits in LDS: short bands for the larger downscales)
    and the two-pass path (a batch holding a 17000-px row) are both bit-exact with PIL; the
    two-pass path's scratch grows geometrically: ever larger batches reallocate
    on fewer steps than they grow, and a second sweep allocates nothing."""
    lib = import_pkg("_lib").load()
    d = J.JpegDecoder(device=0, max_images=16, max_pixels=1 << 22)
    band = [synthetic(640, 480, 51), synthetic(1024, 768, 52, subsampling=2), synthetic(300, 168, 53),
            synthetic(224, 100, 54), synthetic(100, 224, 55, subsampling=1), synthetic(224, 224, 56)]
    for x, data in zip(d.decode_resized(band, 224, 3), band):
        assert np.array_equal(x.cpu().numpy(), _pil_resized(data))
    for x, data in zip(d.decode_resized(band, 224, 2), band):
        assert np.array_equal(x.cpu().numpy(), _pil_resized(data, 224, 2))
    wide, small = synthetic(17000, 12, 57, subsampling=2), synthetic(300, 168, 58)
    rises = []
    for sweep in range(2):
        for n in range(1, 9):
            c0 = lib.rc_alloc_count()
            got = d.decode_resized([wide] + [small] * (n - 1), 224, 3)
            rises.append(lib.rc_alloc_count() > c0)
            if sweep == 0 and n in (1, 8):
                assert np.array_equal(got[0].cpu().numpy(), _pil_resized(wide))
                assert np.array_equal(got[-1].cpu().numpy(), _pil_resized(wide if n == 1 else small))
    assert sum(rises[:8]) <= 6 and not any(rises[8:]), rises
    d.close()


@pytest.mark.parametrize("resample", [3, 2])
def test_decode_resized_single_images_fine_bands(dec, resample):
    """One image per call (the /embed request): the band kernel splits the 224 output rows into
    bands of <= 4 rows (>= 56 blocks for the image) — every decode case alone, bit-exact with PIL
    decode + Image.resize; and a batch of two picks the same bands."""
    cs = cases()
    for name, data in cs:
        got = dec.decode_resized([data], 224, resample)
        assert np.array_equal(got[0].cpu().numpy(), _pil_resized(data, 224, resample)), name
    pair = dec.decode_resized([cs[0][1], cs[-1][1]], 224, resample)
    assert np.array_equal(pair[1].cpu().numpy(), _pil_resized(cs[-1][1], 224, resample))
