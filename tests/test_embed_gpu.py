"""GPU parity of the ViT-MSN embedding path (rc_embed / rc_preprocess) against the oracle.

Reference path replaced: ``embedding/main.py:97-114`` (PIL decode → ViTImageProcessor
→ ViTMSNModel → ``last_hidden_state[:, 0, :]``).  Bars (north star):
  * preprocessing is integer/byte work + an exact f32 LUT → bit-exact pixel_values;
  * embeddings (bf16 MFMA GEMMs, f32 accumulate/residual) agree with the fp32
    reference within 1e-2 cosine distance — tolerance written below as BF16_COS_TOL.
"""
import hashlib
import json
import os

import numpy as np
import pytest
from PIL import Image

from conftest import GOLDEN, import_pkg
from oracle.pil_resample import BICUBIC, BILINEAR
from oracle.preprocess import VIT_MSN_PREPROCESS, preprocess
from oracle.vit import cosine, embed_cls
from oracle.weights import seeded_vit_msn_weights

pytestmark = pytest.mark.gpu

BF16_COS_TOL = 1e-2  # north-star bound for the bf16 path: 1 - cos(got, ref) <= 1e-2
# north-star bound of the fp32 tier.  The bf16 path meets it as well on the 12-layer
# seeded model (measured max 1.1e-4 over the test image + random images,
# tools/precision_probe.py), so it is asserted as this build's regression guard.
FP32_TIER_COS_TOL = 1e-3


@pytest.fixture(scope="module")
def vitmod(cuda):
    return import_pkg("vit")


@pytest.fixture(scope="module")
def weights12():
    return seeded_vit_msn_weights(1907)


@pytest.fixture(scope="module")
def model12(vitmod, weights12, cuda):
    m = vitmod.VitMsnEmbedder(weights12, device=0, max_batch=16)
    yield m
    m.close()


def _test_image():
    return np.array(Image.open(os.path.join(GOLDEN, "test_image.jpeg")).convert("RGB"))


def test_preprocess_test_image_bit_exact(model12):
    import torch

    g = json.load(open(os.path.join(GOLDEN, "golden.json")))
    img = _test_image()
    pv = model12.preprocess(torch.from_numpy(img[None])).cpu().numpy()[0]
    assert hashlib.sha256(pv.tobytes()).hexdigest()[:16] == g["pixel_values_sha16"]


@pytest.mark.parametrize("h,w", [(224, 224), (300, 168), (97, 480), (224, 100), (50, 224), (513, 511), (16, 16)])
@pytest.mark.parametrize("resample", [BICUBIC, BILINEAR])
def test_preprocess_random_sizes_bit_exact(vitmod, weights12, cuda, h, w, resample):
    import torch

    params = dict(VIT_MSN_PREPROCESS, resample=resample)
    m = vitmod.VitMsnEmbedder({k: v for k, v in weights12.items() if "encoder.layer." not in k or ".layer.0." in k},
                              device=0, max_batch=3, preprocess=params)
    rng = np.random.default_rng(h * 1000 + w)
    imgs = rng.integers(0, 256, (3, h, w, 3), dtype=np.uint8)
    got = m.preprocess(torch.from_numpy(imgs)).cpu().numpy()
    ref = np.stack([preprocess(x, params) for x in imgs])
    assert np.array_equal(got, ref)
    m.close()


def test_embed_test_image_matches_reference(model12):
    """Full 12-layer seeded model on the reference's own test image vs transformers' output."""
    import torch

    ref = np.load(os.path.join(GOLDEN, "test_image_embedding_seed1907.npy"))
    img = _test_image()
    raw, nrm = model12.embed(torch.from_numpy(img[None]))
    raw = raw.cpu().numpy()[0]
    assert np.isfinite(raw).all()
    assert 1.0 - cosine(raw, ref) <= BF16_COS_TOL
    assert 1.0 - cosine(raw, ref) <= FP32_TIER_COS_TOL
    nrm = nrm.cpu().numpy()[0]
    assert np.allclose(nrm, raw / np.linalg.norm(raw), atol=1e-6)


def test_embed_two_layer_synthetic(vitmod, cuda):
    import torch

    sd2 = seeded_vit_msn_weights(1907, num_layers=2)
    m = vitmod.VitMsnEmbedder(sd2, device=0, max_batch=2)
    imgs = np.load(os.path.join(GOLDEN, "synthetic_u8_2x224.npy"))
    ref = np.load(os.path.join(GOLDEN, "synthetic_embedding_2layer_seed1907.npy"))
    raw, _ = m.embed(torch.from_numpy(imgs))
    raw = raw.cpu().numpy()
    for i in range(2):
        assert 1.0 - cosine(raw[i], ref[i]) <= BF16_COS_TOL
    m.close()


def test_embed_batch_equals_single_and_deterministic(model12):
    """Rows of a batch are independent: batched == one-by-one, bitwise; repeat runs are bitwise equal."""
    import torch

    rng = np.random.default_rng(7)
    imgs = torch.from_numpy(rng.integers(0, 256, (5, 224, 224, 3), dtype=np.uint8))
    a, _ = model12.embed(imgs)
    b, _ = model12.embed(imgs)
    assert torch.equal(a, b)
    for i in range(5):
        s, _ = model12.embed(imgs[i:i + 1])
        assert torch.equal(s[0], a[i])


def test_embed_matches_numpy_oracle_random(model12, weights12):
    import torch

    rng = np.random.default_rng(9)
    imgs = rng.integers(0, 256, (2, 224, 224, 3), dtype=np.uint8)
    raw, _ = model12.embed(torch.from_numpy(imgs))
    ref = embed_cls(np.stack([preprocess(x) for x in imgs]), weights12)
    raw = raw.cpu().numpy()
    for i in range(2):
        assert 1.0 - cosine(raw[i], ref[i]) <= BF16_COS_TOL
        assert 1.0 - cosine(raw[i], ref[i]) <= FP32_TIER_COS_TOL


def test_embed_full_batch_256_properties(vitmod, weights12, cuda):
    """Config 2's shape (batch 256, 224x224): finite, deterministic, spot rows vs the oracle."""
    import torch

    m = vitmod.VitMsnEmbedder(weights12, device=0, max_batch=256)
    rng = np.random.default_rng(1)
    imgs = rng.integers(0, 256, (256, 224, 224, 3), dtype=np.uint8)
    raw, nrm = m.embed(torch.from_numpy(imgs))
    raw2, _ = m.embed(torch.from_numpy(imgs))
    assert torch.equal(raw, raw2)
    assert torch.isfinite(raw).all()
    assert torch.allclose(nrm.norm(dim=1), torch.ones(256, device=nrm.device), atol=1e-5)
    pick = [0, 131, 255]
    ref = embed_cls(np.stack([preprocess(imgs[i]) for i in pick]), weights12)
    got = raw.cpu().numpy()[pick]
    for j in range(len(pick)):
        assert 1.0 - cosine(got[j], ref[j]) <= BF16_COS_TOL
        assert 1.0 - cosine(got[j], ref[j]) <= FP32_TIER_COS_TOL
    m.close()


@pytest.mark.parametrize("parts", [2, 3, 4])
def test_embed_split_streams_bitwise_equal(vitmod, cuda, parts):
    """A batch encoded as 2-4 concurrent parts on separate streams equals the one-stream result bit for bit."""
    import torch

    from oracle.weights import seeded_vit_msn_weights

    sd = seeded_vit_msn_weights(1907, num_layers=2)
    rng = np.random.default_rng(parts)
    imgs = torch.from_numpy(rng.integers(0, 256, (250, 224, 224, 3), dtype=np.uint8))
    m1 = vitmod.VitMsnEmbedder(sd, device=0, max_batch=250)
    m1.set_parts(1)
    a, an = m1.embed(imgs)
    mp = vitmod.VitMsnEmbedder(sd, device=0, max_batch=250)
    mp.set_parts(parts)
    b, bn = mp.embed(imgs)
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(an, bn)
    m1.close()
    mp.close()


def test_cls_only_last_layer_matches_full_layer(vitmod, weights12, cuda):
    """The CLS-only last layer (default) agrees with the whole last layer and with the oracle.

    Only attention's summation order differs (attention_cls_kernel vs the MFMA
    kernel), so the two paths agree far inside the bf16 bar; both stay within
    BF16_COS_TOL of the fp32 reference.
    """
    import torch

    rng = np.random.default_rng(11)
    imgs = rng.integers(0, 256, (40, 224, 224, 3), dtype=np.uint8)
    m = vitmod.VitMsnEmbedder(weights12, device=0, max_batch=40)
    m.set_last_layer(False)
    full, _ = m.embed(torch.from_numpy(imgs))
    m.set_last_layer(True)
    cls, cls_n = m.embed(torch.from_numpy(imgs))
    torch.cuda.synchronize()
    full, cls = full.cpu().numpy(), cls.cpu().numpy()
    assert np.isfinite(cls).all()
    for i in range(40):
        assert 1.0 - cosine(cls[i], full[i]) <= 1e-4
    assert np.abs(cls - full).max() <= 2e-2 * np.abs(full).max()
    pick = [0, 39]
    ref = embed_cls(np.stack([preprocess(imgs[i]) for i in pick]), weights12)
    for j, i in enumerate(pick):
        assert 1.0 - cosine(cls[i], ref[j]) <= BF16_COS_TOL
        assert 1.0 - cosine(full[i], ref[j]) <= BF16_COS_TOL
    m.close()


def test_ln_fold_matches_unfused_and_oracle(vitmod, weights12, cuda):
    """LayerNorm folded into QKV / fc1 (default) vs the standalone LN kernel: the two agree far
    inside the bf16 bar, both stay within BF16_COS_TOL of the fp32 oracle, and the fold gives
    the same bits at every batch size (tiled GEMMs for 40 images, skinny ones for 1)."""
    import torch

    rng = np.random.default_rng(13)
    imgs = rng.integers(0, 256, (40, 224, 224, 3), dtype=np.uint8)
    m = vitmod.VitMsnEmbedder(weights12, device=0, max_batch=40)
    m.set_ln_fold(False)
    plain, _ = m.embed(torch.from_numpy(imgs))
    m.set_ln_fold(True)
    fold, _ = m.embed(torch.from_numpy(imgs))
    one, _ = m.embed(torch.from_numpy(imgs[7:8]))
    torch.cuda.synchronize()
    assert torch.equal(one[0], fold[7])
    plain, fold = plain.cpu().numpy(), fold.cpu().numpy()
    assert np.isfinite(fold).all()
    for i in range(40):
        assert 1.0 - cosine(fold[i], plain[i]) <= 1e-3
    pick = [0, 39]
    ref = embed_cls(np.stack([preprocess(imgs[i]) for i in pick]), weights12)
    for j, i in enumerate(pick):
        assert 1.0 - cosine(fold[i], ref[j]) <= BF16_COS_TOL
        assert 1.0 - cosine(fold[i], ref[j]) <= FP32_TIER_COS_TOL
    m.close()


def test_embed_massive_activation_channels(vitmod, weights12, cuda):
    """Trained ViTs carry a few residual channels at ~100x the rest (massive activations);
    the seeded weights do not.  With oracle.weights.with_massive_activations the residual
    stream spans 280 vs ~0.5 (560x): the bf16 residual copy and the LayerNorm fold (whose
    mean and rstd the outliers then set) must still match the fp32 oracle — on every
    channel and on the ordinary channels alone (the outliers would dominate the cosine)."""
    import torch

    from oracle.weights import with_massive_activations

    outl = (17, 401)
    sd = with_massive_activations(weights12, channels=outl)
    rng = np.random.default_rng(21)
    imgs = rng.integers(0, 256, (3, 224, 224, 3), dtype=np.uint8)
    imgs[0] = np.array(Image.fromarray(_test_image()).resize((224, 224)))
    ref = embed_cls(np.stack([preprocess(x) for x in imgs]), sd)
    keep = np.ones(768, bool)
    keep[list(outl)] = False
    m = vitmod.VitMsnEmbedder(sd, device=0, max_batch=3)
    outs = {}
    for fold in (True, False):
        m.set_ln_fold(fold)
        raw, _ = m.embed(torch.from_numpy(imgs))
        outs[fold] = raw.cpu().numpy()
        assert np.isfinite(outs[fold]).all()
        for i in range(3):
            assert 1.0 - cosine(outs[fold][i], ref[i]) <= FP32_TIER_COS_TOL
            assert 1.0 - cosine(outs[fold][i][keep], ref[i][keep]) <= FP32_TIER_COS_TOL
    for i in range(3):  # fold vs standalone LayerNorm: measured ~1e-6
        assert 1.0 - cosine(outs[True][i][keep], outs[False][i][keep]) <= 1e-4
    m.close()



def test_from_pretrained_v5_layout_matches_golden(vitmod, cuda, tmp_path):
    """VitMsnEmbedder.from_pretrained on a local checkpoint directory in the transformers-5 key
    layout (config.json + model.safetensors: the offline stand-in for the reference's
    from_pretrained("facebook/vit-msn-base"), embedding/main.py:37-38) embeds the committed
    2-layer golden images like the seeded weights handed over directly."""
    import json as _json

    import torch
    from safetensors.numpy import save_file

    from oracle.weights import to_hf_v5

    sd2 = seeded_vit_msn_weights(1907, num_layers=2)
    d = tmp_path / "ckpt"
    d.mkdir()
    (d / "config.json").write_text(_json.dumps({"num_hidden_layers": 2, "hidden_size": 768}))
    save_file({k: np.ascontiguousarray(v) for k, v in to_hf_v5(sd2).items()}, str(d / "model.safetensors"))
    m = vitmod.VitMsnEmbedder.from_pretrained(str(d), device=0, max_batch=2)
    direct = vitmod.VitMsnEmbedder(sd2, device=0, max_batch=2)
    imgs = torch.from_numpy(np.load(os.path.join(GOLDEN, "synthetic_u8_2x224.npy")))
    ref = np.load(os.path.join(GOLDEN, "synthetic_embedding_2layer_seed1907.npy"))
    raw, _ = m.embed(imgs)
    raw2, _ = direct.embed(imgs)
    assert torch.equal(raw, raw2)
    raw = raw.cpu().numpy()
    for i in range(2):
        assert 1.0 - cosine(raw[i], ref[i]) <= BF16_COS_TOL
    m.close()
    direct.close()


def test_image_aligned_tiles_batch_invariant(vitmod, weights12, cuda):
    """Full batches run the 256-row ping-pong and the two-workgroup 128-row tiles (image rows at any
    position in a tile), a lone image the skinny kernels: every kernel accumulates K in the same
    order, so an image's 12-layer embedding is the same bits whatever batch, slice or tile it lands
    in — a batch of 300 in one or two slices, three batches of 100, single images."""
    import torch

    rng = np.random.default_rng(21)
    imgs = torch.from_numpy(rng.integers(0, 256, (300, 224, 224, 3), dtype=np.uint8))
    m = vitmod.VitMsnEmbedder(weights12, device=0, max_batch=300)
    m.set_parts(1)
    a, an = m.embed(imgs)
    m.set_parts(2)
    b, bn = m.embed(imgs)
    parts = [m.embed(imgs[i:i + 100]) for i in range(0, 300, 100)]
    c = torch.cat([p[0] for p in parts])
    ones = [m.embed(imgs[i:i + 1])[0] for i in (0, 1, 150, 299)]
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(an, bn)
    assert torch.equal(a, c)
    for j, i in enumerate((0, 1, 150, 299)):
        assert torch.equal(a[i:i + 1], ones[j]), i
    m.close()


def test_batch1_graph_replay_matches_stream_form(vitmod, weights12, cuda):
    """A one-image embed replays a captured HIP graph (rc_model_set_graphs, default on): the same
    bits as the stream form, for new contents in the same buffers (the graph reads them at replay),
    for a second buffer triple (a second graph), into pinned host memory, and after a setter (which
    drops the captured graphs: the replay follows the new setting); with more triples than the
    cache keeps, and when every call brings new buffers (churn: the stream form, no capture)."""
    import torch

    rng = np.random.default_rng(31)
    imgs = torch.from_numpy(rng.integers(0, 256, (3, 224, 224, 3), dtype=np.uint8)).to(cuda)
    m = vitmod.VitMsnEmbedder(weights12, device=0, max_batch=4)
    x = torch.empty((1, 224, 224, 3), dtype=torch.uint8, device=cuda)
    raw, nrm = torch.empty((1, 768), device=cuda), torch.empty((1, 768), device=cuda)
    ref = {}
    m.set_graphs(False)
    for i in range(3):
        ref[i] = [t.clone() for t in m.embed(imgs[i:i + 1])]
    m.set_last_layer(False)
    full_ref = m.embed(imgs[0:1])[0].clone()
    m.set_last_layer(True)
    m.set_graphs(True)
    for rep in range(2):
        for i in range(3):
            x.copy_(imgs[i:i + 1])
            m.embed(x, out=(raw, nrm))
            torch.cuda.synchronize()
            assert torch.equal(raw, ref[i][0]) and torch.equal(nrm, ref[i][1]), (rep, i)
    raw2 = torch.empty((1, 768), device=cuda)
    m.embed(imgs[1:2], out=(raw2, None))
    torch.cuda.synchronize()
    assert torch.equal(raw2, ref[1][0])
    host = torch.empty((1, 768), dtype=torch.float32, pin_memory=True)
    x.copy_(imgs[2:3])
    m.embed(x, out=(host, None))
    torch.cuda.synchronize()
    assert torch.equal(host, ref[2][0].cpu())
    # more buffer triples than the cache keeps (8): the least recently used graphs are evicted and
    # re-captured on their next use, the results unchanged
    outs = [torch.empty((1, 768), device=cuda) for _ in range(11)]
    for rep in range(2):
        for i, o in enumerate(outs):
            m.embed(imgs[i % 3:i % 3 + 1], out=(o, None))
        torch.cuda.synchronize()
        for i, o in enumerate(outs):
            assert torch.equal(o, ref[i % 3][0]), (rep, i)
    # 22 misses in a row put the cache in churn mode (new triples run the stream form); a triple
    # used twice in a row is captured again and replayed from then on
    for rep in range(3):
        x.copy_(imgs[rep:rep + 1])
        m.embed(x, out=(raw, nrm))
        torch.cuda.synchronize()
        assert torch.equal(raw, ref[rep][0]) and torch.equal(nrm, ref[rep][1]), rep
    m.set_last_layer(False)
    x.copy_(imgs[0:1])
    m.embed(x, out=(raw, nrm))
    torch.cuda.synchronize()
    assert torch.equal(raw, full_ref)
    m.close()
