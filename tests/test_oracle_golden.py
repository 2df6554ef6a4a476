"""Pin the CPU oracle against the reference's libraries and the committed goldens (CPU only).

* Pillow resize restatement: bit-exact vs Pillow on random sizes (up and down, both filters).
* preprocess: sha of pixel_values equals transformers' ViTImageProcessor output on the
  reference's own fixture image (tests/data/test_image.jpeg, copied as golden data).
* ViT forward: numpy oracle vs transformers ViTMSNModel (seeded weights) within 1e-4 abs.
* cosine top-k: exact top-5 over the planted 10k x 768 index equals the golden.
"""
import hashlib
import json
import os

import numpy as np
import pytest
from PIL import Image

from conftest import GOLDEN
from oracle.cosine_topk import cosine_topk, cosine_topk_f32, planted_index, topk_equal_modulo_ties
from oracle.pil_resample import BICUBIC, BILINEAR, resize_u8
from oracle.preprocess import pixel_lut, preprocess
from oracle.vit import cosine, embed_cls
from oracle.weights import seeded_vit_msn_weights, vit_msn_shapes

G = json.load(open(os.path.join(GOLDEN, "golden.json")))


def sha16(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def test_image_fixture_decodes_as_recorded():
    img = np.array(Image.open(os.path.join(GOLDEN, "test_image.jpeg")).convert("RGB"))
    assert list(img.shape) == G["decoded_shape"] and sha16(img) == G["decoded_sha16"]


@pytest.mark.parametrize("seed", range(12))
def test_resize_bit_exact_vs_pillow(seed):
    rng = np.random.default_rng(seed)
    h, w = int(rng.integers(1, 330)), int(rng.integers(1, 330))
    oh, ow = [224, int(rng.integers(1, 300))][seed % 2], [224, int(rng.integers(1, 300))][(seed // 2) % 2]
    img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    for rs in (BICUBIC, BILINEAR):
        ref = np.array(Image.fromarray(img).resize((ow, oh), resample=rs))
        assert np.array_equal(resize_u8(img, oh, ow, rs), ref)


def test_resize_test_image_hash():
    img = np.array(Image.open(os.path.join(GOLDEN, "test_image.jpeg")).convert("RGB"))
    assert sha16(resize_u8(img, 224, 224, BICUBIC)) == G["resized_u8_sha16"]


def test_preprocess_matches_transformers_hash():
    img = np.array(Image.open(os.path.join(GOLDEN, "test_image.jpeg")).convert("RGB"))
    assert sha16(preprocess(img)) == G["pixel_values_sha16"]


def test_pixel_lut_is_the_preprocess_map():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (224, 224, 3), dtype=np.uint8)
    lut = pixel_lut()
    via_lut = np.stack([lut[c][img[..., c]] for c in range(3)])
    assert np.array_equal(via_lut, preprocess(img))


def test_vit_oracle_two_layer_matches_transformers_golden():
    sd = seeded_vit_msn_weights(1907, num_layers=2)
    imgs = np.load(os.path.join(GOLDEN, "synthetic_u8_2x224.npy"))
    ref = np.load(os.path.join(GOLDEN, "synthetic_embedding_2layer_seed1907.npy"))
    got = embed_cls(np.stack([preprocess(x) for x in imgs]), sd)
    assert np.abs(got - ref).max() < 1e-4


def test_vit_oracle_full_model_matches_transformers_golden():
    sd = seeded_vit_msn_weights(1907)
    img = np.array(Image.open(os.path.join(GOLDEN, "test_image.jpeg")).convert("RGB"))
    ref = np.load(os.path.join(GOLDEN, "test_image_embedding_seed1907.npy"))
    got = embed_cls(preprocess(img)[None], sd)[0]
    assert np.abs(got - ref).max() < 1e-4
    assert 1 - cosine(got, ref) < 1e-9


def test_weights_layout_matches_vit_msn_state_dict():
    shapes = dict(vit_msn_shapes())
    assert len(shapes) == 198
    assert shapes["encoder.layer.11.intermediate.dense.weight"] == (3072, 768)


def test_cosine_topk_golden():
    emb = np.load(os.path.join(GOLDEN, "test_image_embedding_seed1907.npy"))
    X, planted = planted_index(emb)
    rows, scores = cosine_topk(X, emb, 5)
    assert rows[0].tolist() == G["top5_rows"] == planted
    assert np.allclose(scores[0], G["top5_scores"], atol=1e-12)


def test_cosine_topk_f32_path_agrees_with_f64():
    rng = np.random.default_rng(4)
    X = rng.standard_normal((20000, 512)).astype(np.float32)
    Xn = (X / np.linalg.norm(X, axis=1, keepdims=True)).astype(np.float32)
    q = rng.standard_normal(512).astype(np.float32)
    r32, s32 = cosine_topk_f32(Xn, q, 10)
    r64, s64 = cosine_topk(Xn, q, 10, rows_normalized=True)
    assert topk_equal_modulo_ties(r32, s32, r64[0], s64[0])


def test_tie_rule_row_ascending():
    X = np.ones((10, 4), dtype=np.float32)
    r, s = cosine_topk(X, np.ones(4), 3)
    assert r[0].tolist() == [0, 1, 2]


def test_massive_activation_weights_shape_the_residual_stream():
    """oracle.weights.with_massive_activations: only the named channels of the patch bias,
    fc2 biases and LayerNorm gammas change, and the residual stream then carries them at
    ~100x the other channels on the patch tokens (40 after the embedding, +20 per layer, vs ~0.5)."""
    import oracle.vit as V
    from oracle.weights import with_massive_activations

    sd = seeded_vit_msn_weights(1907, num_layers=2)
    mv = with_massive_activations(sd, channels=(3, 700))
    changed = sorted(k for k in sd if not np.array_equal(sd[k], mv[k]))
    assert changed == sorted(["embeddings.patch_embeddings.projection.bias", "layernorm.weight"] +
                             [f"encoder.layer.{i}.{n}" for i in range(2)
                              for n in ("output.dense.bias", "layernorm_before.weight", "layernorm_after.weight")])
    for k in changed:
        d = np.nonzero(sd[k] != mv[k])[0]
        assert set(d.tolist()) <= {3, 700}
    seen = []
    orig = V._ln
    try:
        V._ln = lambda x, w, b: (seen.append(np.abs(x[:, 1:, [3, 700]]).min() / np.median(np.abs(x))), orig(x, w, b))[1]
        rng = np.random.default_rng(0)
        out = embed_cls(preprocess(rng.integers(0, 256, (224, 224, 3), dtype=np.uint8))[None], mv)
    finally:
        V._ln = orig
    assert np.isfinite(out).all()
    assert min(seen) > 50  # the outlier channels stay far above the rest on every patch token
