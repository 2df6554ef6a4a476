"""Local-checkpoint loading (the offline stand-in for ``from_pretrained("facebook/vit-msn-base")``,
reference ``embedding/main.py:37-38``).

A checkpoint directory is written in each key layout a real ViT-MSN checkpoint can carry:
the legacy transformers-4 layout (``encoder.layer.N.attention.attention.query``), the
transformers-5 module names (``layers.N.attention.q_proj``, ``oracle/weights.py:to_hf_v5``),
and the ``ViTMSNForImageClassification`` form (``vit.`` prefix, classifier head, mask token).
``load_checkpoint_dir`` + ``canonical_state_dict`` must give the same tensors for all three,
and must raise on unknown or missing keys — before any GPU work.  No GPU needed; the GPU
test (tests/test_embed_gpu.py::test_from_pretrained_v5_layout_matches_golden) embeds through
the loaded directory.
"""
import json
import os

import numpy as np
import pytest

from conftest import import_pkg
from oracle.weights import seeded_vit_msn_weights, to_hf_v5


@pytest.fixture(scope="module")
def vitmod():
    return import_pkg("vit")


@pytest.fixture(scope="module")
def sd2():
    return seeded_vit_msn_weights(1907, num_layers=2)


def _write(path, sd, layers=2, preprocessor=None, fmt="safetensors"):
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump({"model_type": "vit-msn", "hidden_size": 768, "num_hidden_layers": layers, "num_attention_heads": 12,
                   "intermediate_size": 3072, "image_size": 224, "patch_size": 16, "layer_norm_eps": 1e-6}, f)
    if preprocessor is not None:
        with open(os.path.join(path, "preprocessor_config.json"), "w") as f:
            json.dump(preprocessor, f)
    if fmt == "safetensors":
        from safetensors.numpy import save_file

        save_file({k: np.ascontiguousarray(v) for k, v in sd.items()}, os.path.join(path, "model.safetensors"))
    else:
        import torch

        torch.save({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()},
                   os.path.join(path, "pytorch_model.bin"))


def _classifier_form(sd):
    out = {"vit." + k: v for k, v in sd.items()}
    out["vit.embeddings.mask_token"] = np.zeros((1, 1, 768), np.float32)
    out["classifier.weight"] = np.zeros((1000, 768), np.float32)
    out["classifier.bias"] = np.zeros((1000,), np.float32)
    return out


@pytest.mark.parametrize("layout", ["legacy", "v5", "classifier", "legacy-bin"])
def test_every_layout_loads_to_the_same_state(vitmod, sd2, tmp_path, layout):
    sd = {"legacy": sd2, "legacy-bin": sd2, "v5": to_hf_v5(sd2), "classifier": _classifier_form(sd2)}[layout]
    d = str(tmp_path / layout)
    _write(d, sd, fmt="bin" if layout.endswith("bin") else "safetensors")
    got, cfg, pre = vitmod.load_checkpoint_dir(d)
    assert cfg["num_hidden_layers"] == 2 and cfg["hidden_size"] == 768
    canon = vitmod.canonical_state_dict(got, cfg["num_hidden_layers"])
    assert sorted(canon) == sorted(sd2)
    for k, v in sd2.items():
        assert np.array_equal(np.asarray(canon[k]), v), k


def test_preprocessor_config_is_read(vitmod, sd2, tmp_path):
    d = str(tmp_path / "pre")
    _write(d, sd2, preprocessor={"resample": 2, "rescale_factor": 0.5, "image_mean": [0.5, 0.5, 0.5],
                                 "image_std": [0.25, 0.25, 0.25], "size": {"height": 224, "width": 224}})
    _, _, pre = vitmod.load_checkpoint_dir(d)
    assert pre["resample"] == 2 and pre["rescale_factor"] == 0.5
    assert tuple(pre["image_mean"]) == (0.5, 0.5, 0.5) and tuple(pre["image_std"]) == (0.25, 0.25, 0.25)


def test_unknown_key_raises(vitmod, sd2, tmp_path):
    bad = dict(sd2)
    bad["encoder.layer.0.attention.attention.qkv.weight"] = np.zeros((2304, 768), np.float32)  # a fused-QKV layout
    d = str(tmp_path / "unknown")
    _write(d, bad)
    got, cfg, _ = vitmod.load_checkpoint_dir(d)
    with pytest.raises(ValueError, match="unknown checkpoint keys"):
        vitmod.canonical_state_dict(got, cfg["num_hidden_layers"])


def test_missing_key_raises(vitmod, sd2, tmp_path):
    bad = {k: v for k, v in to_hf_v5(sd2).items() if "layers.1.mlp.fc2.weight" not in k}
    d = str(tmp_path / "missing")
    _write(d, bad)
    got, cfg, _ = vitmod.load_checkpoint_dir(d)
    with pytest.raises(ValueError, match="missing"):
        vitmod.canonical_state_dict(got, cfg["num_hidden_layers"])


def test_mixed_layouts_naming_one_tensor_twice_raises(vitmod, sd2):
    both = dict(sd2)
    both["layers.0.attention.q_proj.weight"] = sd2["encoder.layer.0.attention.attention.query.weight"]
    with pytest.raises(ValueError, match="twice"):
        vitmod.canonical_state_dict(both, 2)


def test_layer_count_mismatch_raises(vitmod, sd2):
    with pytest.raises(ValueError, match="missing"):
        vitmod.canonical_state_dict(sd2, 3)  # config claims 3 layers, the file holds 2
