"""JPEG decode, host side (no GPU): the library's header parse and Huffman decoder
plus the oracle's restatement of libjpeg-turbo's reconstruction (oracle/jpeg.py)
reproduce Pillow's decode (embedding/main.py:97) bit for bit; streams outside the
GPU decoder's scope are reported, not mis-decoded."""
import hashlib
import io

import numpy as np
import pytest
from PIL import Image

from conftest import import_pkg
from jpeg_cases import cases, pil_rgb, synthetic
from oracle.jpeg import reconstruct


@pytest.fixture(scope="module")
def J():
    return import_pkg("jpeg")


@pytest.mark.parametrize("name,data", cases(), ids=[c[0] for c in cases()])
def test_host_entropy_decode_plus_oracle_matches_pillow(J, name, data):
    info, coef, qt = J.decode_coefficients(data)
    assert np.array_equal(reconstruct(info, coef, qt), pil_rgb(data))


def test_reference_fixture_decoded_sha(J):
    # decoded test image sha256 prefix 0feedc7d874a0994
    data = dict(cases())["test_image"]
    info, coef, qt = J.decode_coefficients(data)
    rgb = reconstruct(info, coef, qt)
    assert (info.width, info.height) == (168, 300)
    assert hashlib.sha256(rgb.tobytes()).hexdigest()[:16] == "0feedc7d874a0994"


def test_probe_reports_geometry(J):
    info = J.probe(synthetic(33, 17, 5, quality=90, subsampling=2))
    assert (info.width, info.height, info.ncomp, info.supported) == (33, 17, 3, 1)
    assert (list(info.h), list(info.v)) == ([2, 1, 1], [2, 1, 1])
    assert (info.mcux, info.mcuy) == (3, 2)
    assert info.blocks == 3 * 2 * 4 + 2 * (3 * 2)


def test_unsupported_streams_are_reported(J):
    prog = synthetic(64, 64, 7, quality=80, progressive=True)
    assert J.probe(prog).supported == 0
    assert not J.is_gpu_decodable(prog)
    b = io.BytesIO()
    Image.fromarray(np.zeros((8, 8, 4), np.uint8), "RGBA").convert("CMYK").save(b, format="JPEG")
    assert J.probe(b.getvalue()).supported == 0
    with pytest.raises(J.JpegUnsupported):
        J.decode_coefficients(prog)


def test_not_a_jpeg_is_a_value_error(J):
    b = io.BytesIO()
    Image.fromarray(np.zeros((4, 4, 3), np.uint8)).save(b, format="PNG")
    with pytest.raises(ValueError):
        J.probe(b.getvalue())
    assert not J.is_gpu_decodable(b.getvalue())
    assert not J.is_gpu_decodable(b"")


def test_truncated_stream_is_an_error(J):
    data = synthetic(96, 96, 9, quality=90)
    with pytest.raises(ValueError):
        J.decode_coefficients(data[: len(data) // 2])
