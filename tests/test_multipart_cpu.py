"""The upload parser (``…_amd/multipart.py``): the direct boundary split gives what the standard
library's email parser gives (the parser the routes used before, and still use for any body outside
the common shape), on bodies built by httpx — the encoder behind TestClient and the usual Python
HTTP clients — with binary payloads that contain CRLFs, dashes and boundary-like bytes."""
import random

import httpx
import pytest

from conftest import import_pkg


def _email_parse(body, ctype):
    mp = import_pkg("multipart")
    orig = mp._parse_fast
    mp._parse_fast = lambda b, c: None
    try:
        return mp.parse_form_all(body, ctype)
    finally:
        mp._parse_fast = orig


def _encode(files, data=None):
    req = httpx.Request("POST", "http://x/u", files=files, data=data)
    return req.read(), req.headers["content-type"]


def _same(a, b):
    assert a.keys() == b.keys()
    for k in a:
        assert [(f.filename, f.content_type, f.data) for f in a[k]] == [(f.filename, f.content_type, f.data) for f in b[k]]


@pytest.mark.parametrize("seed", range(12))
def test_fast_split_equals_email_parser(seed):
    mp = import_pkg("multipart")
    rng = random.Random(seed)
    alphabet = [b"\r\n", b"--", b"\r\n--", b"a", b"\x00", b"\xff", b"\r", b"\n", b"-"]
    files = []
    for i in range(rng.randint(1, 4)):
        payload = b"".join(rng.choice(alphabet) + bytes([rng.randrange(256)]) for _ in range(rng.randint(0, 300)))
        name = rng.choice(["file", "files", "files", "x"])
        fname = rng.choice(["a.jpg", "b c.jpeg", 'q"uote.png', "ü.jpg", "x;y.jpg"])
        files.append((name, (fname, payload, rng.choice(["image/jpeg", "application/octet-stream", "IMAGE/PNG"]))))
    body, ctype = _encode(files, data={"note": "hello"} if seed % 3 == 0 else None)
    fast = mp._parse_fast(body, ctype)
    assert fast is not None, "httpx's body shape takes the fast path"
    _same(fast, _email_parse(body, ctype))
    _same(mp.parse_form_all(body, ctype), fast)


def test_unusual_shapes_fall_back():
    mp = import_pkg("multipart")
    body, ctype = _encode([("file", ("a.jpg", b"abc", "image/jpeg"))])
    # a preamble, a quoted boundary, RFC 2231 filename*, a transfer encoding: the email parser decides
    b = body.split(b"\r\n", 1)
    bnd = ctype.split("boundary=")[1]
    assert mp._parse_fast(b"preamble" + body, ctype) is None
    q = f'multipart/form-data; boundary="{bnd}"'
    assert mp._parse_fast(body, q) is not None and mp.parse_form_all(body, q)["file"][0].data == b"abc"
    star = body.replace(b'filename="a.jpg"', b"filename*=utf-8''a.jpg")
    assert mp._parse_fast(star, ctype) is None
    _same(mp.parse_form_all(star, ctype), _email_parse(star, ctype))
    cte = body.replace(b"Content-Type: image/jpeg", b"Content-Type: image/jpeg\r\nContent-Transfer-Encoding: binary")
    assert mp._parse_fast(cte, ctype) is None
    assert mp.parse_form_all(b"x", "text/plain") == {} and len(b) == 2
    assert mp.parse_form(b"", ctype) == {}
