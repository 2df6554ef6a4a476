"""Minimal ``multipart/form-data`` parsing for the ``/embed`` upload.

FastAPI's ``UploadFile = File(...)`` needs ``python-multipart`` (reference pin
``embedding/requirements.txt:6``), which this image does not ship; the route
therefore reads the raw body and parses it with the standard library.  The
HTTP contract is unchanged: field ``file``, 422 when it is missing.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from email.parser import BytesParser
from email.policy import HTTP


@dataclass
class FormFile:
    filename: str | None
    content_type: str | None
    data: bytes


_TOKEN = re.compile(rb'\s*([^\s=;]+)\s*(?:=\s*("(?:[^"\\]|\\.)*"|[^;]*))?\s*(?:;|$)')


def _params(value: bytes) -> tuple[bytes, dict[str, str]] | None:
    """'form-data; name="file"; filename="a.jpg"' -> (b"form-data", {"name": "file", ...});
    None for anything this fast path leaves to the email parser (RFC 2231 ``*`` parameters)."""
    head, _, rest = value.partition(b";")
    out: dict[str, str] = {}
    for m in _TOKEN.finditer(rest):
        if not m.group(0).strip():
            continue
        key = m.group(1).decode("latin-1").lower()
        if key.endswith("*"):
            return None
        v = (m.group(2) or b"").strip()
        if v[:1] == b'"' and v[-1:] == b'"' and len(v) >= 2:
            v = re.sub(rb'\\(.)', rb'\1', v[1:-1])
        out[key] = v.decode("utf-8", "surrogateescape")
    return head.strip().lower(), out


def _parse_fast(body: bytes, content_type: str) -> dict[str, list[FormFile]] | None:
    """Direct split on the boundary (the common shape every HTTP client sends: CRLF lines, no
    Content-Transfer-Encoding, plain parameters).  None → the email parser decides."""
    kind = _params(content_type.encode("latin-1"))
    if kind is None or not kind[1].get("boundary"):
        return None
    delim = b"--" + kind[1]["boundary"].encode("latin-1")
    first = body.find(delim)
    if first < 0 or (first > 0 and body[first - 2:first] != b"\r\n"):
        return None
    out: dict[str, list[FormFile]] = {}
    pos = first + len(delim)
    sep = b"\r\n" + delim
    while True:
        if body[pos:pos + 2] == b"--":
            return out
        if body[pos:pos + 2] != b"\r\n":
            return None
        end = body.find(sep, pos + 2)
        if end < 0:
            return None
        part = body[pos + 2:end]
        hend = part.find(b"\r\n\r\n")
        if hend < 0:
            return None
        name = filename = None
        ctype = "text/plain"
        for line in part[:hend].split(b"\r\n"):
            key, colon, value = line.partition(b":")
            if not colon or line[:1] in (b" ", b"\t"):
                return None
            key = key.strip().lower()
            if key == b"content-disposition":
                pv = _params(value)
                if pv is None or pv[0] != b"form-data":
                    return None
                name, filename = pv[1].get("name"), pv[1].get("filename")
            elif key == b"content-type":
                pv = _params(value)
                if pv is None:
                    return None
                ctype = pv[0].decode("latin-1") if pv[0].count(b"/") == 1 else "text/plain"
            elif key == b"content-transfer-encoding":
                return None
        if name:
            out.setdefault(name, []).append(FormFile(filename, ctype, part[hend + 4:]))
        pos = end + len(sep)


def parse_form_all(body: bytes, content_type: str) -> dict[str, list[FormFile]]:
    """Every part of a multipart/form-data body, by field name, in body order (repeated
    fields — ``files`` of the batched routes — keep all their parts).  A body that is not
    multipart yields {} (the routes answer 422 for the missing field, as FastAPI does).
    The common shape is split directly on the boundary (~20x faster than the email parser on
    a 10 KB upload); anything else goes through the standard library's parser."""
    if not content_type or not content_type.lower().startswith("multipart/form-data"):
        return {}
    fast = _parse_fast(body, content_type)
    if fast is not None:
        return fast
    head = b"Content-Type: " + content_type.encode("latin-1") + b"\r\nMIME-Version: 1.0\r\n\r\n"
    msg = BytesParser(policy=HTTP).parsebytes(head + body)
    if not msg.is_multipart():
        return {}
    out: dict[str, list[FormFile]] = {}
    for part in msg.iter_parts():
        name = part.get_param("name", header="content-disposition")
        if not name:
            continue
        data = part.get_payload(decode=True)
        if data is None:
            data = b""
        out.setdefault(str(name), []).append(FormFile(part.get_filename(), part.get_content_type(), data))
    return out


def parse_form(body: bytes, content_type: str) -> dict[str, FormFile]:
    """One part per field (a repeated field keeps its last part, as Starlette's form.get does)."""
    return {k: v[-1] for k, v in parse_form_all(body, content_type).items()}
