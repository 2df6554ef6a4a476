"""Minimal ``multipart/form-data`` parsing for the ``/embed`` upload.

FastAPI's ``UploadFile = File(...)`` needs ``python-multipart`` (reference pin
``embedding/requirements.txt:6``), which this image does not ship; the route
therefore reads the raw body and parses it with the standard library.  The
HTTP contract is unchanged: field ``file``, 422 when it is missing.
"""
from __future__ import annotations

from dataclasses import dataclass
from email.parser import BytesParser
from email.policy import HTTP


@dataclass
class FormFile:
    filename: str | None
    content_type: str | None
    data: bytes


def parse_form_all(body: bytes, content_type: str) -> dict[str, list[FormFile]]:
    """Every part of a multipart/form-data body, by field name, in body order (repeated
    fields — ``files`` of the batched routes — keep all their parts).  A body that is not
    multipart yields {} (the routes answer 422 for the missing field, as FastAPI does)."""
    if not content_type or not content_type.lower().startswith("multipart/form-data"):
        return {}
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
