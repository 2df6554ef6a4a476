"""Build the gfx950 shared library ``lib/libretrieval_core.so`` in-tree with hipcc.

Each ``csrc/*.hip`` is compiled to an object (in parallel, cached by mtime),
then linked with ``-shared``.  No torch extension machinery: the library is a
plain C-ABI ``.so`` that the host layer opens with ctypes.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
OBJDIR = os.path.join(PKG, "lib", "obj")
LIB = os.path.join(LIBDIR, "libretrieval_core.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

CFLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-I" + os.path.join(REPO, "include"),
    "-I" + CSRC,
    "-Wno-unused-result",
    "-munsafe-fp-atomics",
]


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(REPO, "include", "retrieval_core.h"))
    return hs


def _deps(src: str) -> list[str]:
    """src plus every in-tree header it includes, transitively (#include "...")."""
    import re

    seen, todo = [], [src]
    while todo:
        f = todo.pop()
        if f in seen or not os.path.exists(f):
            continue
        seen.append(f)
        for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', open(f).read(), flags=re.M):
            for d in (os.path.dirname(f), CSRC, os.path.join(REPO, "include")):
                cand = os.path.join(d, inc)
                if os.path.exists(cand):
                    todo.append(cand)
                    break
    return seen


def _compile(src: str, extra: list[str]) -> str:
    obj = os.path.join(OBJDIR, os.path.basename(src) + ".o")
    stamp = obj + ".flags"
    flags = " ".join(CFLAGS + extra)
    newest_dep = max(os.path.getmtime(p) for p in [__file__] + _deps(src))
    same_flags = os.path.exists(stamp) and open(stamp).read() == flags
    if same_flags and os.path.exists(obj) and os.path.getmtime(obj) >= newest_dep:
        return obj
    cmd = [HIPCC, *CFLAGS, *extra, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    with open(stamp, "w") as f:
        f.write(flags)
    return obj


def build(verbose: bool = False, extra: list[str] | None = None, jobs: int | None = None) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    extra = list(extra or [])
    srcs = _sources()
    jobs = jobs or min(len(srcs), max(1, min(8, (os.cpu_count() or 4))))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, extra), srcs))
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    build(verbose=True, extra=sys.argv[1:])
