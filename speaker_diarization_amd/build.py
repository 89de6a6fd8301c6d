"""Build libsdiar.so (HIP kernels + C ABI) for gfx950 with hipcc, in-tree.

Usage: python -m speaker_diarization_amd.build [--force]
Objects are cached under speaker_diarization_amd/lib/obj keyed by source hash.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
OBJDIR = os.path.join(LIBDIR, "obj")
LIB = os.path.join(LIBDIR, "libsdiar.so")
ARCH = os.environ.get("SDIAR_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result",
          "-munsafe-fp-atomics"]


def _sources():
    return sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _headers_digest():
    h = hashlib.sha256()
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(".h"):
            h.update(open(os.path.join(CSRC, f), "rb").read())
    inc = os.path.join(os.path.dirname(PKG), "include", "sdiar.h")
    if os.path.exists(inc):
        h.update(open(inc, "rb").read())
    return h.hexdigest()


def _file_flags(path: str) -> list:
    """Extra compiler flags a source asks for on a line `// sdiar-build: <flags>` (e.g. LLVM options)."""
    out = []
    for line in open(path, encoding="utf-8"):
        if line.startswith("// sdiar-build:"):
            out += line.split(":", 1)[1].split()
    return out


def _compile(src: str, hdr: str, force: bool) -> str:
    path = os.path.join(CSRC, src)
    flags = CFLAGS + _file_flags(path)
    key = hashlib.sha256(open(path, "rb").read() + hdr.encode() + " ".join(flags).encode())
    obj = os.path.join(OBJDIR, f"{src}.{key.hexdigest()[:16]}.o")
    if os.path.exists(obj) and not force:
        return obj
    cmd = [HIPCC, *flags, "-x", "hip", "-c", path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    hdr = _headers_digest()
    srcs = _sources()
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr, force), srcs))
    newest = max(os.path.getmtime(o) for o in objs)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        tmp = LIB + ".tmp"
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        os.replace(tmp, LIB)
        if verbose:
            print(f"[sdiar] built {LIB}")
    # drop stale objects
    keep = set(objs)
    for f in os.listdir(OBJDIR):
        p = os.path.join(OBJDIR, f)
        if p not in keep:
            os.remove(p)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    try:
        build(force=a.force)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
