"""Build libhnm_mi355x.so in-tree with hipcc for gfx950 (no JIT cache, no torch ext).

The shared library is the C-ABI boundary declared in include/hnm.h; it is git-ignored
but travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(REPO, "build", "obj")
LIB = os.path.join(PKG, "libhnm_mi355x.so")
SOURCES = ["api.hip", "score.hip", "dot_cert.hip", "ncf.hip", "ncf_cert.hip", "ncf_deep.hip", "graph.hip",
           "widedeep.hip", "eval.hip", "topk_sort.hip", "collective.hip"]
HEADERS = ["hnm_device.h", "hnm_internal.h", "dot_internal.h", "ncf_internal.h", "sample_kth.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall",
         "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-but-set-variable"]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else 0.0


def _deps_mtime():
    paths = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(REPO, "include", "hnm.h")]
    return max(_mtime(p) for p in paths)


def _compile(src):
    obj = os.path.join(BUILD, src.replace(".hip", ".o"))
    srcp = os.path.join(CSRC, src)
    if _mtime(obj) >= max(_mtime(srcp), _deps_mtime()):
        return obj, None
    cmd = [HIPCC, *FLAGS, "-c", srcp, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


def build_library(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    sources = [s for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    if force:
        for s in sources:
            o = os.path.join(BUILD, s.replace(".hip", ".o"))
            if os.path.exists(o):
                os.remove(o)
    with cf.ThreadPoolExecutor(max_workers=min(4, len(sources))) as ex:
        results = list(ex.map(_compile, sources))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _ in results]
    if force or _mtime(LIB) < max(_mtime(o) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB, *objs,
               "-L/opt/rocm/lib", "-lrccl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"built {LIB}", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build_library(force="--force" in sys.argv)
