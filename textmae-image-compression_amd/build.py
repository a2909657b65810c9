"""Build libtmae.so (gfx950) in-tree with hipcc.

Objects are compiled in parallel and cached by source mtime; the shared library lands in
``<pkg>/lib/libtmae.so`` so it travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_DIR = os.path.join(PKG_DIR, "lib")
OBJ_DIR = os.path.join(LIB_DIR, "obj")
LIB_PATH = os.path.join(LIB_DIR, "libtmae.so")
INCLUDE = os.path.join(os.path.dirname(PKG_DIR), "include")
ARCH = os.environ.get("TMAE_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")

FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", f"-I{INCLUDE}", "-Wno-unused-result"]
HOST_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"-I{INCLUDE}", "-Wall"]
# per-source extras.  attention.hip: the softmax max trees take MFMA results through loop phis, where IEEE-mode
# fmaxf would first quiet each operand (one v_max_f32 x, x per score); scores are finite or the -inf mask.
EXTRA = {"attention.hip": ["-fno-honor-nans"], "qkv_attn.hip": ["-fno-honor-nans"]}


def _sources():
    """device sources (*.hip, hipcc) and host-only sources (*.cpp: the entropy coder, g++)"""
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _deps_mtime():
    files = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    files.append(os.path.join(INCLUDE, "tmae.h"))
    return max(os.path.getmtime(f) for f in files)


def _compile(src: str, hdr_mtime: float, verbose: bool) -> str:
    obj = os.path.join(OBJ_DIR, os.path.basename(src) + ".o")
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_mtime):
        return obj
    if src.endswith(".cpp"):
        cmd = [CXX, *HOST_FLAGS, "-c", src, "-o", obj]
    else:
        cmd = [HIPCC, *FLAGS, *EXTRA.get(os.path.basename(src), []), "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{cmd[0]} failed for {src}:\n{r.stderr}")
    return obj


def build(verbose: bool = False, jobs: int | None = None) -> str:
    os.makedirs(OBJ_DIR, exist_ok=True)
    srcs = _sources()
    hdr = _deps_mtime()
    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 4) // 2), 8)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr, verbose), srcs))
    newest = max(os.path.getmtime(o) for o in objs)
    if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < newest:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB_PATH, *objs]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    return LIB_PATH


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
