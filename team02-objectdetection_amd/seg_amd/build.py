"""Build libsegamd.so (all HIP kernels + the C-ABI) for gfx950 with hipcc.

No torch.utils.cpp_extension: the library is a plain C-ABI shared object
(include/segamd.h) so any FFI can bind it; Python binds it with ctypes
(seg_amd/_lib.py).  The object links libamdhip64.so.7 by soname, so inside a
process that imported torch it shares torch's HIP runtime (and its streams).
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(PKG_DIR), "csrc")
OUT_DIR = os.path.join(PKG_DIR, "_lib")
LIB_PATH = os.path.join(OUT_DIR, "libsegamd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-Wno-unused-result"]


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _stale(obj, src):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    deps = [src] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, jobs: int = 8) -> str:
    os.makedirs(os.path.join(OUT_DIR, "obj"), exist_ok=True)
    srcs = sources()
    objs = [os.path.join(OUT_DIR, "obj", os.path.basename(s)[:-4] + ".o") for s in srcs]

    def compile_one(so):
        s, o = so
        if not _stale(o, s):
            return None
        cmd = [HIPCC, *FLAGS, "-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {s}:\n{r.stderr}")
        return o

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(compile_one, zip(srcs, objs)))
    if not os.path.exists(LIB_PATH) or any(os.path.getmtime(o) > os.path.getmtime(LIB_PATH) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB_PATH, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    return LIB_PATH


if __name__ == "__main__":
    print(build(verbose=True))
