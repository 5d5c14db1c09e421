"""Build a variant of libsegamd.so with extra compile flags, for A/B timing.

    python tools/variant.py NAME [--only a.hip,b.hip] [-DFOO=1 ...]   ->  variants/NAME.so  (travels with gpurun;
git-ignored).  --only: compile just those sources with the extra flags and link the main build's objects
(seg_amd/_lib/obj, current after __graft_entry__.build()) for the rest -- minutes instead of a full rebuild.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "team02-objectdetection_amd"))
from seg_amd.build import ARCH, FLAGS, GEN_DIR, HIPCC, OUT_DIR, _write_hash_source, source_hash, sources  # noqa: E402


def main():
    name, extra = sys.argv[1], sys.argv[2:]
    only = None
    if extra[:1] == ["--only"]:
        only, extra = set(extra[1].split(",")), extra[2:]
    odir = os.path.join(REPO, "tmp_var", name)  # objects stay here (gpurun-ignored)
    os.makedirs(odir, exist_ok=True)

    def one(src):
        if only is not None and os.path.basename(src) not in only:
            return os.path.join(OUT_DIR, "obj", os.path.basename(src)[:-4] + ".o")
        obj = os.path.join(odir, os.path.basename(src)[:-4] + ".o")
        r = subprocess.run([HIPCC, *FLAGS, *extra, "-c", src, "-o", obj], capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(r.stderr)
        return obj
    with ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(one, sources()))
    os.makedirs(GEN_DIR, exist_ok=True)
    hobj = os.path.join(odir, "build_hash.o")  # seg_build_hash: the tree's hash (SEG_LIB_PATH skips the check)
    subprocess.run([HIPCC, "-O2", "-fPIC", "-c", _write_hash_source(source_hash()), "-o", hobj], check=True)
    objs.append(hobj)
    os.makedirs(os.path.join(REPO, "variants"), exist_ok=True)
    out = os.path.join(REPO, "variants", name + ".so")
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out, *objs], check=True)
    print(out)


if __name__ == "__main__":
    main()
