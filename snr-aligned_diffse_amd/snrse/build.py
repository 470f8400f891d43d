"""Build libsnrse_hip.so from csrc/*.hip (+ abi.cpp) with hipcc for gfx950, in-tree.

Plain `hipcc -shared -fPIC` — no torch types cross the boundary, so no cpp_extension.
Objects go to lib/obj/, the library to lib/libsnrse_hip.so (git-ignored, travels to the
GPU box with the gpurun snapshot).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import time

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libsnrse_hip.so")
ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-Wno-unused-result"]
# Files whose kernels interleave VALU work with MFMAs: no SLP vectorisation, which otherwise packs
# adjacent f32 adds / muls / fmas into v_pk_*_f32 -- slower than the scalar forms beside MFMAs
# (MI355X_MICROARCH.md, 'price of one filler beside MFMAs'; measured +1.8 % C2 utt/s, halo GEMM
# 703 -> 686 us per launch, profiles/r02n_noslp_ab.json)
FILE_FLAGS = {name: ["-fno-slp-vectorize"] for name in ("conv.hip", "conv_head.hip", "attn.hip", "score.hip",
                                                          "train.hip")}


def _sources(csrc=CSRC):
    return sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.cpp")))


def _headers(csrc=CSRC):
    return glob.glob(os.path.join(csrc, "*.h"))


def source_hash(csrc=CSRC) -> str:
    """sha256 over the library's sources (csrc/*.hip, *.cpp, *.h) and this build script, by content:
    compiled into the library as snrse_build_id() and written beside it as libsnrse_hip.so.id."""
    h = hashlib.sha256()
    for f in sorted(_sources(csrc) + _headers(csrc), key=os.path.basename) + [os.path.abspath(__file__)]:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


# what the latest build_library() call did (printed by __graft_entry__.build())
LAST_BUILD = {"compiled": False, "build_id": None, "seconds": 0.0, "lib": LIB}


def needs_build() -> bool:
    """The library is rebuilt unless it exists and its recorded source hash equals the tree's (content,
    not mtimes: a checkout or a copy that touches no bytes does not rebuild, an edit always does)."""
    if not os.path.exists(LIB):
        return True
    try:
        with open(LIB + ".id") as f:
            return f.read().strip() != source_hash()
    except OSError:
        return True


def _compile(src: str, obj: str, extra=()):
    cmd = [HIPCC, *FLAGS, *FILE_FLAGS.get(os.path.basename(src), []), *extra, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def _read(path: str):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _obj_key(src: str, common: str, extra=()) -> str:
    """Content key of one object: its source, the shared headers + build script (`common`) and its flags."""
    h = hashlib.sha256(common.encode())
    h.update(" ".join([*FLAGS, *FILE_FLAGS.get(os.path.basename(src), []), *extra]).encode())
    with open(src, "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()


def build_library(force: bool = False, jobs: int = 8, extra_flags=(), lib: str = LIB, csrc: str = CSRC) -> str:
    """Build `lib`.  `extra_flags` (e.g. -DSNRSE_STAMPS for the timing-diagnostic build) go to
    every compile; such builds use their own object directory next to `lib`.  `csrc` selects another
    source tree (A/B builds of an earlier revision, tools/build_variant.py)."""
    bid = source_hash(csrc)
    LAST_BUILD.update(compiled=False, build_id=bid, seconds=0.0, lib=lib)
    if lib == LIB and not force and not needs_build():
        return LIB
    t0 = time.time()
    objdir = os.path.join(os.path.dirname(lib), "obj")
    os.makedirs(objdir, exist_ok=True)
    # objects are reused only when their recorded key -- sha256 of the source, every header, this script and the
    # compile flags, by content -- matches, so the linked objects are the tree's (an mtime-preserving copy of an old
    # object is recompiled); abi.cpp carries the build id and is always recompiled
    common = hashlib.sha256()
    for f in sorted(_headers(csrc), key=os.path.basename) + [os.path.abspath(__file__)]:
        common.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            common.update(fh.read())
    todo, objs = [], []
    for src in _sources(csrc):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        key = _obj_key(src, common.hexdigest(), tuple(extra_flags))
        if force or os.path.basename(src) == "abi.cpp" or _read(obj + ".id") != key or not os.path.exists(obj):
            todo.append((src, obj, key))
    idflag = (f'-DSNRSE_BUILD_ID="{bid}"',)
    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo) or 1))) as ex:
        futs = [(ex.submit(_compile, s, o, tuple(extra_flags) + (idflag if os.path.basename(s) == "abi.cpp" else ())),
                 o, k) for s, o, k in todo]
        for f, o, k in futs:
            f.result()
            with open(o + ".id", "w") as fh:
                fh.write(k + "\n")
    tmp = lib + ".tmp"
    r = subprocess.run([HIPCC, "-shared", f"--offload-arch={ARCH}", *objs, "-o", tmp],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, lib)
    with open(lib + ".id", "w") as f:
        f.write(bid + "\n")
    LAST_BUILD.update(compiled=True, seconds=round(time.time() - t0, 1))
    return lib


if __name__ == "__main__":
    print(build_library(force=True))
