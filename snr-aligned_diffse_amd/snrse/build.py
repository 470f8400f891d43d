"""Build libsnrse_hip.so from csrc/*.hip (+ abi.cpp) with hipcc for gfx950, in-tree.

Plain `hipcc -shared -fPIC` — no torch types cross the boundary, so no cpp_extension.
Objects go to lib/obj/, the library to lib/libsnrse_hip.so (git-ignored, travels to the
GPU box with the gpurun snapshot).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess

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


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(f) > t for f in _sources() + _headers() + [os.path.abspath(__file__)])


def _compile(src: str, obj: str, extra=()):
    cmd = [HIPCC, *FLAGS, *FILE_FLAGS.get(os.path.basename(src), []), *extra, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build_library(force: bool = False, jobs: int = 8, extra_flags=(), lib: str = LIB, csrc: str = CSRC) -> str:
    """Build `lib`.  `extra_flags` (e.g. -DSNRSE_STAMPS for the timing-diagnostic build) go to
    every compile; such builds use their own object directory next to `lib`.  `csrc` selects another
    source tree (A/B builds of an earlier revision, tools/build_variant.py)."""
    if lib == LIB and not force and not needs_build():
        return LIB
    objdir = os.path.join(os.path.dirname(lib), "obj")
    os.makedirs(objdir, exist_ok=True)
    hdr_t = max([os.path.getmtime(h) for h in _headers(csrc) + [os.path.abspath(__file__)]] + [0.0])
    todo, objs = [], []
    for src in _sources(csrc):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_t):
            todo.append((src, obj))
    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo) or 1))) as ex:
        for f in [ex.submit(_compile, s, o, tuple(extra_flags)) for s, o in todo]:
            f.result()
    tmp = lib + ".tmp"
    r = subprocess.run([HIPCC, "-shared", f"--offload-arch={ARCH}", *objs, "-o", tmp],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    print(build_library(force=True))
