#!/usr/bin/env python3
"""Timing-diagnostic builds of libsnrse_hip.so (results are WRONG under them; never used by tests or
bench): one library per ablation macro of the v7 halo GEMM, under snr-aligned_diffse_amd/lib/abl_*/.
Run a micro-bench against one with SNRSE_LIB=<path>."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snr-aligned_diffse_amd"))
from snrse.build import LIBDIR, build_library  # noqa: E402

ABL = {"nosync": ["-DSNRSE_H7_ABL_NOSYNC"], "noepi": ["-DSNRSE_H7_ABL_NOEPI"], "nohalo": ["-DSNRSE_H7_ABL_NOHALO"],
       "mfma_only": ["-DSNRSE_H7_ABL_NOSYNC", "-DSNRSE_H7_ABL_NOEPI", "-DSNRSE_H7_ABL_NOHALO"]}
for name in (sys.argv[1:] or list(ABL)):
    lib = os.path.join(LIBDIR, f"abl_{name}", "libsnrse_hip.so")
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    print(build_library(force=False, extra_flags=ABL[name], lib=lib))
