#!/usr/bin/env python3
"""A/B builds of libsnrse_hip.so: `tools/build_variant.py NAME [--rev GITREV] [-DMACRO=V ...]` builds
snr-aligned_diffse_amd/lib/var_NAME/libsnrse_hip.so from the working tree (or from the csrc/ of git
revision GITREV) with extra compile flags.  Select one at run time with SNRSE_LIB=<path>."""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snr-aligned_diffse_amd"))
from snrse.build import CSRC, LIBDIR, build_library  # noqa: E402

name, args = sys.argv[1], sys.argv[2:]
rev = None
if "--rev" in args:
    i = args.index("--rev")
    rev = args[i + 1]
    args = args[:i] + args[i + 2:]
csrc = CSRC
if rev:
    csrc = tempfile.mkdtemp(prefix=f"csrc_{name}_")
    files = subprocess.run(["git", "-C", ROOT, "ls-tree", "--name-only", rev, "snr-aligned_diffse_amd/csrc/"],
                           check=True, capture_output=True, text=True).stdout.split()
    for f in files:
        blob = subprocess.run(["git", "-C", ROOT, "show", f"{rev}:{f}"], check=True, capture_output=True).stdout
        with open(os.path.join(csrc, os.path.basename(f)), "wb") as fh:
            fh.write(blob)
lib = os.path.join(LIBDIR, f"var_{name}", "libsnrse_hip.so")
os.makedirs(os.path.dirname(lib), exist_ok=True)
print(build_library(force=True, extra_flags=args, lib=lib, csrc=csrc))
