"""Per-level precision budget of the fp32x3 parity mode, by CPU emulation on the reference's
N=5 OUVE PC golden (tests/golden/pc_ouve.npz), as tools/x3_emulate.py does for the whole network: every conv of the
oracle network is computed as the split-bf16 sum hi.hi + hi.lo + lo.hi (the fp32x3 kernels' three products), except
the convs whose input lies at resolution level LEVEL (input height 256 >> LEVEL on the golden's [2, 2, 256, 64]
grid), which use the single product bf16(x).bf16(w) with fp32 accumulation -- the GEMM a one-product (bf16-rate)
kernel would compute there, fp32 activations unchanged.  Reports the absolute RMS error of the PC output against
the golden for each level, and for the all-x3 baseline.  Usage: python tools/x3_level_emulate.py [levels...]
Test infrastructure: reads oracle/ and tests/."""
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "snr-aligned_diffse_amd")]
torch.set_num_threads(int(os.environ.get("EMU_THREADS", "8")))
from conftest import fnormal, golden  # noqa: E402
from oracle import ncsnpp_ref, sde_ref  # noqa: E402
from snrse import formula  # noqa: E402
from test_oracle_golden import Tape  # noqa: E402


def split(x):
    h = x.to(torch.bfloat16).float()
    return h, (x - h).to(torch.bfloat16).float()


LEVEL = None


def conv_emu(x, sd, pre, pad):
    w, b = sd[pre + ".weight"], sd[pre + ".bias"]
    (xh, xl), (wh, wl) = split(x), split(w)
    if LEVEL is not None and x.shape[2] == 256 >> LEVEL:
        out = F.conv2d(xh, wh, None, padding=pad)
    else:
        out = F.conv2d(xh, wh, None, padding=pad) + F.conv2d(xh, wl, None, padding=pad) + F.conv2d(xl, wh, None, padding=pad)
    return out + b[None, :, None, None]


def run(level):
    global LEVEL
    LEVEL = level
    ncsnpp_ref.conv = conv_emu
    with open(os.path.join(ROOT, "tests", "golden", "state_dict_keys.json")) as f:
        shapes = {k: tuple(s) for k, s in json.load(f)["ncsnpp"]}
    sd = ncsnpp_ref.state_dict_to_torch(formula.formula_state_dict(shapes))
    g = golden("pc_ouve.npz")
    Y = torch.from_numpy(fnormal("golden.pc.Y", (2, 1, 256, 64), complex_=True)) * 0.5
    sde = sde_ref.OUVE(1.5, 0.05, 0.5, N=5)

    def score_fn(x, t, y):
        tt = torch.full((x.shape[0],), t, dtype=torch.float32)
        return -ncsnpp_ref.ncsnpp_forward(torch.cat([x, y], 1), tt, sd)

    t0 = time.time()
    xr, _ = sde_ref.pc_sample(sde, score_fn, Y, Tape("golden.pc.noise"))
    d = xr.numpy() - g["out"]
    return {"bf16_level": level, "abs_rms": float(np.sqrt(np.mean(np.abs(d) ** 2))),
            "max_abs": float(np.abs(d).max()), "seconds": round(time.time() - t0, 1)}


if __name__ == "__main__":
    levels = [None if a == "none" else int(a) for a in sys.argv[1:]] or [None, 0, 1, 2, 3, 4, 5, 6]
    for lv in levels:
        print(json.dumps(run(lv)), flush=True)
