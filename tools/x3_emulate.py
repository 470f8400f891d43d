"""CPU emulation of the split-bf16 ("x3") fp32 GEMM arithmetic on the reference's N=5 OUVE PC golden
(tests/golden/pc_ouve.npz): the oracle network with every ResBlock / input / head conv computed as
sum over (i, j) in TERMS of conv(x_i, w_j), x_0 = bf16(x), x_1 = bf16(x - x_0) (and a third piece for x3).
Usage: python tools/x3_emulate.py fp32|x2|x22|x3.  Test infrastructure: reads oracle/ and tests/.
Results (8 cores): fp32 3.3e-6, x2 (the kernel's three products) 6.0e-5, x22 (+ lo*lo) 5.7e-5 abs RMS."""
import os, sys, time, numpy as np, torch, torch.nn.functional as F
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'snr-aligned_diffse_amd')]
torch.set_num_threads(8)
from conftest import fnormal, golden
from oracle import ncsnpp_ref, sde_ref
from snrse import formula
import json
MODE = sys.argv[1]
def split(x, n):
    parts = []; r = x
    for _ in range(n):
        h = r.to(torch.bfloat16).float(); parts.append(h); r = r - h
    return parts
def mm_terms(n):
    if n == 2: return [(0,0),(0,1),(1,0)]
    if n == 22: return [(0,0),(0,1),(1,0),(1,1)]
    if n == 3: return [(0,0),(0,1),(1,0),(0,2),(2,0),(1,1)]
orig_conv = ncsnpp_ref.conv
def conv_emu(x, sd, pre, pad):
    w, b = sd[pre + '.weight'], sd[pre + '.bias']
    n = {'x2': 2, 'x22': 22, 'x3': 3}[MODE]
    ns = 3 if n == 3 else 2
    xs, ws = split(x, ns), split(w, ns)
    out = None
    for i, j in mm_terms(n):
        o = F.conv2d(xs[i], ws[j], None, padding=pad)
        out = o if out is None else out + o
    return out + b[None, :, None, None]
if MODE != 'fp32':
    ncsnpp_ref.conv = conv_emu
with open(os.path.join(ROOT, 'tests', 'golden', 'state_dict_keys.json')) as f:
    shapes = {k: tuple(s) for k, s in json.load(f)['ncsnpp']}
sd = ncsnpp_ref.state_dict_to_torch(formula.formula_state_dict(shapes))
g = golden('pc_ouve.npz')
Y = torch.from_numpy(fnormal('golden.pc.Y', (2, 1, 256, 64), complex_=True)) * 0.5
sde = sde_ref.OUVE(1.5, 0.05, 0.5, N=5)
def score_fn(x, t, y):
    tt = torch.full((x.shape[0],), t, dtype=torch.float32)
    return -ncsnpp_ref.ncsnpp_forward(torch.cat([x, y], 1), tt, sd)
from test_oracle_golden import Tape
tape = Tape('golden.pc.noise')
t0 = time.time()
xr, ns = sde_ref.pc_sample(sde, score_fn, Y, tape)
d = xr.numpy() - g['out']
print(MODE, 'abs_rms', float(np.sqrt(np.mean(np.abs(d)**2))), 'rel', float(np.sqrt(np.mean(np.abs(d)**2))/np.sqrt(np.mean(np.abs(g['out'])**2))), 'max', float(np.abs(d).max()), f'{time.time()-t0:.0f}s')
