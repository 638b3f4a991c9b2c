"""Debug probe: where the split demapper's planes differ from the host chain at
16QAM N=212 r=2/3 (tests/test_gpu_demap_split.py)."""
import sys
import numpy as np
import torch
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import test_gpu_demap_split as T
from oracle import oracle as O
from modulations_amd import demap as D
from modulations_amd import dvb_rcs2_turbo as M

mod, n, rate = "16QAM", 212, "2/3"
rng = np.random.default_rng(sum(map(ord, mod)) + n)
c = M.DVBRCS2_Turbo(n, rate)
bps = 4
S = -(-c.n_coded // bps)
syms = T._adversarial(D.constellation(mod), rng, (130, S))
cons = D.constellation(mod)
_, div32, nve = D.demap_mode(np.complex64, cons.dtype, np.float64(0.04))
B = 130
c.reserve(B)
planes = torch.full((c.planes_bytes(B) // 4,), 7.0, dtype=torch.float32, device="cuda")
c.demap_planes_device(torch.from_numpy(syms).cuda(), cons, bps, nve, planes, div_f32=div32)
flat = syms.reshape(-1)
llr = np.full(flat.size * bps, np.nan, np.float64)
fin = ~np.isnan(flat)
llr.reshape(-1, bps)[fin] = (-O.demap(flat[fin], cons, bps, nve, div_f32=div32)).reshape(-1, bps)
llr = llr.reshape(B, -1)
L = c.handle.llr_len
print("n_coded", c.n_coded, "llr_len", L, "S", S, "S*bps", S * bps)
ref_llr = np.zeros((B, max(c.n_coded, L)), np.float32)
m = min(c.n_coded, llr.shape[1])
ref_llr[:, :m] = llr[:, :m]
ref = torch.empty_like(planes)
c.depuncture_device(torch.from_numpy(ref_llr).cuda(), ref)
torch.cuda.synchronize()
a, r = planes.cpu().numpy(), ref.cpu().numpy()
bad = np.nonzero(~((a == r) | (np.isnan(a) & np.isnan(r))))[0]
print("mismatches", bad.size)
N = n
tf = N * 64 * 6
for i in bad[:20]:
    t, o = divmod(int(i), tf)
    if o < N * 64 * 4:
        k, rem = divmod(o, 256); lane, cc = divmod(rem, 4)
    else:
        o2 = o - N * 64 * 4; k, rem = divmod(o2, 128); lane, cc = divmod(rem, 2); cc += 6
    cw = t * 64 + lane
    print(f"tile {t} k {k} comp {cc} lane {lane} cw {cw}: got {a[i]!r} want {r[i]!r}")
