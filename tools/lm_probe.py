import os, sys, time, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from modulations_amd import dvb_rcs2_turbo as M, tables as T
def p(*a): print(*a, flush=True)
rng = np.random.default_rng(0)
tabs = T.trellis_tables()[:5]
for n in (48, 212):
    Lc = (rng.standard_normal((4, 2, n)) * 3).astype(np.float32); La = rng.standard_normal((2, 2, n))
    t = time.time(); M.bcjr_max_log_map_batch(*Lc, *La, *tabs, n, 0.7, algo="log-map"); p("siso", n, time.time() - t)
for n in (48, 752):
    c = M.DVBRCS2_Turbo(n, "1/3", algo="log-map")
    llr = (rng.standard_normal((2, c.n_coded)) * 3).astype(np.float32)
    t = time.time(); c.decode_batch(llr); p("decode", n, time.time() - t)
