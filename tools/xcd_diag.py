"""Split-arrival repetition check (development tool): 28 segments (config-2 and 60 s shapes)
through the auto and the 3-part split shapes, 4 launches for each of fenced / fence-free x
same-XCD / spread parts (WX_SPLIT_FENCED, WX_SPLIT_XCD_SPREAD), counting segments whose t_start
or spans differ from the oracle and segments recovered after a lost hand-off.

    python tools/xcd_diag.py
"""
import os, sys, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from whisperx_amd import _lib
from oracle import oracle
rng = np.random.default_rng(41)
def cases_(n, T, N, V=32):
    out = []
    for _ in range(n):
        T_ = int(rng.integers(*T)); N_ = int(rng.integers(*N))
        lg = rng.standard_normal((T_, V)).astype(np.float32); lg[:, 0] += 6
        tk = rng.integers(1, V, N_); fr = np.sort(rng.choice(np.arange(1, T_ - 1), N_, replace=False)); lg[fr, tk] += 12
        out.append((torch.log_softmax(torch.from_numpy(lg), -1).numpy(), tk))
    return out
cs = cases_(24, (1400, 1500), (300, 500)) + cases_(4, (2900, 3000), (850, 950))
want = [oracle.align_dp(e, t, 0) for e, t in cs]
b = _lib.Batch([torch.from_numpy(e).cuda() for e, _ in cs], [t.tolist() for _, t in cs], [0] * len(cs), device="cuda:0")
for mode in (-1, 13):
    for fenced in "01":
        for spread in "01":
            os.environ["WX_SPLIT_FENCED"] = fenced; os.environ["WX_SPLIT_XCD_SPREAD"] = spread
            res = []
            for rep in range(4):
                ss, se, sc, ts, st = (x.cpu().numpy() for x in _lib.align_dp(b, mode=mode))
                bad_ts = bad_sp = rec = 0
                for i, (ok, tso, sso, seo, sco) in enumerate(want):
                    a, e_ = b.tok_off[i], b.tok_off[i + 1]
                    bad_ts += int(ts[i] != tso)
                    bad_sp += int(not (np.array_equal(ss[a:e_], sso) and np.array_equal(se[a:e_], seo)))
                    rec += int((st[i] & 16) != 0)
                res.append((bad_ts, bad_sp, rec))
            print(f"mode {mode} fenced {fenced} spread {spread}: (t_start bad, spans bad, recovered) per rep {res}", flush=True)
