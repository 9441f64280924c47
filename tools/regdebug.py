#!/usr/bin/env python
"""Development tool: run the fused DP of one library build on the parity tests' case families
(skewed paths, config 2, random V=32) in every split mode and report, per mismatching segment
against the CPU oracle, where its spans first differ — plus the same segment re-run alone.

    WX_LIB_PATH=tools/ab/libwx_reg.so python tools/regdebug.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import oracle  # noqa: E402
from test_gpu_parity import _random_cases, _skewed_cases  # noqa: E402
from whisperx_amd import _lib  # noqa: E402

DEV = "cuda:0"


def run(cases, mode):
    ems = [torch.from_numpy(c["em"]).to(DEV) for c in cases]
    b = _lib.Batch(ems, [c["tokens"].tolist() for c in cases], [int(c["blank"]) for c in cases], device=DEV)
    ss, se, sc, ts, st = (x.cpu().numpy() for x in _lib.align_dp(b, mode=mode))
    return b, ss, se, ts, st


def check(cases, tag, mode, rerun=True):
    b, ss, se, ts, st = run(cases, mode)
    plan = _lib.align_dp_plan(b.S, b.min_N, b.max_N, b.V, mode)
    bad = 0
    for s, c in enumerate(cases):
        ok, tso, sso, seo, sco = oracle.align_dp(c["em"], c["tokens"], int(c["blank"]))
        a, e = b.tok_off[s], b.tok_off[s + 1]
        good = ts[s] == tso and bool(_lib.status_ok(st[s])) == ok and (
            not ok or (np.array_equal(ss[a:e], sso) and np.array_equal(se[a:e], seo)))
        if good:
            continue
        bad += 1
        T, N = c["em"].shape[0], len(c["tokens"])
        msg = f"  {tag} mode {mode}: seg {s} T={T} N={N} status={st[s]} t_start {ts[s]} vs {tso}"
        if ok and ts[s] == tso:
            d = np.flatnonzero(ss[a:e] != sso)
            if len(d):
                k = int(d[0])
                msg += f"; starts differ at token {k} ({len(d)} tokens): got {ss[a:e][max(k-2,0):k+4].tolist()} " \
                       f"want {sso[max(k-2,0):k+4].tolist()}"
        print(msg, flush=True)
        if rerun:
            b1, ss1, se1, ts1, st1 = run([c], mode)
            ok1 = ts1[0] == tso and (not ok or np.array_equal(ss1[: N], sso))
            print(f"    alone: {'OK' if ok1 else 'BAD'} plan {_lib.align_dp_plan(1, N, N, b.V, mode)}", flush=True)
    print(f"{tag} mode {mode}: {bad} bad of {len(cases)}; plan {plan}", flush=True)
    return bad


def main():
    print(_lib.LIB_PATH, flush=True)
    total = 0
    for mode in (-1, 12, 13, 14, 1):
        total += check(_skewed_cases(np.random.default_rng(7)), "skewed", mode)
        rng = np.random.default_rng(2)
        total += check(_random_cases(rng, 64, (1499, 1500), (300, 501), 32, blank=0), "cfg2", mode)
        rng = np.random.default_rng(32)
        total += check(_random_cases(rng, 16, (50, 1600), (1, 520), 32), "rand32", mode)
        total += check(_random_cases(rng, 16, (50, 1600), (1, 520), 32, quant=16), "ties32", mode)
    print("TOTAL BAD", total, flush=True)


if __name__ == "__main__":
    main()
