#!/usr/bin/env python
"""Development tool: run wx_binarize_ex on the golden VAD cases, check its pre-pass words and
block records against numpy, and print the first region where it differs from the one-pass
kernel and the oracle."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402
from whisperx_amd import _lib  # noqa: E402

DEV = "cuda:0"


def words_np(y, onset, offset):
    F = len(y)
    nw = (F + 63) // 64
    on = np.zeros(nw, np.uint64)
    off = np.zeros(nw, np.uint64)
    mv = np.zeros(nw, np.float32)
    mi = np.full(nw, -1, np.int32)
    for b in range(nw):
        blk = y[64 * b: 64 * b + 64]
        for k, v in enumerate(blk):
            if v > onset:
                on[b] |= np.uint64(1) << np.uint64(k)
            if v < offset:
                off[b] |= np.uint64(1) << np.uint64(k)
        if b == 0 and not y[0] > onset:  # frame 0 decides the initial state: a reset when it does not activate
            off[0] |= np.uint64(1)
        mi[b] = 64 * b + int(np.argmin(blk))
        mv[b] = blk[mi[b] - 64 * b]
    return on, off, mv, mi


def main():
    lib = _lib.load()
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "vad_cases.json")))
    arr = np.load(os.path.join(ROOT, "tests", "golden", "vad_cases.npz"))
    for ci, c in enumerate(meta["cases"]):
        y = arr[f"v{ci:02d}_scores"].astype(np.float32)
        F = len(y)
        onset = np.float32(c["onset"])
        offset = np.float32(c["offset"] or c["onset"])
        geom = (c["sw_start"], c["sw_step"], c["sw_duration"])
        yd = torch.from_numpy(y).to(DEV)
        f_off = torch.tensor([0, F], dtype=torch.int64, device=DEV)
        g = torch.tensor([geom], dtype=torch.float64, device=DEV)
        st0, stp, dur = g[:, 0].contiguous(), g[:, 1].contiguous(), g[:, 2].contiguous()
        rs = torch.empty(F + 1, dtype=torch.float64, device=DEV)
        re = torch.empty(F + 1, dtype=torch.float64, device=DEV)
        r_off = torch.tensor([0, F + 1], dtype=torch.int64, device=DEV)
        cnt = torch.empty(1, dtype=torch.int64, device=DEV)
        wsb = lib.wx_binarize_workspace_bytes(1, F)
        ws = torch.zeros(wsb, dtype=torch.uint8, device=DEV)
        p = _lib._ptr
        rc = lib.wx_binarize_ex(p(yd), p(f_off), 1, F, p(st0), p(stp), p(dur), float(onset), float(offset),
                                float(c["chunk_size"]), 0.0, 0.0, p(rs), p(re), p(r_off), p(cnt), p(ws), wsb,
                                _lib._stream(torch.device(DEV)))
        torch.cuda.synchronize()
        nw = (F >> 6) + 2
        a8 = (nw * 8 + 255) // 256 * 256
        a4 = (nw * 4 + 255) // 256 * 256
        wsh = ws.cpu().numpy()
        on = wsh[:nw * 8].view(np.uint64)
        off = wsh[a8:a8 + nw * 8].view(np.uint64)
        mv = wsh[2 * a8:2 * a8 + nw * 4].view(np.float32)
        mi = wsh[2 * a8 + a4:2 * a8 + a4 + nw * 4].view(np.int32)
        on_r, off_r, mv_r, mi_r = words_np(y, onset, offset)
        k = len(on_r)
        wbad = [name for name, a_, b_ in (("on", on[:k], on_r), ("off", off[:k], off_r), ("mi", mi[:k], mi_r))
                if not np.array_equal(a_, b_)]
        n = int(cnt.item())
        got = list(zip(rs[:n].cpu().tolist(), re[:n].cpu().tolist()))
        want = oracle.binarize(y, *geom, float(onset), float(offset), max_duration=c["chunk_size"])
        (r1, e1), = _lib.binarize([y], [geom], onset, offset, c["chunk_size"], two_pass=False)
        one = list(zip(r1.tolist(), e1.tolist()))
        msg = f"case {ci} F={F} rc={rc} n={n} want={len(want)} one-pass-ok={one == want} words-bad={wbad}"
        if got != want:
            d = next((i for i, (a_, b_) in enumerate(zip(got, want)) if a_ != b_), min(len(got), len(want)))
            msg += f"\n   first diff at region {d}: got {got[max(d - 1, 0):d + 2]} want {want[max(d - 1, 0):d + 2]}"
            fr = lambda t: (t - geom[0] - 0.5 * geom[2]) / geom[1]  # noqa: E731
            if d < len(got):
                msg += f"\n   frames got {[round(fr(t), 2) for t in got[d]]}"
            if d < len(want):
                msg += f" want {[round(fr(t), 2) for t in want[d]]}"
        print(msg, flush=True)


if __name__ == "__main__":
    main()
