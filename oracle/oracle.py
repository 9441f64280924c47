"""CPU oracle for the alignment DP and VAD segmentation — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, and
only as the *checker*.  The product package (whisperx_amd) never imports this module.

Two restatements of the reference live here:

* ``libwxoracle.so`` (wx_oracle.c): plain C, bit-exact against the golden vectors in
  tests/golden (generated from the reference itself), used to check the HIP kernels.
* ``TorchPort``: the same algorithm written with the per-timestep torch CPU tensor ops the
  reference uses (alignment.py:359-454), used only to time a faithful CPU baseline
  (``cpu_baseline.kind = "port"`` in bench.py).
* ``merge_chunks_regions``: the greedy chunk merge of vad.py:292-310 over a region list.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libwxoracle.so")
_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)


def build() -> str:
    """Compile the oracle with gcc (the Makefile next to this file)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(os.path.join(_HERE, "wx_oracle.c")):
            build()
        L = ctypes.CDLL(_LIB)
        L.wxo_trellis.argtypes = [_f32p, ctypes.c_int64, ctypes.c_int32, _i32p, ctypes.c_int64, ctypes.c_int32, _f32p]
        L.wxo_trellis.restype = None
        L.wxo_backtrack.argtypes = [_f32p, _f32p, ctypes.c_int64, ctypes.c_int32, _i32p, ctypes.c_int64,
                                    ctypes.c_int32, _i32p, _i32p, _f32p, _i64p]
        L.wxo_backtrack.restype = ctypes.c_int64
        L.wxo_merge_repeats.argtypes = [_i32p, _i32p, _f32p, ctypes.c_int64, _i32p, _i32p, _i32p, _f64p]
        L.wxo_merge_repeats.restype = ctypes.c_int64
        L.wxo_align_dp.argtypes = [_f32p, ctypes.c_int64, ctypes.c_int32, _i32p, ctypes.c_int64, ctypes.c_int32,
                                   _i32p, _i32p, _f64p, _i64p]
        L.wxo_align_dp.restype = ctypes.c_int
        L.wxo_binarize.argtypes = [_f32p, ctypes.c_int64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                   ctypes.c_float, ctypes.c_float, ctypes.c_double, ctypes.c_double,
                                   ctypes.c_double, _f64p, _f64p, ctypes.c_int64]
        L.wxo_binarize.restype = ctypes.c_int64
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def trellis(em: np.ndarray, tokens, blank: int = 0) -> np.ndarray:
    em = np.ascontiguousarray(em, np.float32)
    tok = np.ascontiguousarray(tokens, np.int32)
    T, V = em.shape
    N = len(tok)
    out = np.empty((T + 1, N + 1), np.float32)
    lib().wxo_trellis(_p(em, _f32p), T, V, _p(tok, _i32p), N, blank, _p(out, _f32p))
    return out


def backtrack(tr: np.ndarray, em: np.ndarray, tokens, blank: int = 0):
    """Returns (t_start, path) with path = (tok[L], time[L], prob[L]) or None."""
    tr = np.ascontiguousarray(tr, np.float32)
    em = np.ascontiguousarray(em, np.float32)
    tok = np.ascontiguousarray(tokens, np.int32)
    T, V = em.shape
    cap = T + 1
    pt, pm, pp = np.empty(cap, np.int32), np.empty(cap, np.int32), np.empty(cap, np.float32)
    ts = np.zeros(1, np.int64)
    L = lib().wxo_backtrack(_p(tr, _f32p), _p(em, _f32p), T, V, _p(tok, _i32p), len(tok), blank,
                            _p(pt, _i32p), _p(pm, _i32p), _p(pp, _f32p), _p(ts, _i64p))
    if L < 0:
        return int(ts[0]), None
    return int(ts[0]), (pt[:L].copy(), pm[:L].copy(), pp[:L].copy())


def merge_repeats(path):
    pt, pm, pp = path
    L = len(pt)
    st, ss, se, sc = (np.empty(max(L, 1), np.int32), np.empty(max(L, 1), np.int32),
                      np.empty(max(L, 1), np.int32), np.empty(max(L, 1), np.float64))
    S = lib().wxo_merge_repeats(_p(np.ascontiguousarray(pt), _i32p), _p(np.ascontiguousarray(pm), _i32p),
                                _p(np.ascontiguousarray(pp), _f32p), L, _p(st, _i32p), _p(ss, _i32p),
                                _p(se, _i32p), _p(sc, _f64p))
    return st[:S], ss[:S], se[:S], sc[:S]


def align_dp(em: np.ndarray, tokens, blank: int = 0):
    """(ok, t_start, seg_start[N], seg_end[N], seg_score[N]) — what align() consumes."""
    em = np.ascontiguousarray(em, np.float32)
    tok = np.ascontiguousarray(tokens, np.int32)
    T, V = em.shape
    N = len(tok)
    ss, se, sc = np.empty(N, np.int32), np.empty(N, np.int32), np.empty(N, np.float64)
    ts = np.zeros(1, np.int64)
    rc = lib().wxo_align_dp(_p(em, _f32p), T, V, _p(tok, _i32p), N, blank, _p(ss, _i32p), _p(se, _i32p),
                            _p(sc, _f64p), _p(ts, _i64p))
    return rc == 0, int(ts[0]), ss, se, sc


def binarize(scores: np.ndarray, sw_start: float, sw_step: float, sw_duration: float,
             onset: float = 0.5, offset=None, max_duration: float = float("inf"),
             pad_onset: float = 0.0, pad_offset: float = 0.0):
    """Region list [(start, end)] of vad.py:118-180 for one class column."""
    y = np.ascontiguousarray(scores, np.float32).reshape(-1)
    offset = offset or onset
    F = len(y)
    cap = F + 1
    rs, re = np.empty(cap, np.float64), np.empty(cap, np.float64)
    n = lib().wxo_binarize(_p(y, _f32p), F, sw_start, sw_step, sw_duration, np.float32(onset),
                           np.float32(offset), float(max_duration), float(pad_onset), float(pad_offset),
                           _p(rs, _f64p), _p(re, _f64p), cap)
    if n < 0:
        raise RuntimeError("oracle binarize failed")
    regs = sorted(set(zip(rs[:n].tolist(), re[:n].tolist())))
    return regs


def merge_chunks_regions(regions, chunk_size):
    """vad.py:285-310 over a sorted region list [(start, end)]."""
    if len(regions) == 0:
        return []
    out = []
    curr_start = regions[0][0]
    curr_end = 0
    seg_idxs = []
    for (s, e) in regions:
        if e - curr_start > chunk_size and curr_end - curr_start > 0:
            out.append({"start": curr_start, "end": curr_end, "segments": seg_idxs})
            curr_start = s
            seg_idxs = []
        curr_end = e
        seg_idxs.append((s, e))
    out.append({"start": curr_start, "end": curr_end, "segments": seg_idxs})
    return out


class TorchPort:
    """The reference algorithm with its per-timestep torch-CPU op structure
    (alignment.py:359-454): used only to time a CPU baseline on the GPU host, where the
    reference itself cannot be shipped.  Calibrated against the reference in the build
    container."""

    def __init__(self):
        import torch
        self.torch = torch

    def trellis(self, em, tokens, blank=0):
        torch = self.torch
        T, N = em.shape[0], len(tokens)
        tr = torch.empty((T + 1, N + 1))
        tr[0, 0] = 0
        tr[1:, 0] = torch.cumsum(em[:, 0], 0)
        tr[0, -N:] = -float("inf")
        tr[-N:, 0] = float("inf")
        for t in range(T):
            row = tr[t]
            tr[t + 1, 1:] = torch.maximum(row[1:] + em[t, blank], row[:-1] + em[t, tokens])
        return tr

    def backtrack(self, tr, em, tokens, blank=0):
        torch = self.torch
        j = tr.size(1) - 1
        t0 = torch.argmax(tr[:, j]).item()
        out = []
        t = t0
        while t > 0:
            stay = tr[t - 1, j] + em[t - 1, blank]
            move = tr[t - 1, j - 1] + em[t - 1, tokens[j - 1]]
            moved = bool(move > stay)
            out.append((j - 1, t - 1, em[t - 1, tokens[j - 1] if moved else 0].exp().item()))
            if moved:
                j -= 1
                if j == 0:
                    return out[::-1]
            t -= 1
        return None

    @staticmethod
    def merge_repeats(path):
        segs = []
        i = 0
        while i < len(path):
            k = i
            while k < len(path) and path[k][0] == path[i][0]:
                k += 1
            segs.append((path[i][0], path[i][1], path[k - 1][1] + 1, sum(p[2] for p in path[i:k]) / (k - i)))
            i = k
        return segs

    def align_dp(self, em, tokens, blank=0):
        tr = self.trellis(em, tokens, blank)
        path = self.backtrack(tr, em, tokens, blank)
        return None if path is None else self.merge_repeats(path)


def vad_aggregate(scores, start_frames, n_frames, missing=np.nan):
    """The VAD producer's overlap-add (whisperx/vad.py:198-240 -> pyannote.audio 3.1.1
    ``Inference.aggregate``, setup.py:23 pins pyannote.audio==3.1.1; pyannote is not installed
    here, so this restates its published algorithm and is itself "parity unpinned"):
    multi-label pre-aggregation hook ``np.max(scores, axis=-1, keepdims=True)``, then, with
    hamming=False, warm_up=(0, 0), skip_average=False, window by window in order:
    ``aggregated[s:s+K] += score * mask``, ``count[s:s+K] += mask``, ``seen = max(seen, mask)``
    (float32 accumulators), ``aggregated / maximum(count, 1e-12)``, ``missing`` where unseen.
    scores [n_chunks, K, n_classes]; returns [n_frames] float32."""
    s = np.max(np.asarray(scores, np.float32), axis=-1, keepdims=True)
    masks = 1 - np.isnan(s)
    s = np.nan_to_num(s, copy=True, nan=0.0)
    K = s.shape[1]
    agg = np.zeros((n_frames, 1), np.float32)
    cnt = np.zeros((n_frames, 1), np.float32)
    seen = np.zeros((n_frames, 1), np.float32)
    for c in range(s.shape[0]):
        f0 = int(start_frames[c])
        agg[f0:f0 + K] += (s[c] * masks[c])[: max(0, min(K, n_frames - f0))]
        cnt[f0:f0 + K] += masks[c][: max(0, min(K, n_frames - f0))]
        seen[f0:f0 + K] = np.maximum(seen[f0:f0 + K], masks[c][: max(0, min(K, n_frames - f0))])
    avg = agg / np.maximum(cnt, 1e-12)
    avg[seen == 0.0] = missing
    return avg[:, 0]
