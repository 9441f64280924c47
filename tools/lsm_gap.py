"""Measure what fusing log_softmax into the DP's emission read would change (development tool;
VERDICT round 4, item 7).  alignment.py:233 computes torch.log_softmax(logits, -1) on the
device and the DP reads the result; a fused kernel would compute x - (m + log(sum exp(x - m)))
per row itself, with a wave's butterfly reduction order.  This restates that fused form in fp32
(numpy, butterfly order over the row's V values, fp32 exp/log) and reports, against
torch.log_softmax on the same logits (on the GPU when one is visible, as the reference's
device path runs it): the max and the distribution of ULP differences of the log-probs, and
the number of segments whose DP result (t_start, token spans; oracle/wx_oracle.c) differs.

    python tools/lsm_gap.py [--out profiles/r5_lsm_gap.json]

Inputs: BASELINE config 2 (64 x T=1499, V=32, the bench's logits generator), config 5
(T=2999, V=40, N~900) and the golden DP cases' emissions used as logits."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def fused_log_softmax(x: np.ndarray) -> np.ndarray:
    """Row-wise x - (m + log(sum exp(x - m))) in fp32, the sum in xor-butterfly order over the
    V values padded to a power of two with zeros (a wave reduction's order)."""
    x = np.asarray(x, np.float32)
    T, V = x.shape
    P = 1 << (V - 1).bit_length()
    m = x.max(axis=1, keepdims=True)
    e = np.zeros((T, P), np.float32)
    e[:, :V] = np.exp((x - m).astype(np.float32)).astype(np.float32)
    off = 1
    while off < P:
        idx = np.arange(P) ^ off
        e = (e + e[:, idx]).astype(np.float32)
        off <<= 1
    lse = (m[:, 0] + np.log(e[:, 0]).astype(np.float32)).astype(np.float32)
    return (x - lse[:, None]).astype(np.float32)


def ulp_diff(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    ia = a.view(np.int32).astype(np.int64)
    ib = b.view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = np.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    return np.abs(ia - ib)


def cases_cfg(rng, S, T, V, n_lo, n_hi):
    out = []
    for _ in range(S):
        N = int(rng.integers(n_lo, n_hi + 1))
        logits = rng.standard_normal((T, V)).astype(np.float32)
        logits[:, 0] += 6.0
        toks = rng.integers(1, V, N)
        fr = np.sort(rng.choice(np.arange(1, T - 1), N, replace=False))
        logits[fr, toks] += 12.0
        out.append((logits, toks, 0))
    return out


def golden_cases():
    d = np.load(os.path.join(ROOT, "tests", "golden", "dp_cases.npz"), allow_pickle=False)
    ids = sorted({k.split("_")[0] for k in d.keys() if k.endswith("_em")})
    return [(d[f"{i}_em"].astype(np.float32), d[f"{i}_tokens"], int(d[f"{i}_blank"])) for i in ids]


def measure(name, cases, dev):
    from oracle import oracle

    ulps, n_rows, diff_rows, diff_paths, diff_scores = [], 0, 0, 0, 0
    for logits, toks, blank in cases:
        ref = torch.log_softmax(torch.from_numpy(logits).to(dev), -1).cpu().numpy()
        fus = fused_log_softmax(logits)
        fin = np.isfinite(ref) & np.isfinite(fus)
        u = ulp_diff(ref[fin], fus[fin])
        ulps.append(u)
        n_rows += ref.shape[0]
        diff_rows += int((~np.all(ref == fus, axis=1)).sum())
        a = oracle.align_dp(ref, toks, blank)
        b = oracle.align_dp(fus, toks, blank)
        same = a[0] == b[0] and a[1] == b[1] and (not a[0] or (np.array_equal(a[2], b[2]) and np.array_equal(a[3], b[3])))
        diff_paths += 0 if same else 1
        if same and a[0] and not np.array_equal(a[4], b[4]):
            diff_scores += 1
    u = np.concatenate(ulps) if ulps else np.zeros(0, np.int64)
    return {"segments": len(cases), "rows": n_rows, "rows_differing": diff_rows,
            "values": int(u.size), "values_differing": int((u > 0).sum()), "max_ulp": int(u.max()) if u.size else 0,
            "ulp_hist": {str(k): int((u == k).sum()) for k in range(0, 5)} | {">4": int((u > 4).sum())},
            "segments_with_differing_dp_result": diff_paths, "segments_same_path_different_scores": diff_scores}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    rng = np.random.default_rng(1000)
    res = {"torch_log_softmax_device": dev, "fused_form": "x - (max + log(sum exp(x - max))), fp32, butterfly sum"}
    res["config2_64x1499_V32"] = measure("cfg2", cases_cfg(rng, 64, 1499, 32, 300, 500), dev)
    res["config5_4x2999_V40"] = measure("cfg5", cases_cfg(rng, 4, 2999, 40, 850, 951), dev)
    res["golden_dp_cases"] = measure("golden", golden_cases(), dev)
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
