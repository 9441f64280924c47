#!/usr/bin/env python
"""Kernel A/B harness for wx_align_dp (development tool, not the bench contract).

Times the fused DP on three shapes — the config-2 batch (64 x T=1499, latency shape), a
saturated T=1499 batch and the north star's T=3000 x V=32 batch — for one or more builds of
libwxalign.so, and checks every build's outputs against the first build's (bit-exact).

    python tools/satbench.py [--libs a.so,b.so] [--cases b64,sat1499,sat3000] [--steps K]

Each build runs in its own subprocess (the library path is fixed at import).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = {  # name: (segments, T, N range)
    "b64": (64, 1499, (300, 500)),
    "b16": (16, 1499, (300, 500)),
    "b32": (32, 1499, (300, 500)),
    "b128": (128, 1499, (300, 500)),
    "b64n900": (64, 2999, (850, 951)),
    "b64p3": (64, 1499, (300, 400)),   # three parts per segment (column N in part 2)
    "b64p4": (64, 1499, (430, 530)),   # four parts
    "b64p2": (64, 1499, (170, 280)),   # two parts
    "sat1499": (4096, 1499, (300, 500)),
    "sat3000": (2048, 2999, (850, 951)),
    "sat3000_1024": (1024, 2999, (850, 951)),
    "sat3000_1536": (1536, 2999, (850, 951)),
    "sat3000_1792": (1792, 2999, (850, 951)),
    "sat3000_4096": (4096, 2999, (850, 951)),
}


def make_batch(S, T, V, n_lo, n_hi, seed, device):
    import numpy as np
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    rng = np.random.default_rng(seed)
    logits = torch.randn((S, T, V), generator=g, device=device)
    logits[:, :, 0] += 6.0
    toks = []
    for s in range(S):
        N = int(rng.integers(n_lo, n_hi + 1))
        tk = rng.integers(1, V, N)
        fr = np.sort(rng.choice(np.arange(1, T - 1), N, replace=False))
        logits[s, torch.from_numpy(fr).to(device), torch.from_numpy(tk).to(device)] += 12.0
        toks.append(tk.tolist())
    em = torch.log_softmax(logits, -1)
    return [em[s] for s in range(S)], toks


def make_ragged(S, V, seed, device):
    """S segments of T ~ U[100, 1499] frames, N ~ U[T/6, T/3] tokens (VAD-chunk-like shapes)."""
    import numpy as np
    import torch

    rng = np.random.default_rng(seed)
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    ems, toks = [], []
    for _ in range(S):
        T = int(rng.integers(100, 1500))
        N = int(rng.integers(max(1, T // 6), max(2, T // 3)))
        logits = torch.randn((T, V), generator=g, device=device)
        logits[:, 0] += 6.0
        tk = rng.integers(1, V, N)
        fr = np.sort(rng.choice(np.arange(1, T - 1), N, replace=False))
        logits[torch.from_numpy(fr).to(device), torch.from_numpy(tk).to(device)] += 12.0
        ems.append(torch.log_softmax(logits, -1))
        toks.append(tk.tolist())
    return ems, toks


def child(args):
    import numpy as np
    import torch

    sys.path.insert(0, ROOT)
    from whisperx_amd import _lib

    dev = torch.device("cuda", 0)
    out = {}
    for case in args.cases.split(","):
        if case.startswith("tr"):  # materialised trellis (wx_trellis): HBM-write-bound
            S, T, (lo, hi) = CASES[case[2:]]
            ems, toks = make_batch(S, T, 32, lo, hi, 1234, dev)
            b = _lib.Batch(ems, toks, [0] * S, device=dev)
            del ems
            tr, offs = _lib.trellis(b)
            torch.cuda.synchronize()
            ms = []
            for _ in range(args.steps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                _lib.load().wx_trellis(_lib._ptr(b.em), _lib._ptr(b.em_off_d), b.V, _lib._ptr(b.tok),
                                       _lib._ptr(b.tok_off_d), _lib._ptr(b.blank), b.S, b.max_N, _lib._ptr(tr),
                                       _lib._ptr(_lib._dev_i64(offs, dev)), _lib._stream(dev))
                e1.record()
                torch.cuda.synchronize()
                ms.append(e0.elapsed_time(e1))
            med = float(np.median(ms))
            Bytes = sum(4 * t * 32 + 4 * n + 4 * (t + 1) * (n + 1) for t, n in zip(b.Ts, b.Ns))
            cells = float(sum(t * n for t, n in zip(b.Ts, b.Ns)))
            digest = [int(np.int64(hash(tr[: min(tr.numel(), 1 << 24)].cpu().numpy().tobytes()) & 0x7FFFFFFF))]
            out[case] = {"ms_med": med, "ms_min": float(min(ms)), "cells_per_s": cells / (med / 1e3),
                         "GBps": Bytes / (med / 1e3) / 1e9, "frac": Bytes / (med / 1e3) / 8e12, "digest": digest}
            del tr, b
            torch.cuda.empty_cache()
            continue
        if case.startswith("rag"):  # ragged: rag64, rag16
            S = int(case[3:])
            ems, toks = make_ragged(S, 32, 4321, dev)
        else:
            S, T, (lo, hi) = CASES[case]
            ems, toks = make_batch(S, T, 32, lo, hi, 1234, dev)
        b = _lib.Batch(ems, toks, [0] * S, device=dev)
        del ems
        p = _lib.AlignPlan(b, mode=args.mode)
        for _ in range(2):
            p.run()
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        for a, e in ev:
            a.record(st)
            p.run()
            e.record(st)
        torch.cuda.synchronize()
        ms = [a.elapsed_time(e) for a, e in ev]
        cells = float(sum(t * n for t, n in zip(b.Ts, b.Ns)))
        Bytes = sum(4 * t * 32 + 4 * n + (t * n) // 8 + 16 * n for t, n in zip(b.Ts, b.Ns))
        med = float(np.median(ms))
        res = [x.cpu().numpy() for x in p.run()]
        torch.cuda.synchronize()
        # results (starts, ends, scores, t_start, and the outcome bits of the status) apart from
        # the route flags (recovered hand-off / generic forward): a recovered hand-off changes
        # the route, never the result, and the two must be told apart
        outcome = res[4] & _lib.STATUS_MASK
        digest = [int(np.int64(hash(r.tobytes()) & 0x7FFFFFFF)) for r in res[:4] + [outcome]]
        out[case] = {"ms_med": med, "ms_min": float(min(ms)), "cells_per_s": cells / (med / 1e3),
                     "GBps": Bytes / (med / 1e3) / 1e9, "frac": Bytes / (med / 1e3) / 8e12, "digest": digest,
                     "status": _lib.status_summary(res[4][: b.S])}
        if args.phases:
            import ctypes
            lib = _lib.load()
            n = min(S * args.parts, 8192)  # one row per workgroup (split: S * parts)
            buf = (ctypes.c_ulonglong * (6 * n))()
            lib.wx_debug_phases(buf, n)
            ph = np.frombuffer(buf, dtype=np.uint64).reshape(n, 6).astype(np.int64)
            # split grids: block ((s // 8) * P + p) * 8 + s % 8 -> row s * P + p (S % 8 == 0)
            P = args.parts
            perm = np.array([((s // 8) * P + q) * 8 + s % 8 for s in range(n // P) for q in range(P)]) \
                if P > 1 else np.arange(n)
            ph = ph[perm]
            fwd, walk, mrg = ph[:, 1] - ph[:, 0], ph[:, 2] - ph[:, 1], ph[:, 3] - ph[:, 2]
            if args.parts > 1:
                pf = fwd.reshape(-1, args.parts)
                out[case]["fwd_by_part_med"] = [float(np.median(pf[:, i])) for i in range(args.parts)]
                ent = (ph[:, 4] - ph[:, 4].min()).reshape(-1, args.parts) / 100.0
                out[case]["entry_by_part_med_us"] = [float(np.median(ent[:, i])) for i in range(args.parts)]
                ex = (ph[:, 5] - ph[:, 4].min()).reshape(-1, args.parts) / 100.0
                out[case]["exit_by_part_med_us"] = [float(np.median(ex[:, i])) for i in range(args.parts)]
                out[case]["exit_max_us"] = float(ex.max())
                seg_exit = ex.max(axis=1)
                Ns = np.array(b.Ns[: len(seg_exit)])
                by = {}
                for lo, hi in ((0, 288), (288, 416), (416, 448), (448, 1 << 30)):
                    m = (Ns > lo) & (Ns <= hi)
                    if m.any():
                        by[f"N({lo},{hi}]"] = [int(m.sum()), round(float(np.median(seg_exit[m])), 2), round(float(seg_exit[m].max()), 2)]
                out[case]["seg_exit_us_by_N(count,med,max)"] = by
            out[case]["phases_cyc_med"] = {"forward": float(np.median(fwd)), "walk": float(np.median(walk)),
                                           "merge": float(np.median(mrg)), "per_step_fwd": float(np.median(fwd)) / T,
                                           "per_step_walk": float(np.median(walk)) / T,
                                           "walk_max": float(walk.max()), "fwd_max": float(fwd.max())}
            if args.parts > 1 and hasattr(lib, "wx_debug_cq"):
                cbuf = (ctypes.c_ulonglong * (n * 48 * 3))()
                lib.wx_debug_cq(cbuf, n)
                cq = np.frombuffer(cbuf, dtype=np.uint64).reshape(n, 48, 3).astype(np.int64)[perm]
                cq = cq.reshape(-1, args.parts, 48, 3)
                t0 = cq[:, 0, 0, 0][:, None, None]
                rel = (cq - t0[..., None]) / 100.0  # us since part 0 passed barrier 0
                nq = (T + 31) // 32
                out[case]["chunk_start_us_by_part_med"] = [[round(float(np.median(rel[:, p_, q, 0])), 2) for q in range(0, nq, 4)]
                                                           for p_ in range(args.parts)]
                out[case]["granule_store_us_by_part_med"] = [[round(float(np.median(rel[:, p_, q, 1])), 2) for q in range(1, nq, 4)]
                                                             for p_ in range(args.parts)]
                out[case]["granule_seen_us_by_part_med"] = [[round(float(np.median(rel[:, p_, q, 2])), 2) for q in range(1, nq, 4)]
                                                            for p_ in range(args.parts)]
            lbuf = (ctypes.c_ulonglong * (n * 32 * 3))()
            lib.wx_debug_loop(lbuf, n)
            lp = np.frombuffer(lbuf, dtype=np.uint64).reshape(n, 32, 3).astype(np.int64)[perm]
            out[case]["loop_med_per_wave"] = [[float(np.median(lp[:, w, i])) for i in range(3)] for w in range(8)
                                              if lp[:, w, 0].max() > 0]
            if args.parts > 1:
                lq = lp.reshape(-1, args.parts, 32, 3)
                out[case]["loop_med_by_part"] = [[[float(np.median(lq[:, q, w, i])) for i in range(3)]
                                                  for w in range(8) if lq[:, q, w, 0].max() > 0]
                                                 for q in range(args.parts)]
                out[case]["handoff_by_part"] = [[float(np.median(lq[:, q, 14, i])) for i in range(3)]
                                                for q in range(args.parts)]
            xk = lp[:, 14, :]
            xk = xk[xk[:, 1] > 0]
            if len(xk):
                out[case]["handoff_med(misses,wait_cyc,slack_cyc)"] = [float(np.median(xk[:, i])) for i in range(3)]
            rk = lp[:, 13, :]
            rk = rk[rk[:, 2] > 0]
            if len(rk):
                out[case]["walk_rl_med(cycles,changes,blocks)"] = [float(np.median(rk[:, i])) for i in range(3)]
            sw_ = lp[:, 6:13, :]
            sw_ = sw_[sw_[:, 0, 2] > 0]  # (the workgroups that walked)
            if len(sw_):  # walk_spec per wave (slots 6 + wave)
                out[case]["spec_by_wave_med"] = [[float(np.median(sw_[:, w, i])) for i in range(3)]
                                                 for w in range(7) if sw_[:, w, 1].max() > 0]
            ww = lp[:, 16:24, :]
            ww = ww[ww[:, 0, 2] > 0]
            if len(ww):  # walk_range per wave: window-wait cycles, run-length cycles, blocks
                out[case]["walk_by_wave_med(win,rl,blocks)"] = [[float(np.median(ww[:, w, i])) for i in range(3)]
                                                                for w in range(8) if ww[:, w, 2].max() > 0]
                w2 = lp[:, 24, :]
                w2 = w2[w2[:, 2] > 0]
                if len(w2):
                    out[case]["walk_by_wave_med(win,rl,blocks)"].append([float(np.median(w2[:, i])) for i in range(3)])
            wk = lp[:, 15, :]
            wk = wk[wk[:, 1] > 0]
            if len(wk):
                out[case]["walk_split_med(argmax,walk,compact)"] = [float(np.median(wk[:, i])) for i in range(3)]
            rt = (ph[:, 5] - ph[:, 4]) / 100.0  # s_memrealtime ticks at 100 MHz -> us
            out[case]["seg_us_med"] = float(np.median(rt))
            ent = (ph[:, 4] - ph[:, 4].min()) / 100.0
            out[case]["entry_us_q"] = [float(np.quantile(ent, q)) for q in (0.1, 0.5, 0.75, 0.9, 0.99, 1.0)]
            out[case]["clock_GHz"] = float(np.median((ph[:, 3] - ph[:, 0]) / np.maximum(rt, 1e-9) / 1e3))
        del p, b
        torch.cuda.empty_cache()
    print("RESULT " + json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default=os.path.join(ROOT, "whisperx_amd", "libwxalign.so"))
    ap.add_argument("--cases", default="b64,sat1499,sat3000")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--mode", type=int, default=-1)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--phases", action="store_true", help="library built with -DWX_PHASE_TIMING")
    ap.add_argument("--parts", type=int, default=1, help="workgroups per segment of the timed launch (phases)")
    args = ap.parse_args()
    if args.child:
        child(args)
        return
    results = {}
    for lib in args.libs.split(","):
        env = dict(os.environ, WX_LIB_PATH=os.path.abspath(lib), PYTHONHASHSEED="0")
        t0 = time.time()
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--cases", args.cases,
                            "--steps", str(args.steps), "--mode", str(args.mode)] + (["--phases", "--parts", str(args.parts)] if args.phases else []),
                           env=env, capture_output=True, text=True, timeout=600)
        line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")]
        if r.returncode != 0 or not line:
            print(f"{lib}: FAILED rc={r.returncode}\n{r.stderr[-3000:]}", flush=True)
            sys.exit(1)
        results[lib] = json.loads(line[0][7:])
        print(f"{os.path.basename(lib)} ({time.time() - t0:.0f}s):", flush=True)
        for case, v in results[lib].items():
            print(f"  {case:9s} {v['ms_med']:9.4f} ms  {v['cells_per_s']:.3e} cells/s  frac {v['frac']:.3f}", flush=True)
            if "phases_cyc_med" in v:
                print(f"            phases {v['phases_cyc_med']} seg_us {v['seg_us_med']:.1f} clk {v['clock_GHz']:.2f} GHz entry_us_q {v['entry_us_q']}", flush=True)
                for k in ("seg_exit_us_by_N(count,med,max)", "chunk_start_us_by_part_med", "granule_store_us_by_part_med", "granule_seen_us_by_part_med",
                          "fwd_by_part_med", "entry_by_part_med_us", "exit_by_part_med_us", "exit_max_us",
                          "loop_med_per_wave", "loop_med_by_part", "handoff_by_part", "walk_rl_med(cycles,changes,blocks)", "walk_split_med(argmax,walk,compact)", "spec_by_wave_med", "walk_by_wave_med(win,rl,blocks)",
                          "handoff_med(misses,wait_cyc,slack_cyc)"):
                    if k in v:
                        print(f"            {k} {v[k]}", flush=True)
    libs = list(results)
    for lib in libs:
        for case, v in results[lib].items():
            st = v.get("status", {})
            if st.get("recovered_segments") or st.get("generic_forward_segments") or st.get("not_computed"):
                print(f"ROUTE {lib} {case}: {st}", flush=True)
    for lib in libs[1:]:
        for case in results[lib]:
            if results[lib][case]["digest"] != results[libs[0]][case]["digest"]:
                print(f"RESULT MISMATCH {lib} {case} vs {libs[0]}", flush=True)


if __name__ == "__main__":
    main()
