"""HIP path (through the C ABI) against the reference's golden vectors and the CPU oracle.

Tolerances: token paths, t_start, frame spans, timestamps and trellis values are bit-exact.
Path probabilities: <= 1 fp32 ULP from the reference (its torch-CPU exp is MKL's; the GPU
uses the correctly rounded exp, as the oracle does, so GPU == oracle bit for bit);
merge_repeats scores: relative 2.5e-7 from the reference, == oracle (fp64, 1e-15 rel)."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from align_helpers import compare, jsonable, run_scenario, scenarios
from conftest import GOLDEN, ulp_diff
from oracle import oracle

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
# throughput; latency (auto parts); latency on one CU; split over 2 / 3 / 4 CUs
MODES = [-1, 0, 1, 2, 12, 13, 14]  # -1: WX_MODE_AUTO (small batches: split over 4 CUs)


@pytest.fixture(scope="module", autouse=True)
def _device():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from whisperx_amd import _lib

    _lib.load()


def _batch(cases):
    from whisperx_amd import _lib

    ems = [torch.from_numpy(c["em"]).to(DEV) for c in cases]
    toks = [c["tokens"].tolist() for c in cases]
    blanks = [int(c["blank"]) for c in cases]
    return _lib.Batch(ems, toks, blanks, device=DEV)


def _by_vocab(dp_cases):
    groups = {}
    for i in range(len(dp_cases)):
        c = dp_cases[i]
        groups.setdefault(c["em"].shape[1], []).append((i, c))
    return groups


# --------------------------------------------------------------------- fused align DP
def test_align_dp_matches_reference_golden(dp_cases):
    from whisperx_amd import _lib

    for V, items in _by_vocab(dp_cases).items():
        cases = [c for _, c in items]
        b = _batch(cases)
        ss, se, sc, ts, st = (x.cpu().numpy() for x in _lib.align_dp(b))
        for s, (i, c) in enumerate(items):
            assert ts[s] == int(c["t_start"]), f"case {i}: t_start {ts[s]} != {int(c['t_start'])}"
            ok = int(c["path_ok"]) == 1
            assert (st[s] & _lib.STATUS_MASK) == (0 if ok else 1), f"case {i}: status {st[s]}"
            if not ok:
                continue
            a, e = b.tok_off[s], b.tok_off[s + 1]
            assert np.array_equal(ss[a:e], c["seg_start"]), f"case {i}: seg_start"
            assert np.array_equal(se[a:e], c["seg_end"]), f"case {i}: seg_end"
            assert np.allclose(sc[a:e], c["seg_score"], rtol=2.5e-7, atol=0, equal_nan=True), f"case {i}"
            okc, tso, sso, seo, sco = oracle.align_dp(c["em"], c["tokens"], int(c["blank"]))
            assert np.array_equal(sc[a:e], sco, equal_nan=True) or np.allclose(sc[a:e], sco, rtol=1e-15,
                                                                               equal_nan=True), f"case {i}"


def _random_cases(rng, n, T_range, N_range, V, quant=None, blank=None):
    cases = []
    for _ in range(n):
        T = int(rng.integers(*T_range))
        N = int(rng.integers(*N_range))
        bl = int(rng.integers(0, V)) if blank is None else blank
        logits = rng.standard_normal((T, V)).astype(np.float32)
        logits[:, bl] += 6.0
        nb = np.array([v for v in range(V) if v != bl])
        toks = nb[rng.integers(0, len(nb), N)]
        if N <= T - 2:
            fr = np.sort(rng.choice(np.arange(1, T - 1), N, replace=False))
            logits[fr, toks] += 12.0
        em = torch.log_softmax(torch.from_numpy(logits), -1).numpy()
        if quant:
            em = (np.round(em * quant) / quant).astype(np.float32)
        cases.append({"em": np.ascontiguousarray(em), "tokens": toks.astype(np.int64), "blank": np.int64(bl)})
    return cases


def _check_vs_oracle(cases, tag, mode=-1, status_out=None):
    from whisperx_amd import _lib

    b = _batch(cases)
    ss, se, sc, ts, st = (x.cpu().numpy() for x in _lib.align_dp(b, mode=mode))
    if status_out is not None:
        status_out.append(st[: b.S].copy())
    mism = 0
    for s, c in enumerate(cases):
        ok, tso, sso, seo, sco = oracle.align_dp(c["em"], c["tokens"], int(c["blank"]))
        assert ts[s] == tso, f"{tag} seg {s}: t_start {ts[s]} vs {tso}"
        assert bool(_lib.status_ok(st[s])) == ok, f"{tag} seg {s}: status {st[s]}"
        if ok:
            a, e = b.tok_off[s], b.tok_off[s + 1]
            assert np.array_equal(ss[a:e], sso) and np.array_equal(se[a:e], seo), f"{tag} seg {s}: spans"
            mism += int((sc[a:e] != sco).sum())
            assert np.allclose(sc[a:e], sco, rtol=1e-12, atol=0, equal_nan=True), f"{tag} seg {s}: scores"
    return mism


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("V", [29, 32, 40, 64])
def test_align_dp_random_mixed_buckets_vs_oracle(V, mode):
    rng = np.random.default_rng(V)
    cases = []
    # every cells-per-lane bucket: N in (1..64], (64..128], ... (1536..2048]
    for lo, hi in [(1, 65), (65, 129), (129, 257), (257, 385), (385, 513), (513, 769), (769, 1025),
                   (1025, 1537), (1537, 2049)]:
        cases += _random_cases(rng, 2, (max(hi + 8, 40), hi + 700), (lo, hi), V)
    cases += _random_cases(rng, 6, (20, 300), (1, 60), V, quant=16)  # exact ties
    cases += _random_cases(rng, 4, (5, 40), (20, 60), V)  # N > T: backtrack fails
    _check_vs_oracle(cases, f"V{V} mode {mode}", mode)


def test_align_dp_concurrent_streams_vs_oracle():
    """The wrapper is as reentrant as the ABI: align_dp batches enqueued back to back on two
    streams (and from two threads) without a sync between them each use their own workspace
    and hand-off region (keyed by (device, stream)), and each equals the oracle."""
    import threading

    from whisperx_amd import _lib

    rng = np.random.default_rng(77)
    sets = [_random_cases(rng, 24, (1200, 1500), (300, 500), 32),   # split launch (4 CUs each)
            _random_cases(rng, 300, (200, 700), (20, 200), 32),     # throughput buckets
            _random_cases(rng, 40, (900, 1500), (100, 400), 29)]
    batches = [_batch(c) for c in sets]
    streams = [torch.cuda.Stream(device=DEV) for _ in batches]
    torch.cuda.synchronize()
    want = [[oracle.align_dp(c["em"], c["tokens"], int(c["blank"])) for c in cases] for cases in sets]

    def check(outs, tag):
        for k, (b, out) in enumerate(zip(batches, outs)):
            ss, se, sc, ts, st = (x.cpu().numpy() for x in out)
            for s, (ok, tso, sso, seo, sco) in enumerate(want[k]):
                assert ts[s] == tso and bool(_lib.status_ok(st[s])) == ok, f"{tag} batch {k} seg {s}"
                if ok:
                    a, e = b.tok_off[s], b.tok_off[s + 1]
                    assert np.array_equal(ss[a:e], sso) and np.array_equal(se[a:e], seo), f"{tag} {k}/{s}: spans"
                    assert np.allclose(sc[a:e], sco, rtol=1e-12, atol=0, equal_nan=True), f"{tag} {k}/{s}: scores"

    outs = [None] * len(batches)
    for rep in range(3):
        for i, (b, st) in enumerate(zip(batches, streams)):
            with torch.cuda.stream(st):
                outs[i] = _lib.align_dp(b)
        torch.cuda.synchronize()
        check(outs, f"streams rep {rep}")
        errs = []

        def run(i):
            try:
                with torch.cuda.stream(streams[i]):
                    outs[i] = _lib.align_dp(batches[i])
                streams[i].synchronize()
            except Exception as e:  # noqa: BLE001 - reported below
                errs.append(e)

        th = [threading.Thread(target=run, args=(i,)) for i in range(len(batches))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs
        torch.cuda.synchronize()
        check(outs, f"threads rep {rep}")


def _skewed_cases(rng, V=32):
    """Segments whose path is far from the straight line the speculative walk guesses from
    (walk_spec): all tokens in the last or first fifth, bursts, flat noise, exact ties."""
    cases = []
    for kind in ("late", "early", "bursts", "flat", "ties"):
        for _ in range(3):
            T = int(rng.integers(900, 1500))
            N = int(rng.integers(150, 420))
            logits = rng.standard_normal((T, V)).astype(np.float32)
            toks = rng.integers(1, V, N)
            if kind == "late":
                fr = np.sort(rng.choice(np.arange(T - T // 5, T - 1), min(N, T // 5 - 2), replace=False))
            elif kind == "early":
                fr = np.sort(rng.choice(np.arange(1, T // 5), min(N, T // 5 - 2), replace=False))
            elif kind == "bursts":
                lo = np.concatenate([np.arange(s, s + 60) for s in range(20, T - 80, 240)])
                fr = np.sort(rng.choice(lo, min(N, len(lo)), replace=False))
            else:
                fr = np.sort(rng.choice(np.arange(1, T - 1), N, replace=False))
            toks = toks[: len(fr)]
            if kind != "flat":
                logits[:, 0] += 6.0
                logits[fr, toks] += 12.0
            em = torch.log_softmax(torch.from_numpy(logits), -1).numpy()
            if kind == "ties":
                em = (np.round(em * 4) / 4).astype(np.float32)
            cases.append({"em": np.ascontiguousarray(em), "tokens": toks.astype(np.int64), "blank": np.int64(0)})
    return cases


@pytest.mark.parametrize("mode", MODES)
def test_align_dp_speculative_walk_skewed_paths(mode):
    """The multi-wave kernels walk the backtrack in segments from guessed columns and keep a
    segment only where the true walk merged with it; paths far from the guess must still
    equal the oracle's."""
    _check_vs_oracle(_skewed_cases(np.random.default_rng(7)), f"skewed mode {mode}", mode)


def test_align_dp_speculative_walk_trimmed_segments():
    """walk_spec drops speculative segments that would start past block 0 (too few blocks for
    the wave count).  With 8-wave workgroups that happens for T in 993-1024, 1185-1248 and
    1441-1472 frames (the segment lengths are computed host-side below, as the kernel does);
    those segments, in the one-CU latency buckets (1, 7, 1) and (2, 7, 1), equal the oracle,
    random and tie-quantised."""
    from whisperx_amd import _lib

    def trimmed(T, nw=8):
        top = (T - 1) >> 5
        K = min(nw, (top + 1) // 4)
        L = max((top + 1 + 3 + K - 1) // K, 1)
        L0 = max(L - 3, 1)
        lo = lambda k: max(top - L0 - k * L + 1, 0)
        return K > 1 and lo(K - 2) == 0

    rng = np.random.default_rng(99)
    Ts = (993, 1010, 1024, 1185, 1200, 1248, 1441, 1472)
    assert all(trimmed(T) for T in Ts) and not trimmed(992) and not trimmed(1473)
    for quant in (None, 4):
        cases = []
        for T in Ts:
            for N in (200, 600):
                cases += _random_cases(rng, 1, (T, T + 1), (N, N + 1), 32, quant=quant)
        plan = _lib.align_dp_plan(len(cases), 200, 600, 32, 2)
        assert plan == ["void wx::align_dp_kernel<1, 32, 7, 1>(wx::AlignArgs)",
                        "void wx::align_dp_kernel<2, 32, 7, 1>(wx::AlignArgs)"], plan
        _check_vs_oracle(cases, f"trimmed walk segments quant={quant}", mode=2)


def _capacity(C, W):
    """Tokens a (C cells/lane, W waves) bucket holds: waves >= 1 give ceil(32/C) lanes to the
    chunk halo (wx_align.hip, Geometry)."""
    return C * (64 + (W - 1) * (64 - ((32 + C - 1) // C if W > 1 else 0)))


THROUGHPUT_BUCKETS = [(1, 1), (2, 1), (4, 1), (6, 1), (8, 1), (8, 2), (8, 4), (8, 8), (16, 8)]
SPLIT_BUCKETS = [(1, 3), (1, 4), (2, 3), (4, 3)]


def _split_capacity(C, W, P):
    """Tokens a split bucket holds: the chunk halo runs through all W * P virtual waves."""
    return C * (64 + (W * P - 1) * (64 - (32 + C - 1) // C))
LATENCY_BUCKETS = [(1, 1), (1, 3), (1, 7), (2, 7), (4, 7), (8, 7), (16, 8)]


@pytest.mark.parametrize("mode", MODES)
def test_align_dp_bucket_capacity_edges(mode):
    """N at every bucket capacity and one past it (column N in the last lane of the last wave,
    halo lanes holding column N's left neighbours), in both launch shapes, V=32 (16-byte
    staging) and V=29 (row staging)."""
    rng = np.random.default_rng(100 + mode)
    Ns = set()
    for C, W in (THROUGHPUT_BUCKETS if mode == 0 else LATENCY_BUCKETS):
        cap = _capacity(C, W)
        if cap <= 4001 or (mode == 0 and cap <= 8000):
            Ns.update({cap, cap + 1})
    if mode != 0:  # split buckets (every part count: the auto mode picks one from the batch size)
        for P in (2, 3, 4):
            for C, W in SPLIT_BUCKETS:
                cap = _split_capacity(C, W, P)
                Ns.update({cap, cap + 1})
    for V in (32, 29):
        cases = []
        for N in sorted(Ns):
            T = N + int(rng.integers(2, 70))
            cases += _random_cases(rng, 1, (T, T + 1), (N, N + 1), V, blank=0)
        _check_vs_oracle(cases, f"edges V{V} mode {mode}", mode)
        if mode != 0:  # a split launch runs the bucket of its longest segment: one batch per N too
            for c in cases:
                _check_vs_oracle([c, cases[0]], f"edge N={len(c['tokens'])} V{V} mode {mode}", mode)


def _large_vocab_cases(rng, V, n, T_range, N_range, distinct):
    """ja/zh-like: a V-symbol vocabulary, each segment using `distinct` of its symbols."""
    cases = []
    for _ in range(n):
        T = int(rng.integers(*T_range))
        N = int(rng.integers(*N_range))
        bl = int(rng.integers(0, V))
        logits = rng.standard_normal((T, V)).astype(np.float32)
        logits[:, bl] += 6.0
        pool = rng.choice(np.array([v for v in range(V) if v != bl]), size=min(distinct, V - 1), replace=False)
        toks = pool[rng.integers(0, len(pool), N)]
        if N <= T - 2:
            fr = np.sort(rng.choice(np.arange(1, T - 1), N, replace=False))
            logits[fr, toks] += 12.0
        em = torch.log_softmax(torch.from_numpy(logits), -1).numpy()
        cases.append({"em": np.ascontiguousarray(em), "tokens": toks.astype(np.int64), "blank": np.int64(bl)})
    return cases


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("V", [100, 1000, 4000])
def test_align_dp_large_vocabulary_vs_oracle(V, mode):
    """V > 64 (e.g. the ja/zh wav2vec2 character vocabularies): each segment's used columns
    are gathered into a compact LDS row; up to 254 distinct tokens + blank + column 0."""
    rng = np.random.default_rng(V + mode)
    cases = _large_vocab_cases(rng, V, 6, (300, 900), (40, 280), 60)
    cases += _large_vocab_cases(rng, V, 3, (700, 1500), (250, 600), min(V - 2, 250))
    cases += _large_vocab_cases(rng, V, 2, (10, 40), (30, 60), 30)  # N > T: backtrack fails
    _check_vs_oracle(cases, f"V{V} mode {mode}", mode)


@pytest.mark.parametrize("mode", MODES)
def test_align_dp_large_vocabulary_too_many_columns(mode):
    """More than 256 distinct columns in one segment: the compact LDS row cannot hold them,
    so the segment is recomputed in-kernel by the generic forward (status 2 before round 2);
    results equal the oracle, neighbours unaffected."""
    rng = np.random.default_rng(9)
    ok_cases = _large_vocab_cases(rng, 1000, 2, (600, 700), (100, 200), 40)
    big = _large_vocab_cases(rng, 1000, 2, (900, 1000), (600, 700), 400)
    tie = _large_vocab_cases(rng, 1000, 1, (300, 400), (280, 290), 300)
    tie[0]["em"] = (np.round(tie[0]["em"] * 16) / 16).astype(np.float32)  # exact ties
    nofit = _large_vocab_cases(rng, 1000, 1, (10, 40), (300, 320), 300)  # N > T: backtrack fails
    sts = []
    cases = [ok_cases[0], big[0], ok_cases[1], big[1], tie[0], nofit[0]]
    _check_vs_oracle(cases, f"many columns mode {mode}", mode, status_out=sts)
    from whisperx_amd import _lib

    wide = [len(set(c["tokens"].tolist()) | {0, int(c["blank"])}) > _lib.MAX_SEGMENT_COLUMNS for c in cases]
    assert wide[1] and wide[3] and not wide[0]
    generic = (sts[0] & _lib.STATUS_GENERIC) != 0  # the route is reported per segment
    assert generic.tolist() == wide, sts[0]


def test_align_dp_lost_handoff_recovered(monkeypatch):
    """A split segment whose cross-CU hand-off is lost (WX_SPIN_LIMIT=0: no consumer part
    waits for its predecessor) is recomputed in-kernel by the last part to arrive; results
    still equal the oracle, in the auto (split) shape and every explicit split, and every
    such segment carries WX_STATUS_RECOVERED (none does once the hand-offs wait again)."""
    from whisperx_amd import _lib

    rng = np.random.default_rng(12)
    cases = _random_cases(rng, 12, (1400, 1600), (300, 500), 32)
    cases += _random_cases(rng, 2, (2900, 3000), (850, 950), 32)
    cases += _random_cases(rng, 2, (20, 200), (10, 60), 32, quant=16)
    monkeypatch.setenv("WX_SPIN_LIMIT", "0")
    for mode in (-1, 12, 13, 14):
        sts = []
        _check_vs_oracle(cases, f"lost hand-offs mode {mode}", mode, status_out=sts)
        rec = (sts[0] & _lib.STATUS_RECOVERED) != 0
        # the 60 s segments (N 850-950) span more than one part in every split shape, so a
        # consumer part lost its hand-off; a 30 s segment that fits in part 0 has no hand-off
        assert rec[12:14].all(), f"mode {mode}: 60 s split segments not flagged recovered: {sts[0]}"
        assert not rec[14:].any(), f"mode {mode}: {sts[0]}"
    monkeypatch.delenv("WX_SPIN_LIMIT")
    sts = []
    _check_vs_oracle(cases, "after recovery", -1, status_out=sts)
    assert int(((sts[0] & _lib.STATUS_RECOVERED) != 0).sum()) == 0, sts[0]


def _column0_variants(rng, T):
    """Columns 0 that exercise every branch of the fused DP's column-0 routine (col0_scan's
    binade scan, its one-row sequential steps, the sequential-chain fallback): log-probs,
    tiny values, mixed signs, 2^-4-quantised values (exact ties), magnitudes over 2^-40..2^40,
    -inf rows, a NaN row, +inf after -inf (NaN sums)."""
    out = {}
    lg = rng.standard_normal((T, 32)).astype(np.float32)
    lg[:, 0] += 6.0
    out["logprob"] = torch.log_softmax(torch.from_numpy(lg), -1).numpy()[:, 0]
    out["tiny"] = (-rng.random(T) * 1e-7).astype(np.float32)
    out["mixed"] = (rng.standard_normal(T) * 3).astype(np.float32)
    out["ties"] = (np.round(rng.standard_normal(T) * 16) / 16).astype(np.float32)
    out["wide"] = (-np.exp(rng.standard_normal(T) * 9)).astype(np.float32)
    out["alt_pow2"] = (np.where(np.arange(T) % 2, 1.0, -1.0) * 2.0 ** rng.integers(-20, 20, T)).astype(np.float32)
    x = (-rng.random(T)).astype(np.float32)
    x[T // 3] = -np.inf
    out["neg_inf"] = x.copy()
    x[2 * T // 3] = np.inf
    out["inf_nan"] = x.copy()
    y = (-rng.random(T)).astype(np.float32)
    y[T // 2] = np.nan
    out["nan"] = y
    return out


def test_column0_cumsum_bit_exact():
    """wx_column0_cumsum (the fused DP's column-0 routine) equals the sequential fp64 running
    sum of em[:, 0] (alignment.py:367, torch's CPU cumsum accumulates in double) bit for bit,
    NaN for NaN, on every variant and at chunk edges."""
    from whisperx_amd import _lib

    rng = np.random.default_rng(31)
    for T in (0, 1, 2, 31, 32, 33, 64, 65, 1499, 3001):
        for name, col in _column0_variants(rng, max(T, 1)).items():
            col = col[:T]
            em = np.zeros((T, 3), np.float32)
            em[:, 0] = col
            got = _lib.column0_cumsum(torch.from_numpy(em).to(DEV)).cpu().numpy()
            want = np.concatenate([[0.0], np.cumsum(col.astype(np.float64))])  # sequential (np accumulate)
            same = (got.view(np.uint64) == want.view(np.uint64)) | (np.isnan(got) & np.isnan(want))
            assert same.all(), f"T={T} {name}: first difference at t={int(np.argmin(same))}"


def test_align_dp_column0_edge_values_vs_oracle():
    """The split kernels' column 0 (col0_pre via col0_chunk) on the column-0 variants above,
    config-2-sized segments, in the auto (split) and every explicit split shape."""
    rng = np.random.default_rng(32)
    cases = []
    for name, col in _column0_variants(rng, 1499).items():
        c = _random_cases(rng, 1, (1499, 1500), (300, 500), 32, blank=3)[0]
        c["em"] = c["em"].copy()
        c["em"][:, 0] = col
        cases.append(c)
    for mode in (-1, 12, 13, 14):
        _check_vs_oracle(cases, f"column-0 variants mode {mode}", mode)


def test_align_dp_split_arrival_fenced_equals_write_through_across_xcds(monkeypatch):
    """The split kernels hand their decision words and column-N history to the last part with
    write-through (sc1) stores and loads and no fences (measured behaviour on gfx950, not an
    architectural guarantee).  With each segment's parts forced onto different XCDs
    (WX_SPLIT_XCD_SPREAD=1), the fence-free and the fenced arrival (WX_SPLIT_FENCED=1: the
    memory model's release / acquire on top) give bit-identical results equal to the oracle,
    in every split shape and on the lost-hand-off recovery path (WX_SPIN_LIMIT=0)."""
    from whisperx_amd import _lib

    rng = np.random.default_rng(41)
    cases = _random_cases(rng, 20, (1400, 1500), (300, 500), 32, blank=0)
    cases += _random_cases(rng, 2, (2900, 3000), (850, 950), 32)
    cases += _random_cases(rng, 2, (300, 900), (100, 280), 32, quant=16)
    cases += _random_cases(rng, 2, (5, 40), (20, 60), 32)  # N > T
    b = _batch(cases)
    for spin in (None, "0"):
        if spin is None:
            monkeypatch.delenv("WX_SPIN_LIMIT", raising=False)
        else:
            monkeypatch.setenv("WX_SPIN_LIMIT", spin)
        for mode in (-1, 12, 13, 14):
            ref = None
            for fenced in ("0", "1"):
                for spread in ("0", "1"):
                    monkeypatch.setenv("WX_SPLIT_FENCED", fenced)
                    monkeypatch.setenv("WX_SPLIT_XCD_SPREAD", spread)
                    tag = f"spin {spin} mode {mode} fenced {fenced} spread {spread}"
                    ss, se, sc, ts, st = (x.cpu().numpy() for x in _lib.align_dp(b, mode=mode))
                    # per segment: t_start, outcome and, where a path exists, its spans and scores
                    # (a failed segment's token slots are not written)
                    out = []
                    for s in range(b.S):
                        a, e = b.tok_off[s], b.tok_off[s + 1]
                        ok = bool(_lib.status_ok(st[s]))
                        out.append((int(ts[s]), int(st[s]) & _lib.STATUS_MASK,
                                    (ss[a:e].tobytes(), se[a:e].tobytes(), sc[a:e].tobytes()) if ok else None))
                    if ref is None:
                        ref = out
                        _check_vs_oracle(cases, tag, mode)
                    else:
                        diff = [s for s in range(b.S) if out[s] != ref[s]]
                        assert not diff, f"{tag}: segments {diff} differ from the unfenced same-XCD launch"
    monkeypatch.delenv("WX_SPLIT_FENCED")
    monkeypatch.delenv("WX_SPLIT_XCD_SPREAD")


def test_align_dp_handoff_region_reuse():
    """wx_align_dp_ex: one caller-owned hand-off region reused across launches of different
    batch layouts (granules of earlier launches stay behind in other slots: their epochs
    never match) gives oracle results every time, and its arrival counters are left at zero;
    and foreign data in a workspace-carved region (wx_align_dp_mode) is zeroed first."""
    from whisperx_amd import _lib

    rng = np.random.default_rng(13)
    cases = _random_cases(rng, 16, (1400, 1600), (300, 500), 32)
    other = _random_cases(rng, 9, (700, 2600), (200, 700), 32)
    for c in (cases, other, cases[3:], other, cases):
        _check_vs_oracle(c, "handoff reuse", 14)
    b = _batch(cases)
    plan = _lib.AlignPlan(b, mode=14)
    for _ in range(3):
        plan.run()
    torch.cuda.synchronize()
    xg = plan.hob - (b.S + 1) * 8
    arrive = plan.ho[plan.hob - ((b.S + 1) * 8 + 255) // 256 * 256:].view(torch.int64)[: b.S]
    assert int(arrive.count_nonzero()) == 0 and xg > 0
    # a workspace full of tag-like garbage through the memset path
    lib = _lib.load()
    wsb = lib.wx_align_dp_workspace_bytes(b.S, b.sum_T, b.max_N)
    ws = torch.full((wsb // 8 + 1,), -1, dtype=torch.int64, device=DEV)
    outs = [torch.empty(max(b.tok_off[-1], 1), dtype=t, device=DEV) for t in (torch.int32, torch.int32, torch.float64)]
    ts = torch.empty(b.S, dtype=torch.int32, device=DEV)
    st = torch.empty(b.S, dtype=torch.int32, device=DEV)
    _lib._check(lib.wx_align_dp_mode(_lib._ptr(b.em), _lib._ptr(b.em_off_d), b.V, _lib._ptr(b.tok),
                                     _lib._ptr(b.tok_off_d), _lib._ptr(b.blank), b.S, b.min_N, b.max_N, b.sum_T,
                                     *[_lib._ptr(o) for o in outs], _lib._ptr(ts), _lib._ptr(st), _lib._ptr(ws), wsb,
                                     14, _lib._stream(torch.device(DEV))))
    ss, se = outs[0].cpu().numpy(), outs[1].cpu().numpy()
    for s_, c in enumerate(cases):
        ok, tso, sso, seo, sco = oracle.align_dp(c["em"], c["tokens"], int(c["blank"]))
        a, e = b.tok_off[s_], b.tok_off[s_ + 1]
        assert ok and int(st[s_]) == 0 and np.array_equal(ss[a:e], sso) and np.array_equal(se[a:e], seo)


def test_trellis_large_vocabulary_vs_oracle():
    from whisperx_amd import _lib

    rng = np.random.default_rng(31)
    cases = _large_vocab_cases(rng, 500, 4, (50, 400), (5, 120), 50)
    b = _batch(cases)
    flat, offs = _lib.trellis(b)
    flat = flat.cpu().numpy()
    for s_, c in enumerate(cases):
        T, N = c["em"].shape[0], len(c["tokens"])
        got = flat[offs[s_]:offs[s_] + (T + 1) * (N + 1)].reshape(T + 1, N + 1)
        exp = oracle.trellis(c["em"], c["tokens"], int(c["blank"]))
        assert np.array_equal(got, exp, equal_nan=True), f"segment {s_}"


@pytest.mark.parametrize("V", [32, 29])
def test_trellis_every_bucket_vs_oracle(V):
    """get_trellis over every launch bucket (N at each capacity and one past it, short
    lanes, multi-wave chunk halos), T spanning several 32-row chunks: bit-exact rows (the
    row stores go through the LDS transpose)."""
    from whisperx_amd import _lib

    rng = np.random.default_rng(300 + V)
    Ns = {1, 2, 3, 5, 63, 64, 65, 100}
    for C, W in THROUGHPUT_BUCKETS:
        cap = _capacity(C, W)
        if cap <= 4001:
            Ns.update({cap, cap + 1, cap - 7})
    cases = []
    for N in sorted(Ns):
        T = N + int(rng.integers(2, 90)) if N > 60 else int(rng.integers(N + 2, 140))
        cases += _random_cases(rng, 1, (T, T + 1), (N, N + 1), V)
    cases += _random_cases(rng, 3, (5, 40), (20, 60), V)  # N > T
    cases += _random_cases(rng, 3, (20, 300), (1, 60), V, quant=16)  # exact ties
    b = _batch(cases)
    flat, offs = _lib.trellis(b)
    flat = flat.cpu().numpy()
    for s_, c in enumerate(cases):
        T, N = c["em"].shape[0], len(c["tokens"])
        got = flat[offs[s_]:offs[s_] + (T + 1) * (N + 1)].reshape(T + 1, N + 1)
        exp = oracle.trellis(c["em"], c["tokens"], int(c["blank"]))
        assert np.array_equal(got, exp, equal_nan=True), f"V{V} segment {s_} (T={T}, N={N})"


@pytest.mark.parametrize("mode", MODES)
def test_align_dp_long_segments_and_chunk_edges(mode):
    """T > 8192 (walk change masks in global memory instead of LDS), T at multiples of the
    32-row chunk and one off, T < 32, N = 1 and N = T - 1."""
    rng = np.random.default_rng(55 + mode)
    cases = _random_cases(rng, 2, (9000, 9400), (1200, 1800), 32, blank=0)
    cases += _random_cases(rng, 1, (40, 41), (1, 2), 32)    # N = 1
    cases += _random_cases(rng, 1, (90, 91), (89, 90), 32)  # N = T - 1
    _check_vs_oracle(cases, f"long mode {mode}", mode)
    edges = []
    for T in (31, 32, 33, 63, 64, 65, 1023, 1024, 1025):
        edges += _random_cases(rng, 1, (T, T + 1), (max(1, T // 4), max(2, T // 3)), 29)
    _check_vs_oracle(edges, f"chunk edges mode {mode}", mode)


def test_align_dp_config2_batch_vs_oracle():
    """BASELINE config 2: 64 x 30 s segments (T=1499, V=32, N~U[300,500])."""
    rng = np.random.default_rng(2)
    cases = _random_cases(rng, 64, (1499, 1500), (300, 501), 32, blank=0)
    for mode in MODES:
        _check_vs_oracle(cases, f"cfg2 mode {mode}", mode)


def test_align_dp_config5_long_form_vs_oracle():
    """BASELINE config 5: DE large-xlsr-shaped, T=2999, V=40, N~900."""
    rng = np.random.default_rng(5)
    cases = _random_cases(rng, 8, (2999, 3000), (850, 951), 40, blank=0)
    for mode in MODES:
        _check_vs_oracle(cases, f"cfg5 mode {mode}", mode)


def test_align_dp_deterministic_and_order_independent():
    from whisperx_amd import _lib

    rng = np.random.default_rng(11)
    cases = _random_cases(rng, 12, (300, 900), (20, 280), 32)
    b = _batch(cases)
    r1 = [x.cpu().numpy() for x in _lib.align_dp(b)]
    r2 = [x.cpu().numpy() for x in _lib.align_dp(_batch(cases))]
    for a, c in zip(r1, r2):
        assert np.array_equal(a, c, equal_nan=True)
    assert (r1[4][:12] == 0).all(), "all segments align (N < T)"
    # a segment's result does not depend on its batch neighbours
    single = [x.cpu().numpy() for x in _lib.align_dp(_batch(cases[5:6]))]
    a0, a1 = b.tok_off[5], b.tok_off[6]
    for k in (0, 1, 2):
        assert np.array_equal(r1[k][a0:a1], single[k][: a1 - a0])


# --------------------------------------------------------------- get_trellis / backtrack
def test_trellis_matches_reference_golden(dp_cases):
    from whisperx_amd import _lib

    for V, items in _by_vocab(dp_cases).items():
        b = _batch([c for _, c in items])
        flat, offs = _lib.trellis(b)
        flat = flat.cpu().numpy()
        for s, (i, c) in enumerate(items):
            T, N = c["em"].shape[0], len(c["tokens"])
            tr = flat[offs[s]:offs[s + 1]].reshape(T + 1, N + 1)
            if "trellis" in c:
                assert np.array_equal(tr, c["trellis"], equal_nan=True), f"case {i}"
            if not np.isnan(tr).any():
                assert hashlib.sha256(tr.tobytes()).digest() == c["trellis_sha"].tobytes(), f"case {i}"
            assert np.array_equal(tr[:, -1], c["trellis_colN"], equal_nan=True), f"case {i}"


def test_backtrack_matches_reference_golden(dp_cases):
    from whisperx_amd import _lib

    for V, items in _by_vocab(dp_cases).items():
        b = _batch([c for _, c in items])
        flat, offs = _lib.trellis(b)
        pt, pm, pp, plen, ts = (x.cpu().numpy() for x in _lib.backtrack(b, flat, offs))
        for s, (i, c) in enumerate(items):
            assert ts[s] == int(c["t_start"]), f"case {i}"
            if not int(c["path_ok"]):
                assert plen[s] == -1, f"case {i}"
                continue
            L = plen[s]
            o = b.em_off[s]
            assert L == len(c["path_tok"]), f"case {i}: len {L}"
            assert np.array_equal(pt[o:o + L], c["path_tok"]) and np.array_equal(pm[o:o + L], c["path_time"])
            assert ulp_diff(pp[o:o + L], c["path_prob"].astype(np.float32)).max() <= 1, f"case {i}"


def test_merge_repeats_kernel_on_reference_paths(dp_cases):
    from whisperx_amd import _lib

    paths = [dp_cases[i] for i in range(len(dp_cases)) if int(dp_cases[i]["path_ok"])]
    off = [0]
    for c in paths:
        off.append(off[-1] + len(c["path_tok"]))
    cat = lambda k, dt: torch.from_numpy(np.concatenate([c[k] for c in paths]).astype(dt)).to(DEV)  # noqa: E731
    st, ss, se, sc, cnt = _lib.merge_repeats(cat("path_tok", np.int32), cat("path_time", np.int32),
                                             cat("path_prob", np.float32),
                                             torch.tensor(off[:-1], dtype=torch.int64).to(DEV),
                                             torch.tensor([len(c["path_tok"]) for c in paths], dtype=torch.int32).to(DEV),
                                             DEV)
    ss, se, sc, cnt = ss.cpu().numpy(), se.cpu().numpy(), sc.cpu().numpy(), cnt.cpu().numpy()
    for p, c in enumerate(paths):
        G = cnt[p]
        o = off[p]
        assert G == len(c["seg_start"])
        assert np.array_equal(ss[o:o + G], c["seg_start"]) and np.array_equal(se[o:o + G], c["seg_end"])
        # probabilities fed as the reference's own fp32 values -> scores bit-exact
        assert np.array_equal(sc[o:o + G], c["seg_score"], equal_nan=True)


def test_python_api_objects(dp_cases):
    from whisperx_amd import backtrack, get_trellis, merge_repeats, merge_words

    c = dp_cases[26]
    em = torch.from_numpy(c["em"])
    toks = c["tokens"].tolist()
    tr = get_trellis(em, toks, int(c["blank"]))
    assert tr.device.type == "cpu" and tuple(tr.shape) == (em.shape[0] + 1, len(toks) + 1)
    assert hashlib.sha256(tr.numpy().tobytes()).digest() == c["trellis_sha"].tobytes()
    path = backtrack(tr, em, toks, int(c["blank"]))
    assert [p.token_index for p in path] == c["path_tok"].tolist()
    assert [p.time_index for p in path] == c["path_time"].tolist()
    transcript = "".join(chr(97 + (int(x) % 26)) for x in toks)
    segs = merge_repeats(path, transcript)
    assert [s.start for s in segs] == c["seg_start"].tolist()
    assert [s.end for s in segs] == c["seg_end"].tolist()
    assert [ord(s.label) for s in segs] == c["seg_label"].tolist()
    words = merge_words(segs, separator=transcript[0])
    assert [w.start for w in words] == c["word_start"].tolist()
    assert [w.end for w in words] == c["word_end"].tolist()
    assert np.allclose([w.score for w in words], c["word_score"], rtol=1e-6)
    # failure -> None
    bad = dp_cases[4]
    em = torch.from_numpy(bad["em"])
    tr = get_trellis(em, bad["tokens"].tolist(), 0)
    assert backtrack(tr, em, bad["tokens"].tolist(), 0) is None


# ------------------------------------------------------------------------ align() e2e
@pytest.mark.parametrize("si", range(len(scenarios())))
def test_align_end_to_end_matches_reference(si, capsys):
    """Fake CTC model on the GPU: log_softmax runs on the device, the DP in the fused kernel.
    Timestamps must match the reference to within one frame; in practice they are exact."""
    from whisperx_amd import align

    sc, logits = scenarios()[si]
    stats = {}
    out, mutated = run_scenario(align, sc, logits, DEV)
    compare(jsonable(out), sc["result"], time_tol=0.02 + 1e-9, score_tol=1e-3 + 1e-9, stats=stats)
    assert jsonable(mutated) == sc["mutated"]
    if stats.get("abs_err"):
        assert float(np.mean(stats["abs_err"])) * 1000 <= 1.0  # word-boundary MAE (ms)


@pytest.mark.parametrize("si", range(len(scenarios())))
def test_align_device_cpu_matches_reference(si, capsys):
    """Config 1's literal call, align(..., device='cpu'): the model forward and log_softmax on
    the CPU (alignment.py:226-235 with device='cpu'), the DP on GPU 0 (_dp_device), the
    emissions copied over once per group.  Same golden results as the reference."""
    from whisperx_amd import align

    sc, logits = scenarios()[si]
    stats = {}
    out, mutated = run_scenario(align, sc, logits, "cpu")
    compare(jsonable(out), sc["result"], time_tol=0.02 + 1e-9, score_tol=1e-3 + 1e-9, stats=stats)
    assert jsonable(mutated) == sc["mutated"]
    if stats.get("abs_err"):
        assert float(np.mean(stats["abs_err"])) * 1000 <= 1.0


# ------------------------------------------------------------------------------ VAD
def _vad():
    with open(os.path.join(GOLDEN, "vad_cases.json")) as f:
        meta = json.load(f)
    return meta, np.load(os.path.join(GOLDEN, "vad_cases.npz"))


def test_binarize_and_merge_chunks_match_reference():
    from whisperx_amd.vad import Binarize, SlidingWindow, SlidingWindowFeature, merge_chunks

    from whisperx_amd import _lib

    meta, arr = _vad()
    kernels = set()
    for ci, c in enumerate(meta["cases"]):
        sc = arr[f"v{ci:02d}_scores"]
        kernels.add(_lib.binarize_plan(c["onset"], c["offset"] if c["offset"] is not None else c["onset"])[-1])
        feat = SlidingWindowFeature(sc[:, None], SlidingWindow(c["sw_start"], c["sw_step"], c["sw_duration"]))
        ann = Binarize(max_duration=c["chunk_size"], onset=c["onset"], offset=c["offset"])(feat)
        assert [[s.start, s.end] for s in ann.get_timeline()] == c["regions"], f"vad case {ci}"
        chunks = merge_chunks(feat, c["chunk_size"], onset=c["onset"], offset=c["offset"])
        got = [{"start": x["start"], "end": x["end"], "segments": [list(p) for p in x["segments"]]} for x in chunks]
        assert got == c["chunks"], f"vad case {ci}"
    # the golden cases reach both wx_binarize_ex routes (offset > onset since round 4)
    assert kernels == {"void wx::binarize_scan_kernel(wx::BinScanArgs)",
                       "void wx::binarize_fsm_kernel(wx::BinarizeArgs, wx::BinWords)"}
    m = meta["min_duration_on"]
    sc = arr["vmin_scores"]
    feat = SlidingWindowFeature(sc[:, None], SlidingWindow(0.0, 0.016875, 0.0619375))
    ann = Binarize(onset=m["onset"], offset=m["offset"], min_duration_on=m["min_duration_on"])(feat)
    assert [[s.start, s.end] for s, _ in ann.itertracks()] == m["regions"]


def test_binarize_one_hour_vs_oracle():
    """BASELINE config 3 scale: 1 h of VAD scores (213,333 frames), several chunk sizes."""
    from whisperx_amd import _lib

    rng = np.random.default_rng(3)
    F = 213_333
    x = rng.standard_normal(F + 40)
    y = np.convolve(x, np.ones(40) / 40, mode="valid")[:F] * 4 * np.sqrt(40) / 3
    sc = (1 / (1 + np.exp(-y))).astype(np.float32)
    for chunk in (30, 10, 2.5):
        regs = oracle.binarize(sc, 0.0, 0.016875, 0.0619375, 0.5, 0.363, max_duration=chunk)
        (rs, re), = _lib.binarize([sc], [(0.0, 0.016875, 0.0619375)], 0.5, 0.363, chunk)
        assert list(zip(rs.tolist(), re.tolist())) == regs, f"chunk {chunk}"
    # many files in one launch
    cols = [sc[i * 20000:(i + 1) * 20000 + i * 7] for i in range(8)]
    outs = _lib.binarize(cols, [(0.25 * i, 0.016875, 0.0619375) for i in range(8)], 0.5, 0.363, 30)
    for i, (rs, re) in enumerate(outs):
        assert list(zip(rs.tolist(), re.tolist())) == oracle.binarize(cols[i], 0.25 * i, 0.016875, 0.0619375,
                                                                       0.5, 0.363, max_duration=30)


def _binarize_both(cols, geom, onset, offset, maxd):
    from whisperx_amd import _lib

    two = _lib.binarize(cols, geom, onset, offset, maxd, two_pass=True)
    one = _lib.binarize(cols, geom, onset, offset, maxd, two_pass=False)
    for i, c in enumerate(cols):
        want = oracle.binarize(c, *geom[i], onset, offset, max_duration=maxd)
        for tag, (rs, re) in (("two-pass", two[i]), ("one-pass", one[i])):
            assert list(zip(rs.tolist(), re.tolist())) == want, (tag, i, len(c), onset, offset, maxd)


def test_binarize_dense_events_nan_and_ragged_files():
    """wx_binarize_ex (bit-word pre-pass, then the parallel scan for offset <= onset or the
    event-jumping state machine binarize_fsm_kernel for offset > onset — the plan is asserted
    per pair) and the one-pass scan wx_binarize, against the oracle, where every other frame
    is an event (noise thresholded near its median), min-cuts span many 64-frame blocks, blocks
    hold NaNs (np.argmin takes the first NaN), and files are 0, 1, 2, 63, 64, 65 ... frames
    long (partial words, words of one frame)."""
    from whisperx_amd import _lib

    rng = np.random.default_rng(11)
    lens = [0, 1, 2, 63, 64, 65, 127, 128, 129, 1000, 4095, 4096, 4097, 0, 9000, 30001]
    cols = []
    for k, n in enumerate(lens):
        y = rng.random(n).astype(np.float32)
        if k % 3 == 0 and n > 10:
            y[rng.integers(0, n, max(n // 200, 1))] = np.nan
        if k % 4 == 1:  # ties: quantised scores
            y = np.round(y * 8) / 8
        cols.append(y)
    geom = [(0.1 * i, 0.016875, 0.0619375) for i in range(len(cols))]
    scan = "void wx::binarize_scan_kernel(wx::BinScanArgs)"
    fsm = "void wx::binarize_fsm_kernel(wx::BinarizeArgs, wx::BinWords)"
    for onset, offset, maxd in ((0.5, 0.5, 30.0), (0.5, 0.363, 1.0), (0.2, 0.1, 0.5), (0.95, 0.9, 0.05),
                                (0.5, 0.4, float("inf")), (0.0, 0.0, 2.0),
                                # offset > onset: binarize_fsm_kernel
                                (0.4, 0.6, 30.0), (0.5, 0.55, 1.0), (0.3, 0.9, 0.5), (0.45, 0.5, float("inf")),
                                (0.0, 1.0, 2.0), (0.5, 0.5000001, 0.05)):
        want = fsm if np.float32(offset) > np.float32(onset) else scan
        assert _lib.binarize_plan(onset, offset, sum(len(c) for c in cols))[-1] == want, (onset, offset)
        _binarize_both(cols, geom, onset, offset, maxd)


def test_binarize_all_active_many_splits():
    """Scores above onset everywhere: one region cut at every max_duration, each cut an argmin
    over ~half the current list (block records + two partial blocks), with NaN runs and
    constant stretches (ties go to the first frame)."""
    rng = np.random.default_rng(12)
    F = 50_000
    y = (0.6 + 0.4 * rng.random(F)).astype(np.float32)
    y[10_000:10_300] = 0.7  # a constant stretch: the first minimum wins
    y[20_000:20_070] = np.nan
    y[33_333] = np.nan
    geom = [(0.0, 0.016875, 0.0619375)]
    for maxd in (30.0, 7.3, 1.1, 0.02):
        _binarize_both([y], geom, 0.5, 0.5, maxd)


def test_binarize_and_merge_chunks_device_scores_dense():
    """merge_chunks on device-resident dense-event scores equals the oracle's reference loop
    over the oracle's regions (the VAD producer's untrained-model case)."""
    import torch
    from whisperx_amd.vad import SlidingWindow, SlidingWindowFeature, merge_chunks

    rng = np.random.default_rng(13)
    y = rng.random(213_333).astype(np.float32)
    med = float(np.median(y))
    sw = SlidingWindow(0.0, 0.016875, 0.0619375)
    got = merge_chunks(SlidingWindowFeature(torch.from_numpy(y)[:, None].to("cuda:0"), sw), 30, onset=med, offset=med)
    regs = oracle.binarize(y, 0.0, 0.016875, 0.0619375, med, med, max_duration=30)
    want = oracle.merge_chunks_regions(regs, 30)
    assert got == want
