"""align() host logic (text prep, timestamps, sentence/word aggregation, NaN interpolation,
(start,end) grouping) against the reference's align() outputs, with the DP supplied by
the CPU oracle (checker) so that the host code is tested exactly without a GPU."""
import numpy as np
import pytest
import torch

from align_helpers import compare, jsonable, run_scenario, scenarios
from oracle import oracle


def _oracle_dp(ems, toks, blanks, dev):
    out = []
    for em, tk, bl in zip(ems, toks, blanks):
        ok, ts, ss, se, sc = oracle.align_dp(em.cpu().numpy(), tk, bl)
        out.append((ok, ss, se, sc, em.shape[0]))
    return out


@pytest.fixture
def cpu_align(monkeypatch):
    from whisperx_amd import alignment

    monkeypatch.setattr(alignment, "_run_dp", _oracle_dp)
    monkeypatch.setattr(alignment, "_dp_device", lambda device: torch.device("cpu"))
    return alignment.align


@pytest.mark.parametrize("si", range(len(scenarios())))
def test_align_host_logic_matches_reference(cpu_align, si, capsys):
    sc, logits = scenarios()[si]
    out, mutated = run_scenario(cpu_align, sc, logits, "cpu")
    compare(jsonable(out), sc["result"])
    assert jsonable(mutated) == sc["mutated"]


def test_word_score_uses_numpy_rounding():
    from whisperx_amd.alignment import _nanmean

    # pandas mean -> np.float64; round() on it is numpy's (0.1235 -> 0.124, Python's: 0.123)
    assert round(_nanmean([0.1235]), 3) == np.round(0.1235, 3)
    assert round(_nanmean([float("nan"), 0.5, 0.25]), 3) == 0.375


def test_interpolate_nans_list_and_series():
    import pandas as pd

    from whisperx_amd.utils import interpolate_nans

    vals = [float("nan"), 1.0, float("nan"), float("nan"), 4.0, float("nan")]
    for m in ("nearest", "linear"):
        ref = pd.Series(vals).interpolate(method=m).ffill().bfill().tolist()
        assert interpolate_nans(vals, m) == ref
        assert interpolate_nans(pd.Series(vals), m).tolist() == ref
    assert interpolate_nans([float("nan"), 2.0], "nearest") == [2.0, 2.0]
    assert interpolate_nans([1.0, 2.0], "nearest") == [1.0, 2.0]


def test_pack_ranges():
    """The packed encoder's segment ranges: consecutive, at most `cap` frames each, a longer
    segment alone."""
    from whisperx_amd import alignment

    assert alignment._pack_ranges([], 10) == []
    assert alignment._pack_ranges([4, 4, 4], 10) == [(0, 2), (2, 3)]
    assert alignment._pack_ranges([12, 1, 9, 1], 10) == [(0, 1), (1, 3), (3, 4)]
    assert alignment._pack_ranges([5, 5], 10) == [(0, 2)]
    # a last pack of >= 8 segments leaves its last eighth to a pack of its own
    assert alignment._pack_ranges([1499] * 16, 49152) == [(0, 14), (14, 16)]
    assert alignment._pack_ranges([1] * 9, 6) == [(0, 6), (6, 9)]
    assert alignment._pack_ranges([1] * 20, 12) == [(0, 12), (12, 19), (19, 20)]


def test_packed_segments_layout():
    from whisperx_amd import _lib

    s = _lib.PackedSegments([3, 0, 40])
    assert s.offsets == [0, 3, 3, 43] and s.rows == 43


def test_round3_matches_python_round():
    """alignment._round3 (vectorised char-timestamp rounding) equals Python's round(v, 3) on
    random values, exact decimal ties, their neighbouring doubles and timestamp-like products."""
    import math

    import numpy as np

    from whisperx_amd import alignment

    rng = np.random.default_rng(3)
    vals = list(rng.random(20000) * 7200) + list(rng.random(2000))
    ties = [k / 1000 + 0.0005 for k in range(0, 200000, 7)]
    vals += ties + [math.nextafter(v, 0) for v in ties] + [math.nextafter(v, 1e9) for v in ties]
    vals += [int(f) * (30.0 / 1499) + 30.0 * s for f in range(1499) for s in (0, 7, 113)]
    vals += [-v for v in vals[:500]] + [0.0, -0.0, 1e-9, 0.0005, 0.0015, 2.675]
    x = np.array(vals, dtype=np.float64)
    got = alignment._round3(x)
    for v, g in zip(vals, got):
        r = round(v, 3)
        assert g == r and math.copysign(1, g) == math.copysign(1, r), (v, g, r)


def test_nanmean_matches_numpy_sum():
    import math

    import numpy as np

    from whisperx_amd import alignment

    rng = np.random.default_rng(4)
    for n in range(1, 20):
        for _ in range(300):
            vals = [round(float(v), 3) for v in rng.random(n)]
            if n > 2:
                vals[int(rng.integers(n))] = math.nan
            cnt = sum(1 for v in vals if v == v)
            ref = np.float64(np.array([v if v == v else 0.0 for v in vals]).sum() / cnt)
            assert alignment._nanmean(vals) == ref


def test_np_round3_matches_numpy_scalar_round():
    import math

    import numpy as np

    from whisperx_amd import alignment

    rng = np.random.default_rng(5)
    vals = list(rng.random(20000)) + [k / 1000 + 0.0005 for k in range(3000)] + [2.675, 0.0005, -0.0004, -0.0, 0.0]
    vals += [math.nan, math.inf, -math.inf, 1e300]
    for v in vals:
        ref = round(np.float64(v), 3)
        got = alignment._np_round3(np.float64(v))
        assert type(got) is type(ref)
        assert (got == ref and math.copysign(1, got) == math.copysign(1, ref)) or (ref != ref and got != got), (v, got, ref)


def test_has_alignable_matches_prepare():
    """align() decides which segments get a forward with _has_alignable before _prepare runs:
    it must agree with _prepare's clean_char on every text (stripped range, lower-casing,
    ' ' -> '|' in languages with spaces, multi-char lower-case forms)."""
    from whisperx_amd import alignment

    rng = np.random.default_rng(5)
    pool = list("abc ABC|.,!?-'♪123 \t\nİßÅé日本")
    dicts = [{"a": 1, "|": 2}, {"b": 1}, {"i̇": 1, "x": 2}, {"日": 1}, {"|": 1}, {}]
    for _ in range(3000):
        text = "".join(rng.choice(pool, int(rng.integers(0, 12))))
        d = dicts[int(rng.integers(0, len(dicts)))]
        lang = ["en", "ja", "de"][int(rng.integers(0, 3))]
        seg = {"text": text}
        alignment._prepare(seg, d, lang)
        assert alignment._has_alignable(text, d, lang) == (len(seg["clean_char"]) > 0), (text, d, lang)


def test_align_runs_no_forward_for_segments_it_skips(cpu_align, capsys):
    """A segment with no alignable char (music, digits, a script the model lacks) and one past
    the audio get no forward (the reference never calls the model for them,
    alignment.py:185-202): the fake model holds logits for the two alignable segments only."""
    from align_helpers import FakeCTC

    rng = np.random.default_rng(3)
    d = {"<pad>": 0, "|": 1, "a": 2, "b": 3}
    T = 99  # frames of a 2 s segment

    def peaky(n_tok):
        lg = rng.standard_normal((T, 4)).astype(np.float32)
        lg[:, 0] += 6
        fr = np.sort(rng.choice(np.arange(1, T - 1), n_tok, replace=False))
        lg[fr, rng.integers(1, 4, n_tok)] += 12
        return lg

    model = FakeCTC([peaky(5), peaky(2)])
    segs = [{"start": 0.0, "end": 2.0, "text": "ab ba"}, {"start": 2.0, "end": 4.0, "text": " ♪123♪ "},
            {"start": 4.0, "end": 6.0, "text": "ab"}, {"start": 9.0, "end": 10.0, "text": "ab"}]
    out = cpu_align(segs, model, {"language": "en", "dictionary": d, "type": "huggingface"},
                    np.zeros(6 * 16000, np.float32), "cpu")
    assert not model.queue
    assert [s["text"] for s in out["segments"]] == ["ab ba", " ♪123♪ ", "ab", "ab"]
    assert out["segments"][1]["words"] == [] and out["segments"][3]["words"] == []
    assert len(out["segments"][0]["words"]) == 2 and len(out["segments"][2]["words"]) == 1
    msg = capsys.readouterr().out
    assert "no characters in this segment found in model dictionary" in msg
    assert "original start time longer than audio duration" in msg
