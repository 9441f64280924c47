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
