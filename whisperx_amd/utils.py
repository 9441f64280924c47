"""Small host utilities mirrored from whisperx/utils.py (LANGUAGES_WITHOUT_SPACES :127,
interpolate_nans :433-437)."""
from __future__ import annotations

import math

LANGUAGES_WITHOUT_SPACES = ["ja", "zh"]


def interpolate_nans(x, method="nearest"):
    """utils.py:433-437: interpolate NaNs (pandas semantics), then ffill/bfill.

    Accepts a pandas Series (returns a Series, like the reference) or a list of floats
    (returns a list; NaN-free input is returned as is without touching pandas)."""
    if type(x).__name__ == "Series":
        if x.notnull().sum() > 1:
            return x.interpolate(method=method).ffill().bfill()
        return x.ffill().bfill()
    vals = [float(v) for v in x]
    if all(v == v for v in vals):
        return vals
    import pandas as pd  # (only when there is something to interpolate: its import costs ~1 s)

    s = pd.Series(vals, dtype="float64")
    if s.notnull().sum() > 1:
        s = s.interpolate(method=method)
    s = s.ffill().bfill()
    return [float(v) for v in s.tolist()]


def isnan(v) -> bool:
    return isinstance(v, float) and math.isnan(v)
