"""Shared helpers to replay tests/golden/align_cases.* through whisperx_amd.align()."""
import json
import math
import os
from types import SimpleNamespace

import numpy as np
import torch

from conftest import GOLDEN


def test_splitter(text):
    """Same sentence splitter make_golden.py used for its "split" scenarios (a sentence ends
    after '. '); the reference's Punkt stand-in for those fixtures."""
    start = 0
    n = len(text.rstrip())
    i = 0
    out = []
    while i < n:
        if text[i] == "." and i + 1 < n and text[i + 1] == " ":
            out.append((start, i + 1))
            j = i + 1
            while j < n and text[j] == " ":
                j += 1
            start = j
            i = j
            continue
        i += 1
    if start < n:
        out.append((start, n))
    return out


def single_span(text):
    return [(0, len(text.rstrip()))]


class FakeCTC(torch.nn.Module):
    """A Wav2Vec2ForCTC stand-in returning queued logits (.logits), one per forward."""

    def __init__(self, queue):
        super().__init__()
        self.queue = list(queue)

    def forward(self, x):
        lg = self.queue.pop(0)
        return SimpleNamespace(logits=torch.from_numpy(lg)[None].to(x.device))


def scenarios():
    with open(os.path.join(GOLDEN, "align_cases.json")) as f:
        meta = json.load(f)
    arr = np.load(os.path.join(GOLDEN, "align_cases.npz"))
    out = []
    for si, sc in enumerate(meta):
        logits = [arr[f"s{si:02d}_logits{k:02d}"] for k in range(sc["n_logits"])]
        out.append((sc, logits))
    return out


def run_scenario(align_fn, sc, logits, device):
    from whisperx_amd import alignment

    alignment.set_sentence_splitter(test_splitter if sc["split"] == "split" else single_span)
    try:
        segs = [dict(s) for s in sc["segments"]]
        audio = np.zeros(int(sc["audio_sec"] * 16000), np.float32)
        model = FakeCTC(logits)
        meta = {"language": sc["lang"], "dictionary": sc["dictionary"], "type": "huggingface"}
        out = align_fn(segs, model, meta, audio, device, interpolate_method=sc["interpolate_method"],
                       return_char_alignments=sc["return_char_alignments"])
        assert not model.queue
        mutated = [{k: s[k] for k in ("clean_char", "clean_cdx", "clean_wdx", "sentence_spans")} for s in segs]
        return out, mutated
    finally:
        alignment.set_sentence_splitter(None)


def jsonable(x):
    if isinstance(x, dict):
        return {str(k): jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [jsonable(v) for v in x]
    if isinstance(x, np.floating):
        return float(x)
    if isinstance(x, np.integer):
        return int(x)
    if isinstance(x, float) and math.isnan(x):
        return "NaN"
    return x


def compare(got, exp, path="", time_tol=0.0, score_tol=0.0, stats=None):
    """Structural comparison; numbers under 'start'/'end' within time_tol, 'score' within
    score_tol, everything else exact.  Key sets and order must match."""
    if isinstance(exp, dict):
        assert isinstance(got, dict), path
        assert list(got.keys()) == list(exp.keys()), f"{path}: keys {list(got.keys())} != {list(exp.keys())}"
        for k in exp:
            compare(got[k], exp[k], f"{path}.{k}", time_tol, score_tol, stats)
        return
    if isinstance(exp, list):
        assert isinstance(got, list) and len(got) == len(exp), f"{path}: len {len(got)} != {len(exp)}"
        for i, (g, e) in enumerate(zip(got, exp)):
            compare(g, e, f"{path}[{i}]", time_tol, score_tol, stats)
        return
    if isinstance(exp, float) and not isinstance(exp, bool):
        key = path.rsplit(".", 1)[-1]
        tol = time_tol if key in ("start", "end") else (score_tol if key == "score" else 0.0)
        if stats is not None:
            stats["n"] = stats.get("n", 0) + 1
            if got != exp:
                stats["diff"] = stats.get("diff", 0) + 1
            if key in ("start", "end"):
                stats.setdefault("abs_err", []).append(abs(got - exp))
        assert abs(got - exp) <= tol + 1e-12, f"{path}: {got} != {exp} (tol {tol})"
        return
    assert got == exp, f"{path}: {got!r} != {exp!r}"
