"""Seeded synthetic workloads of BASELINE.json's configs for the bench and
the GPU tests.  There is no network here or on the GPU box: no audio corpus, no VAD or
wav2vec2 checkpoints.  Everything below is shaped like the real inputs, never the real data.

* ``corpus_durations``: config 4's corpus, 40 files with log-uniform durations in 1-60 min
  summing to 10 h.
* ``vad_scores``: a file's VAD scores, smoothed Gaussian noise through a sigmoid, on the
  pyannote segmentation model's frame geometry (16.875 ms step, 61.9375 ms window).
* ``Transcriber``: the ASR stage's output stand-in, random lower-case words at ~14 chars/s
  for each VAD chunk, with the chunk bounds rounded to 3 decimals as asr.py:226-232 does.
* ``SyntheticCTC``: a cheap, deterministic CTC "model" with wav2vec2's frame geometry and
  ``.logits`` / ``.lm_head`` like Wav2Vec2ForCTC, for parity tests that re-derive the same
  emissions on the CPU oracle side.
"""
from __future__ import annotations

from types import SimpleNamespace
from typing import List

import numpy as np
import torch

from .emission import n_frames

W2V_VOCAB = ["<pad>", "<s>", "</s>", "<unk>", "|", "E", "T", "A", "O", "N", "I", "H", "S", "R",
             "D", "L", "U", "M", "W", "C", "F", "G", "Y", "P", "B", "V", "K", "'", "X", "J", "Q", "Z"]
VAD_STEP = 0.016875
VAD_DURATION = 0.0619375
LETTERS = "etaoinshrdlucmfwypvbgkqjxz"


def w2v_dictionary():
    """wav2vec2-base-960h's {char.lower(): id} (alignment.py:93): '<pad>' = 0 is the blank."""
    return {c.lower(): i for i, c in enumerate(W2V_VOCAB)}


# A German character vocabulary of BASELINE config 5's size (V = 40), laid out like the HF
# xlsr CTC tokenizers the DEFAULT_ALIGN_MODELS_HF entries use: '<pad>' first (the blank),
# '|' for the word boundary, lower-case letters with umlauts and sharp s.
DE_VOCAB = ["<pad>", "<s>", "</s>", "<unk>", "|", "'", "-"] + list("abcdefghijklmnopqrstuvwxyz") + \
           ["ä", "ö", "ü", "ß", "é", "à", "."]
DE_LETTERS = "enisratdhulcgmobwfkzvpüäößjyxq"


def de_dictionary():
    """config 5's {char: id} (V = 40, '<pad>' = 0 the blank)."""
    assert len(DE_VOCAB) == 40
    return {c: i for i, c in enumerate(DE_VOCAB)}


def corpus_durations(seed: int = 4, n_files: int = 40, total_s: float = 36000.0, lo_s: float = 60.0,
                     hi_s: float = 3600.0) -> List[float]:
    """Log-uniform durations in [lo_s, hi_s], rescaled to sum to total_s (clipped, re-spread)."""
    rng = np.random.default_rng(seed)
    d = np.exp(rng.uniform(np.log(lo_s), np.log(hi_s), n_files))
    for _ in range(50):
        d = d * (total_s / d.sum())
        d = np.clip(d, lo_s, hi_s)
        if abs(d.sum() - total_s) < 1e-6:
            break
    return [float(round(x, 3)) for x in d]


def vad_scores(seed: int, duration_s: float):
    """[F, 1] fp32 speech probabilities for a file (F = duration / 16.875 ms): 40-frame moving
    average of N(0,1), scaled, sigmoid.  Returns a SlidingWindowFeature."""
    from .vad import SlidingWindow, SlidingWindowFeature

    rng = np.random.default_rng(seed)
    F = max(int(duration_s / VAD_STEP), 1)
    x = rng.standard_normal(F + 40)
    y = np.convolve(x, np.ones(40) / 40, mode="valid")[:F] * 4 * np.sqrt(40) / 3
    data = (1 / (1 + np.exp(-y))).astype(np.float32)[:, None]
    return SlidingWindowFeature(data, SlidingWindow(start=0.0, duration=VAD_DURATION, step=VAD_STEP))


class Transcriber:
    """ASR stand-in: each VAD chunk becomes a segment {start, end, text} with start/end
    rounded to 3 decimals (asr.py:226-232) and ~14 chars/s of random words."""

    def __init__(self, seed: int, pool_words: int = 200_000, letters: str = LETTERS):
        rng = np.random.default_rng(seed)
        lens = rng.integers(2, 9, pool_words)
        idx = rng.integers(0, len(letters), int(lens.sum()))
        text = np.array(list(letters))[idx]
        cuts = np.concatenate([[0], np.cumsum(lens)])
        self.words = ["".join(text[cuts[i]:cuts[i + 1]]) for i in range(pool_words)]
        self.pos = 0

    def _take(self, n):
        if self.pos + n > len(self.words):
            self.pos = 0
        out = self.words[self.pos:self.pos + n]
        self.pos += n
        return out

    def segments(self, chunks):
        segs = []
        for c in chunks:
            n_words = max(1, int((c["end"] - c["start"]) * 14 / 5.5))
            segs.append({"start": round(c["start"], 3), "end": round(c["end"], 3),
                         "text": " ".join(self._take(n_words))})
        return segs


class SyntheticCTC(torch.nn.Module):
    """Deterministic CTC emissions with wav2vec2's frame count: frame t sees samples
    [320 t, 320 t + 400), projected to V logits (blank column raised by `blank_bias`).
    Looks like Wav2Vec2ForCTC to align(): forward(x).logits and lm_head.out_features."""

    def __init__(self, V: int = 32, seed: int = 0, blank_bias: float = 2.0, scale: float = 40.0):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.lm_head = torch.nn.Linear(400, V, bias=True)
        with torch.no_grad():
            self.lm_head.weight.copy_(torch.randn(V, 400, generator=g) * (scale / 20.0))
            self.lm_head.bias.zero_()
            self.lm_head.bias[0] = blank_bias

    def forward(self, x):
        S = int(x.shape[-1])
        T = n_frames(S)
        fr = x[0, : 320 * (T - 1) + 400].unfold(0, 400, 320)  # [T, 400]
        return SimpleNamespace(logits=self.lm_head(fr)[None])
