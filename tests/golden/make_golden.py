"""Golden-vector generator for the forced-alignment + VAD-segmentation path.

TEST INFRASTRUCTURE ONLY — run by hand in the build container, never on the GPU box,
never imported by the package or by the tests.  It imports the *reference* whisperX
(`/root/reference/whisperx`, read-only) behind small stand-ins for the modules this
image lacks (torchaudio, nltk, pyannote), runs the reference functions on seeded
synthetic inputs and writes only their inputs/outputs as fixtures:

  dp_cases.npz      get_trellis / backtrack / merge_repeats     (alignment.py:359-454)
  align_cases.npz   align() end to end with a fake CTC model    (alignment.py:100-354)
  align_cases.json  expected align() outputs
  vad_cases.npz     Binarize / merge_chunks                     (vad.py:61-195, 264-311)
  vad_cases.json    expected regions and chunks

No reference source text is copied into the repository: only numbers produced by it.

Stand-ins (recipe of SURVEY.md §8(c)):
  * torchaudio: empty ``pipelines`` so ``load_align_model`` takes the HF branch.
  * nltk Punkt: ``span_tokenize`` returns one span ``(0, len(text.rstrip()))``
    (NLTK 3.8's final slice for single-sentence text — parity for multi-sentence text
    is unpinned).  For the aggregation tests a second mode splits after ". " so that the
    reference's multi-sentence pandas aggregation is exercised; the build accepts the
    same splitter through ``whisperx_amd.alignment.set_sentence_splitter``.
  * pyannote.core: Segment/SlidingWindow/SlidingWindowFeature/Annotation with the
    semantics listed in SURVEY.md §8(c) (empty segments skipped, sorted timeline).

Usage:  python tests/golden/make_golden.py      (writes next to this file)
"""
from __future__ import annotations

import dataclasses
import importlib.util
import json
import math
import os
import sys
import types
from importlib.machinery import ModuleSpec
from types import SimpleNamespace

import numpy as np

REF = "/root/reference/whisperx"
OUT = os.path.dirname(os.path.abspath(__file__))

# --------------------------------------------------------------------------- stubs
import transformers  # noqa: E402,F401  (must come before the torchaudio stand-in)
import torch  # noqa: E402

SPLIT_MODE = {"mode": "single"}


def _install_stubs():
    ta = types.ModuleType("torchaudio")
    ta.__spec__ = ModuleSpec("torchaudio", None)
    ta.pipelines = SimpleNamespace(__all__=[])
    sys.modules["torchaudio"] = ta

    nltk = types.ModuleType("nltk")
    tok = types.ModuleType("nltk.tokenize")
    punkt = types.ModuleType("nltk.tokenize.punkt")

    class PunktParameters:
        def __init__(self):
            self.abbrev_types = set()

    class PunktSentenceTokenizer:
        def __init__(self, params=None):
            self.params = params

        def span_tokenize(self, text):
            if SPLIT_MODE["mode"] == "single":
                yield (0, len(text.rstrip()))
                return
            # test splitter: a sentence ends after ". " ; spans exclude the blank
            start = 0
            n = len(text.rstrip())
            i = 0
            while i < n:
                if text[i] == "." and i + 1 < n and text[i + 1] == " ":
                    yield (start, i + 1)
                    j = i + 1
                    while j < n and text[j] == " ":
                        j += 1
                    start = j
                    i = j
                    continue
                i += 1
            if start < n:
                yield (start, n)

    punkt.PunktParameters = PunktParameters
    punkt.PunktSentenceTokenizer = PunktSentenceTokenizer
    tok.punkt = punkt
    nltk.tokenize = tok
    for m in (nltk, tok, punkt):
        m.__spec__ = ModuleSpec(m.__name__, None)
    sys.modules.update({"nltk": nltk, "nltk.tokenize": tok, "nltk.tokenize.punkt": punkt})

    # pyannote ------------------------------------------------------------------
    @dataclasses.dataclass(frozen=True, order=True)
    class Segment:
        start: float = 0.0
        end: float = 0.0

        def __bool__(self):
            return bool((self.end - self.start) > 1e-6)

        @property
        def middle(self):
            return 0.5 * (self.start + self.end)

        @property
        def duration(self):
            return self.end - self.start if self else 0.0

    class SlidingWindow:
        def __init__(self, start=0.0, step=0.0, duration=0.0):
            self.start, self.step, self.duration = start, step, duration

        def __getitem__(self, i):
            s = self.start + i * self.step
            return Segment(s, s + self.duration)

    class SlidingWindowFeature:
        def __init__(self, data, sliding_window, labels=None):
            self.data, self.sliding_window, self.labels = data, sliding_window, labels

    class Annotation:
        def __init__(self):
            self._tracks = {}

        def __setitem__(self, key, label):
            seg, track = key
            if not seg:
                return
            self._tracks[(seg, track)] = label

        def __delitem__(self, key):
            del self._tracks[key]

        def get_timeline(self):
            return sorted({s for (s, _t) in self._tracks})

        def itertracks(self):
            for (s, t) in sorted(self._tracks, key=lambda st: (st[0], str(st[1]))):
                yield s, t

    pa = types.ModuleType("pyannote")
    paa = types.ModuleType("pyannote.audio")
    paa.Model = object
    paa.Pipeline = object
    pac = types.ModuleType("pyannote.audio.core")
    paci = types.ModuleType("pyannote.audio.core.io")
    paci.AudioFile = object
    pap = types.ModuleType("pyannote.audio.pipelines")
    pap.VoiceActivityDetection = object
    papu = types.ModuleType("pyannote.audio.pipelines.utils")
    papu.PipelineModel = object
    pcore = types.ModuleType("pyannote.core")
    pcore.Annotation, pcore.Segment, pcore.SlidingWindowFeature = Annotation, Segment, SlidingWindowFeature
    pcore.SlidingWindow = SlidingWindow
    for m in (pa, paa, pac, paci, pap, papu, pcore):
        m.__spec__ = ModuleSpec(m.__name__, None)
        sys.modules[m.__name__] = m
    return SimpleNamespace(Segment=Segment, SlidingWindow=SlidingWindow,
                           SlidingWindowFeature=SlidingWindowFeature, Annotation=Annotation)


def _load_reference():
    pc = _install_stubs()
    pkg = types.ModuleType("whisperx")
    pkg.__path__ = [REF]
    pkg.__spec__ = ModuleSpec("whisperx", None, is_package=True)
    sys.modules["whisperx"] = pkg
    mods = {}
    for name in ("alignment", "vad"):
        spec = importlib.util.spec_from_file_location(f"whisperx.{name}", os.path.join(REF, f"{name}.py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[f"whisperx.{name}"] = mod
        spec.loader.exec_module(mod)
        mods[name] = mod
    return mods["alignment"], mods["vad"], pc


# --------------------------------------------------------------------------- inputs
def peaky_emission(rng, T, V, N, blank=0, quant=None):
    """SURVEY.md §8(d) emission generator: N(0,1) logits, +6 on the blank column, +12 at N
    sorted distinct frames for uniform tokens in [1,V) (blank excluded), fp32 log_softmax."""
    logits = rng.standard_normal((T, V)).astype(np.float32)
    logits[:, blank] += 6.0
    nonblank = np.array([v for v in range(V) if v != blank])
    toks = nonblank[rng.integers(0, len(nonblank), N)]
    if N <= max(T - 2, 0):
        frames = np.sort(rng.choice(np.arange(1, T - 1), N, replace=False))
        logits[frames, toks] += 12.0
    em = torch.log_softmax(torch.from_numpy(logits), dim=-1).numpy()
    if quant:
        em = (np.round(em * quant) / quant).astype(np.float32)
    return np.ascontiguousarray(em), toks.astype(np.int64)


def dp_reference(A, em, toks, blank):
    e = torch.from_numpy(em)
    tl = [int(x) for x in toks]
    tr = A.get_trellis(e, tl, blank)
    path = A.backtrack(tr, e, tl, blank)
    tstart = int(torch.argmax(tr[:, tr.size(1) - 1]).item())
    return tr.numpy(), tstart, path


def build_dp_cases(A):
    rng = np.random.default_rng(1234)
    cases = []
    # (T, V, N, blank, quant, nonfinite)
    specs = [
        (1, 29, 1, 0, None, None), (2, 29, 1, 0, None, None), (3, 32, 2, 0, None, None),
        (5, 32, 4, 0, None, None), (10, 32, 11, 0, None, None), (10, 32, 10, 0, None, None),
        (10, 32, 9, 0, None, None), (12, 32, 12, 0, None, None),
        (40, 29, 1, 0, None, None), (40, 29, 39, 0, None, None), (40, 29, 40, 0, None, None),
        (40, 29, 41, 0, None, None), (64, 32, 63, 5, None, None),
        (100, 32, 30, 0, 16, None), (100, 32, 60, 0, 16, None), (200, 32, 80, 0, 4, None),
        (300, 40, 120, 3, 16, None), (257, 32, 64, 0, None, None), (257, 32, 65, 0, None, None),
        (333, 32, 128, 31, None, None), (500, 29, 200, 0, None, None), (640, 32, 129, 0, 8, None),
        (150, 32, 100, 0, None, "neginf"), (60, 32, 58, 0, None, "neginf"),
        (80, 32, 30, 0, None, "nan"), (90, 32, 89, 0, None, "neginf_blank"),
        (1499, 32, 420, 0, None, None), (1499, 32, 364, 0, 16, None),
        (2999, 40, 900, 0, None, None), (700, 32, 2100, 0, None, None),
        (2100, 32, 1100, 0, None, None),
    ]
    for ci, (T, V, N, blank, quant, nf) in enumerate(specs):
        em, toks = peaky_emission(rng, T, V, N, blank, quant)
        if nf == "neginf":
            m = rng.random(em.shape) < 0.05
            em[m] = -np.inf
        elif nf == "nan":
            em[rng.integers(0, T), rng.integers(0, V)] = np.nan
            em[rng.integers(0, T), 0] = np.nan
        elif nf == "neginf_blank":
            em[rng.integers(0, T, 5), blank] = -np.inf
            em[rng.integers(0, T, 5), toks[0]] = -np.inf
        tr, tstart, path = dp_reference(A, em, toks, blank)
        transcript = "".join(chr(97 + (int(x) % 26)) for x in toks)
        c = {"em": em, "tokens": toks, "blank": np.int64(blank), "t_start": np.int64(tstart)}
        if path is None:
            c["path_ok"] = np.int64(0)
        else:
            c["path_ok"] = np.int64(1)
            c["path_tok"] = np.array([p.token_index for p in path], np.int64)
            c["path_time"] = np.array([p.time_index for p in path], np.int64)
            c["path_prob"] = np.array([p.score for p in path], np.float64)
            segs = A.merge_repeats(path, transcript)
            c["seg_start"] = np.array([s.start for s in segs], np.int64)
            c["seg_end"] = np.array([s.end for s in segs], np.int64)
            c["seg_score"] = np.array([s.score for s in segs], np.float64)
            c["seg_label"] = np.array([ord(s.label) for s in segs], np.int64)
            words = A.merge_words(segs, separator=transcript[0])
            c["word_start"] = np.array([w.start for w in words], np.int64)
            c["word_end"] = np.array([w.end for w in words], np.int64)
            c["word_score"] = np.array([w.score for w in words], np.float64)
            c["word_text"] = np.array([sum(ord(ch) * (k + 1) for k, ch in enumerate(w.label)) for w in words], np.int64)
        if tr.size <= 400_000:
            c["trellis"] = tr
        c["trellis_sha"] = np.frombuffer(__import__("hashlib").sha256(np.ascontiguousarray(tr).tobytes()).digest(), np.uint8)
        c["trellis_colN"] = tr[:, -1].copy()
        c["trellis_rowT"] = tr[-1, :].copy()
        for k, v in c.items():
            cases.append((f"c{ci:03d}_{k}", v))
    arrays = dict(cases)
    arrays["n_cases"] = np.int64(len(specs))
    np.savez_compressed(os.path.join(OUT, "dp_cases.npz"), **arrays)
    print("dp cases:", len(specs))


# --------------------------------------------------------------------------- align()
W2V_BASE_VOCAB = ["<pad>", "<s>", "</s>", "<unk>", "|", "E", "T", "A", "O", "N", "I", "H", "S", "R",
                  "D", "L", "U", "M", "W", "C", "F", "G", "Y", "P", "B", "V", "K", "'", "X", "J", "Q", "Z"]


def n_frames(samples):
    return (samples - 400) // 320 + 1 if samples >= 400 else 1


class FakeCTC(torch.nn.Module):
    """Returns queued logits, like a HF Wav2Vec2ForCTC (`.logits`), one per forward call."""

    def __init__(self, queue):
        super().__init__()
        self.queue = list(queue)

    def forward(self, x):
        lg = self.queue.pop(0)
        return SimpleNamespace(logits=torch.from_numpy(lg)[None].to(x.device))


def text_logits(rng, text, dictionary, lang, T, V, blank, sharp=12.0):
    """Peaky logits that spell the clean text over T frames (so that alignment is meaningful)."""
    logits = rng.standard_normal((T, V)).astype(np.float32)
    logits[:, blank] += 5.0
    chars = []
    for ch in text.strip().lower():
        c = ch if lang in ("ja", "zh") else ch.replace(" ", "|")
        if c in dictionary:
            chars.append(dictionary[c])
    if chars and T > len(chars) + 2:
        frames = np.sort(rng.choice(np.arange(1, T - 1), len(chars), replace=False))
        logits[frames, np.array(chars)] += sharp
    return logits


ALIGN_TEXTS = [
    " Hello world, this is a test of the forced alignment.",
    "The quick brown fox jumps over the lazy dog 42 times!  ",
    "  Mr. Smith went to Washington. He stayed for 3 days. Then he left.",
    "No problem at all",
    "1234 5678",
    "It's   spaced   out   oddly .",
    "Dr. Who vs. the daleks, said prof. X.",
    "a",
    "Short.",
    "We hold these truths to be self-evident, that all men are created equal, that they are endowed "
    "by their Creator with certain unalienable Rights, that among these are Life, Liberty and the "
    "pursuit of Happiness.",
]


def build_align_cases(A):
    rng = np.random.default_rng(77)
    dictionary = {c.lower(): i for i, c in enumerate(W2V_BASE_VOCAB)}
    V = len(W2V_BASE_VOCAB)
    arrays = {}
    expected = []
    scenarios = []
    audio_sec = 120.0
    # scenario list: (lang, split_mode, return_chars, interp, segments)
    def segs_from(texts, t0=0.5, gap=0.7):
        out, t = [], t0
        for tx in texts:
            dur = round(0.9 + 0.065 * len(tx.strip()) + rng.random(), 3)
            out.append({"start": round(t, 3), "end": round(t + dur, 3), "text": tx})
            t += dur + gap
        return out

    scenarios.append(("en", "single", False, "nearest", segs_from(ALIGN_TEXTS)))
    scenarios.append(("en", "single", True, "nearest", segs_from(ALIGN_TEXTS[:6])))
    scenarios.append(("en", "split", True, "nearest", segs_from(ALIGN_TEXTS)))
    scenarios.append(("en", "split", False, "linear", segs_from(ALIGN_TEXTS[2:7])))
    # failure modes: t1 >= duration, backtrack failure (text longer than frames), very short segment (<400 samples)
    fail = [{"start": 130.0, "end": 131.0, "text": "beyond the end"},
            {"start": 3.0, "end": 3.3, "text": "this text is far too long for a third of a second of audio"},
            {"start": 5.0, "end": 5.02, "text": "x"},
            {"start": 6.0, "end": 7.5, "text": "ok then"}]
    scenarios.append(("en", "single", True, "nearest", fail))
    # language without spaces: use the same char dictionary extended with CJK chars
    scenarios.append(("ja", "single", True, "nearest",
                      [{"start": 1.0, "end": 3.0, "text": "こんにちは世界"}, {"start": 4.0, "end": 5.5, "text": " 日本語 テスト "}]))
    # long-ish segment with many words, single sentence, chars returned
    scenarios.append(("en", "single", True, "nearest", segs_from([ALIGN_TEXTS[9] * 2], t0=10.0)))

    cjk = {ch: V + i for i, ch in enumerate("こんにちは世界日本語テスト")}
    for si, (lang, mode, ret_chars, interp, segments) in enumerate(scenarios):
        dct = dict(dictionary)
        VV = V
        if lang == "ja":
            dct.update(cjk)
            VV = V + len(cjk)
        audio = np.zeros(int(audio_sec * 16000), np.float32)
        queue = []
        for s in segments:
            f1, f2 = int(s["start"] * 16000), int(s["end"] * 16000)
            samples = max(0, min(f2, len(audio)) - f1)
            T = n_frames(max(samples, 400))
            queue.append(text_logits(rng, s["text"], dct, lang, T, VV, 0))
        # the reference only calls the model for segments that pass the checks; we record
        # every candidate logit and let the fake model pop them in call order.
        model = FakeCTC(queue)
        calls = []
        orig_forward = model.forward

        def fwd(x, _orig=orig_forward, _calls=calls):
            out = _orig(x)
            _calls.append(out.logits.shape[1])
            return out

        model.forward = fwd
        SPLIT_MODE["mode"] = mode
        segs_in = [dict(s) for s in segments]
        # pre-filter the queue to the segments that will reach the forward (same checks as
        # alignment.py:199-207) so logits stay matched to their segment
        clean_ok = []
        for s in segs_in:
            text = s["text"]
            nl = len(text) - len(text.lstrip())
            nt = len(text) - len(text.rstrip())
            ok = False
            for cdx, ch in enumerate(text):
                c = ch.lower()
                if lang not in ("ja", "zh"):
                    c = c.replace(" ", "|")
                if cdx < nl or cdx > len(text) - nt - 1:
                    continue
                if c in dct:
                    ok = True
            clean_ok.append(ok and s["start"] < audio_sec)
        model.queue = [q for q, ok in zip(queue, clean_ok) if ok]
        fed = list(model.queue)
        meta = {"language": lang, "dictionary": dct, "type": "huggingface"}
        out = A.align(segs_in, model, meta, audio, "cpu", interpolate_method=interp,
                      return_char_alignments=ret_chars)
        assert not model.queue, "logit queue not consumed"
        for k, lg in enumerate(fed):
            arrays[f"s{si:02d}_logits{k:02d}"] = lg
        mutated = [{k: s[k] for k in ("clean_char", "clean_cdx", "clean_wdx", "sentence_spans")} for s in segs_in]
        expected.append({"lang": lang, "split": mode, "return_char_alignments": ret_chars,
                         "interpolate_method": interp, "segments": segments, "n_logits": len(fed),
                         "audio_sec": audio_sec, "dictionary": dct, "result": _jsonable(out),
                         "mutated": _jsonable(mutated)})
    SPLIT_MODE["mode"] = "single"
    np.savez_compressed(os.path.join(OUT, "align_cases.npz"), **arrays)
    with open(os.path.join(OUT, "align_cases.json"), "w") as f:
        json.dump(expected, f, ensure_ascii=False, indent=0)
    print("align scenarios:", len(scenarios))


def _jsonable(x):
    if isinstance(x, dict):
        return {str(k): _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    if isinstance(x, (np.floating,)):
        return float(x)
    if isinstance(x, (np.integer,)):
        return int(x)
    if isinstance(x, float) and math.isnan(x):
        return "NaN"
    return x


# --------------------------------------------------------------------------- VAD
def vad_scores(rng, F, smooth=40, bias=0.0, scale=4.0):
    x = rng.standard_normal(F + smooth).astype(np.float64)
    k = np.ones(smooth) / smooth
    y = np.convolve(x, k, mode="valid")[:F] * scale * math.sqrt(smooth) / 3.0 + bias
    return (1.0 / (1.0 + np.exp(-y))).astype(np.float32)


def build_vad_cases(Vd, pc):
    rng = np.random.default_rng(99)
    arrays, expected = {}, []
    STEP, DUR = 0.016875, 0.0619375
    specs = [
        # (F, smooth, bias, onset, offset, chunk, sw_start)
        (200, 10, 0.0, 0.5, 0.363, 30, 0.0),
        (5000, 40, 0.0, 0.5, 0.363, 30, 0.0),
        (5000, 40, 0.0, 0.5, 0.363, 5, 0.0),
        (5000, 40, 1.5, 0.5, 0.363, 3, 0.0),
        (20000, 60, 0.5, 0.5, 0.363, 30, 0.0),
        (20000, 60, 0.5, 0.6, None, 10, 0.25),
        (35556, 40, 0.0, 0.5, 0.363, 30, 0.0),   # 10 minutes
        (35556, 80, 3.0, 0.5, 0.363, 30, 0.0),   # mostly speech -> min-cut splits
        (3000, 40, -8.0, 0.5, 0.363, 30, 0.0),   # silence
        (3000, 40, 9.0, 0.5, 0.363, 30, 0.0),    # all speech
        (1, 1, 0.0, 0.5, 0.363, 30, 0.0),
        (2, 1, 5.0, 0.5, 0.363, 30, 0.0),
        (4000, 30, 0.0, 0.5, 0.363, 1, 0.0),
    ]
    for ci, (F, smooth, bias, onset, offset, chunk, sw0) in enumerate(specs):
        sc = vad_scores(rng, F, smooth, bias)
        if ci == 1:  # exact threshold ties
            sc[::97] = np.float32(0.5)
            sc[5::89] = np.float32(0.363)
        sw = pc.SlidingWindow(start=sw0, step=STEP, duration=DUR)
        feat = pc.SlidingWindowFeature(sc[:, None], sw)
        b = Vd.Binarize(max_duration=chunk, onset=onset, offset=offset)
        ann = b(feat)
        regions = [[s.start, s.end] for s in ann.get_timeline()]
        chunks = Vd.merge_chunks(feat, chunk, onset=onset, offset=offset)
        arrays[f"v{ci:02d}_scores"] = sc
        expected.append({"F": F, "onset": onset, "offset": offset, "chunk_size": chunk,
                         "sw_start": sw0, "sw_step": STEP, "sw_duration": DUR,
                         "regions": regions,
                         "chunks": [{"start": c["start"], "end": c["end"],
                                     "segments": [list(p) for p in c["segments"]]} for c in chunks]})
    # Binarize with min_duration_on (no pads / min_duration_off: those need pyannote's support())
    sc = vad_scores(rng, 8000, 20, 0.0)
    arrays["vmin_scores"] = sc
    sw = pc.SlidingWindow(start=0.0, step=STEP, duration=DUR)
    ann = Vd.Binarize(onset=0.5, offset=0.363, min_duration_on=0.25)(pc.SlidingWindowFeature(sc[:, None], sw))
    expected_min = [[s.start, s.end] for s, _t in ann.itertracks()]
    # offset > onset (transcribe.py:42-43 --vad_onset/--vad_offset): a frame can both set and
    # reset the hysteresis state (vad.py:146-175).  Own generator, so the cases above keep
    # their scores.
    rng2 = np.random.default_rng(4242)
    specs2 = [
        (5000, 40, 0.0, 0.4, 0.6, 30, 0.0),
        (5000, 40, 0.0, 0.5, 0.55, 30, 0.0),
        (4000, 30, 0.0, 0.4, 0.6, 1, 0.0),
        (4000, 30, 0.0, 0.5, 0.55, 1, 0.0),
        (35556, 80, 3.0, 0.4, 0.6, 30, 0.0),    # mostly speech: min-cut splits
        (35556, 80, 3.0, 0.5, 0.55, 30, 0.125),
        (20000, 60, 0.5, 0.45, 0.7, 10, 0.25),
        (3000, 40, 9.0, 0.4, 0.6, 1, 0.0),      # all speech, a cut every second
        (3000, 20, 0.0, 0.3, 0.9, 5, 0.0),
    ]
    base = len(specs)
    for k, (F, smooth, bias, onset, offset, chunk, sw0) in enumerate(specs2):
        ci = base + k
        sc = vad_scores(rng2, F, smooth, bias)
        if k == 0:  # exact threshold ties
            sc[::83] = np.float32(0.4)
            sc[7::71] = np.float32(0.6)
        sw = pc.SlidingWindow(start=sw0, step=STEP, duration=DUR)
        feat = pc.SlidingWindowFeature(sc[:, None], sw)
        ann = Vd.Binarize(max_duration=chunk, onset=onset, offset=offset)(feat)
        chunks = Vd.merge_chunks(feat, chunk, onset=onset, offset=offset)
        arrays[f"v{ci:02d}_scores"] = sc
        expected.append({"F": F, "onset": onset, "offset": offset, "chunk_size": chunk,
                         "sw_start": sw0, "sw_step": STEP, "sw_duration": DUR,
                         "regions": [[s.start, s.end] for s in ann.get_timeline()],
                         "chunks": [{"start": c["start"], "end": c["end"],
                                     "segments": [list(p) for p in c["segments"]]} for c in chunks]})
    np.savez_compressed(os.path.join(OUT, "vad_cases.npz"), **arrays)
    with open(os.path.join(OUT, "vad_cases.json"), "w") as f:
        json.dump({"cases": expected, "min_duration_on": {"onset": 0.5, "offset": 0.363,
                   "min_duration_on": 0.25, "regions": expected_min}}, f, indent=0)
    print("vad cases:", len(specs) + len(specs2) + 1)


if __name__ == "__main__":
    torch.set_num_threads(1)
    A, Vd, pc = _load_reference()
    build_dp_cases(A)
    build_align_cases(A)
    build_vad_cases(Vd, pc)
