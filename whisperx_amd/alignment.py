"""Forced alignment for WhisperX on MI355X — drop-in for ``whisperx.alignment``.

Same public API and semantics as the reference (NADOOIT/whisperX @ 2025-01-12,
whisperx/alignment.py):

  load_align_model(language_code, device, model_name=None, model_dir=None)   :64-97
  align(transcript, model, align_model_metadata, audio, device, ...)           :100-354
  get_trellis(emission, tokens, blank_id=0)                                   :359-379
  backtrack(trellis, emission, tokens, blank_id=0)                            :387-421
  merge_repeats(path, transcript)                                             :438-454
  merge_words(segments, separator="|")                                        :456-470
  Point, Segment                                                              :381-436

What changes is where the work runs:
  * The emission forward stays a PyTorch-ROCm model call, one per segment (padding a
    batch would change wav2vec2's logits), queued back to back on the device with no
    host round trip; log_softmax stays on the device.
  * The whole DP for all segments of a call is ONE launch of the fused HIP kernel
    (libwxalign.so: wx_align_dp): trellis recurrence with a 1-bit decision map,
    argmax, backtrack and merge_repeats.  Only per-token (start, end, score) come back.
  * The per-segment pandas aggregation (:282-347) is re-implemented with plain Python/
    numpy, reproducing pandas' results (NaN-skipping min/max, numpy-summed means,
    np.round on word scores, groupby sort/NaN-drop, interpolate_nans).
There is no CPU fallback: without a HIP device the DP raises.
"""
from __future__ import annotations

import bisect
import contextlib
import math
import os
import time
from dataclasses import dataclass
from typing import Callable, Iterable, List, Optional, Union

import numpy as np
import torch

from . import _lib, emission, punkt
from .audio import SAMPLE_RATE, load_audio
from .types import AlignedTranscriptionResult, SingleAlignedSegment, SingleSegment, SingleWordSegment
from .utils import interpolate_nans

PUNKT_ABBREVIATIONS = ["dr", "vs", "mr", "mrs", "prof"]

LANGUAGES_WITHOUT_SPACES = ["ja", "zh"]

DEFAULT_ALIGN_MODELS_TORCH = {
    "en": "WAV2VEC2_ASR_BASE_960H",
    "fr": "VOXPOPULI_ASR_BASE_10K_FR",
    "de": "VOXPOPULI_ASR_BASE_10K_DE",
    "es": "VOXPOPULI_ASR_BASE_10K_ES",
    "it": "VOXPOPULI_ASR_BASE_10K_IT",
}

DEFAULT_ALIGN_MODELS_HF = {
    "ja": "jonatasgrosman/wav2vec2-large-xlsr-53-japanese",
    "zh": "jonatasgrosman/wav2vec2-large-xlsr-53-chinese-zh-cn",
    "nl": "jonatasgrosman/wav2vec2-large-xlsr-53-dutch",
    "uk": "Yehor/wav2vec2-xls-r-300m-uk-with-small-lm",
    "pt": "jonatasgrosman/wav2vec2-large-xlsr-53-portuguese",
    "ar": "jonatasgrosman/wav2vec2-large-xlsr-53-arabic",
    "cs": "comodoro/wav2vec2-xls-r-300m-cs-250",
    "ru": "jonatasgrosman/wav2vec2-large-xlsr-53-russian",
    "pl": "jonatasgrosman/wav2vec2-large-xlsr-53-polish",
    "hu": "jonatasgrosman/wav2vec2-large-xlsr-53-hungarian",
    "fi": "jonatasgrosman/wav2vec2-large-xlsr-53-finnish",
    "fa": "jonatasgrosman/wav2vec2-large-xlsr-53-persian",
    "el": "jonatasgrosman/wav2vec2-large-xlsr-53-greek",
    "tr": "mpoyraz/wav2vec2-xls-r-300m-cv7-turkish",
    "da": "saattrupdan/wav2vec2-xls-r-300m-ftspeech",
    "he": "imvladikon/wav2vec2-xls-r-300m-hebrew",
    "vi": "nguyenvulebinh/wav2vec2-base-vi",
    "ko": "kresnik/wav2vec2-large-xlsr-korean",
    "ur": "kingabzpro/wav2vec2-large-xls-r-300m-Urdu",
    "te": "anuragshas/wav2vec2-large-xlsr-53-telugu",
    "hi": "theainerd/Wav2Vec2-large-xlsr-hindi",
    "ca": "softcatala/wav2vec2-large-xlsr-catala",
    "ml": "gvs/wav2vec2-large-xlsr-malayalam",
    "no": "NbAiLab/nb-wav2vec2-1b-bokmaal",
    "nn": "NbAiLab/nb-wav2vec2-300m-nynorsk",
    "sk": "comodoro/wav2vec2-xls-r-300m-sk-cv8",
    "sl": "anton-l/wav2vec2-large-xlsr-53-slovenian",
    "hr": "classla/wav2vec2-xls-r-parlaspeech-hr",
}


# ------------------------------------------------------------------------------- loading
def load_align_model(language_code, device, model_name=None, model_dir=None):
    """alignment.py:64-97.  torchaudio bundles when torchaudio is installed; otherwise a
    Hugging Face Wav2Vec2ForCTC from a hub name or (offline) a local directory."""
    if model_name is None:
        if language_code in DEFAULT_ALIGN_MODELS_TORCH:
            model_name = DEFAULT_ALIGN_MODELS_TORCH[language_code]
        elif language_code in DEFAULT_ALIGN_MODELS_HF:
            model_name = DEFAULT_ALIGN_MODELS_HF[language_code]
        else:
            print(f"There is no default alignment model set for this language ({language_code}).\
                Please find a wav2vec2.0 model finetuned on this language in https://huggingface.co/models, then pass the model name in --align_model [MODEL_NAME]")
            raise ValueError(f"No default align-model for language: {language_code}")

    pipelines = _torchaudio_pipelines()
    if model_name in pipelines:
        import torchaudio

        pipeline_type = "torchaudio"
        bundle = torchaudio.pipelines.__dict__[model_name]
        align_model = bundle.get_model(dl_kwargs={"model_dir": model_dir}).to(device)
        labels = bundle.get_labels()
        align_dictionary = {c.lower(): i for i, c in enumerate(labels)}
    else:
        try:
            from transformers import Wav2Vec2ForCTC, Wav2Vec2Processor

            processor = Wav2Vec2Processor.from_pretrained(model_name, cache_dir=model_dir)
            align_model = Wav2Vec2ForCTC.from_pretrained(model_name, cache_dir=model_dir)
        except Exception as e:
            print(e)
            print("Error loading model from huggingface, check https://huggingface.co/models for finetuned wav2vec2.0 models")
            raise ValueError(f'The chosen align_model "{model_name}" could not be found in huggingface (https://huggingface.co/models) or torchaudio (https://pytorch.org/audio/stable/pipelines.html#id14)')
        pipeline_type = "huggingface"
        align_model = align_model.to(device)
        align_dictionary = {char.lower(): code for char, code in processor.tokenizer.get_vocab().items()}

    align_metadata = {"language": language_code, "dictionary": align_dictionary, "type": pipeline_type}
    return align_model, align_metadata


def _torchaudio_pipelines():
    try:
        import torchaudio  # noqa: F401

        return set(torchaudio.pipelines.__all__)
    except Exception:
        return set()


# ------------------------------------------------------------------------ sentence spans
_sentence_splitter: Optional[Callable[[str], list]] = None


def set_sentence_splitter(fn: Optional[Callable[[str], list]]):
    """Override the sentence splitter (fn(text) -> [(start, end)]); None restores Punkt."""
    global _sentence_splitter
    _sentence_splitter = fn


_punkt = None


def _sentence_spans(text: str):
    if _sentence_splitter is not None:
        return list(_sentence_splitter(text))
    global _punkt
    if _punkt is None:
        try:
            from nltk.tokenize.punkt import PunktParameters, PunktSentenceTokenizer

            params = PunktParameters()
            params.abbrev_types = set(PUNKT_ABBREVIATIONS)
            _punkt = PunktSentenceTokenizer(params)
        except Exception:
            _punkt = False
    if _punkt:
        return list(_punkt.span_tokenize(text))
    # nltk absent: the restated untrained-Punkt splitter (parity unpinned, whisperx_amd/punkt.py)
    return punkt.span_tokenize(text, PUNKT_ABBREVIATIONS)


# ------------------------------------------------------------------------------- align()
# WX_PROFILE=1: synchronise at align()'s phase boundaries and accumulate wall time per phase
# in PHASE_TIMES (diagnostics only; the sync points remove the overlap of the phases)
_PROFILE = bool(os.environ.get("WX_PROFILE"))
PHASE_TIMES: dict = {}


class _Phase:
    def __init__(self, name):
        self.name = name

    def __enter__(self):
        if _PROFILE:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self.t0 = time.perf_counter()

    def __exit__(self, *exc):
        if _PROFILE:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            PHASE_TIMES[self.name] = PHASE_TIMES.get(self.name, 0.0) + time.perf_counter() - self.t0


def _prepare(segment: dict, dictionary, lang: str):
    """alignment.py:137-177: clean chars/indices, clean words, sentence spans (mutates)."""
    text = segment["text"]
    num_leading = len(text) - len(text.lstrip())
    num_trailing = len(text) - len(text.rstrip())
    per_word = text.split(" ") if lang not in LANGUAGES_WITHOUT_SPACES else text
    spaces = lang not in LANGUAGES_WITHOUT_SPACES
    last = len(text) - num_trailing - 1
    clean_char, clean_cdx = [], []
    for cdx in range(num_leading, last + 1):
        c = text[cdx].lower()
        if spaces:
            c = c.replace(" ", "|")
        if c in dictionary:
            clean_char.append(c)
            clean_cdx.append(cdx)
    clean_wdx = [wdx for wdx, wrd in enumerate(per_word) if any(c in dictionary for c in wrd)]
    segment["clean_char"] = clean_char
    segment["clean_cdx"] = clean_cdx
    segment["clean_wdx"] = clean_wdx
    segment["sentence_spans"] = _sentence_spans(text)


def _has_alignable(text: str, dictionary, lang: str) -> bool:
    """Whether _prepare would keep any char of `text` (a non-empty clean_char, alignment.py:
    137-151): the same stripped range, lower-casing and space -> '|' rule, without building the
    lists.  align() queues a segment's forward only then, as the reference runs the model only
    for segments it does not skip (alignment.py:199-202)."""
    spaces = lang not in LANGUAGES_WITHOUT_SPACES
    for ch in text.strip():
        c = ch.lower()
        if spaces:
            c = c.replace(" ", "|")
        if c in dictionary:
            return True
    return False


class _PackedUnsupported(Exception):
    """The packed encoder cannot run this model (its frame geometry is not n_frames'): align()
    redoes the emissions on the per-segment route with the model prepared."""


def _logits(model, model_type, waveform_segment, device):
    """alignment.py:217-232 on the device: the [1, T, V] logits of one unpadded forward."""
    if waveform_segment.shape[-1] < 400:
        lengths = torch.as_tensor([waveform_segment.shape[-1]]).to(device)
        waveform_segment = torch.nn.functional.pad(waveform_segment, (0, 400 - waveform_segment.shape[-1]))
    else:
        lengths = None
    with torch.inference_mode():
        if model_type == "torchaudio":
            emissions, _ = model(waveform_segment.to(device), lengths=lengths)
        elif model_type == "huggingface":
            emissions = model(waveform_segment.to(device)).logits
        else:
            raise NotImplementedError(f"Align model of type {model_type} not supported.")
    return emissions


def _emission(model, model_type, waveform_segment, device):
    """alignment.py:217-235 without the host copy: the [T, V] log-probabilities (on device)."""
    with torch.inference_mode():
        return torch.log_softmax(_logits(model, model_type, waveform_segment, device), dim=-1)[0].detach()


class _EmissionsCSR:
    """Log-probabilities of S segments packed as one [sum_T, V] fp32 device matrix (the DP
    kernel's input layout); iterating yields each segment's [T, V] row slice."""

    def __init__(self, em: torch.Tensor, Ts, events=None):
        self.em = em
        self.Ts = list(Ts)
        self.off = [0]
        for T in self.Ts:
            self.off.append(self.off[-1] + T)
        self.events = events  # per segment: recorded on its forward's stream after log_softmax
        self.streams = []
        self.groups = None  # packed encoder: the packs' segment ranges

    def sub(self, a: int, b: int) -> "_EmissionsCSR":
        """Segments [a, b) as their own packed matrix (a row-range view: no copy)."""
        ev = self.events[a:b] if self.events is not None else None
        return _EmissionsCSR(self.em[self.off[a]: self.off[b]], self.Ts[a:b], ev)

    def wait(self, stream):
        """Make `stream` wait for these segments' forwards."""
        seen = set()
        for ev in self.events or ():
            if id(ev) not in seen:  # (a pack's segments share its event)
                seen.add(id(ev))
                stream.wait_event(ev)

    def __len__(self):
        return len(self.Ts)

    def __getitem__(self, i):
        return self.em[self.off[i]: self.off[i + 1]]

    def __iter__(self):
        return (self[i] for i in range(len(self)))


def _vocab_size(model, model_type):
    if model_type == "huggingface":
        head = getattr(model, "lm_head", None)
    else:
        head = getattr(model, "aux", None)
    n = getattr(head, "out_features", None)
    return int(n) if n else None


_EMISSION_STREAMS = {}


def _emissions(model, model_type, waveforms, device, n_streams: int = int(os.environ.get("WX_EMISSION_STREAMS", "8")),
               allow_packed: bool = True):
    """Emissions of every segment, one unpadded forward each (padding would change wav2vec2's
    logits, alignment.py:217-233), issued round-robin on `n_streams` (8; A/B on config 3: 2 / 4 / 8 streams 803 / 790 / 755 ms) HIP streams: one 30 s
    forward's GEMMs (1,499 rows) fill a fraction of the GPU, so consecutive segments overlap.
    On a HIP device each forward's log_softmax writes straight into its rows of one packed
    [sum_T, V] matrix (returned as _EmissionsCSR), which the DP reads in place; the model's
    convolutions take the length-agnostic GEMM route (emission.prepare_model) unless
    WX_MIOPEN_CONV=1.  Joined back onto the current stream."""
    dev = torch.device(device) if not isinstance(device, torch.device) else device
    if dev.type != "cuda":
        return [_emission(model, model_type, w, device) for w in waveforms]
    packed = (allow_packed and not os.environ.get("WX_MIOPEN_CONV") and model_type == "huggingface"
              and emission.packed_supported(model))
    if not os.environ.get("WX_MIOPEN_CONV") and not packed:
        emission.prepare_model(model)
        # cached weight_norm weights are built here, on the current stream, before the
        # side streams wait on it (a lazily built cache would race between the streams)
        emission.materialize_weights(model)
    V = _vocab_size(model, model_type)
    cfg_model = model if model_type == "huggingface" else None
    Ts = [emission.n_frames(int(w.shape[-1]), cfg_model) for w in waveforms]
    main = torch.cuda.current_stream(dev)
    if V is None or not waveforms:
        return [_emission(model, model_type, w, device) for w in waveforms]
    csr = _EmissionsCSR(torch.empty((max(sum(Ts), 1), V), dtype=torch.float32, device=dev), Ts)
    if sum(Ts) == 0:
        csr.em = csr.em[:0]
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), n_streams)
    streams = _EMISSION_STREAMS.get(key)
    if streams is None:
        streams = [torch.cuda.Stream(device=dev) for _ in range(max(n_streams, 1))]
        _EMISSION_STREAMS[key] = streams
    for st in streams:
        st.wait_stream(main)
    if packed:
        try:
            csr.groups = _pack_ranges(Ts)
            csr.events = _packed_emissions(model, waveforms, csr, streams)
            csr.streams = streams
            return csr
        except ValueError:  # a model whose frame geometry is not n_frames': per-segment path
            # whatever the packs queued on streams[0] finishes before anything else touches
            # those rows or the model, and the caller redoes the call on the prepared route
            main.wait_stream(streams[0])
            for st in streams:
                st.wait_stream(streams[0])
            raise _PackedUnsupported() from None
    bad = False
    csr.events = []
    for i, w in enumerate(waveforms):
        st = streams[i % len(streams)]
        with torch.cuda.stream(st):
            lg = _logits(model, model_type, w, device)
            if tuple(lg.shape) != (1, Ts[i], V):
                bad = True  # the model's frame geometry is not wav2vec2's: fall back below
                break
            with torch.inference_mode():
                emission.log_softmax_into(lg[0], csr[i])
            ev = torch.cuda.Event()
            ev.record(st)
            csr.events.append(ev)
    if bad:
        for st in streams:
            main.wait_stream(st)
        return [_emission(model, model_type, w, device) for w in waveforms]
    # not joined here: align() runs the DP group by group as their forwards finish, then
    # joins every stream back onto the current one
    csr.streams = streams
    return csr


_PACK_ROWS = 49152  # encoder rows per pack (~16 min of audio; WX_PACK_ROWS overrides)


def _pack_ranges(Ts, cap: Optional[int] = None):
    """Consecutive segment ranges [a, b) of at most `cap` frames each (a longer segment alone).
    WX_PACK_PLAN="12,4" (development A/B): explicit segments per pack instead."""
    plan = os.environ.get("WX_PACK_PLAN")
    if plan and cap is None:
        packs, a = [], 0
        for k in (int(x) for x in plan.split(",")):
            if a < len(Ts):
                packs.append((a, min(len(Ts), a + k)))
                a = packs[-1][1]
        if a < len(Ts):
            packs.append((a, len(Ts)))
        return packs
    cap = int(os.environ.get("WX_PACK_ROWS", _PACK_ROWS)) if cap is None else cap
    packs, a, rows = [], 0, 0
    for i, T in enumerate(Ts):
        if i > a and rows + T > cap:
            packs.append((a, i))
            a, rows = i, 0
        rows += T
    if Ts:
        packs.append((a, len(Ts)))
    # the last pack's eighth as a pack of its own: the host aggregates the rest of it while
    # the GPU runs that tail, leaving only the tail's aggregation after the last kernel
    # (e2e_align, 16 x 30 s: one pack 85.6 ms, 12 + 4 84.6 ms, 8 + 8 86.9 ms; after the host
    # work was cut, 12 + 4 75.2 ms, 13 + 3 76.4 ms, 14 + 2 73.6 ms)
    a, b = packs[-1] if packs else (0, 0)
    if b - a >= 8:
        t = (b - a) // 8
        packs[-1:] = [(a, b - t), (b - t, b)]
    return packs


def _packed_emissions(model, waveforms, csr, streams):
    """The packed-encoder route of _emissions (emission.packed_logits): segments in the packs
    csr.groups (consecutive ranges, _pack_ranges), all on streams[0] (the others only serve
    packed_logits' per-segment feature-encoder fallback), log_softmax of the whole pack into
    its CSR rows.  Returns the per-segment events (a pack's segments share its event)."""
    events = []
    # every pack on one stream: pack p finishes (and its DP and host aggregation start) as
    # early as possible instead of sharing the GPU with pack p + 1
    ps = streams[0]
    for a, b in csr.groups:
        with torch.cuda.stream(ps):
            lg = emission.packed_logits(model, waveforms[a:b], _lib.PackedSegments(csr.Ts[a:b]), streams)
            with torch.inference_mode():
                emission.log_softmax_into(lg, csr.em[csr.off[a]: csr.off[b]])
            ev = torch.cuda.Event()
            ev.record(ps)
        events += [ev] * (b - a)
    return events


def _dp_device(device):
    """Device on which the DP runs: the model's device if it is a HIP device, else GPU 0."""
    d = torch.device(device) if not isinstance(device, torch.device) else device
    if d.type == "cuda":
        return d if d.index is not None else torch.device("cuda", torch.cuda.current_device())
    if not torch.cuda.is_available():
        raise _lib.WXError("whisperx_amd.align needs a HIP device for the alignment DP (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def blank_id_of(dictionary) -> int:
    """alignment.py:237-240 (the last '[pad]'/'<pad>' entry wins, default 0)."""
    blank_id = 0
    for char, code in dictionary.items():
        if char == "[pad]" or char == "<pad>":
            blank_id = code
    return blank_id


def align(
    transcript: Iterable[SingleSegment],
    model: torch.nn.Module,
    align_model_metadata: dict,
    audio: Union[str, np.ndarray, torch.Tensor],
    device: str,
    interpolate_method: str = "nearest",
    return_char_alignments: bool = False,
    print_progress: bool = False,
    combined_progress: bool = False,
) -> AlignedTranscriptionResult:
    """Align phoneme recognition predictions to known transcription (alignment.py:100-354)."""
    if not torch.is_tensor(audio):
        if isinstance(audio, str):
            audio = load_audio(audio)
        audio = torch.from_numpy(audio)
    if len(audio.shape) == 1:
        audio = audio.unsqueeze(0)

    MAX_DURATION = audio.shape[1] / SAMPLE_RATE

    model_dictionary = align_model_metadata["dictionary"]
    model_lang = align_model_metadata["language"]
    model_type = align_model_metadata["type"]

    # 2a. the emission forward of every segment that starts inside the audio, queued on the
    # device first, so that the host prepares the transcripts (step 1) while the GPU runs them.
    # A segment whose text has no alignable char wastes its forward: the reference skips it
    # (alignment.py:185-195), and so do the DP and the aggregation below.
    blank_id = blank_id_of(model_dictionary)
    dp_dev = _dp_device(device)
    if torch.device(device).type == "cuda" and not audio.is_cuda:
        # one host->device copy of the waveform: per-segment copies from pageable memory would
        # each wait for their stream's earlier forwards, keeping the host in lock-step with them
        audio = audio.to(dp_dev)
    fwd_pos = {}  # transcript index -> index of its forward
    wavs = []
    for sdx, segment in enumerate(transcript):
        t1, t2 = segment["start"], segment["end"]
        # no forward for a segment the reference skips before its model call: past the audio,
        # or no alignable char (music, a script the model lacks: a long one would otherwise pay
        # a full wav2vec2 forward the reference never runs)
        if t1 >= MAX_DURATION or not _has_alignable(segment["text"], model_dictionary, model_lang):
            continue
        fwd_pos[sdx] = len(wavs)
        wavs.append(audio[:, int(t1 * SAMPLE_RATE): int(t2 * SAMPLE_RATE)])
    # the model is prepared (GEMM convolutions, wx attention) for this call only: the caller's
    # model is restored when align() returns, after every forward has been joined
    gpu_route = torch.device(device).type == "cuda" and not os.environ.get("WX_MIOPEN_CONV")
    # the packed encoder runs the model from its weights: no forward is patched, so the model
    # is not prepared (prepare + restore cost ~5 ms of host time per call before the first kernel)
    packed = gpu_route and model_type == "huggingface" and emission.packed_supported(model)
    with contextlib.ExitStack() as model_ctx:
        if gpu_route and not packed:
            model_ctx.enter_context(emission.prepared(model))
        with _Phase("emission"):
            try:
                ems = _emissions(model, model_type, wavs, device)
            except _PackedUnsupported:  # per-segment route, model prepared for this call
                model_ctx.enter_context(emission.prepared(model))
                ems = _emissions(model, model_type, wavs, device, allow_packed=False)

        # 1. text preparation (mutates the input segments like the reference)
        total_segments = len(transcript)
        with _Phase("prepare"):
            for sdx, segment in enumerate(transcript):
                if print_progress:
                    base_progress = ((sdx + 1) / total_segments) * 100
                    percent_complete = (50 + base_progress / 2) if combined_progress else base_progress
                    print(f"Progress: {percent_complete:.2f}%...")
                _prepare(segment, model_dictionary, model_lang)

        plan = []  # per segment: ("nochars" | "toolate", None) | ("dp", index of its forward)
        dummy = [0 if blank_id != 0 else 1]  # (tokens of a forwarded segment the DP result of which is unused)
        toks = [dummy] * len(wavs)
        blanks = [blank_id] * len(wavs)
        meta = [("", 1)] * len(wavs)
        for sdx, segment in enumerate(transcript):
            if len(segment["clean_char"]) == 0:
                plan.append(("nochars", None))
                continue
            if segment["start"] >= MAX_DURATION:
                plan.append(("toolate", None))
                continue
            i = fwd_pos[sdx]
            text_clean = "".join(segment["clean_char"])
            toks[i] = [model_dictionary[c] for c in text_clean]
            meta[i] = (text_clean, wavs[i].size(0))
            plan.append(("dp", i))

        # 2b. the fused DP, one launch per group of segments, and 2c. timestamps and aggregation
        # in segment order (same prints, same order).  A group's DP waits only for its own
        # forwards, so the host aggregates group g while the GPU still runs the later forwards.
        with _Phase("dp+aggregate"):
            results = _GroupedDP(ems, toks, blanks, dp_dev)
            try:
                aligned_segments = _aggregate_all(transcript, plan, results, meta, model_lang, interpolate_method,
                                                  return_char_alignments)
            finally:
                if isinstance(ems, _EmissionsCSR):
                    main = torch.cuda.current_stream(dp_dev)
                    for st in ems.streams:
                        main.wait_stream(st)
    word_segments: List[SingleWordSegment] = []
    for segment in aligned_segments:
        word_segments += segment["words"]
    return {"segments": aligned_segments, "word_segments": word_segments}


def _aggregate_all(transcript, plan, results, meta, model_lang, interpolate_method, return_char_alignments):
    aligned_segments: List[SingleAlignedSegment] = []
    for sdx, segment in enumerate(transcript):
        t1, t2, text = segment["start"], segment["end"], segment["text"]
        aligned_seg: SingleAlignedSegment = {"start": t1, "end": t2, "text": text, "words": []}
        if return_char_alignments:
            aligned_seg["chars"] = []
        kind, bi = plan[sdx]
        if kind == "nochars":
            print(f'Failed to align segment ("{segment["text"]}"): no characters in this segment found in model dictionary, resorting to original...')
            aligned_segments.append(aligned_seg)
            continue
        if kind == "toolate":
            print(f'Failed to align segment ("{segment["text"]}"): original start time longer than audio duration, skipping...')
            aligned_segments.append(aligned_seg)
            continue
        ok, starts, ends, scores, T = results[bi]
        if not ok:
            print(f'Failed to align segment ("{segment["text"]}"): backtrack failed, resorting to original...')
            aligned_segments.append(aligned_seg)
            continue
        _, n_channels = meta[bi]
        aligned_segments += aggregate_segment(segment, starts, ends, scores, T, n_channels, model_lang,
                                              interpolate_method, return_char_alignments)
    return aligned_segments


class _GroupedDP:
    """DP results by segment index, computed one group of segments at a time on first use
    (each group: one wx_align_dp launch after that group's forwards, one host copy)."""

    def __init__(self, ems, toks, blanks, dev, n_groups: int = 4, min_group: int = 8):
        self.ems, self.toks, self.blanks, self.dev = ems, toks, blanks, dev
        n = len(ems)
        self.res = [None] * n
        groups = getattr(ems, "groups", None)  # the packed encoder's packs: one DP per pack
        if not groups:
            size = max(min_group, -(-n // n_groups)) if n else 1
            groups = [(a, min(n, a + size)) for a in range(0, n, size)]
        self.group_of = [None] * n
        for g in groups:
            for i in range(g[0], g[1]):
                self.group_of[i] = g

    def __getitem__(self, i):
        if self.res[i] is None:
            a, b = self.group_of[i]
            sub = self.ems.sub(a, b) if isinstance(self.ems, _EmissionsCSR) else self.ems[a:b]
            self.res[a:b] = _run_dp(sub, self.toks[a:b], self.blanks[a:b], self.dev)
        return self.res[i]


def _run_dp(ems, toks, blanks, dev):
    if isinstance(ems, _EmissionsCSR) and ems.em.device == dev:
        ems.wait(torch.cuda.current_stream(dev))
        batch = _lib.Batch.from_csr(ems.em, ems.Ts, toks, blanks)
    else:
        batch = _lib.Batch(list(ems), toks, blanks, device=dev)
    seg_start, seg_end, seg_score, t_start, status = _lib.align_dp(batch)
    # one device->host copy of everything the host needs
    ss = seg_start.cpu().numpy()
    se = seg_end.cpu().numpy()
    sc = seg_score.cpu().numpy()
    st = status.cpu().numpy()
    outcome = st & _lib.STATUS_MASK
    if (outcome >= 2).any():  # the in-kernel generic forward could not hold the segment either
        i = int(np.flatnonzero(outcome >= 2)[0])
        if outcome[i] == 3:
            raise _lib.WXError(f"segment {i} ({batch.Ns[i]} tokens): a cross-CU hand-off was lost and the segment "
                               f"is too long for the in-kernel recovery forward (status 3); this is transient "
                               f"(the GPU was busy with other work), re-running the call normally succeeds")
        raise _lib.WXError(f"segment {i} ({batch.Ns[i]} tokens) uses more than {_lib.MAX_SEGMENT_COLUMNS} distinct "
                           f"emission columns and is too long for the generic forward (status 2); split it into "
                           f"shorter segments")
    DP_STATS["recovered_segments"] += int(((st & _lib.STATUS_RECOVERED) != 0).sum())
    DP_STATS["segments"] += batch.S
    out = []
    for i in range(batch.S):
        a, b = batch.tok_off[i], batch.tok_off[i + 1]
        out.append((outcome[i] == 0, ss[a:b], se[a:b], sc[a:b], batch.Ts[i]))
    return out


# over the process: DP segments, and those recomputed in-kernel after a lost hand-off
# (WX_STATUS_RECOVERED); the bench legs report the difference across each leg
DP_STATS = {"segments": 0, "recovered_segments": 0}


# ------------------------------------------------------------------ host post-processing
def _nanmin(vals):
    m = math.nan
    for v in vals:
        if v == v and (m != m or v < m):
            m = v
    return np.float64(m)


def _nanmax(vals):
    m = math.nan
    for v in vals:
        if v == v and (m != m or v > m):
            m = v
    return np.float64(m)


def _nanmean(vals):
    """pandas Series.mean(): NaNs zeroed, numpy (pairwise) sum, / non-NaN count.  numpy sums
    fewer than 8 float64 values sequentially from 0.0 (its pairwise sum's base case), which
    the Python loop reproduces exactly without an array round trip."""
    cnt = sum(1 for v in vals if v == v)
    if cnt == 0:
        return np.float64(math.nan)
    if len(vals) < 8:
        s = 0.0
        for v in vals:
            if v == v:
                s += v
            else:
                s += 0.0
        return np.float64(s / cnt)
    arr = np.array([v if v == v else 0.0 for v in vals], dtype=np.float64)
    return np.float64(arr.sum() / cnt)


def _np_round3(v):
    """round(np.float64 v, 3) as numpy computes it (the reference rounds pandas' mean, a numpy
    scalar: rint(v * 1000) / 1000, not Python's correctly rounded round) without numpy's
    per-scalar overhead; Python's round(float) is round-half-even like rint."""
    if v != v or v in (math.inf, -math.inf):
        return np.float64(v)
    y = float(v) * 1000.0
    r = float(round(y))
    if r == 0.0:
        r = math.copysign(0.0, y)  # (rint keeps the sign of a zero)
    return np.float64(r / 1000.0)


def _round3(x: np.ndarray) -> list:
    """[round(v, 3) for v in x] (Python's correctly rounded round) for a float64 array,
    vectorised: rint(v * 1000) / 1000 is the same double (an exact integer over 1000,
    correctly rounded by the division, as round's decimal -> double step) unless v * 1000 lies
    within its rounding error of a half-integer, where the product may round across the tie;
    those values go through round() itself."""
    y = x * 1000.0
    out = np.rint(y) / 1000.0
    near = np.abs(y - np.floor(y) - 0.5) <= 1e-6
    res = out.tolist()
    if near.any():
        xs = x.tolist()
        for i in np.flatnonzero(near).tolist():
            res[i] = round(xs[i], 3)
    return res


def aggregate_segment(segment, starts, ends, scores, T, n_channels, model_lang, interpolate_method,
                      return_char_alignments):
    """alignment.py:252-347 for one aligned segment: char timestamps, sentence/word records,
    NaN interpolation and the (start, end) grouping.  Returns the list of sub-segments."""
    t1, t2, text = segment["start"], segment["end"], segment["text"]
    duration = t2 - t1
    ratio = duration * n_channels / T
    no_spaces = model_lang in LANGUAGES_WITHOUT_SPACES
    n = len(text)
    cdx = segment["clean_cdx"]
    if len(cdx):
        # round(int(start) * ratio + t1, 3) etc. per clean char (the same double operations),
        # NaN for the other chars
        m = len(cdx)
        ci = np.asarray(cdx, dtype=np.int64)
        cols = []
        for v in (np.asarray(starts[:m], dtype=np.int64).astype(np.float64) * ratio + t1,
                  np.asarray(ends[:m], dtype=np.int64).astype(np.float64) * ratio + t1,
                  np.asarray(scores[:m], dtype=np.float64)):
            col = np.full(n, np.nan)
            col[ci] = _round3(v)
            cols.append(col.tolist())
        c_start, c_end, c_score = cols
    else:
        c_start = [math.nan] * n
        c_end = [math.nan] * n
        c_score = [math.nan] * n
    # words: the reference's word index advances after every char followed by a space (after
    # every char for languages without spaces), so word k is the char run [wb[k], wb[k + 1]):
    # it starts at 0 and at every space after position 0
    if no_spaces:
        wb = list(range(n + 1))
    else:
        wb = [0]
        p = text.find(" ", 1)
        while p != -1:
            wb.append(p)
            p = text.find(" ", p + 1)
        wb.append(n)

    subs = []
    for (sstart, send) in segment["sentence_spans"]:
        lo, hi = max(sstart, 0), min(send, n - 1)
        rows = range(lo, hi + 1) if hi >= lo else range(0)
        sentence_text = text[sstart:send]
        sentence_start = _nanmin(c_start[r] for r in rows)
        sentence_end = _nanmax(c_end[r] for r in rows if text[r] != " ")
        words = []
        # the words meeting rows [lo, hi], each clipped to them, in order
        k0 = bisect.bisect_right(wb, lo) - 1 if hi >= lo else len(wb)
        for k in range(k0, len(wb) - 1):
            a, b = max(wb[k], lo), min(wb[k + 1], hi + 1)
            if a >= b:
                break
            word_text = text[a:b].strip()
            if len(word_text) == 0:
                continue
            idx = [r for r in range(a, b) if text[r] != " "]
            word_start = _nanmin(c_start[r] for r in idx)
            word_end = _nanmax(c_end[r] for r in idx)
            word_score = _np_round3(_nanmean([c_score[r] for r in idx]))
            rec = {"word": word_text}
            if word_start == word_start:
                rec["start"] = word_start
            if word_end == word_end:
                rec["end"] = word_end
            if word_score == word_score:
                rec["score"] = word_score
            words.append(rec)
        sub = {"text": sentence_text, "start": sentence_start, "end": sentence_end, "words": words}
        if return_char_alignments:
            chars = []
            for r in rows:
                rec = {"char": text[r]}
                for key, v in (("start", c_start[r]), ("end", c_end[r]), ("score", c_score[r])):
                    v = -1.0 if v != v else v
                    if v != -1:
                        rec[key] = float(v)
                chars.append(rec)
            sub["chars"] = chars
        subs.append(sub)

    if not subs:
        return []
    starts_s = interpolate_nans([s["start"] for s in subs], interpolate_method)
    ends_s = interpolate_nans([s["end"] for s in subs], interpolate_method)
    # groupby(["start", "end"], sort=True, dropna=True) + agg, rows in original order per group
    keyed = [(starts_s[i], ends_s[i], i) for i in range(len(subs)) if starts_s[i] == starts_s[i] and ends_s[i] == ends_s[i]]
    keyed.sort(key=lambda k: (k[0], k[1]))
    sep = "" if model_lang in LANGUAGES_WITHOUT_SPACES else " "
    out = []
    i = 0
    while i < len(keyed):
        j = i
        while j < len(keyed) and keyed[j][0] == keyed[i][0] and keyed[j][1] == keyed[i][1]:
            j += 1
        members = sorted(k[2] for k in keyed[i:j])
        rec = {"start": float(keyed[i][0]), "end": float(keyed[i][1]),
               "text": sep.join(subs[m]["text"] for m in members),
               "words": [w for m in members for w in subs[m]["words"]]}
        if return_char_alignments:
            rec["chars"] = [c for m in members for c in subs[m]["chars"]]
        out.append(rec)
        i = j
    return out


# ------------------------------------------------------------------- DP-level APIs
@dataclass
class Point:
    token_index: int
    time_index: int
    score: float


@dataclass
class Segment:
    label: str
    start: int
    end: int
    score: float

    def __repr__(self):
        return f"{self.label}\t({self.score:4.2f}): [{self.start:5d}, {self.end:5d})"

    @property
    def length(self):
        return self.end - self.start


def _as_tokens(tokens):
    if torch.is_tensor(tokens):
        return [int(x) for x in tokens.reshape(-1).tolist()]
    return [int(x) for x in tokens]


def get_trellis(emission, tokens, blank_id=0):
    """alignment.py:359-379 on the GPU.  Returns the [T+1, N+1] fp32 trellis on the
    emission's device (a CPU emission gets a CPU trellis back)."""
    em = emission if torch.is_tensor(emission) else torch.as_tensor(emission)
    dev = em.device if em.is_cuda else _dp_device("cuda")
    toks = _as_tokens(tokens)
    b = _lib.Batch([em], [toks], [blank_id], device=dev)
    flat, offs = _lib.trellis(b)
    out = flat[: offs[1]].view(b.Ts[0] + 1, len(toks) + 1)
    return out if em.is_cuda else out.cpu()


def backtrack(trellis, emission, tokens, blank_id=0):
    """alignment.py:387-421 on the GPU: list[Point] or None."""
    em = emission if torch.is_tensor(emission) else torch.as_tensor(emission)
    dev = em.device if em.is_cuda else _dp_device("cuda")
    toks = _as_tokens(tokens)
    b = _lib.Batch([em], [toks], [blank_id], device=dev)
    tr = torch.as_tensor(trellis, dtype=torch.float32).to(dev).contiguous().reshape(-1)
    pt, pm, pp, plen, ts = _lib.backtrack(b, tr, [0, tr.numel()])
    L = int(plen[0].item())
    if L < 0:
        return None
    tok_h = pt[:L].cpu().tolist()
    time_h = pm[:L].cpu().tolist()
    prob_h = pp[:L].cpu().tolist()
    return [Point(a, t, p) for a, t, p in zip(tok_h, time_h, prob_h)]


def merge_repeats(path, transcript):
    """alignment.py:438-454 on the GPU (run-length grouping, fp64 left-to-right means of
    the fp32 path probabilities, as backtrack() produces them)."""
    if not path:
        return []
    dev = _dp_device("cuda")
    pt = torch.tensor([p.token_index for p in path], dtype=torch.int32).to(dev)
    pm = torch.tensor([p.time_index for p in path], dtype=torch.int32).to(dev)
    pp = torch.tensor([p.score for p in path], dtype=torch.float32).to(dev)
    off = torch.zeros(1, dtype=torch.int64).to(dev)
    ln = torch.tensor([len(path)], dtype=torch.int32).to(dev)
    st, ss, se, sc, cnt = _lib.merge_repeats(pt, pm, pp, off, ln, dev)
    G = int(cnt[0].item())
    st, ss, se, sc = st[:G].cpu().tolist(), ss[:G].cpu().tolist(), se[:G].cpu().tolist(), sc[:G].cpu().tolist()
    return [Segment(transcript[a], s, e, c) for a, s, e, c in zip(st, ss, se, sc)]


def merge_words(segments, separator="|"):
    """alignment.py:456-470 (host; not on the align() path): words between separator
    labels, score weighted by segment length."""
    words = []
    run = []
    for seg in list(segments) + [None]:
        if seg is None or seg.label == separator:
            if run:
                label = "".join(x.label for x in run)
                num = sum(x.score * x.length for x in run)
                den = sum(x.length for x in run)
                words.append(Segment(label, run[0].start, run[-1].end, num / den))
            run = []
        else:
            run.append(seg)
    return words
