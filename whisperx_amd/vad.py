"""VAD segmentation for WhisperX on MI355X — drop-in for ``whisperx.vad``'s
``Binarize`` (vad.py:61-195) and ``merge_chunks`` (vad.py:264-311).

The hysteresis/min-cut state machine runs on the GPU (libwxalign.so: wx_binarize, one
wave per score column, event-driven scan); the greedy chunk merge over the resulting
region list is O(#regions) host work, as in the reference.

pyannote.core is an optional dependency: when it is installed its containers are used for
the returned Annotation; otherwise this module's small stand-ins with the same interface
(Segment, SlidingWindow, SlidingWindowFeature, Annotation) are used.  The frame geometry
is read from ``scores.sliding_window`` (start, step, duration); frame i is centred at
0.5*(s + (s + duration)) with s = start + i*step, as pyannote's SlidingWindow.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from . import _lib

try:  # pragma: no cover - pyannote is not part of this image
    from pyannote.core import Annotation, Segment, SlidingWindow, SlidingWindowFeature  # type: ignore

    HAVE_PYANNOTE = True
except Exception:  # stand-ins with pyannote.core semantics
    HAVE_PYANNOTE = False

    class Segment:
        """Time interval; falsy when shorter than 1e-6 s (pyannote SEGMENT_PRECISION)."""

        __slots__ = ("start", "end")

        def __init__(self, start: float = 0.0, end: float = 0.0):
            self.start = start
            self.end = end

        def __bool__(self):
            return bool((self.end - self.start) > 1e-6)

        @property
        def duration(self):
            return self.end - self.start if self else 0.0

        @property
        def middle(self):
            return 0.5 * (self.start + self.end)

        def _key(self):
            return (self.start, self.end)

        def __eq__(self, other):
            return isinstance(other, Segment) and self._key() == other._key()

        def __lt__(self, other):
            return self._key() < other._key()

        def __hash__(self):
            return hash(self._key())

        def __repr__(self):
            return f"<Segment({self.start}, {self.end})>"

    class SlidingWindow:
        def __init__(self, start: float = 0.0, step: float = 0.0, duration: float = 0.0):
            self.start, self.step, self.duration = start, step, duration

        def __getitem__(self, i: int) -> "Segment":
            s = self.start + i * self.step
            return Segment(s, s + self.duration)

    class SlidingWindowFeature:
        def __init__(self, data, sliding_window, labels=None):
            self.data = data
            self.sliding_window = sliding_window
            self.labels = labels

    class Annotation:
        """(segment, track) -> label store; empty segments are ignored on assignment."""

        def __init__(self):
            self._tracks = {}

        def __setitem__(self, key, label):
            seg, track = key
            if not seg:
                return
            self._tracks[(seg, track)] = label

        def __delitem__(self, key):
            del self._tracks[key]

        def __getitem__(self, key):
            return self._tracks[key]

        def __len__(self):
            return len(self._tracks)

        def get_timeline(self):
            return sorted({s for (s, _t) in self._tracks}, key=Segment._key)

        def itertracks(self, yield_label: bool = False):
            for (s, t) in sorted(self._tracks, key=lambda st: (st[0].start, st[0].end, str(st[1]))):
                yield (s, t, self._tracks[(s, t)]) if yield_label else (s, t)

        def labels(self):
            return sorted(set(self._tracks.values()), key=str)

        def support(self, collar: float = 0.0) -> "Annotation":
            """Per label, merge segments that overlap or are separated by a gap < collar
            (pyannote Annotation.support; parity unpinned — pyannote is not installed)."""
            out = Annotation()
            for label in self.labels():
                segs = sorted(s for (s, t), lab in self._tracks.items() if lab == label)
                merged = []
                for s in segs:
                    if merged and (s.start <= merged[-1].end or s.start - merged[-1].end < collar):
                        if s.end > merged[-1].end:
                            merged[-1] = Segment(merged[-1].start, s.end)
                    else:
                        merged.append(Segment(s.start, s.end))
                for i, s in enumerate(merged):
                    out[s, f"{label}_{i}"] = label
            return out


class SegmentX:
    """whisperx.diarize.Segment (diarize.py:70-74): start, end, speaker."""

    def __init__(self, start, end, speaker=None):
        self.start = start
        self.end = end
        self.speaker = speaker


class Binarize:
    """Hysteresis thresholding with WhisperX's min-cut (vad.py:61-195), on the GPU.

    Same constructor and call semantics as the reference: ``offset`` defaults to
    ``onset`` (``offset or onset``), a region longer than ``max_duration`` is cut at the
    lowest score in the second half of its current score list, pads/min_duration_off
    trigger ``Annotation.support`` (not allowed together with a finite max_duration), and
    regions shorter than ``min_duration_on`` are removed."""

    def __init__(self, onset: float = 0.5, offset: Optional[float] = None, min_duration_on: float = 0.0,
                 min_duration_off: float = 0.0, pad_onset: float = 0.0, pad_offset: float = 0.0,
                 max_duration: float = float("inf")):
        self.onset = onset
        self.offset = offset or onset
        self.pad_onset = pad_onset
        self.pad_offset = pad_offset
        self.min_duration_on = min_duration_on
        self.min_duration_off = min_duration_off
        self.max_duration = max_duration

    def regions(self, scores):
        """GPU state machine: [(starts, ends)] per class column (float64 arrays).  Scores may
        be a device tensor (the VAD producer's output): they are then read in place."""
        data = scores.data
        if torch.is_tensor(data) and data.is_cuda:
            data = data.reshape(data.shape[0], -1) if data.dim() > 1 else data[:, None]
            cols = [data[:, k].contiguous() for k in range(data.shape[1])]
        else:
            data = np.asarray(data, dtype=np.float32)
            if data.ndim == 1:
                data = data[:, None]
            cols = [np.ascontiguousarray(data[:, k]) for k in range(data.shape[1])]
        sw = scores.sliding_window
        geom = [(float(sw.start), float(sw.step), float(sw.duration))] * len(cols)
        return _lib.binarize(cols, geom, self.onset, self.offset, self.max_duration, self.pad_onset,
                             self.pad_offset)

    def __call__(self, scores) -> "Annotation":
        active = Annotation()
        for k, (rs, re) in enumerate(self.regions(scores)):
            label = k if scores.labels is None else scores.labels[k]
            for a, b in zip(rs.tolist(), re.tolist()):
                active[Segment(a, b), k] = label
        if self.pad_offset > 0.0 or self.pad_onset > 0.0 or self.min_duration_off > 0.0:
            if self.max_duration < float("inf"):
                raise NotImplementedError("This would break current max_duration param")
            active = active.support(collar=self.min_duration_off)
        if self.min_duration_on > 0:
            for segment, track in list(active.itertracks()):
                if segment.duration < self.min_duration_on:
                    del active[segment, track]
        return active


def merge_chunks(segments, chunk_size, onset: float = 0.5, offset: Optional[float] = None):
    """vad.py:264-311: binarize with max_duration=chunk_size, then greedily merge speech
    regions into chunks no longer than chunk_size (unless a single region is)."""
    assert chunk_size > 0
    binarize = Binarize(max_duration=chunk_size, onset=onset, offset=offset)
    # no pads / min durations here, so the Annotation's timeline is the sorted set of the
    # regions of all columns: taken from the region arrays without building the Annotation
    s, e = _timeline(binarize.regions(segments))
    if len(s) == 0:
        print("No active speech found in audio")
        return []
    return _greedy_chunks_arrays(s, e, chunk_size)


def _timeline(cols):
    """Annotation.get_timeline() over the regions of every column: unique (start, end)
    pairs in (start, end) order, as float64 arrays."""
    if len(cols) == 1:
        s, e = (np.asarray(x, dtype=np.float64) for x in cols[0])
    else:
        s = np.concatenate([np.asarray(c[0], dtype=np.float64) for c in cols]) if cols else np.zeros(0)
        e = np.concatenate([np.asarray(c[1], dtype=np.float64) for c in cols]) if cols else np.zeros(0)
    if len(s) > 1:
        ordered = (s[1:] > s[:-1]) | ((s[1:] == s[:-1]) & (e[1:] > e[:-1]))
        if not ordered.all():  # several columns (or out-of-order input): sort and drop repeats
            o = np.lexsort((e, s))
            s, e = s[o], e[o]
            keep = np.ones(len(s), dtype=bool)
            keep[1:] = (s[1:] != s[:-1]) | (e[1:] != e[:-1])
            s, e = s[keep], e[keep]
    return s, e


def _greedy_chunks_arrays(s, e, chunk_size):
    """_greedy_chunks over (start, end) arrays in timeline order.  With non-decreasing ends
    (one VAD column always has them) the region that flushes a chunk started at cs is the
    first later one with end - cs > chunk_size — a monotone predicate, so each chunk is one
    binary search instead of a per-region loop; the regions are only touched to build the
    chunks' segment lists."""
    n = len(s)
    if n > 1 and not bool(np.all(e[1:] >= e[:-1])):
        return _greedy_chunks([SegmentX(a, b, "UNKNOWN") for a, b in zip(s.tolist(), e.tolist())], chunk_size)
    sl, el = s.tolist(), e.tolist()
    merged = []
    if el[0] - sl[0] > chunk_size and 0 - sl[0] > 0:  # the reference's chunk_end = 0 start state
        merged.append({"start": sl[0], "end": 0, "segments": []})
    a = 0
    while True:
        cs = sl[a]
        r = max(int(np.searchsorted(e, cs + chunk_size, side="right")), a + 1)
        while r > a + 1 and el[r - 1] - cs > chunk_size:  # settle on the exact fp64 predicate
            r -= 1
        while r < n and not (el[r] - cs > chunk_size):
            r += 1
        # every region in (a, r) ends after cs (ends are non-decreasing and regions non-empty),
        # so the reference's chunk_end - chunk_start > 0 condition holds at r
        merged.append({"start": cs, "end": el[r - 1], "segments": list(zip(sl[a:r], el[a:r]))})
        if r >= n:
            return merged
        a = r


def _greedy_chunks(regions, chunk_size):
    """vad.py:290-310.  A chunk is flushed when adding the next region would stretch it
    past chunk_size (and the chunk is non-empty in time)."""
    merged = []
    chunk_start = regions[0].start
    chunk_end = 0
    members = []
    for r in regions:
        if r.end - chunk_start > chunk_size and chunk_end - chunk_start > 0:
            merged.append({"start": chunk_start, "end": chunk_end, "segments": members})
            chunk_start = r.start
            members = []
        chunk_end = r.end
        members.append((r.start, r.end))
    merged.append({"start": chunk_start, "end": chunk_end, "segments": members})
    return merged
