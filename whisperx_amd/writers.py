"""Result writers: txt / vtt / srt / tsv / json / aud files of an aligned transcript.

Same classes, options and byte-for-byte output as the reference's writers
(whisperx/utils.py:171-431: format_timestamp, ResultWriter, WriteTXT, SubtitlesWriter,
WriteVTT, WriteSRT, WriteTSV, WriteAudacity, WriteJSON, get_writer); pinned by
tests/golden/writer_cases.json.gz, which the reference's own writers produced.

Subtitle cues (SubtitlesWriter.iterate_result) are built by a small line packer:
  * a word continues the current line when the line is non-empty, the word fits in
    max_line_width (1000 when unset), it does not start a new segment (segments are kept
    whole unless both max_line_width and max_line_count are set) and it is not a pause of
    more than 3 s after the previous timed word (only checked when segments are not kept);
  * otherwise the word (stripped) starts a new line; the cue is closed first when it is a
    segment start, or max_line_count lines are full / a long pause occurred;
  * a cue takes the start/end of the segment its first word belongs to; with
    highlight_words every timed word also gets its own cue with the word underlined, and
    gaps between word cues are filled with the plain text.
"""
from __future__ import annotations

import json
import os
import re
from typing import Callable, Iterator, List, Optional, TextIO, Tuple

from .alignment import LANGUAGES_WITHOUT_SPACES

__all__ = ["format_timestamp", "ResultWriter", "WriteTXT", "SubtitlesWriter", "WriteVTT", "WriteSRT",
           "WriteTSV", "WriteAudacity", "WriteJSON", "get_writer"]


def format_timestamp(seconds: float, always_include_hours: bool = False, decimal_marker: str = ".") -> str:
    """[hh:]mm:ss<marker>mmm of a non-negative time, milliseconds rounded half to even."""
    assert seconds >= 0, "non-negative timestamp expected"
    ms = round(seconds * 1000.0)
    h, rem = divmod(ms, 3_600_000)
    m, rem = divmod(rem, 60_000)
    s, ms = divmod(rem, 1_000)
    head = f"{h:02d}:" if (always_include_hours or h > 0) else ""
    return f"{head}{m:02d}:{s:02d}{decimal_marker}{ms:03d}"


class ResultWriter:
    extension: str

    def __init__(self, output_dir: str):
        self.output_dir = output_dir

    def __call__(self, result: dict, audio_path: str, options: dict):
        stem = os.path.splitext(os.path.basename(audio_path))[0]
        path = os.path.join(self.output_dir, f"{stem}.{self.extension}")
        with open(path, "w", encoding="utf-8") as f:
            self.write_result(result, file=f, options=options)

    def write_result(self, result: dict, file: TextIO, options: dict):
        raise NotImplementedError


class WriteTXT(ResultWriter):
    extension: str = "txt"

    def write_result(self, result: dict, file: TextIO, options: dict):
        file.write("".join(seg["text"].strip() + "\n" for seg in result["segments"]))
        file.flush()


_UNDERLINE = re.compile(r"^(\s*)(.*)$")


class _CuePacker:
    """Groups the words of all segments into cues (lists of word dicts) with their
    owning segments' (start, end, speaker)."""

    def __init__(self, first_start: float, max_width: int, max_lines: Optional[int], keep_segments: bool):
        self.max_width, self.max_lines, self.keep_segments = max_width, max_lines, keep_segments
        self.prev_start = first_start
        self.width = 0
        self.lines = 1
        self.words: List[dict] = []
        self.owners: List[tuple] = []

    def _flush(self):
        cue = (self.words, self.owners)
        self.words, self.owners, self.lines = [], [], 1
        return cue

    def add(self, segment: dict, index: int, word: dict):
        """Adds one word; returns a finished cue or None."""
        w = dict(word)
        text = w["word"]
        pause = (not self.keep_segments) and ("start" in w) and (w["start"] - self.prev_start > 3.0)
        new_segment = self.keep_segments and index == 0 and bool(self.words)
        fits = self.width + len(text) <= self.max_width
        done = None
        if self.width > 0 and fits and not pause and not new_segment:
            self.width += len(text)
        else:
            text = text.strip()
            cue_full = self.max_lines is not None and (pause or self.lines >= self.max_lines)
            if (self.words and cue_full) or new_segment:
                done = self._flush()
            elif self.width > 0:
                self.lines += 1
                text = "\n" + text
            w["word"] = text
            self.width = len(text.strip())
        self.words.append(w)
        self.owners.append((segment["start"], segment["end"], segment.get("speaker")))
        if "start" in w:
            self.prev_start = w["start"]
        return done


class SubtitlesWriter(ResultWriter):
    always_include_hours: bool
    decimal_marker: str

    def format_timestamp(self, seconds: float) -> str:
        return format_timestamp(seconds, self.always_include_hours, self.decimal_marker)

    def _cues(self, result: dict, options: dict) -> Iterator[Tuple[list, list]]:
        width = options["max_line_width"]
        lines = options["max_line_count"]
        packer = _CuePacker(result["segments"][0]["start"], 1000 if width is None else width, lines,
                            keep_segments=(lines is None or width is None))
        for seg in result["segments"]:
            for i, word in enumerate(seg["words"]):
                cue = packer.add(seg, i, word)
                if cue is not None:
                    yield cue
        if packer.words:
            yield packer._flush()

    def iterate_result(self, result: dict, options: dict) -> Iterator[Tuple[str, str, str]]:
        segments = result["segments"]
        if not segments:
            return
        if "words" not in segments[0]:  # segment-level cues
            for seg in segments:
                text = seg["text"].strip().replace("-->", "->")
                if "speaker" in seg:
                    text = f"[{seg['speaker']}]: {text}"
                yield self.format_timestamp(seg["start"]), self.format_timestamp(seg["end"]), text
            return
        joiner = "" if result["language"] in LANGUAGES_WITHOUT_SPACES else " "
        highlight = options["highlight_words"]
        for words, owners in self._cues(result, options):
            seg_start, seg_end, speaker = owners[0]
            cue_start, cue_end = self.format_timestamp(seg_start), self.format_timestamp(seg_end)
            tokens = [w["word"] for w in words]
            text = joiner.join(tokens)
            prefix = "" if speaker is None else f"[{speaker}]: "
            if not (highlight and any("start" in w for w in words)):
                yield cue_start, cue_end, prefix + text
                continue
            cursor = cue_start
            for i, w in enumerate(words):
                if "start" not in w:
                    continue
                a, b = self.format_timestamp(w["start"]), self.format_timestamp(w["end"])
                if cursor != a:
                    yield cursor, a, prefix + text
                marked = list(tokens)
                marked[i] = _UNDERLINE.sub(r"\1<u>\2</u>", marked[i])
                yield a, b, prefix + " ".join(marked)
                cursor = b


class WriteVTT(SubtitlesWriter):
    extension: str = "vtt"
    always_include_hours: bool = False
    decimal_marker: str = "."

    def write_result(self, result: dict, file: TextIO, options: dict):
        file.write("WEBVTT\n\n")
        for a, b, text in self.iterate_result(result, options):
            file.write(f"{a} --> {b}\n{text}\n\n")
        file.flush()


class WriteSRT(SubtitlesWriter):
    extension: str = "srt"
    always_include_hours: bool = True
    decimal_marker: str = ","

    def write_result(self, result: dict, file: TextIO, options: dict):
        for n, (a, b, text) in enumerate(self.iterate_result(result, options), start=1):
            file.write(f"{n}\n{a} --> {b}\n{text}\n\n")
        file.flush()


class WriteTSV(ResultWriter):
    """start<TAB>end<TAB>text, times in integer milliseconds (round half to even)."""

    extension: str = "tsv"

    def write_result(self, result: dict, file: TextIO, options: dict):
        rows = ["start\tend\ttext\n"]
        for seg in result["segments"]:
            rows.append(f"{round(1000 * seg['start'])}\t{round(1000 * seg['end'])}\t"
                        f"{seg['text'].strip().replace(chr(9), ' ')}\n")
        file.write("".join(rows))
        file.flush()


class WriteAudacity(ResultWriter):
    """Audacity label track: start<TAB>end<TAB>[[speaker]]text, times in seconds."""

    extension: str = "aud"

    def write_result(self, result: dict, file: TextIO, options: dict):
        for seg in result["segments"]:
            who = f"[[{seg['speaker']}]]" if "speaker" in seg else ""
            file.write(f"{seg['start']}\t{seg['end']}\t{who}{seg['text'].strip().replace(chr(9), ' ')}\n")
        file.flush()


class WriteJSON(ResultWriter):
    extension: str = "json"

    def write_result(self, result: dict, file: TextIO, options: dict):
        json.dump(result, file, ensure_ascii=False)


_WRITERS = {"txt": WriteTXT, "vtt": WriteVTT, "srt": WriteSRT, "tsv": WriteTSV, "json": WriteJSON}
_OPTIONAL_WRITERS = {"aud": WriteAudacity}


def get_writer(output_format: str, output_dir: str) -> Callable[[dict, str, dict], None]:
    """A writer for one format; "all" writes txt, vtt, srt, tsv and json (not aud)."""
    if output_format == "all":
        every = [cls(output_dir) for cls in _WRITERS.values()]

        def write_all(result: dict, audio_path: str, options: dict):
            for w in every:
                w(result, audio_path, options)

        return write_all
    cls = _OPTIONAL_WRITERS.get(output_format) or _WRITERS[output_format]
    return cls(output_dir)
