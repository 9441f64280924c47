"""Result types of the alignment path — same TypedDicts as whisperx/types.py:4-58."""
from typing import List, Optional, TypedDict


class SingleWordSegment(TypedDict):
    word: str
    start: float
    end: float
    score: float


class SingleCharSegment(TypedDict):
    char: str
    start: float
    end: float
    score: float


class SingleSegment(TypedDict):
    start: float
    end: float
    text: str


class SingleAlignedSegment(TypedDict):
    start: float
    end: float
    text: str
    words: List[SingleWordSegment]
    chars: Optional[List[SingleCharSegment]]


class TranscriptionResult(TypedDict):
    segments: List[SingleSegment]
    language: str


class AlignedTranscriptionResult(TypedDict):
    segments: List[SingleAlignedSegment]
    word_segments: List[SingleWordSegment]
