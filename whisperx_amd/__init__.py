"""whisperx_amd — MI355X-native forced alignment + VAD segmentation for WhisperX.

Drop-in for the reference's alignment path (whisperx/__init__.py:2 re-exports
load_align_model/align) and its VAD post-processing (whisperx/vad.py Binarize,
merge_chunks).  Compute runs in libwxalign.so (HIP, gfx950); see DESIGN.md.
"""
from .alignment import (  # noqa: F401
    DEFAULT_ALIGN_MODELS_HF,
    DEFAULT_ALIGN_MODELS_TORCH,
    LANGUAGES_WITHOUT_SPACES,
    PUNKT_ABBREVIATIONS,
    Point,
    Segment,
    align,
    backtrack,
    get_trellis,
    load_align_model,
    merge_repeats,
    merge_words,
)
from .audio import SAMPLE_RATE, load_audio  # noqa: F401
from .vad import Binarize, merge_chunks  # noqa: F401

__version__ = "0.1.0"
