"""whisperx_amd — MI355X-native forced alignment + VAD segmentation for WhisperX.

Drop-in for the reference's alignment path (whisperx/__init__.py:2 re-exports
load_align_model/align) and its VAD post-processing (whisperx/vad.py Binarize,
merge_chunks).  Compute runs in libwxalign.so (HIP, gfx950); see DESIGN.md.
"""
import os as _os

# wav2vec2's convolutions see a new input length for almost every VAD chunk.  MIOpen's
# default find mode searches (and JIT-compiles) kernels per new shape: ~1.2 s each on a
# fresh MI355X; FAST picks by heuristic (~10 ms forward for a 30 s chunk either way).
# Set before the first convolution; a user's own setting wins.
_os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
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
from .writers import get_writer, format_timestamp  # noqa: F401
from .integration import install  # noqa: F401

__version__ = "0.1.0"
