"""Switch an installed reference whisperX over to this package.

The reference binds the alignment/VAD names at import time in several modules, so changing
``whisperx/__init__.py:2`` alone leaves the CLI on the CPU path:

  whisperx/__init__.py:2    from .alignment import load_align_model, align
  whisperx/transcribe.py:9  from .alignment import align, load_align_model   (CLI, :188,:201,:203)
  whisperx/asr.py:13        from .vad import load_vad_model, merge_chunks      (:187)
  whisperx/transcribe.py:13 from .utils import ... get_writer ...

``install()`` rebinds every one of those names, in every module of the package that holds
one, to this package's implementations.  Call it once, before ``whisperx.transcribe.cli()``
or a user's own pipeline runs:

    import whisperx, whisperx_amd
    whisperx_amd.install(whisperx)
"""
from __future__ import annotations

import importlib
import sys
from typing import Dict, List, Optional, Tuple


def _targets() -> Dict[str, Dict[str, object]]:
    from . import alignment, vad, writers

    align_names = {n: getattr(alignment, n) for n in
                   ("align", "load_align_model", "get_trellis", "backtrack", "merge_repeats", "merge_words",
                    "Point", "Segment")}
    return {
        "": {"align": alignment.align, "load_align_model": alignment.load_align_model},
        "alignment": align_names,
        "transcribe": {"align": alignment.align, "load_align_model": alignment.load_align_model,
                       "get_writer": writers.get_writer},
        "asr": {"merge_chunks": vad.merge_chunks},
        "vad": {"merge_chunks": vad.merge_chunks, "Binarize": vad.Binarize},
        "utils": {"get_writer": writers.get_writer},
    }


def install(whisperx=None, import_missing: bool = True) -> List[Tuple[str, str]]:
    """Rebind the reference package's alignment / VAD-segmentation / writer names to
    whisperx_amd's.  `whisperx` is the reference package object (default: ``import whisperx``).
    Submodules not imported yet are imported first when `import_missing` (a submodule whose
    own dependencies are absent is skipped).  Only names the module already defines are
    replaced.  Returns the (module, name) pairs rebound."""
    if whisperx is None:
        whisperx = importlib.import_module("whisperx")
    base = whisperx.__name__
    done: List[Tuple[str, str]] = []
    for sub, names in _targets().items():
        modname = f"{base}.{sub}" if sub else base
        mod = sys.modules.get(modname)
        if mod is None and import_missing:
            try:
                mod = importlib.import_module(modname)
            except Exception:
                mod = None
        if mod is None:
            continue
        for name, obj in names.items():
            if hasattr(mod, name):
                setattr(mod, name, obj)
                done.append((modname, name))
    return done


def installed(whisperx=None) -> Optional[bool]:
    """True when every loaded reference module's align/merge_chunks binding is ours."""
    if whisperx is None:
        whisperx = sys.modules.get("whisperx")
        if whisperx is None:
            return None
    base = whisperx.__name__
    for sub, names in _targets().items():
        mod = sys.modules.get(f"{base}.{sub}" if sub else base)
        if mod is None:
            continue
        for name, obj in names.items():
            if hasattr(mod, name) and getattr(mod, name) is not obj:
                return False
    return True
