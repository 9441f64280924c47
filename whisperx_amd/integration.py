"""Switch an installed reference whisperX over to this package.

The reference binds the alignment/VAD names at import time in several modules, so changing
``whisperx/__init__.py:2`` alone leaves the CLI on the CPU path:

  whisperx/__init__.py:2    from .alignment import load_align_model, align
  whisperx/transcribe.py:9  from .alignment import align, load_align_model   (CLI, :188,:201,:203)
  whisperx/asr.py:13        from .vad import load_vad_model, merge_chunks      (:187, :347)
  whisperx/transcribe.py:13 from .utils import ... get_writer ...

``install()`` rebinds every one of those names, in every module of the package that holds
one, to this package's implementations.  Call it once, before ``whisperx.transcribe.cli()``
or a user's own pipeline runs:

    import whisperx, whisperx_amd
    whisperx_amd.install(whisperx)
"""
from __future__ import annotations

import importlib
import os
import sys
from typing import Dict, List, Optional, Tuple


def _vad_loader(reference_loader):
    """The drop-in for the reference's load_vad_model (vad.py:20-59, bound at asr.py:13 and
    called at asr.py:347): this package's producer (PyanNet + wx_vad_aggregate, scores kept on
    the device) when the checkpoint loads without executing anything from it; otherwise —
    a pickled Lightning checkpoint, another key layout, or no local file (the reference then
    downloads it) — the reference's own pyannote pipeline, with a one-line notice.  The default
    checkpoint (model_fp None: the whisperX file the reference caches) is read tensors-only by
    vad_model.read_checkpoint_tensors; WX_VAD_STATE_DICT names a state_dict file of one's own to
    use instead (no SHA256 check).  A digest mismatch raises RuntimeError, as the reference does."""
    from . import vad_model

    def load_vad_model(device, vad_onset=0.500, vad_offset=0.363, use_auth_token=None, model_fp=None):
        own = os.environ.get("WX_VAD_STATE_DICT")  # an exported state_dict of one's own (no digest check)
        try:
            if own and model_fp is None:
                return vad_model.load_vad_model(device, vad_onset=vad_onset, vad_offset=vad_offset,
                                                use_auth_token=use_auth_token, model_fp=own, check_sha256=False)
            return vad_model.load_vad_model(device, vad_onset=vad_onset, vad_offset=vad_offset,
                                            use_auth_token=use_auth_token, model_fp=model_fp)
        except (vad_model.CheckpointNotLoadable, FileNotFoundError) as e:
            print(f"whisperx_amd: VAD producer not used ({str(e).splitlines()[0][:160]}); "
                  f"falling back to the reference's pyannote pipeline")
            return reference_loader(device, vad_onset=vad_onset, vad_offset=vad_offset,
                                    use_auth_token=use_auth_token, model_fp=model_fp)

    load_vad_model._wx_reference = reference_loader
    load_vad_model.__doc__ = _vad_loader.__doc__
    return load_vad_model


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
        "asr": {"merge_chunks": vad.merge_chunks, "load_vad_model": _vad_loader},
        "vad": {"merge_chunks": vad.merge_chunks, "Binarize": vad.Binarize, "load_vad_model": _vad_loader},
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
                if obj is _vad_loader:  # wraps the module's own loader (its fallback)
                    cur = getattr(mod, name)
                    if hasattr(cur, "_wx_reference"):
                        continue  # installed already
                    obj = _vad_loader(cur)
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
            if not hasattr(mod, name):
                continue
            cur = getattr(mod, name)
            if (obj is _vad_loader and not hasattr(cur, "_wx_reference")) or (obj is not _vad_loader and cur is not obj):
                return False
    return True
