"""The drop-in boundary, proven on the reference package itself (build container only):
import /root/reference/whisperx behind stand-ins for the modules this image lacks (SURVEY.md
§8(c) recipe, plus ctranslate2 / faster_whisper for asr.py), apply whisperx_amd.install(),
and check that every call site the CLI and the ASR pipeline use now resolves to
whisperx_amd's functions (transcribe.py:9,188,201,203; asr.py:13,187; __init__.py:2).

Runs in a subprocess: the stand-ins must not leak into the other tests' sys.modules."""
import os
import subprocess
import sys
import textwrap

import pytest

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent(r'''
    import sys, types
    from importlib.machinery import ModuleSpec
    from types import SimpleNamespace
    import transformers, torch  # transformers before the torchaudio stand-in

    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__spec__ = ModuleSpec(name, None)
        for k, v in attrs.items():
            setattr(m, k, v)
        sys.modules[name] = m
        return m

    mod("torchaudio", pipelines=SimpleNamespace(__all__=[]))
    class PunktParameters:
        def __init__(self): self.abbrev_types = set()
    class PunktSentenceTokenizer:
        def __init__(self, params=None): pass
        def span_tokenize(self, text): yield (0, len(text.rstrip()))
    punkt = mod("nltk.tokenize.punkt", PunktParameters=PunktParameters, PunktSentenceTokenizer=PunktSentenceTokenizer)
    mod("nltk.tokenize", punkt=punkt); mod("nltk")
    mod("pyannote"); mod("pyannote.audio", Model=object, Pipeline=object); mod("pyannote.audio.core")
    mod("pyannote.audio.core.io", AudioFile=object)
    mod("pyannote.audio.pipelines", VoiceActivityDetection=object)
    mod("pyannote.audio.pipelines.utils", PipelineModel=object)
    mod("pyannote.core", Annotation=object, Segment=object, SlidingWindowFeature=object, SlidingWindow=object)
    mod("ctranslate2", StorageView=object)
    fw_tok = mod("faster_whisper.tokenizer", Tokenizer=object)
    fw_tr = mod("faster_whisper.transcribe", TranscriptionOptions=object, get_ctranslate2_storage=None)
    mod("faster_whisper", WhisperModel=object, tokenizer=fw_tok, transcribe=fw_tr)

    sys.path.insert(0, sys.argv[1])   # /root/reference
    sys.path.insert(0, sys.argv[2])   # this repo
    import whisperx
    import whisperx.transcribe, whisperx.asr, whisperx.alignment, whisperx.vad, whisperx.utils
    ref_align = whisperx.transcribe.align
    assert ref_align is whisperx.alignment.align          # before: the reference CPU path

    # the reference's load_vad_model downloads (vad.py:28-43): a recording stand-in for it
    ref_vad_calls = []
    def ref_load_vad_model(device, vad_onset=0.5, vad_offset=0.363, use_auth_token=None, model_fp=None):
        ref_vad_calls.append(model_fp)
        return "reference-pyannote-pipeline"
    whisperx.vad.load_vad_model = ref_load_vad_model
    whisperx.asr.load_vad_model = ref_load_vad_model

    import whisperx_amd
    from whisperx_amd import vad as amd_vad, writers as amd_writers
    rebound = whisperx_amd.install(whisperx)
    assert whisperx_amd.integration.installed(whisperx)

    # module attributes
    assert whisperx.align is whisperx_amd.align and whisperx.load_align_model is whisperx_amd.load_align_model
    assert whisperx.transcribe.align is whisperx_amd.align
    assert whisperx.transcribe.load_align_model is whisperx_amd.load_align_model
    assert whisperx.transcribe.get_writer is amd_writers.get_writer
    assert whisperx.alignment.align is whisperx_amd.align
    assert whisperx.alignment.get_trellis is whisperx_amd.get_trellis
    assert whisperx.asr.merge_chunks is amd_vad.merge_chunks
    assert whisperx.vad.merge_chunks is amd_vad.merge_chunks
    # what the call sites resolve at call time (module globals of the calling functions)
    assert whisperx.transcribe.cli.__globals__["align"] is whisperx_amd.align
    assert whisperx.transcribe.cli.__globals__["load_align_model"] is whisperx_amd.load_align_model
    assert whisperx.asr.FasterWhisperPipeline.transcribe.__globals__["merge_chunks"] is amd_vad.merge_chunks

    # load_vad_model (asr.py:13, called by load_model at asr.py:347) is the drop-in producer,
    # falling back to the reference's loader for what it cannot read
    lv = whisperx.asr.load_model.__globals__["load_vad_model"]
    assert lv is whisperx.asr.load_vad_model and lv._wx_reference is ref_load_vad_model
    assert whisperx.vad.load_vad_model._wx_reference is ref_load_vad_model
    whisperx_amd.install(whisperx)  # a second install must not wrap the drop-in again
    assert whisperx.asr.load_vad_model._wx_reference is ref_load_vad_model
    import hashlib, os, tempfile
    from whisperx_amd import vad_model as amd_vm
    tmp = tempfile.mkdtemp()
    assert lv("cpu", model_fp=os.path.join(tmp, "absent.bin")) == "reference-pyannote-pipeline"
    pickled = os.path.join(tmp, "lightning.bin")          # pickles a non-tensor object (Lightning layout)
    torch.save({"state_dict": amd_vm.PyanNet().state_dict(), "loops": SimpleNamespace(epoch=3)}, pickled)
    plain = os.path.join(tmp, "plain.bin")
    torch.save(amd_vm.PyanNet().state_dict(), plain)
    garbage = os.path.join(tmp, "garbage.bin")            # no tensors to read: the reference's pipeline
    open(garbage, "wb").write(b"neither zip nor pickle" * 8)
    for fp, want_ref in ((pickled, False), (plain, False), (garbage, True)):
        digest = hashlib.sha256(open(fp, "rb").read()).hexdigest()   # as if it were the whisperX file
        amd_vm.VAD_SEGMENTATION_URL = "https://x/segmentation/" + digest + "/pytorch_model.bin"
        got = lv("cpu", vad_onset=0.45, model_fp=fp)
        if want_ref:
            assert got == "reference-pyannote-pipeline", got
        else:
            assert isinstance(got, amd_vm.VoiceActivitySegmentation) and got.hyperparameters["onset"] == 0.45
    assert ref_vad_calls == [os.path.join(tmp, "absent.bin"), garbage], ref_vad_calls
    # the default checkpoint (model_fp None) replaced by an exported state_dict of one's own
    os.environ["WX_VAD_STATE_DICT"] = plain
    got = lv("cpu", vad_onset=0.4)
    assert isinstance(got, amd_vm.VoiceActivitySegmentation) and got.hyperparameters["onset"] == 0.4
    del os.environ["WX_VAD_STATE_DICT"]
    print("rebound", len(rebound))
''')


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "whisperx")), reason="reference tree absent (GPU box)")
def test_install_rebinds_reference_call_sites():
    r = subprocess.run([sys.executable, "-c", SCRIPT, REF, ROOT], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rebound" in r.stdout


def test_install_on_a_package_without_reference_modules():
    import types

    import whisperx_amd

    pkg = types.ModuleType("fake_whisperx_pkg")
    pkg.align = None
    sys.modules["fake_whisperx_pkg"] = pkg
    try:
        done = whisperx_amd.install(pkg, import_missing=False)
        assert done == [("fake_whisperx_pkg", "align")]
        assert pkg.align is whisperx_amd.align
    finally:
        del sys.modules["fake_whisperx_pkg"]
