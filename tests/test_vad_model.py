"""The VAD producer's segmentation model takes a pyannote/segmentation checkpoint (vad.py:20-59,
Model.from_pretrained of whisperX's VAD_SEGMENTATION_URL file): pyannote's module tree and
parameter names, SincNet's band-pass filterbank materialised from the checkpoint's band edges,
and load_vad_model's file / checksum handling.  pyannote.audio and asteroid-filterbanks are
absent, so the filterbank's values are checked by their defining properties (parity
unpinned), and the checkpoint by a synthetic state_dict with the real key set and shapes."""
import numpy as np
import pytest
import torch

# pyannote.audio 3.1 PyanNet (SincNet + monolithic BiLSTM + 2 linear + classifier) state_dict
PYANNOTE_KEYS = {
    "sincnet.wav_norm1d.weight": (1,), "sincnet.wav_norm1d.bias": (1,),
    "sincnet.conv1d.0.filterbank.low_hz_": (40, 1), "sincnet.conv1d.0.filterbank.band_hz_": (40, 1),
    "sincnet.conv1d.0.filterbank.n_": (1, 125), "sincnet.conv1d.0.filterbank.window_": (125,),
    "sincnet.conv1d.1.weight": (60, 80, 5), "sincnet.conv1d.1.bias": (60,),
    "sincnet.conv1d.2.weight": (60, 60, 5), "sincnet.conv1d.2.bias": (60,),
    "sincnet.norm1d.0.weight": (80,), "sincnet.norm1d.0.bias": (80,),
    "sincnet.norm1d.1.weight": (60,), "sincnet.norm1d.1.bias": (60,),
    "sincnet.norm1d.2.weight": (60,), "sincnet.norm1d.2.bias": (60,),
    "linear.0.weight": (128, 256), "linear.0.bias": (128,), "linear.1.weight": (128, 128), "linear.1.bias": (128,),
    "classifier.weight": (3, 128), "classifier.bias": (3,),
}
for _l in range(2):
    for _sfx in ("", "_reverse"):
        _in = 60 if _l == 0 else 256
        PYANNOTE_KEYS[f"lstm.weight_ih_l{_l}{_sfx}"] = (512, _in)
        PYANNOTE_KEYS[f"lstm.weight_hh_l{_l}{_sfx}"] = (512, 128)
        PYANNOTE_KEYS[f"lstm.bias_ih_l{_l}{_sfx}"] = (512,)
        PYANNOTE_KEYS[f"lstm.bias_hh_l{_l}{_sfx}"] = (512,)


def _synthetic_checkpoint(seed=0):
    from whisperx_amd.vad_model import PyanNet

    g = torch.Generator().manual_seed(seed)
    ref = PyanNet().state_dict()
    sd = {}
    for k, shape in PYANNOTE_KEYS.items():
        if k.endswith(("n_", "window_")):
            sd[k] = ref[k].clone()  # buffers: fixed by the filterbank geometry
        elif k.endswith("low_hz_"):
            sd[k] = torch.linspace(40.0, 6000.0, 40).view(40, 1)
        elif k.endswith("band_hz_"):
            sd[k] = torch.full((40, 1), 120.0)
        else:
            sd[k] = torch.randn(shape, generator=g) * 0.1
    return sd


def test_pyannet_state_dict_has_pyannote_names_and_shapes():
    from whisperx_amd.vad_model import PyanNet

    sd = PyanNet().state_dict()
    assert {k: tuple(v.shape) for k, v in sd.items()} == PYANNOTE_KEYS


def test_sinc_filterbank_properties():
    """Cosine filters are even, sine filters odd, the centre tap of a cosine filter is 1
    (2 band / 2 band), and every filter's magnitude response peaks inside its band."""
    from whisperx_amd.vad_model import SincFilterbank

    fb = SincFilterbank()
    with torch.no_grad():
        f = fb.filters()[:, 0].numpy().astype(np.float64)
    assert f.shape == (80, 251)
    cos, sin = f[:40], f[40:]
    np.testing.assert_allclose(cos, cos[:, ::-1], atol=1e-6)
    np.testing.assert_allclose(sin, -sin[:, ::-1], atol=1e-6)
    np.testing.assert_allclose(cos[:, 125], 1.0, atol=1e-6)
    low = 50.0 + np.abs(fb.low_hz_.detach().numpy()[:, 0])
    high = np.minimum(low + 50.0 + np.abs(fb.band_hz_.detach().numpy()[:, 0]), 8000.0)
    freqs = np.fft.rfftfreq(8192, 1 / 16000)
    for k in range(40):
        mag = np.abs(np.fft.rfft(cos[k], 8192))
        peak = freqs[np.argmax(mag)]
        assert low[k] - 60 <= peak <= high[k] + 60, (k, low[k], high[k], peak)


def test_from_pyannote_state_dict_loads_the_checkpoint_weights():
    from whisperx_amd.vad_model import PyanNet

    sd = _synthetic_checkpoint()
    m = PyanNet.from_pyannote_state_dict({"state_dict": sd, "epoch": 3})  # Lightning layout
    for k, v in m.state_dict().items():
        assert torch.equal(v, sd[k]), k
    enc = m.sincnet.conv1d[0]
    with torch.no_grad():
        w = enc.weight()
        # the filters follow the loaded band edges (40 Hz + 50 Hz floor ... 6000 Hz)
        assert torch.equal(w, enc.filterbank.filters())
        y = m.eval()(torch.randn(2, 1, 80000))
    assert y.shape == (2, 293, 3)
    bad = dict(sd)
    bad.pop("linear.1.bias")
    with pytest.raises(RuntimeError, match="linear.1.bias"):
        PyanNet.from_pyannote_state_dict(bad)
    with pytest.raises(KeyError):
        PyanNet.from_pyannote_state_dict({"foo": torch.zeros(1)})


def test_load_vad_model_local_file(tmp_path):
    from whisperx_amd import vad_model

    fp = str(tmp_path / "seg.bin")
    torch.save({"state_dict": _synthetic_checkpoint(1)}, fp)
    with pytest.raises(RuntimeError, match="SHA256 checksum"):
        vad_model.load_vad_model("cpu", model_fp=fp)  # the reference checks its download's digest
    pipe = vad_model.load_vad_model("cpu", vad_onset=0.45, model_fp=fp, check_sha256=False)
    assert pipe.hyperparameters == {"onset": 0.45, "offset": 0.363, "min_duration_on": 0.1, "min_duration_off": 0.1}
    assert torch.equal(pipe.model.classifier.bias, _synthetic_checkpoint(1)["classifier.bias"])
    with pytest.raises(FileNotFoundError):
        vad_model.load_vad_model("cpu", model_fp=str(tmp_path / "missing.bin"))
    with pytest.raises(RuntimeError, match="not a regular file"):
        vad_model.load_vad_model("cpu", model_fp=str(tmp_path))


# --- a Lightning-style checkpoint whose pickle names code: the no-code reader ----------------
_SIDE_EFFECTS = []


def _record_side_effect(tag):
    """What unpickling _Trap would call.  The no-code reader must never reach it."""
    _SIDE_EFFECTS.append(tag)
    return tag


class _Trap:
    """Pickled into the checkpoint beside the state_dict (as Lightning pickles its hyper-parameter
    and callback objects): a normal unpickler calls _record_side_effect while loading."""

    def __reduce__(self):
        return (_record_side_effect, ("executed",))


class _Hparams(dict):
    """A dict subclass with state (NEWOBJ + SETITEMS + BUILD opcodes)."""

    def __init__(self, **kw):
        super().__init__(**kw)
        self.note = "built"


def test_read_checkpoint_tensors_executes_nothing(tmp_path):
    from whisperx_amd import vad_model

    sd = _synthetic_checkpoint(2)
    fp = str(tmp_path / "lightning.ckpt")
    torch.save({"state_dict": sd, "epoch": 7, "trap": _Trap(), "hyper_parameters": _Hparams(lr=1e-3, trap=_Trap()),
                "callbacks": [_Trap(), {"x": _Trap()}]}, fp)
    _SIDE_EFFECTS.clear()
    with pytest.raises(Exception):  # torch's own safe loader refuses the file
        torch.load(fp, map_location="cpu", weights_only=True)
    got = vad_model.read_checkpoint_tensors(fp)
    assert _SIDE_EFFECTS == []  # the trap's callable was never called
    assert set(got) == set(sd) and all(torch.equal(got[k], sd[k]) for k in sd)
    # load_vad_model takes that path on its own when weights_only refuses the file
    pipe = vad_model.load_vad_model("cpu", model_fp=fp, check_sha256=False)
    assert _SIDE_EFFECTS == []
    assert torch.equal(pipe.model.classifier.bias, sd["classifier.bias"])


def test_unreadable_checkpoint_still_falls_back(tmp_path):
    from whisperx_amd import vad_model

    fp = tmp_path / "garbage.bin"
    fp.write_bytes(b"not a checkpoint at all" * 10)
    with pytest.raises(vad_model.CheckpointNotLoadable):
        vad_model.load_vad_model("cpu", model_fp=str(fp), check_sha256=False)
    other = str(tmp_path / "other.ckpt")  # readable, but not a PyanNet state_dict
    torch.save({"state_dict": {"encoder.weight": torch.zeros(3)}, "trap": _Trap()}, other)
    with pytest.raises(vad_model.CheckpointNotLoadable):
        vad_model.load_vad_model("cpu", model_fp=other, check_sha256=False)
    assert _SIDE_EFFECTS == []
