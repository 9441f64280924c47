"""VAD producer on the GPU: the speech scores that merge_chunks
binarises, computed where merge_chunks then reads them.

Reference: ``VoiceActivitySegmentation.apply`` (whisperx/vad.py:198-240), called from
``FasterWhisperPipeline.transcribe`` (asr.py:186) through pyannote.audio 3.1:

1. ``Inference.slide``: 5 s windows every 0.5 s (10 % of the window) over the waveform; the
   last, incomplete window is zero-padded to 5 s;
2. the segmentation model (pyannote/segmentation, PyanNet: SincNet front-end, 2-layer BiLSTM,
   2 linear layers, 3-speaker multi-label sigmoid head) on batches of windows;
3. the multi-label pre-aggregation hook: max over the speaker classes;
4. ``Inference.aggregate``: overlap-add of the window frames onto the file's frame grid
   (16.875 ms step, 61.9375 ms receptive field), averaged over the windows covering a frame.

Here steps 1-2 are PyTorch-ROCm (one batched forward per group of windows; every window has
the same 5 s shape, so MIOpen tunes each convolution once) and steps 3-4 are one HIP kernel
(``wx_vad_aggregate``: one thread per output frame, gathering its windows in window order, so
the fp32 sums are the reference's sequential ones).  The scores stay on the device:
``Binarize``/``merge_chunks`` read them in place (``wx_binarize``).

The whisperX VAD checkpoint (``VAD_SEGMENTATION_URL``, pyannote/segmentation) cannot be fetched
offline, but a local copy loads: ``PyanNet`` has pyannote's module tree and parameter names
(``sincnet.wav_norm1d``, ``sincnet.conv1d.0.filterbank.{low_hz_,band_hz_,n_,window_}``,
``sincnet.conv1d.{1,2}``, ``sincnet.norm1d.*``, ``lstm.*``, ``linear.*``, ``classifier``), the first
convolution being the SincNet band-pass filterbank materialised from its learnt band edges
(``SincFilterbank``), so ``load_vad_model(model_fp=...)`` / ``PyanNet.load_pyannote_state_dict``
take the checkpoint's ``state_dict`` as it is.  The benchmarks time random weights.  Parity of the
aggregation is pinned to a restatement of pyannote's published algorithm (oracle.vad_aggregate),
not to pyannote itself, which is absent; the filterbank restates asteroid-filterbanks'
ParamSincFB (absent too): "parity unpinned" at the pyannote boundary.
"""
from __future__ import annotations

import hashlib
import math
import os
import pickle
import types
import weakref
from typing import Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib
from .vad import SlidingWindow, SlidingWindowFeature

SAMPLE_RATE = 16000


def _to_mel(hz):
    return 2595.0 * np.log10(1.0 + hz / 700.0)


def _to_hz(mel):
    return 700.0 * (10.0 ** (mel / 2595.0) - 1.0)


class SincFilterbank(torch.nn.Module):
    """SincNet's parametrised band-pass filterbank (Ravanelli & Bengio 2018, in the form of
    asteroid-filterbanks' ParamSincFB that pyannote's SincNet uses): n_filters / 2 learnt
    (low edge, band width) pairs in Hz, each giving a cosine-phase and a sine-phase windowed
    band-pass filter of `kernel_size` taps (n_filters in all, cosine ones first).  Parameters
    and buffers carry the checkpoint's names (low_hz_, band_hz_ [n/2, 1]; n_ [1, half];
    window_ [half]).  Initialised on the mel scale between 30 Hz and sr/2 - 100 Hz."""

    def __init__(self, n_filters: int = 80, kernel_size: int = 251, sample_rate: int = SAMPLE_RATE,
                 min_low_hz: float = 50.0, min_band_hz: float = 50.0):
        super().__init__()
        if kernel_size % 2 == 0:
            kernel_size += 1
        self.n_filters, self.kernel_size, self.sample_rate = n_filters, kernel_size, sample_rate
        self.min_low_hz, self.min_band_hz = float(min_low_hz), float(min_band_hz)
        half = kernel_size // 2
        mel = np.linspace(_to_mel(30.0), _to_mel(sample_rate / 2 - (min_low_hz + min_band_hz)), n_filters // 2 + 1,
                          dtype=np.float32)
        hz = _to_hz(mel)
        self.low_hz_ = torch.nn.Parameter(torch.from_numpy(hz[:-1]).view(-1, 1))
        self.band_hz_ = torch.nn.Parameter(torch.from_numpy(np.diff(hz)).view(-1, 1))
        self.register_buffer("window_", torch.from_numpy(np.hamming(kernel_size)[:half]).float())
        self.register_buffer("n_", 2 * math.pi * torch.arange(-half, 0.0).view(1, -1) / sample_rate)

    def filters(self) -> torch.Tensor:
        """[n_filters, 1, kernel_size]: per band, the left half of the windowed band-pass
        impulse response (difference of the two edges' sinc kernels), its centre tap and the
        mirrored right half, normalised by twice the band width."""
        low = self.min_low_hz + torch.abs(self.low_hz_)
        high = torch.clamp(low + self.min_band_hz + torch.abs(self.band_hz_), self.min_low_hz, self.sample_rate / 2)
        band = (high - low)[:, 0]
        ft_low = torch.matmul(low, self.n_)
        ft_high = torch.matmul(high, self.n_)
        out = []
        for phase in ("cos", "sin"):
            if phase == "cos":
                left = ((torch.sin(ft_high) - torch.sin(ft_low)) / (self.n_ / 2)) * self.window_
                centre = 2 * band.view(-1, 1)
                right = torch.flip(left, dims=[1])
            else:
                left = ((torch.cos(ft_low) - torch.cos(ft_high)) / (self.n_ / 2)) * self.window_
                centre = torch.zeros_like(band.view(-1, 1))
                right = -torch.flip(left, dims=[1])
            bp = torch.cat([left, centre, right], dim=1) / (2 * band[:, None])
            out.append(bp.view(self.n_filters // 2, 1, self.kernel_size))
        return torch.cat(out, dim=0)


_PATCH_BYTES = int(os.environ.get("WX_VAD_PATCH_MB", "1024")) << 20  # conv1d_batched: patch buffer per chunk of windows (Cin == 1)


_CT_CACHE: dict = {}


def _conv_taps_weights(w: torch.Tensor) -> torch.Tensor:
    """w [Cout, Cin, k] packed for wx_conv1d_taps_tm ([k][CINP / 4][64][4], zero-padded),
    cached per weight tensor (identity and version)."""
    ver = w._version if not w.is_inference() else -1
    hit = _CT_CACHE.get(id(w))
    c = hit[2] if hit is not None and hit[0]() is w and hit[1] == ver else None
    if c is None:
        Cout, Cin, k = w.shape
        cinp = 64 if Cin <= 64 else 80
        with torch.no_grad():
            wp = torch.zeros((k, cinp, 64), dtype=torch.float32, device=w.device)
            wp[:, :Cin, :Cout] = w.detach().permute(2, 1, 0)
            c = wp.view(k, cinp // 4, 4, 64).permute(0, 1, 3, 2).contiguous()
        if len(_CT_CACHE) > 16:
            _CT_CACHE.clear()
        _CT_CACHE[id(w)] = (weakref.ref(w), ver, c)  # (the weakref: an id reused by another tensor misses)
    return c


def conv1d_batched(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], stride: int) -> torch.Tensor:
    """F.conv1d(x, w, b, stride) (no padding, dilation 1, one group) for a batch of windows
    through a few large GEMMs.  MIOpen's choice for these shapes depends on the state of its
    kernel cache: on a fresh MI355X box the first forward settles on one im2col + GEMM per
    window for the whole process (21,573 im2col launches per hour of audio, half the producer's
    GPU time: profiles/r3_vad1h_kernel_stats.csv; 1 h in 544 ms), on a warm one on an implicit
    GEMM (200 ms).  These GEMMs take the same time either way (tools/vad_conv_probe.py: 14.4 /
    7.9 / 2.8 ms per 2,048-window batch vs MIOpen's best 15.5 / 5.3 / 1.8 ms).  Returns [B, Cout, Lout] as the transposed view of a
    time-major [B, Lout, Cout] buffer.

    * Cin == 1 (the sinc filterbank, k = 251, stride 10): the taps are zero-padded to a multiple
      of the stride, so patch row t is the contiguous slice x[s*t : s*t + k'] — an unfold view,
      materialised for ~1 GB worth of windows at a time and multiplied by the [k', Cout] filters;
    * Cin > 1, stride 1 (k = 5): the windows are flattened time-major into [B*L, Cin] and the
      output is the sum over the k taps of one GEMM on the row-shifted view each; the rows that
      straddle two windows (the last k - 1 of every window) are computed and dropped."""
    B, Cin, L = x.shape
    Cout, _, k = w.shape
    Lout = (L - k) // stride + 1
    if Cin == 1:
        kp = -(-k // stride) * stride
        xs = x.reshape(B, L)
        if kp > k:
            xs = F.pad(xs, (0, kp - k))
        wp = F.pad(w.reshape(Cout, k), (0, kp - k)).t().contiguous()  # [kp, Cout]
        pat = xs.unfold(1, kp, stride)[:, :Lout]  # [B, Lout, kp] view
        out = torch.empty((B, Lout, Cout), dtype=x.dtype, device=x.device)
        cb = max(1, _PATCH_BYTES // max(1, Lout * kp * x.element_size()))
        for i in range(0, B, cb):
            p = pat[i:i + cb].reshape(-1, kp)
            o = out[i:i + cb].view(-1, Cout)
            if b is not None:
                torch.addmm(b, p, wp, out=o)
            else:
                torch.mm(p, wp, out=o)
        return out.transpose(1, 2)
    assert stride == 1
    xt = x.transpose(1, 2)
    if (not os.environ.get("WX_NO_CONV_KERNEL") and x.is_cuda and k == 5 and Cout <= 64 and Cin <= 80 and Cin % 4 == 0
            and xt.is_contiguous() and x.dtype == torch.float32 and xt.data_ptr() % 16 == 0 and B <= 65535):
        # every window's conv in one kernel (wx_conv1d_taps_tm): the activation read once
        from . import _lib

        return _lib.conv1d_taps_tm(xt, _conv_taps_weights(w), b, Cout, k).transpose(1, 2)
    X = xt.reshape(B * L, Cin)  # time-major copy
    R = B * L - k + 1
    full = torch.empty((B * L, Cout), dtype=x.dtype, device=x.device)
    wt = w.permute(2, 1, 0)  # [k, Cin, Cout]
    for j in range(k):
        if j == 0:
            if b is not None:
                torch.addmm(b, X[0:R], wt[0], out=full[:R])
            else:
                torch.mm(X[0:R], wt[0], out=full[:R])
        else:
            full[:R].addmm_(X[j:j + R], wt[j])
    return full.view(B, L, Cout)[:, :Lout].transpose(1, 2)


class SincEncoder(torch.nn.Module):
    """The filterbank as a bias-free strided convolution (asteroid Encoder).  The filters are
    a function of the band edges only: they are materialised once per parameter version and
    cached (inference), not rebuilt by every forward."""

    def __init__(self, stride: int = 10, **fb):
        super().__init__()
        self.filterbank = SincFilterbank(**fb)
        self.stride = stride
        self._cache = None

    def weight(self) -> torch.Tensor:
        fb = self.filterbank
        if torch.is_grad_enabled():
            return fb.filters()
        key = tuple((p.data_ptr(), p._version, p.device) for p in (fb.low_hz_, fb.band_hz_))
        if self._cache is None or self._cache[0] != key:
            with torch.no_grad():
                self._cache = (key, fb.filters())
        return self._cache[1]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if _gemm_conv(x):
            return conv1d_batched(x, self.weight(), None, self.stride)
        return F.conv1d(x, self.weight(), stride=self.stride)


def _gemm_conv(x: torch.Tensor) -> bool:
    """Inference forwards on a HIP device take conv1d_batched (WX_MIOPEN_CONV=1: MIOpen)."""
    return x.is_cuda and not torch.is_grad_enabled() and not os.environ.get("WX_MIOPEN_CONV")


class SincNet(torch.nn.Module):
    """pyannote's SincNet block: waveform InstanceNorm, then [sinc filterbank (|.|), conv(80->60,
    k=5), conv(60->60, k=5)], each followed by MaxPool(3) -> InstanceNorm -> LeakyReLU."""

    def __init__(self, sample_rate: int = SAMPLE_RATE, stride: int = 10):
        super().__init__()
        self.wav_norm1d = torch.nn.InstanceNorm1d(1, affine=True)
        self.conv1d = torch.nn.ModuleList([SincEncoder(stride=stride, sample_rate=sample_rate),
                                           torch.nn.Conv1d(80, 60, 5), torch.nn.Conv1d(60, 60, 5)])
        self.pool1d = torch.nn.ModuleList([torch.nn.MaxPool1d(3, stride=3) for _ in range(3)])
        self.norm1d = torch.nn.ModuleList([torch.nn.InstanceNorm1d(80, affine=True), torch.nn.InstanceNorm1d(60, affine=True),
                                           torch.nn.InstanceNorm1d(60, affine=True)])

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.stages(self.wav_norm1d(x), 0)

    def stages(self, x: torch.Tensor, first: int) -> torch.Tensor:
        """Stages first..2 on x (the normalised waveform for stage 0, else the previous stage's
        [B, C, L] output)."""
        for i, (conv, pool, norm) in enumerate(zip(self.conv1d, self.pool1d, self.norm1d)):
            if i < first:
                continue
            gemm = _gemm_conv(x)
            if i > 0 and gemm:
                x = conv1d_batched(x, conv.weight, conv.bias, conv.stride[0])
            else:
                x = conv(x)
            if gemm and _fused_epilogue(pool, norm, x):
                # |.| -> max-pool -> instance norm -> leaky ReLU in one HIP kernel on the
                # time-major conv output (wx_sincnet_stage), returned as the [B, C, L/3] view
                x = _lib.sincnet_stage(x.transpose(1, 2), i == 0, norm.weight, norm.bias, norm.eps).transpose(1, 2)
                continue
            if i == 0:
                x = torch.abs(x)
            x = F.leaky_relu(norm(pool(x)))
        return x


def _conv_global(x: torch.Tensor, w: torch.Tensor, stride: int) -> torch.Tensor:
    """The bias-free strided convolution of one long signal x [n] with filters w [C, k]:
    [(n - k) // stride + 1, C] time-major, as row-chunked GEMMs on the unfold view (taps
    zero-padded to a multiple of the stride; ~1 GB of patch rows at a time)."""
    C, k = w.shape
    n = x.shape[0]
    F_out = (n - k) // stride + 1
    kp = -(-k // stride) * stride
    wp = F.pad(w, (0, kp - k)).t().contiguous()  # [kp, C]
    if (x.is_cuda and C == 80 and kp == 260 and stride <= 16 and x.dtype == torch.float32
            and not os.environ.get("WX_NO_SINC_KERNEL")):
        # wx_sinc_filterbank: the rows read where they lie (no patch copy)
        from . import _lib

        return _lib.sinc_filterbank(x.contiguous(), wp, k, stride)
    xs = F.pad(x, (0, kp - k)) if kp > k else x
    pat = xs.unfold(0, kp, stride)[:F_out]  # [F, kp] view
    out = torch.empty((F_out, C), dtype=x.dtype, device=x.device)
    rows = max(1, _PATCH_BYTES // (kp * x.element_size()))
    for r in range(0, F_out, rows):
        torch.mm(pat[r:r + rows], wp, out=out[r:r + rows])
    return out


def _shared_sinc_ok(model, w: torch.Tensor, hop: int) -> bool:
    """Whether chunk_scores may run the sinc filterbank once over the waveform
    (VoiceActivitySegmentation._shared_sinc_scores): this package's PyanNet on a HIP device
    with the GEMM convolutions and the fused stage epilogue, a window hop that is a multiple
    of the filterbank stride, and the waveform InstanceNorm using instance statistics
    (WX_NO_SHARED_SINC=1: one convolution per window)."""
    if os.environ.get("WX_NO_SHARED_SINC") or not isinstance(model, PyanNet) or not _gemm_conv(w):
        return False
    sn = model.sincnet
    enc, wn = sn.conv1d[0], sn.wav_norm1d
    if not isinstance(enc, SincEncoder) or hop % enc.stride or os.environ.get("WX_NO_SINC_EPILOGUE"):
        return False
    if not isinstance(wn, torch.nn.InstanceNorm1d) or wn.num_features != 1 or (wn.track_running_stats and not wn.training):
        return False
    pool, norm = sn.pool1d[0], sn.norm1d[0]
    C = int(enc.weight().shape[0])  # the checkpoint's filter count (the probe's channels)
    probe = torch.empty((1, C, 3), device=w.device).transpose(1, 2).contiguous().transpose(1, 2)
    return _fused_epilogue(pool, norm, probe)


def _fused_epilogue(pool, norm, x) -> bool:
    """Whether a SincNet stage's pool / norm / activation take wx_sincnet_stage: pyannote's
    shapes (MaxPool1d(3, 3), InstanceNorm1d using instance statistics, <= 128 channels, a
    multiple of 4) on a time-major float32 conv output (WX_NO_SINC_EPILOGUE=1: torch's ops)."""
    if os.environ.get("WX_NO_SINC_EPILOGUE") or x.dtype != torch.float32:
        return False
    if not (isinstance(pool, torch.nn.MaxPool1d) and pool.kernel_size in (3, (3,)) and pool.stride in (3, (3,))
            and pool.padding in (0, (0,)) and pool.dilation in (1, (1,)) and not pool.ceil_mode):
        return False
    if not isinstance(norm, torch.nn.InstanceNorm1d) or (norm.track_running_stats and not norm.training):
        return False
    C = x.shape[1]
    xt = x.transpose(1, 2)
    return C % 4 == 0 and C <= 128 and xt.stride(2) == 1 and xt.stride(1) == C


_LSTM_CACHE: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


def _lstm_weights(lstm: torch.nn.LSTM, layer: int):
    """(W_ih of both directions [8H, in], b_ih + b_hh [8H], weight_hh [2, 4H, H]) of one layer,
    cached per module until a parameter changes."""
    # (an inference tensor — a model built or loaded under torch.inference_mode() — has no
    # version counter: -1, as emission._version)
    key = (layer,) + tuple((p.data_ptr(), -1 if p.is_inference() else p._version) for p in lstm.parameters())
    c = _LSTM_CACHE.get(lstm)
    if c is None or c[0][1:] != key[1:]:
        c = (key, {})
        _LSTM_CACHE[lstm] = c
    if layer not in c[1]:
        sfx = [f"_l{layer}", f"_l{layer}_reverse"]
        with torch.no_grad():
            wih = torch.cat([getattr(lstm, "weight_ih" + s) for s in sfx], 0).detach().contiguous()
            b = torch.cat([(getattr(lstm, "bias_ih" + s) + getattr(lstm, "bias_hh" + s)) for s in sfx]).detach()
            whh = torch.stack([getattr(lstm, "weight_hh" + s) for s in sfx], 0).detach().contiguous()
        c[1][layer] = (wih, b, whh)
    return c[1][layer]


def lstm_forward(lstm: torch.nn.LSTM, x: torch.Tensor) -> torch.Tensor:
    """lstm(x)[0] for a batch-first input [B, T, in]: PyanNet's bidirectional LSTM (H = 128,
    biases, no projection) of an inference forward on a HIP device runs layer by layer as one
    input-projection GEMM (both directions) + wx_lstm_bidir_layer (the recurrence of both
    directions in one persistent kernel) instead of MIOpen's per-step launches
    (WX_NO_LSTM_KERNEL=1: torch's LSTM)."""
    if (os.environ.get("WX_NO_LSTM_KERNEL") or not x.is_cuda or torch.is_grad_enabled() or lstm.training
            or not lstm.bidirectional or not lstm.batch_first or lstm.hidden_size != 128 or not lstm.bias
            or getattr(lstm, "proj_size", 0) or x.dtype != torch.float32 or x.dim() != 3):
        return lstm(x)[0]
    from . import _lib

    B, T, _ = x.shape
    for layer in range(lstm.num_layers):
        wih, b, whh = _lstm_weights(lstm, layer)
        xp = torch.addmm(b, x.reshape(B * T, -1), wih.t()).view(B, T, 2, 4 * lstm.hidden_size)
        x = _lib.lstm_bidir_layer(xp, whh, B, T)
    return x


class PyanNet(torch.nn.Module):
    """pyannote/segmentation's PyanNet (pyannote.audio PyanNet defaults, module names as in its
    checkpoints): SincNet (stride 10) -> BiLSTM(128, 2 layers, batch-first) -> 2 x (Linear(128)
    + LeakyReLU) -> Linear(n_classes) -> sigmoid (multi-label: whisperX's VAD checkpoint has 3
    speaker classes).  Output: [batch, frames, n_classes]; 293 frames per 5 s window
    (270-sample step, 991-sample receptive field)."""

    def __init__(self, n_classes: int = 3, lstm_hidden: int = 128, lstm_layers: int = 2, linear_hidden: int = 128):
        super().__init__()
        self.sincnet = SincNet()
        self.lstm = torch.nn.LSTM(60, lstm_hidden, num_layers=lstm_layers, bidirectional=True, batch_first=True)
        self.linear = torch.nn.ModuleList([torch.nn.Linear(2 * lstm_hidden, linear_hidden),
                                           torch.nn.Linear(linear_hidden, linear_hidden)])
        self.classifier = torch.nn.Linear(linear_hidden, n_classes)
        # frame geometry of the conv/pool chain (pyannote's receptive field arithmetic)
        self.frame_step = 10 * 3 * 3 * 3 / SAMPLE_RATE                          # 270 samples
        self.frame_duration = (251 + (3 - 1) * 10 + (5 - 1) * 30 + (3 - 1) * 30 + (5 - 1) * 90
                               + (3 - 1) * 90) / SAMPLE_RATE                      # 991 samples

    @staticmethod
    def n_frames(n_samples: int) -> int:
        L = (n_samples - 251) // 10 + 1
        L = L // 3
        L = (L - 5) + 1
        L = L // 3
        L = (L - 5) + 1
        return L // 3

    def forward(self, waveforms: torch.Tensor) -> torch.Tensor:
        return self.head(self.sincnet(waveforms))

    def head(self, x: torch.Tensor) -> torch.Tensor:
        """LSTM -> linear layers -> classifier on the SincNet features [B, 60, frames]."""
        x = lstm_forward(self.lstm, x.transpose(1, 2))
        for lin in self.linear:
            x = F.leaky_relu(lin(x))
        return torch.sigmoid(self.classifier(x))

    @classmethod
    def from_pyannote_state_dict(cls, state_dict) -> "PyanNet":
        """A PyanNet holding a pyannote/segmentation checkpoint's weights: the model's
        ``state_dict`` (or a Lightning checkpoint dict holding one under "state_dict"), keys as
        pyannote names them.  The class count is read from the classifier; the load is strict
        (a missing or unexpected key raises, naming it)."""
        sd = state_dict.get("state_dict", state_dict) if isinstance(state_dict, dict) else state_dict
        w = sd.get("classifier.weight")
        if w is None:
            raise KeyError("not a pyannote PyanNet state_dict: no 'classifier.weight'")
        m = cls(n_classes=int(w.shape[0]))
        m.load_state_dict(sd, strict=True)
        return m

    def load_pyannote_state_dict(self, state_dict):
        sd = state_dict.get("state_dict", state_dict) if isinstance(state_dict, dict) else state_dict
        return self.load_state_dict(sd, strict=True)


def closest_frame(t: float, start: float, duration: float, step: float) -> int:
    """pyannote SlidingWindow.closest_frame: int(rint((t - start - duration / 2) / step))."""
    return int(round((t - start - 0.5 * duration) / step))  # Python round == numpy rint (half to even)


class VoiceActivitySegmentation:
    """vad.py:198-240: speech scores of a waveform as a SlidingWindowFeature [frames, 1] whose
    data stays a device tensor.  ``duration``/``step`` are the sliding windows (5 s / 0.5 s),
    ``batch_size`` the windows per model forward.  pyannote's default is 32; the forward is
    host-bound at that size (MIOpen's LSTM costs ~25 ms of host time per call), so the
    default here is 1024 windows (~2.6 GB of activations; MIOpen's LSTM rejects batches of
    ~7,000).  MI355X, 1 h of audio at 2,048 windows per batch: 225 ms."""

    def __init__(self, segmentation: Optional[torch.nn.Module] = None, device="cuda", duration: float = 5.0,
                 step: Optional[float] = None, batch_size: int = 1024):
        self.device = torch.device(device)
        self.model = (segmentation if segmentation is not None else PyanNet()).to(self.device).eval()
        self.duration = float(duration)
        self.step = float(step) if step is not None else 0.1 * self.duration
        self.batch_size = int(batch_size)

    def windows(self, n_samples: int):
        """(number of full windows, whether a zero-padded last window follows) — Inference.slide."""
        win = round(self.duration * SAMPLE_RATE)
        hop = round(self.step * SAMPLE_RATE)
        if n_samples < win:
            return 0, True
        n = (n_samples - win) // hop + 1
        return n, (n_samples - win) % hop > 0

    def chunk_scores(self, waveform: torch.Tensor) -> torch.Tensor:
        """Model outputs of every window: [n_windows, frames, classes] on the device."""
        win = round(self.duration * SAMPLE_RATE)
        hop = round(self.step * SAMPLE_RATE)
        w = waveform.reshape(1, -1).to(self.device, dtype=torch.float32)
        n_full, has_last = self.windows(w.shape[1])
        outs = []
        with torch.inference_mode():
            if n_full and _shared_sinc_ok(self.model, w, hop):
                outs.extend(self._shared_sinc_scores(w, n_full, win, hop))
            elif n_full:
                chunks = w.unfold(1, win, hop)[0]  # [n_full, win] (a view)
                for i in range(0, n_full, self.batch_size):
                    outs.append(self.model(chunks[i:i + self.batch_size].unsqueeze(1).contiguous()))
            if has_last:
                last = w[:, n_full * hop:]
                last = F.pad(last, (0, win - last.shape[1]))
                outs.append(self.model(last.unsqueeze(1)))
        return torch.cat(outs, 0)

    def _shared_sinc_scores(self, w: torch.Tensor, n_full: int, win: int, hop: int):
        """The full windows' outputs with the sinc filterbank run once over the waveform.

        Windows overlap tenfold (5 s every 0.5 s), and the filterbank is a bias-free strided
        convolution, so window b's stage-1 convolution is rows [b * hop / 10, + 7975) of the
        convolution of the whole span (computed per batch of windows: that batch's span).  The
        waveform InstanceNorm of the window (pyannote's
        `wav_norm1d`) is an affine of its input — (x - mean_b) / std_b * g + h — and commutes
        into the convolution: conv(x_norm)[t, c] = (g / std_b) conv(x)[t, c] + (h - g mean_b /
        std_b) * sum(filter c).  wx_sincnet_stage_ex applies that per-window affine while it
        reads the shared output, then |.| -> max-pool -> InstanceNorm -> LeakyReLU as before.
        Float noise only (the sums are reassociated); stages 2-3 and the rest are unchanged."""
        sn = self.model.sincnet
        enc, norm0 = sn.conv1d[0], sn.norm1d[0]
        wn = sn.wav_norm1d
        wf = enc.weight()  # [80, 1, k]
        C, _, k = wf.shape
        s = enc.stride
        L1 = (win - k) // s + 1
        fpw = hop // s
        # the windows' waveform statistics (InstanceNorm1d: biased variance, eps), in fp64.
        # Windows overlap tenfold, so they come from per-hop block sums: sum and sum of squares
        # of each hop of samples accumulated in fp64 straight from the fp32 waveform (no fp64
        # copy), a window being win / hop consecutive blocks.  (A var_mean over each window's
        # own fp64 copy read every sample ten times: ~3 ms per hour of copies and reductions.)
        # var = E[x^2] - E[x]^2 in fp64: its cancellation error is far below fp32 resolution.
        if win % hop == 0:
            nb = n_full - 1 + win // hop
            blk = w[0, : nb * hop].view(nb, hop)
            s1 = blk.sum(1, dtype=torch.float64)
            s2 = torch.linalg.vector_norm(blk, dim=1, dtype=torch.float64).square()
            m = win // hop  # blocks per window
            c1 = F.pad(s1.cumsum(0), (1, 0))
            c2 = F.pad(s2.cumsum(0), (1, 0))
            mean = (c1[m:m + n_full] - c1[:n_full]) / win
            var = ((c2[m:m + n_full] - c2[:n_full]) / win - mean * mean).clamp_min(0.0)
        else:  # windows not a whole number of hops: each window's own fp64 statistics
            chunks = w.unfold(1, win, hop)[0]
            mean = torch.empty(n_full, dtype=torch.float64, device=w.device)
            var = torch.empty_like(mean)
            for i in range(0, n_full, 1024):
                c = chunks[i:i + 1024].to(torch.float64)
                var[i:i + 1024], mean[i:i + 1024] = torch.var_mean(c, dim=1, unbiased=False)
        inv = torch.rsqrt(var + float(wn.eps))
        g = wn.weight.double()[0] if wn.weight is not None else torch.ones((), dtype=torch.float64, device=w.device)
        h = wn.bias.double()[0] if wn.bias is not None else torch.zeros((), dtype=torch.float64, device=w.device)
        scale = (g * inv).float()
        tapsum = wf.reshape(C, k).double().sum(1)
        shift = ((h - g * mean * inv)[:, None] * tapsum[None, :]).float()
        outs = []
        for i in range(0, n_full, self.batch_size):
            B = min(self.batch_size, n_full - i)
            # the batch's span only: [frames, C] time-major, ~50 MB per 2,048 windows (the whole
            # file's would be ~1.8 GB per hour); hop is a multiple of the stride, so the span's
            # rows are the whole-waveform convolution's rows from window i on
            span = (B - 1) * hop + win
            G = _conv_global(w[0, i * hop:i * hop + span], wf.reshape(C, k), s)
            x1 = G.as_strided((B, L1, C), (fpw * C, C, 1), G.storage_offset())
            y1 = _lib.sincnet_stage(x1, True, norm0.weight, norm0.bias, norm0.eps, in_scale=scale[i:i + B],
                                    in_shift=shift[i:i + B])
            outs.append(self.model.head(sn.stages(y1.transpose(1, 2), 1)))
        return outs

    def __call__(self, audio) -> SlidingWindowFeature:
        wav = audio["waveform"] if isinstance(audio, dict) else audio
        wav = torch.as_tensor(wav)
        scores = self.chunk_scores(wav)
        n_chunks, K, _ = scores.shape
        fd, fs = self.model.frame_duration, self.model.frame_step
        # Inference.aggregate's grid: frames = SlidingWindow(start=chunks.start, frames' duration/step)
        starts = [closest_frame(0.0 + c * self.step + 0.5 * fd, 0.0, fd, fs) for c in range(n_chunks)]
        n_frames = closest_frame(0.0 + self.duration + (n_chunks - 1) * self.step + 0.5 * fd, 0.0, fd, fs) + 1
        data = _lib.vad_aggregate(scores, starts, n_frames, missing=math.nan)
        return SlidingWindowFeature(data[:, None], SlidingWindow(start=0.0, duration=fd, step=fs))

    def instantiate(self, hyperparameters: dict) -> "VoiceActivitySegmentation":
        """pyannote Pipeline.instantiate: keeps the binarisation hyper-parameters (onset,
        offset, min_duration_on/off), which transcribe passes to merge_chunks separately."""
        self.hyperparameters = dict(hyperparameters)
        return self


class CheckpointNotLoadable(RuntimeError):
    """The segmentation checkpoint cannot be read without executing code from it (a pickled
    Lightning checkpoint) or is not a PyanNet state_dict.  whisperx_amd.install()'s drop-in
    load_vad_model then falls back to the reference's own pyannote pipeline."""


class _Inert:
    """Stands for every global a checkpoint names outside torch's tensor-rebuild allow-list
    (Lightning / pyannote classes, hyper-parameter objects, anything else): constructing it,
    calling it, setting its state or adding items to it records nothing and runs nothing."""

    def __init__(self, *args, **kwargs):
        pass

    def __call__(self, *args, **kwargs):
        return type(self)()

    def __setstate__(self, state):
        pass

    def __setitem__(self, key, value):
        pass

    def append(self, x):
        pass

    def extend(self, xs):
        pass


def _allowed_globals() -> dict:
    """torch's own weights_only allow-list (tensor/parameter/storage rebuilds, dtypes, Size,
    OrderedDict): the globals a tensor checkpoint needs and nothing that runs code."""
    try:
        from torch._weights_only_unpickler import _get_allowed_globals

        return dict(_get_allowed_globals())
    except Exception:  # (a torch without it: the tensor rebuilds by name)
        import collections
        import torch._utils as tu

        out = {f"torch._utils.{n}": getattr(tu, n) for n in ("_rebuild_tensor", "_rebuild_tensor_v2",
                                                              "_rebuild_parameter") if hasattr(tu, n)}
        out["collections.OrderedDict"] = collections.OrderedDict
        out["torch.Size"] = torch.Size
        return out


class _NoCodeUnpickler(pickle.Unpickler):
    """find_class returns torch's tensor-rebuild globals by name and an inert stand-in
    (_Inert subclass) for every other global, so loading executes nothing from the file."""

    _ALLOWED = None

    def find_class(self, module, name):
        if _NoCodeUnpickler._ALLOWED is None:
            _NoCodeUnpickler._ALLOWED = _allowed_globals()
        obj = _NoCodeUnpickler._ALLOWED.get(f"{module}.{name}")
        if obj is not None:
            return obj
        return type(f"Inert[{module}.{name}]"[:200], (_Inert,), {})


def _nocode_load(f, **kwargs):
    return _NoCodeUnpickler(f, **kwargs).load()


_NOCODE_PICKLE = types.SimpleNamespace(__name__="whisperx_amd.nocode_pickle", Unpickler=_NoCodeUnpickler,
                                       load=_nocode_load)


def read_checkpoint_tensors(path: str) -> dict:
    """The tensors of a pickled checkpoint (e.g. pyannote's Lightning file) without executing
    anything from it: torch.load's zip/storage handling with an unpickler that allow-lists
    torch's tensor-rebuild globals and maps every other global to an inert stub.  Returns the
    'state_dict' entry when there is one (Lightning layout), else the loaded mapping; only
    tensor values are kept."""
    obj = torch.load(path, map_location="cpu", pickle_module=_NOCODE_PICKLE, weights_only=False)
    sd = obj.get("state_dict", obj) if isinstance(obj, dict) else None
    if not isinstance(sd, dict):
        raise CheckpointNotLoadable(f"{path}: no state_dict mapping in the checkpoint")
    return {k: v for k, v in sd.items() if isinstance(k, str) and torch.is_tensor(v)}


VAD_SEGMENTATION_URL = ("https://whisperx.s3.eu-west-2.amazonaws.com/model_weights/segmentation/"
                        "0b5b3216d60a2d32fc086b47ea8c67589aaeb26b7e07fcbe620d6d0b83e209ea/pytorch_model.bin")


def load_vad_model(device, vad_onset=0.500, vad_offset=0.363, use_auth_token=None, model_fp=None,
                   check_sha256: bool = True) -> VoiceActivitySegmentation:
    """vad.py:20-59 without the download: the segmentation checkpoint at `model_fp` (default:
    torch hub's whisperx-vad-segmentation.bin, where the reference caches its download) is
    checked against the SHA256 in VAD_SEGMENTATION_URL like the reference does
    (`check_sha256=False` for a checkpoint of one's own), read with
    ``torch.load(..., weights_only=True)`` or — a pickled Lightning checkpoint, which that
    refuses — read_checkpoint_tensors (torch's tensor-rebuild globals, inert stubs for every
    other global: nothing in the file is executed either way) and loaded into a PyanNet;
    returns the producer pipeline with the reference's hyper-parameters.  A file that is
    absent raises FileNotFoundError (offline: there is nothing to fetch it from); one whose
    tensors cannot be read that way, or whose keys are not PyanNet's, raises
    CheckpointNotLoadable.  Loading the real whisperX checkpoint (a pyannote/Lightning file)
    is untested here — pyannote and the file are absent — so its parity is unpinned: the
    expected layout is pyannote 3.1's PyanNet state_dict (sincnet.wav_norm1d,
    sincnet.conv1d.{0,1,2}, sincnet.norm1d.{0,1,2}, lstm.weight_ih_l{k}[_reverse] ...,
    linear.{0,1}, classifier), as ``PyanNet().state_dict()`` lists it."""
    if model_fp is None:
        model_fp = os.path.join(torch.hub._get_torch_home(), "whisperx-vad-segmentation.bin")
    if os.path.exists(model_fp) and not os.path.isfile(model_fp):
        raise RuntimeError(f"{model_fp} exists and is not a regular file")
    if not os.path.isfile(model_fp):
        raise FileNotFoundError(f"{model_fp}: no VAD segmentation checkpoint (whisperx_amd does not download; "
                                f"place the file from {VAD_SEGMENTATION_URL} there or pass model_fp)")
    if check_sha256:
        with open(model_fp, "rb") as f:
            digest = hashlib.sha256(f.read()).hexdigest()
        if digest != VAD_SEGMENTATION_URL.split("/")[-2]:
            raise RuntimeError("Model has been downloaded but the SHA256 checksum does not not match. "
                               "Please retry loading the model.")
    try:
        ckpt = torch.load(model_fp, map_location="cpu", weights_only=True)
    except Exception as e:  # a Lightning checkpoint with pickled non-tensor objects
        try:  # its tensors through the no-code unpickler (stubs for every other global)
            ckpt = read_checkpoint_tensors(model_fp)
        except Exception as e2:
            raise CheckpointNotLoadable(
                f"{model_fp}: torch.load(weights_only=True) refused the file ({str(e).splitlines()[0][:160]}) and "
                f"its tensors could not be read without executing it ({str(e2).splitlines()[0][:160]})") from e2
    try:
        model = PyanNet.from_pyannote_state_dict(ckpt)
    except (KeyError, RuntimeError, AttributeError) as e:
        raise CheckpointNotLoadable(f"{model_fp}: not a PyanNet segmentation state_dict ({e})") from e
    pipeline = VoiceActivitySegmentation(segmentation=model, device=torch.device(device))
    return pipeline.instantiate({"onset": vad_onset, "offset": vad_offset, "min_duration_on": 0.1,
                                 "min_duration_off": 0.1})
