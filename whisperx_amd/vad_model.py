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

The whisperX VAD checkpoint (``VAD_SEGMENTATION_URL``) cannot be fetched offline: ``PyanNet``
builds the architecture with random weights, which is what the benchmarks time; a state_dict
loads with ``load_state_dict`` (read the file with ``torch.load(..., weights_only=True)``).  Parity of the aggregation is pinned to a restatement of pyannote's
published algorithm (oracle.vad_aggregate), not to pyannote itself, which is absent:
"parity unpinned" at the pyannote boundary.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib
from .vad import SlidingWindow, SlidingWindowFeature

SAMPLE_RATE = 16000


class PyanNet(torch.nn.Module):
    """pyannote/segmentation's PyanNet shape (pyannote.audio PyanNet / SincNet defaults):
    waveform InstanceNorm -> [conv(1->80, k=251, s=10) |abs|, conv(80->60, k=5),
    conv(60->60, k=5)] each followed by MaxPool(3) -> InstanceNorm -> LeakyReLU -> BiLSTM(128, 2
    layers) -> 2 x (Linear(128) + LeakyReLU) -> Linear(n_classes) -> sigmoid.  The first conv
    is a plain Conv1d here (SincNet's band-pass parametrisation only shapes its weights).
    Output: [batch, frames, n_classes]; 293 frames per 5 s window (270-sample step)."""

    def __init__(self, n_classes: int = 3, lstm_hidden: int = 128, lstm_layers: int = 2, linear_hidden: int = 128):
        super().__init__()
        self.wav_norm = torch.nn.InstanceNorm1d(1, affine=True)
        self.conv = torch.nn.ModuleList([torch.nn.Conv1d(1, 80, 251, stride=10), torch.nn.Conv1d(80, 60, 5),
                                         torch.nn.Conv1d(60, 60, 5)])
        self.pool = torch.nn.MaxPool1d(3, stride=3)
        self.norm = torch.nn.ModuleList([torch.nn.InstanceNorm1d(80, affine=True), torch.nn.InstanceNorm1d(60, affine=True),
                                         torch.nn.InstanceNorm1d(60, affine=True)])
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
        x = self.wav_norm(waveforms)
        for i, (conv, norm) in enumerate(zip(self.conv, self.norm)):
            x = conv(x)
            if i == 0:
                x = torch.abs(x)
            x = F.leaky_relu(norm(self.pool(x)))
        x, _ = self.lstm(x.transpose(1, 2))
        for lin in self.linear:
            x = F.leaky_relu(lin(x))
        return torch.sigmoid(self.classifier(x))


def closest_frame(t: float, start: float, duration: float, step: float) -> int:
    """pyannote SlidingWindow.closest_frame: int(rint((t - start - duration / 2) / step))."""
    return int(round((t - start - 0.5 * duration) / step))  # Python round == numpy rint (half to even)


class VoiceActivitySegmentation:
    """vad.py:198-240: speech scores of a waveform as a SlidingWindowFeature [frames, 1] whose
    data stays a device tensor.  ``duration``/``step`` are the sliding windows (5 s / 0.5 s),
    ``batch_size`` the windows per model forward.  pyannote's default is 32; the forward is
    host-bound at that size (MIOpen's LSTM costs ~25 ms of host time per call), so the
    default here is 1024 windows (~2.6 GB of activations; 1 h: 2.2 s at 128, 1.15 s at 2048 on
    MI355X; MIOpen's LSTM rejects batches of ~7,000)."""

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
            if n_full:
                chunks = w.unfold(1, win, hop)[0]  # [n_full, win] (a view)
                for i in range(0, n_full, self.batch_size):
                    outs.append(self.model(chunks[i:i + self.batch_size].unsqueeze(1).contiguous()))
            if has_last:
                last = w[:, n_full * hop:]
                last = F.pad(last, (0, win - last.shape[1]))
                outs.append(self.model(last.unsqueeze(1)))
        return torch.cat(outs, 0)

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
