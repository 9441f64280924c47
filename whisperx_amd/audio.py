"""Audio constants and loader used by align() (whisperx/audio.py:13, :25-65).

Only what the alignment path needs: SAMPLE_RATE and load_audio() (ffmpeg decode to 16 kHz
mono float32 in a subprocess — the same process boundary as the reference)."""
from __future__ import annotations

import subprocess

import numpy as np

SAMPLE_RATE = 16000


def load_audio(file: str, sr: int = SAMPLE_RATE) -> np.ndarray:
    try:
        cmd = ["ffmpeg", "-nostdin", "-threads", "0", "-i", file, "-f", "s16le", "-ac", "1",
               "-acodec", "pcm_s16le", "-ar", str(sr), "-"]
        out = subprocess.run(cmd, capture_output=True, check=True).stdout
    except FileNotFoundError as e:
        raise RuntimeError("ffmpeg is required to decode audio files; pass a waveform array instead") from e
    except subprocess.CalledProcessError as e:
        raise RuntimeError(f"Failed to load audio: {e.stderr.decode()}") from e
    return np.frombuffer(out, np.int16).flatten().astype(np.float32) / 32768.0
