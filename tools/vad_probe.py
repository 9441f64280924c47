"""VAD producer probe (development tool, GPU box): time 10 min of audio through
VoiceActivitySegmentation at a few batch sizes, and a torch-profiler kernel table."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from whisperx_amd.vad_model import VoiceActivitySegmentation  # noqa: E402


def main():
    torch.manual_seed(0)
    wav = (torch.randn(1, 3600 * 16000) * 0.1).cuda()
    for bs in (512, 2048, 8192):
        vad = VoiceActivitySegmentation(device="cuda:0", batch_size=bs)
        vad({"waveform": wav[:, : 60 * 16000]})
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        vad({"waveform": wav})
        torch.cuda.synchronize()
        print(f"batch {bs}: {1000 * (time.perf_counter() - t0):.1f} ms for 3600 s", flush=True)
    from torch.profiler import ProfilerActivity, profile
    vad = VoiceActivitySegmentation(device="cuda:0", batch_size=128)
    vad({"waveform": wav[:, : 60 * 16000]})
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        vad({"waveform": wav})
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=22), flush=True)


if __name__ == "__main__":
    main()
