"""Producer timing per call in one process (development tool): the VAD producer over 1 h three
times, with the convolutions through MIOpen (WX_MIOPEN_CONV=1) or conv1d_batched (default).

    python tools/vad_probe2.py [pre]   (pre: run the three convolutions through MIOpen first)"""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
dev = torch.device("cuda", 0)
tag = sys.argv[1] if len(sys.argv) > 1 else "nopre"
if tag == "pre":
    with torch.inference_mode():
        for shp, w in (((2048, 1, 80000), (80, 1, 251)), ((2048, 80, 2658), (60, 80, 5)), ((2048, 60, 884), (60, 60, 5))):
            F.conv1d(torch.randn(*shp, device=dev), torch.randn(*w, device=dev), stride=10 if shp[1] == 1 else 1)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
from whisperx_amd.vad_model import VoiceActivitySegmentation  # noqa: E402

torch.manual_seed(5)
vad = VoiceActivitySegmentation(device=dev, batch_size=2048)
wav = (torch.randn(1, 3600 * 16000, generator=torch.Generator().manual_seed(5)) * 0.1).to(dev)
for i in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    vad({"waveform": wav, "sample_rate": 16000})
    torch.cuda.synchronize()
    print(tag, os.environ.get("WX_MIOPEN_CONV", "gemm"), i, round(1000 * (time.perf_counter() - t0), 1), "ms", flush=True)
