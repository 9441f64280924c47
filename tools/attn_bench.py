"""wx_attention_f32 vs torch's fp32 SDPA (development tool): per-call time at wav2vec2 shapes.

    python tools/attn_bench.py"""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from whisperx_amd import _lib  # noqa: E402


def timeit(fn, n=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / n


for B, H, T in ((1, 12, 1499), (1, 12, 1450), (1, 16, 2999), (8, 12, 1499)):
    proj = [torch.randn(B, T, H * 64, device="cuda") for _ in range(3)]
    q, k, v = (p.view(B, T, H, 64).transpose(1, 2) for p in proj)
    with torch.inference_mode():
        t_wx = timeit(lambda: _lib.attention_f32(q, k, v, 0.125))
        t_sdpa = timeit(lambda: F.scaled_dot_product_attention(q, k, v, scale=0.125))
    fl = 4.0 * B * H * T * T * 64
    print(f"B={B} H={H} T={T}: wx {t_wx:8.1f} us ({fl / t_wx / 1e6:6.1f} TF/s)   sdpa {t_sdpa:8.1f} us "
          f"({fl / t_sdpa / 1e6:6.1f} TF/s)", flush=True)
