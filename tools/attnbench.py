"""Development tool: time wx_attention_f32 on a 30 s wav2vec2 segment's shape (B=1, H=12/16,
T=1499, head dim 64), alone and on 8 concurrent streams, for each library given."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def run(H, streams, iters=50):
    import whisperx_amd._lib as L
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    qkv = [torch.randn(1, 1499, H, 64, generator=g).to(dev).transpose(1, 2) for _ in range(3)]
    if os.environ.get("ATTN_LAYOUT") == "contig":  # [B, H, T, 64] storage: row stride 256 B
        qkv = [t.contiguous() for t in qkv]
    ref = torch.nn.functional.scaled_dot_product_attention(*qkv, scale=0.125).transpose(1, 2)
    out = L.attention_f32(*qkv, 0.125)
    err = (out - ref).abs().max().item()
    sts = [torch.cuda.Stream(device=dev) for _ in range(streams)]
    for _ in range(30):
        L.attention_f32(*qkv, 0.125)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(iters):
        for st in sts:
            with torch.cuda.stream(st):
                L.attention_f32(*qkv, 0.125)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / (iters * streams)
    fl = 4 * H * 1499 * 1499 * 64
    return dt, fl / dt / 1e12, err


def run_packed(H, nseg, split, iters=20):
    """wx_attention_f32_packed on the packed encoder's layout: nseg segments of 1499 rows in one
    fused [1, R, 3 H 64] q/k/v projection (views), one launch."""
    import whisperx_amd._lib as L
    dev = torch.device("cuda", 0)
    segs = L.PackedSegments([1499] * nseg)
    R = segs.rows
    qkv = torch.randn(1, R, 3 * H * 64, device=dev)
    q, k, v = (qkv[..., i * H * 64:(i + 1) * H * 64].view(1, R, H, 64).transpose(1, 2) for i in range(3))
    for _ in range(5):
        L.attention_f32_packed(q, k, v, 0.125, segs, split)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        L.attention_f32_packed(q, k, v, 0.125, segs, split)
    e1.record()
    torch.cuda.synchronize()
    dt = e0.elapsed_time(e1) / 1e3 / iters
    fl = 4 * H * 1499 * 1499 * 64 * nseg
    return dt, fl / dt / 1e12


if __name__ == "__main__":
    if os.environ.get("ATTN_PACKED"):  # ATTN_PACKED=12 python tools/attnbench.py: packed launches, this library
        n = int(os.environ["ATTN_PACKED"])
        run_packed(12, n, 0)
        for sp in (1, 2, 4):
            dt, tf = run_packed(12, n, sp)
            print(f"packed H=12 segments={n} split={sp}: {dt*1e6:8.1f} us/call {tf:6.1f} TFLOP/s", flush=True)
        sys.exit(0)
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if not a.child:  # one subprocess per build: the library path is fixed at import
        import subprocess
        for lib in a.libs.split(","):
            env = dict(os.environ, WX_LIB_PATH=os.path.abspath(lib))
            subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--libs", lib], env=env, check=True)
        sys.exit(0)
    lib = a.libs
    run(12, 1, iters=200)  # the first shape timed in a process runs ~2x slow (clocks ramping)
    for H in (int(x) for x in os.environ.get("ATTN_HS", "12,16").split(",")):
        for ns in (1, 8):
            dt, tf, err = run(H, ns)
            print(f"{os.path.basename(lib):14s} H={H} streams={ns}: {dt*1e6:7.1f} us/call {tf:6.1f} TFLOP/s maxerr {err:.2e}", flush=True)
