"""VAD producer convolution probe (development tool): times SincNet's three convolutions at a
2,048-window batch through MIOpen under several solver settings, and the whole producer over
1 h in steady state.  (Round 3, MI355X: sinc 15.5 ms, conv2 5.3 ms, conv3 1.8 ms per batch under
every setting; batched-GEMM forms of the same convolutions measured 14.4 / 7.9 / 2.8 ms and were
dropped; producer 199 ms per hour.)  Each MIOpen setting runs in its own process
(MIOpen reads its environment once).

    python tools/vad_conv_probe.py"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(tag):
    import torch
    import torch.nn.functional as F

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    B = 2048
    x0 = torch.randn(B, 1, 80000, device=dev)
    w0 = torch.randn(80, 1, 251, device=dev) * 0.05
    x1 = torch.randn(B, 80, 2658, device=dev)
    w1 = torch.randn(60, 80, 5, device=dev) * 0.05
    b1 = torch.randn(60, device=dev)
    x2 = torch.randn(B, 60, 884, device=dev)
    w2 = torch.randn(60, 60, 5, device=dev) * 0.05
    b2 = torch.randn(60, device=dev)

    def timeit(fn, n=3):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return 1000 * (time.perf_counter() - t0) / n

    out = {}
    with torch.inference_mode():
        out["sinc_miopen_ms"] = timeit(lambda: F.conv1d(x0, w0, stride=10))
        out["conv2_miopen_ms"] = timeit(lambda: F.conv1d(x1, w1, b1))
        out["conv3_miopen_ms"] = timeit(lambda: F.conv1d(x2, w2, b2))
        del x0, x1, x2
        torch.cuda.empty_cache()
    if True:  # (the model is built outside inference_mode: its parameters must be normal tensors)
        from whisperx_amd.vad_model import VoiceActivitySegmentation

        torch.manual_seed(5)
        vad = VoiceActivitySegmentation(device=dev, batch_size=2048)
        wav = (torch.randn(1, 3600 * 16000, generator=torch.Generator().manual_seed(5)) * 0.1).to(dev)
        out["producer_1h_ms"] = timeit(lambda: vad({"waveform": wav, "sample_rate": 16000}), n=2)
    print("RESULT " + json.dumps(out), flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    variants = {"default": {}, "no_gemm_solver": {"MIOPEN_DEBUG_CONV_GEMM": "0"},
                "find_normal": {"MIOPEN_FIND_MODE": "NORMAL"}}
    for tag, env in variants.items():
        e = dict(os.environ, **env)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", tag], env=e, capture_output=True,
                           text=True, timeout=500)
        line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")]
        print(tag, line[0][7:] if line else f"FAILED rc={r.returncode} {r.stderr[-1500:]}", flush=True)


if __name__ == "__main__":
    main()
