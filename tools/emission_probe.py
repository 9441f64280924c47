"""Emission-producer probe (development tool, GPU box): wav2vec2-base forward time per *new*
input length with MIOpen convolutions vs the GEMM route (whisperx_amd.emission), the
steady-state split by kernel, and the GPU-vs-CPU log-prob difference."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import whisperx_amd  # noqa: F401  (MIOPEN_FIND_MODE=FAST default)
from whisperx_amd import emission


def fwd(model, x):
    with torch.inference_mode():
        return torch.log_softmax(model(x).logits, -1)


def timed(model, x):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    y = fwd(model, x)
    torch.cuda.synchronize()
    return 1000 * (time.perf_counter() - t0), y


def main():
    from transformers import Wav2Vec2Config, Wav2Vec2ForCTC

    torch.manual_seed(0)
    dev = "cuda:0"
    model = Wav2Vec2ForCTC(Wav2Vec2Config(vocab_size=32)).eval()
    gm = model.to(dev)
    rng = np.random.default_rng(0)
    base = torch.from_numpy(rng.standard_normal(31 * 16000).astype(np.float32) * 0.1)
    x30 = base[: 30 * 16000][None].to(dev)
    fwd(gm, x30)
    torch.cuda.synchronize()
    res = {}
    for name, lens in (("miopen", [5.13, 9.71, 12.37, 17.05, 21.9, 26.41, 29.33, 14.2]),
                       ("gemm", [5.17, 9.73, 12.39, 17.07, 21.93, 26.43, 29.35, 14.23]),
                       ("gemm+eager", [5.19, 9.75, 12.41, 17.09, 21.95, 26.45, 29.37, 14.25])):
        if name == "gemm":
            emission.prepare_model(gm)
        if name == "gemm+eager":
            try:
                gm.set_attn_implementation("eager")
            except Exception as e:  # older transformers
                print("set_attn_implementation failed", repr(e))
                gm.config._attn_implementation = "eager"
            print("attn:", gm.config._attn_implementation, flush=True)
        first, second = [], []
        for sec in lens:
            x = base[: int(sec * 16000)][None].to(dev)
            a, _ = timed(gm, x)
            b, _ = timed(gm, x)
            first.append(a)
            second.append(b)
        t30 = [timed(gm, x30)[0] for _ in range(5)]
        res[name] = {"first_ms": [round(v, 1) for v in first], "again_ms": [round(v, 1) for v in second],
                     "fixed30_ms": round(min(t30), 2)}
        print(name, res[name], flush=True)
    # GEMM route vs MIOpen on the same input, and vs CPU
    y_e = fwd(gm, x30).float().cpu()
    try:
        gm.set_attn_implementation("sdpa")
    except Exception:
        gm.config._attn_implementation = "sdpa"
    y_g = fwd(gm, x30).float().cpu()
    d = (y_e - y_g).abs()
    print("eager-vs-sdpa max", float(d.max()), flush=True)
    emission.restore_model(gm)
    y_m = fwd(gm, x30).float().cpu()
    y_c = fwd(model.cpu(), x30.cpu())
    for a, b, lab in ((y_g, y_m, "gemm-vs-miopen"), (y_g, y_c, "gemm-vs-cpu"), (y_m, y_c, "miopen-vs-cpu")):
        d = (a - b).abs()
        print(lab, "max", float(d.max()), "mean", float(d.mean()),
              "argmax agree", float((a.argmax(-1) == b.argmax(-1)).float().mean()), flush=True)
    model.to(dev)
    emission.prepare_model(model)
    try:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for _ in range(3):
                fwd(model, x30)
            torch.cuda.synchronize()
        print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25), flush=True)
    except Exception as e:
        print("profiler failed", repr(e))


if __name__ == "__main__":
    main()
