"""One bench leg in isolation, for rocprofv3 runs (development tool): the program after
`rocprofv3 ... --` runs exactly this leg's kernel K times after W warm-ups.

    python tools/legs.py cfg2|cfg5|sat3000|trellis3000|vad1h|e2e|e2e5 [--steps K] [--warmup W]

cfg2: the headline step (64 x T=1499, V=32, wx_align_dp in the default shape);
cfg5: BASELINE config 5's DP (64 x T=2999, V=40, N~U[850,950], default shape);
e2e / e2e5: align() end to end, 16 x 30 s wav2vec2-base / 8 x 60 s large-xlsr shape (config 5);
sat3000: 2048 x T=2999, V=32, N~U[850,951], wx_align_dp (throughput shape);
trellis3000: get_trellis materialised (wx_trellis) on the sat3000 batch;
vad1h: the VAD producer (PyanNet-shaped segmentation forward + wx_vad_aggregate) over 1 h."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import torch

    from satbench import make_batch
    from whisperx_amd import _lib

    ap = argparse.ArgumentParser()
    ap.add_argument("leg")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    if a.leg == "vad1h":  # the VAD producer over 1 h of audio (warm-up: one whole hour)
        from whisperx_amd.vad_model import VoiceActivitySegmentation

        torch.manual_seed(5)
        vad = VoiceActivitySegmentation(device=dev, batch_size=int(os.environ.get("WX_VAD_BATCH", "2048")))
        wav = (torch.randn(1, 3600 * 16000, generator=torch.Generator().manual_seed(5)) * 0.1).to(dev)
        vad({"waveform": wav, "sample_rate": 16000})
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            vad({"waveform": wav, "sample_rate": 16000})
        e1.record()
        torch.cuda.synchronize()
        print(f"vad1h: {e0.elapsed_time(e1) / a.steps:.4f} ms per launch, 1 h of audio", flush=True)
        return
    if a.leg in ("e2e", "e2e5"):  # align() end to end (bench.e2e_align's / config5_leg's inputs)
        import bench

        if a.leg == "e2e":
            segs, audio, model, meta = bench.e2e_leg_inputs(dev)
        else:
            segs, audio, model, meta = bench.config5_inputs(dev)
        import whisperx_amd

        for _ in range(max(1, a.warmup)):
            whisperx_amd.align(segs, model, meta, audio, dev)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            whisperx_amd.align(segs, model, meta, audio, dev)
        e1.record()
        torch.cuda.synchronize()
        print(f"e2e: {e0.elapsed_time(e1) / a.steps:.4f} ms per launch, {len(segs)} segments", flush=True)
        from whisperx_amd import alignment

        if alignment.PHASE_TIMES:  # WX_PROFILE=1: per-phase wall time (synchronised phases)
            n = a.steps + max(1, a.warmup)
            print("phases (ms per launch): " + ", ".join(f"{k} {1000 * v / n:.2f}"
                                                        for k, v in alignment.PHASE_TIMES.items()), flush=True)
        return
    if a.leg == "cfg2":
        ems, toks = make_batch(64, 1499, 32, 300, 500, 1000, dev)
    elif a.leg == "cfg5":
        ems, toks = make_batch(64, 2999, 40, 850, 950, 55, dev)
    else:
        ems, toks = make_batch(2048, 2999, 32, 850, 951, 78, dev)
    b = _lib.Batch(ems, toks, [0] * len(ems), device=dev)
    del ems
    if a.leg == "trellis3000":
        flat, offs = _lib.trellis(b)
        offs_d = _lib._dev_i64(offs, dev)
        lib = _lib.load()

        def run():
            _lib._check(lib.wx_trellis(_lib._ptr(b.em), _lib._ptr(b.em_off_d), b.V, _lib._ptr(b.tok),
                                       _lib._ptr(b.tok_off_d), _lib._ptr(b.blank), b.S, b.max_N, _lib._ptr(flat),
                                       _lib._ptr(offs_d), _lib._stream(dev)))
    else:
        plan = _lib.AlignPlan(b)
        run = plan.run
    for _ in range(a.warmup):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        run()
    e1.record()
    torch.cuda.synchronize()
    print(f"{a.leg}: {e0.elapsed_time(e1) / a.steps:.4f} ms per launch, {b.S} segments", flush=True)


if __name__ == "__main__":
    main()
