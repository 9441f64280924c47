#!/usr/bin/env python
"""bench.py — throughput of the MI355X forced-alignment DP (BASELINE.json metric
"aligned audio-sec/s + word-boundary MAE(ms) vs ref, 1/2/4/8 GPU").

Workload (BASELINE.json configs[1]): one step = the fused HIP alignment DP
(libwxalign.so wx_align_dp: trellis recurrence + decision bits + argmax + backtrack +
merge_repeats) over a batch of 64 synthetic 30 s English segments — T=1499 emission
frames, V=32 (wav2vec2-base-960h vocabulary), N~U[300,500] characters — with the
log-probability emissions already resident in HBM.  Multi-GPU: one process per GPU,
each aligning its own batch (per-file data parallel, weak scaling); the character
vocabulary is broadcast over RCCL at start-up; no collective on the data path.

Reported beside the value (rank 0):
  roofline      dominant kernel's algorithmic HBM bytes / time vs 8 TB/s
  cpu_baseline  the reference algorithm with its per-timestep torch-CPU op structure
                (oracle TorchPort, 1 thread) on a bounded sample of the same batch
  mae_ms        word/char-boundary MAE of the GPU result vs the CPU oracle (same emission)
  extra         C-oracle throughput, saturated-batch roofline, end-to-end align()

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu] [--no-e2e] [--no-scale]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from whisperx_amd.synthetic import W2V_VOCAB  # noqa: E402  (no GPU touched at import)
FRAME_S = 0.02  # wav2vec2 frame hop (320 samples at 16 kHz)
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
STEP_CYCLES = 20  # one register-resident DP step: 5 dependent-chain VALU instructions x 4 cycles (wave64)
ENGINE_PEAK_GHZ = 2.4  # MI355X peak engine clock (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_batch(rng, n_seg, T, V, n_lo, n_hi, device):
    """Peaky CTC emissions: N(0,1) logits, +6 on blank, +12 at N sorted
    frames for tokens in [1,V), fp32 log_softmax.  Returns (emissions on device, tokens)."""
    ems, toks = [], []
    for _ in range(n_seg):
        N = int(rng.integers(n_lo, n_hi + 1))
        logits = rng.standard_normal((T, V)).astype(np.float32)
        logits[:, 0] += 6.0
        tk = rng.integers(1, V, N)
        fr = np.sort(rng.choice(np.arange(1, T - 1), N, replace=False))
        logits[fr, tk] += 12.0
        em = torch.log_softmax(torch.from_numpy(logits).to(device), -1)
        ems.append(em.contiguous())
        toks.append(tk.tolist())
    return ems, toks


def algorithmic_bytes(Ts, Ns, V):
    """Per segment: emission read 4TV + tokens 4N + decision bits T*N/8 + outputs 16N."""
    return int(sum(4 * T * V + 4 * N + (T * N) // 8 + 16 * N for T, N in zip(Ts, Ns)))


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/r*_pmc_traffic.json: separate FETCH_SIZE / WRITE_SIZE passes over this same
    command, gfx950 FETCH_SIZE correction applied) — or None when none matches."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r*_pmc_traffic*.json")))
    for f in reversed(files):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("kernel") == kernel:
            return int(d["traffic_bytes_per_launch"]), os.path.basename(f)
    return None, None


def time_steps(plan, steps, warmup, dist_on):
    """W untimed warm-up steps, then exactly K steps between two barriers + synchronize; the
    device time comes from one event pair around the K steps (no per-step event commands
    between the launches).  A separate, untimed pass with an event pair around every launch
    gives the kernel's mean duration for the roofline (time_steps.last_launch_s)."""
    for _ in range(warmup):
        plan.run()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    # per-launch kernel time (roofline leg): events on the stream the kernel runs on
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(min(steps, 20))]
    for a, b in ev:
        a.record(stream)
        plan.run()
        b.record(stream)
    torch.cuda.synchronize()
    time_steps.last_launch_s = float(np.mean([a.elapsed_time(b) / 1000.0 for a, b in ev]))
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        plan.run()
    e1.record(stream)
    torch.cuda.synchronize()
    if dist_on:
        torch.distributed.barrier()
    host_s = time.perf_counter() - t0
    dev_s = e0.elapsed_time(e1) / 1000.0
    return host_s, dev_s


def cpu_port_baseline(ems_cpu, toks, budget_s=15.0):
    """Reference-structured torch-CPU port (oracle.TorchPort), 1 thread, bounded sample."""
    from oracle.oracle import TorchPort

    torch.set_num_threads(1)
    port = TorchPort()
    done, audio, t_used = 0, 0.0, 0.0
    for em, tk in zip(ems_cpu, toks):
        t0 = time.perf_counter()
        port.align_dp(em, tk, 0)
        t_used += time.perf_counter() - t0
        done += 1
        audio += em.shape[0] * FRAME_S
        if t_used >= budget_s:
            break
    return {"value": audio / t_used, "unit": "audio-sec/s", "cores": 1, "kind": "port",
            "sample": f"{done} of the batch's 30 s segments (T=1499, V=32), torch-CPU port of "
                      f"alignment.py:359-454, 1 thread, {t_used:.1f} s"}


def c_oracle_baseline(ems_np, toks):
    from oracle import oracle

    t0 = time.perf_counter()
    for em, tk in zip(ems_np, toks):
        oracle.align_dp(em, tk, 0)
    dt = time.perf_counter() - t0
    return {"value": sum(e.shape[0] for e in ems_np) * FRAME_S / dt, "unit": "audio-sec/s", "cores": 1,
            "kind": "port", "sample": f"{len(ems_np)} segments, C restatement (oracle/wx_oracle.c), 1 thread"}


def mae_vs_oracle(ems_np, toks, plan):
    """Char-boundary MAE (ms) of the GPU DP vs the CPU oracle on the same emissions."""
    from oracle import oracle

    ss, se, sc, ts, st = (x.cpu().numpy() for x in (plan.seg_start, plan.seg_end, plan.seg_score,
                                                       plan.t_start, plan.status))
    errs, n_tok, n_bad_path = [], 0, 0
    for i, (em, tk) in enumerate(zip(ems_np, toks)):
        ok, tso, sso, seo, sco = oracle.align_dp(em, tk, 0)
        a, b = plan.b.tok_off[i], plan.b.tok_off[i + 1]
        if not ok or (st[i] & 15) != 0:
            n_bad_path += int(ok != ((st[i] & 15) == 0))
            continue
        ratio_ms = 1000.0 * FRAME_S
        errs.append(np.abs(ss[a:b] - sso) * ratio_ms)
        errs.append(np.abs(se[a:b] - seo) * ratio_ms)
        n_tok += b - a
        n_bad_path += int(not (np.array_equal(ss[a:b], sso) and np.array_equal(se[a:b], seo)))
    mae = float(np.concatenate(errs).mean()) if errs else 0.0
    return mae, n_tok, n_bad_path


def e2e_leg_inputs(device, n_seg=16, seed=7):
    """e2e_align's inputs: (segments, audio, random-weight wav2vec2-base, align metadata)."""
    from transformers import Wav2Vec2Config, Wav2Vec2ForCTC

    torch.manual_seed(seed)
    model = Wav2Vec2ForCTC(Wav2Vec2Config(vocab_size=32)).to(device).eval()
    dictionary = {c.lower(): i for i, c in enumerate(W2V_VOCAB)}
    meta = {"language": "en", "dictionary": dictionary, "type": "huggingface"}
    rng = np.random.default_rng(seed)
    letters = "etaoinshrdlucmfwypvbgkqjxz"
    segs = []
    for k in range(n_seg):
        words = ["".join(rng.choice(list(letters), int(rng.integers(2, 9)))) for _ in range(70)]
        segs.append({"start": 30.0 * k, "end": 30.0 * (k + 1), "text": " ".join(words)})
    audio = torch.from_numpy(rng.standard_normal(int(30 * n_seg * 16000)).astype(np.float32) * 0.1)
    return segs, audio, model, meta


def e2e_align(device, n_seg=16, seed=7, reps=3):
    """End-to-end align() on the GPU: random-weight wav2vec2-base (same architecture as
    WAV2VEC2_ASR_BASE_960H) + fused DP + host aggregation, 30 s segments of synthetic
    audio with ~14 chars/s transcripts."""
    import whisperx_amd

    segs, audio, model, meta = e2e_leg_inputs(device, n_seg, seed)
    # warm-up: the timed call itself, once (its pack shapes' GEMM heuristics, allocations);
    # a 2-segment warm-up left the first 16-segment call ~8% slow (driver round 5: 78.7 ms)
    whisperx_amd.align([dict(s) for s in segs], model, meta, audio, device)
    torch.cuda.synchronize()
    st0 = _dp_stats()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = whisperx_amd.align([dict(s) for s in segs], model, meta, audio, device)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    dt = float(np.median(ts))
    n_words = len(out["word_segments"])
    return {"value": 30.0 * n_seg / dt, "unit": "audio-sec/s", "segments": n_seg, "words": n_words,
            "ms_per_segment": 1000 * dt / n_seg, "calls_ms": [1000 * t for t in ts],
            "timing": f"median of {reps} calls after one untimed warm-up call of the same segments",
            "dp": _recovered_since(st0),
            "note": "align() incl. random-weight wav2vec2-base fp32 forward on the GPU: the packed encoder "
                    "(segments stacked by rows through one transformer pass, per-segment attention and "
                    "positional conv), fused DP, host aggregation overlapped with the forwards"}


def e2e_config3(device, seed=3):
    """BASELINE config 3 shape: 1 h of audio, VAD scores (smoothed noise -> sigmoid, 16.875 ms
    frames) -> GPU Binarize + merge_chunks(30 s) -> ~120 chunks -> align()
    (random-weight wav2vec2-base fp32 forward per chunk, fused DP, host aggregation).
    Synthetic audio and transcripts (~14 chars/s): timings only."""
    from transformers import Wav2Vec2Config, Wav2Vec2ForCTC

    import whisperx_amd
    from whisperx_amd.vad import SlidingWindow, SlidingWindowFeature, merge_chunks

    rng = np.random.default_rng(seed)
    F = 213_333
    x = rng.standard_normal(F + 40)
    y = np.convolve(x, np.ones(40) / 40, mode="valid")[:F] * 4 * np.sqrt(40) / 3
    scores = SlidingWindowFeature((1 / (1 + np.exp(-y))).astype(np.float32)[:, None],
                                  SlidingWindow(start=0.0, duration=0.0619375, step=0.016875))
    torch.manual_seed(seed)
    model = Wav2Vec2ForCTC(Wav2Vec2Config(vocab_size=32)).to(device).eval()
    dictionary = {c.lower(): i for i, c in enumerate(W2V_VOCAB)}
    meta = {"language": "en", "dictionary": dictionary, "type": "huggingface"}
    audio = torch.from_numpy(rng.standard_normal(3600 * 16000).astype(np.float32) * 0.1)
    letters = "etaoinshrdlucmfwypvbgkqjxz"
    merge_chunks(scores, 30, 0.5, 0.363)  # warm-up
    whisperx_amd.align([{"start": 0.0, "end": 30.0, "text": "warm up"}], model, meta, audio, device)
    torch.cuda.synchronize()
    vad_s = []
    for _ in range(3):
        t0 = time.perf_counter()
        chunks = merge_chunks(scores, 30, 0.5, 0.363)
        vad_s.append(time.perf_counter() - t0)
    t0, t1 = 0.0, min(vad_s)
    segs = []
    for c in chunks:
        n_words = max(1, int((c["end"] - c["start"]) * 14 / 5.5))
        words = ["".join(rng.choice(list(letters), int(rng.integers(2, 9)))) for _ in range(n_words)]
        segs.append({"start": round(c["start"], 3), "end": round(c["end"], 3), "text": " ".join(words)})
    st0 = _dp_stats()
    t2 = time.perf_counter()
    out = whisperx_amd.align(segs, model, meta, audio, device)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    speech = sum(c["end"] - c["start"] for c in chunks)
    return {"audio_sec": 3600.0, "chunks": len(chunks), "speech_sec": speech, "dp": _recovered_since(st0),
            "vad_merge_chunks_ms": 1000 * (t1 - t0), "align_ms": 1000 * (t3 - t2),
            "audio_sec_per_s": 3600.0 / ((t1 - t0) + (t3 - t2)),
            "words": len(out["word_segments"]),
            "note": "merge_chunks (GPU Binarize) + align() incl. per-chunk wav2vec2-base fp32 forward; "
                    "synthetic scores/audio/transcripts"}


def _smooth_vad_scores(seed, F=213_333):
    """Config 3's synthetic VAD scores: smoothed noise through a sigmoid (~2 regions/min)."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(F + 40)
    y = np.convolve(x, np.ones(40) / 40, mode="valid")[:F] * 4 * np.sqrt(40) / 3
    return (1 / (1 + np.exp(-y))).astype(np.float32)


def binarize_1h(device, reps=20):
    """Binarize on 1 h of scores (213,333 frames), the device-side call of merge_chunks:
    smooth config-3 scores and dense ones (uniform noise thresholded at its median: an event
    every ~2 frames, the random-weight producer's case), both kernels.  ms = HIP events
    around _lib.binarize on device-resident scores (pre-pass + state machine + region
    count read-back), best of reps; merge_chunks_dense_ms = the whole host call."""
    from whisperx_amd import _lib
    from whisperx_amd.vad import SlidingWindow, SlidingWindowFeature, merge_chunks

    geom = [(0.0, 0.016875, 0.0619375)]
    dense = np.random.default_rng(8).random(213_333).astype(np.float32)
    med = float(np.median(dense))
    cases = {"smooth": (_smooth_vad_scores(3), 0.5, 0.363), "dense": (dense, med, med)}
    out = {}
    for name, (y, on, off) in cases.items():
        yd = torch.from_numpy(y).to(device)
        for tp in (True, False):
            ts = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                (rs, _re), = _lib.binarize([yd], geom, on, off, 30.0, device=device, two_pass=tp)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            out[f"{name}_{'two' if tp else 'one'}_pass_ms"] = min(ts)
        out[f"{name}_regions"] = int(len(rs))
    feat = SlidingWindowFeature(torch.from_numpy(dense)[:, None].to(device), SlidingWindow(0.0, 0.016875, 0.0619375))
    ws = []
    for _ in range(3):
        t0 = time.perf_counter()
        chunks = merge_chunks(feat, 30, med, med)
        ws.append(time.perf_counter() - t0)
    out["merge_chunks_dense_ms"] = 1000 * min(ws)
    out["merge_chunks_dense_chunks"] = len(chunks)
    out["note"] = "1 h = 213,333 frames of 16.875 ms; max_duration 30 s"
    return out


def vad_producer_1h(device, seed=5, batch_size=2048):
    """VAD producer (vad.py:198-240) on 1 h of audio: 7,191 five-second windows every 0.5 s
    through the random-weight PyanNet-shaped segmentation model (batched) and the overlap-add
    HIP kernel.  Timing only (random weights: merge_chunks over these scores is exercised by
    tests/test_vad_producer.py; the config-3 leg binarises smooth synthetic scores)."""
    from whisperx_amd.vad_model import VoiceActivitySegmentation

    torch.manual_seed(seed)
    vad = VoiceActivitySegmentation(device=device, batch_size=batch_size)
    g = torch.Generator().manual_seed(seed)
    wav = torch.randn(1, 3600 * 16000, generator=g) * 0.1
    wav_d = wav.to(device)
    # warm-up over the whole hour: every batch shape of the timed call (2,048 windows and the
    # last partial batch) has been seen by MIOpen's LSTM / conv solvers before the clock starts
    vad({"waveform": wav_d, "sample_rate": 16000})
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    feat = vad({"waveform": wav_d, "sample_rate": 16000})
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    n_win = sum(vad.windows(wav.shape[1]))
    return {"audio_sec": 3600.0, "windows": int(n_win), "frames": int(feat.data.shape[0]),
            "producer_ms": 1000 * (t1 - t0), "audio_sec_per_s": 3600.0 / (t1 - t0), "batch_size": batch_size,
            "note": "PyanNet-shaped random-weight segmentation forward (fp32, 5 s windows every 0.5 s) + "
                    "wx_vad_aggregate; scores left on the device for merge_chunks; audio resident on the GPU"}


def e2e_config3_waveform(device, seed=6):
    """BASELINE config 3 from the waveform: 1 h of audio -> VAD producer (PyanNet-shaped
    random-weight segmentation model + wx_vad_aggregate, vad.py:198-240) -> merge_chunks on the
    device-resident scores (GPU Binarize, 30 s, asr.py:186-192) -> chunk bounds rounded
    (asr.py:226-232) -> align() (random-weight wav2vec2-base forward per chunk + fused DP).
    A random-weight segmentation model's scores hover around one value, so the hysteresis
    thresholds are put at their median (onset = offset) to get a realistic number of chunks;
    timings only.  The synthetic transcripts are made outside the clock."""
    import whisperx_amd
    from whisperx_amd import synthetic
    from whisperx_amd.vad import merge_chunks
    from whisperx_amd.vad_model import VoiceActivitySegmentation

    torch.manual_seed(seed)
    vad = VoiceActivitySegmentation(device=device, batch_size=2048)
    model = _w2v_base(device, seed)
    meta = {"language": "en", "dictionary": synthetic.w2v_dictionary(), "type": "huggingface"}
    g = torch.Generator().manual_seed(seed)
    wav = (torch.randn(1, 3600 * 16000, generator=g) * 0.1).to(device)
    tr = synthetic.Transcriber(seed)
    # warm-up outside the clock: producer (MIOpen, LSTM: every batch shape of the hour), Binarize, align
    vad({"waveform": wav, "sample_rate": 16000})
    feat = vad({"waveform": wav[:, : 120 * 16000], "sample_rate": 16000})
    thr = float(torch.nanmedian(feat.data).item())
    merge_chunks(feat, 30, thr, thr)
    whisperx_amd.align(tr.segments([{"start": 0.0, "end": 30.0}]), model, meta, wav[0, : 60 * 16000], device)
    torch.cuda.synchronize()
    st0 = _dp_stats()
    t0 = time.perf_counter()
    feat = vad({"waveform": wav, "sample_rate": 16000})
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    chunks = merge_chunks(feat, 30, thr, thr)
    t2 = time.perf_counter()
    segs = tr.segments(chunks)
    t3 = time.perf_counter()
    out = whisperx_amd.align(segs, model, meta, wav[0], device)
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    wall = (t1 - t0) + (t2 - t1) + (t4 - t3)
    return {"audio_sec": 3600.0, "chunks": len(chunks), "producer_ms": 1000 * (t1 - t0),
            "merge_chunks_ms": 1000 * (t2 - t1), "align_ms": 1000 * (t4 - t3), "audio_sec_per_s": 3600.0 / wall,
            "words": len(out["word_segments"]), "dp": _recovered_since(st0), "threshold": thr,
            "note": "waveform -> VAD producer -> GPU merge_chunks -> align() incl. per-chunk wav2vec2-base fp32 "
                    "forward; random weights (thresholds at the scores' median), synthetic audio/transcripts"}


def _w2v_base(device, seed):
    """Random-weight wav2vec2-base (WAV2VEC2_ASR_BASE_960H's architecture, V=32): there are
    no checkpoints offline, and the forward's cost does not depend on the weights."""
    from transformers import Wav2Vec2Config, Wav2Vec2ForCTC

    torch.manual_seed(seed)
    return Wav2Vec2ForCTC(Wav2Vec2Config(vocab_size=32)).to(device).eval()


def corpus_config4(device, rank, world, dist_on, seed=4):
    """BASELINE config 4: a 10 h corpus of 40 files (log-uniform 1-60 min), sharded over the
    ranks longest-first (distributed.shard_files); per file, as transcribe.py:172-205 runs it
    one file after another: VAD scores -> merge_chunks (GPU Binarize, 30 s chunks,
    asr.py:187) -> segments rounded to 3 dp (asr.py:226-232) -> align() with the random-weight
    wav2vec2-base forward per chunk and the fused DP.  Inputs (scores, audio, transcripts) are
    synthetic and resident before the clock starts; the clock covers merge_chunks + align()
    for every file of every rank (barrier, max over ranks)."""
    import whisperx_amd
    from whisperx_amd import synthetic
    from whisperx_amd.distributed import shard_files
    from whisperx_amd.vad import merge_chunks

    durs = synthetic.corpus_durations(seed)
    mine = shard_files(durs, world)[rank]
    model = _w2v_base(device, seed)
    meta = {"language": "en", "dictionary": synthetic.w2v_dictionary(), "type": "huggingface"}
    longest = max([durs[i] for i in mine], default=30.0)
    g = torch.Generator().manual_seed(seed)
    audio_buf = torch.randn(int(longest * 16000) + 16000, generator=g) * 0.1
    files = [(i, synthetic.vad_scores(seed * 1000 + i, durs[i]), audio_buf[: int(durs[i] * 16000)]) for i in mine]
    tr = synthetic.Transcriber(seed + rank)
    # warm-up outside the clock (kernels, GEMM heuristics, streams)
    whisperx_amd.align(tr.segments([{"start": 0.0, "end": 30.0}, {"start": 30.0, "end": 47.3}]), model, meta,
                       audio_buf[: 60 * 16000], device)
    merge_chunks(synthetic.vad_scores(1, 60.0), 30, 0.5, 0.363)
    torch.cuda.synchronize()
    if dist_on:
        torch.distributed.barrier()
    st0 = _dp_stats()
    t0 = time.perf_counter()
    n_seg, n_words = 0, 0
    for i, scores, audio in files:
        chunks = merge_chunks(scores, 30, 0.5, 0.363)
        segs = tr.segments(chunks)
        out = whisperx_amd.align(segs, model, meta, audio, device)
        n_seg += len(segs)
        n_words += len(out["word_segments"])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist_on:
        torch.distributed.barrier()
        el_max = _allreduce([el], "max")[0]
        n_seg_all, n_words_all, n_files = _allreduce([n_seg, n_words, len(mine)], "sum")
    else:
        el_max, n_seg_all, n_words_all, n_files = el, n_seg, n_words, len(mine)
    total = float(sum(durs))
    rec = _recovered_since(st0)
    if dist_on:
        rec = dict(zip(rec, (int(x) for x in _allreduce(list(rec.values()), "sum"))))
    return {"files": int(n_files), "audio_sec": total, "n_gpus": world, "segments": int(n_seg_all), "dp": rec,
            "words": int(n_words_all), "wall_s": el_max, "audio_sec_per_s": total / el_max,
            "segments_per_s": n_seg_all / el_max, "scaling": "strong (fixed 10 h corpus)",
            "shard": "LPT by duration (distributed.shard_files)",
            "note": "per file: GPU merge_chunks(30 s) + align() incl. random-weight wav2vec2-base fp32 "
                    "forward per chunk; synthetic VAD scores/audio/transcripts resident before the clock"}


def _cpu_reference_align(segs, model_cpu, dictionary, audio, lang="en", chars=False):
    """The reference's CPU align() path (device='cpu'): CPU forward + log_softmax per segment
    (alignment.py:209-235), the DP on the CPU (oracle TorchPort: get_trellis / backtrack /
    merge_repeats with the reference's per-timestep torch ops, :359-454), then the host
    timestamps/aggregation (whisperx_amd.alignment.aggregate_segment: the pandas-free
    restatement of :252-347, faster than the reference's pandas, so the baseline is
    conservative).  Returns (result dicts, seconds per phase)."""
    from oracle.oracle import TorchPort
    from whisperx_amd import alignment as A

    port = TorchPort()
    t_fwd = t_dp = t_agg = 0.0
    out = []
    for seg in segs:
        seg = dict(seg)
        A._prepare(seg, dictionary, lang)
        tokens = [dictionary[c] for c in "".join(seg["clean_char"])]
        wav = audio[:, int(seg["start"] * 16000): int(seg["end"] * 16000)]
        t0 = time.perf_counter()
        with torch.inference_mode():
            em = torch.log_softmax(model_cpu(wav).logits, -1)[0]
        t1 = time.perf_counter()
        merged = port.align_dp(em, tokens, 0)
        t2 = time.perf_counter()
        if merged is not None:
            ss = np.array([m[1] for m in merged])
            se = np.array([m[2] for m in merged])
            sc = np.array([m[3] for m in merged])
            out += A.aggregate_segment(seg, ss, se, sc, em.shape[0], 1, lang, "nearest", chars)
        t3 = time.perf_counter()
        t_fwd, t_dp, t_agg = t_fwd + t1 - t0, t_dp + t2 - t1, t_agg + t3 - t2
    return out, (t_fwd, t_dp, t_agg)


def _e2e_inputs(n_seg, seed):
    from whisperx_amd import synthetic

    tr = synthetic.Transcriber(seed)
    segs = tr.segments([{"start": 30.0 * k, "end": 30.0 * (k + 1)} for k in range(n_seg)])
    g = torch.Generator().manual_seed(seed)
    audio = torch.randn(30 * n_seg * 16000, generator=g) * 0.1
    return segs, audio


def cpu_align_baseline(threads, budget_s=20.0, seed=11):
    """BASELINE config 1 on the host CPU: one 30 s EN clip through the reference-structured
    CPU align() (random-weight wav2vec2-base forward, T=1499, ~70 words), at `threads` torch
    threads, repeated until `budget_s`."""
    from whisperx_amd import synthetic

    old = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        model = _w2v_base("cpu", seed)
        segs, audio = _e2e_inputs(1, seed)
        audio = audio[None]
        _cpu_reference_align(segs, model, synthetic.w2v_dictionary(), audio)  # warm-up
        n, tot = 0, [0.0, 0.0, 0.0]
        while sum(tot) < budget_s and n < 50:
            _, ph = _cpu_reference_align(segs, model, synthetic.w2v_dictionary(), audio)
            tot = [a + b for a, b in zip(tot, ph)]
            n += 1
            log(f"bench: cpu align clip {n} ({threads} threads): {sum(ph):.2f} s")
    finally:
        torch.set_num_threads(old)
    el = sum(tot)
    return {"value": 30.0 * n / el, "unit": "audio-sec/s", "threads": threads, "clips": n,
            "ms_per_clip": 1000 * el / n, "forward_ms": 1000 * tot[0] / n, "dp_ms": 1000 * tot[1] / n,
            "aggregate_ms": 1000 * tot[2] / n}


def _w2v_large(device, seed, V=40):
    """Random-weight wav2vec2-large-xlsr-shaped CTC model (BASELINE config 5 / the layer-norm
    family of the HF default alignment models, alignment.py:32-61): 24 layers of 1024, layer-norm
    feature encoder with conv bias, stable layer norm."""
    from transformers import Wav2Vec2Config, Wav2Vec2ForCTC

    torch.manual_seed(seed)
    cfg = Wav2Vec2Config(vocab_size=V, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                         intermediate_size=4096, feat_extract_norm="layer", do_stable_layer_norm=True,
                         conv_bias=True)
    return Wav2Vec2ForCTC(cfg).to(device).eval()


def mae_e2e(device, n_seg=4, seed=7, large=False, seg_s=30.0):
    """north_star parity on the real emission path: the same random-weight wav2vec2 and the
    same audio through (a) align() on the GPU (GPU forward + fused HIP DP) and (b) the
    reference's CPU path (CPU forward + CPU DP).  Word start/end MAE in ms, and the segments
    whose char (token path) times differ.  large=True: config 5 (wav2vec2-large-xlsr shape,
    V = 40 German characters, 60 s segments)."""
    import whisperx_amd
    from whisperx_amd import synthetic

    if large:
        model, model_cpu = _w2v_large(device, seed), _w2v_large("cpu", seed)
        dictionary, letters, lang = synthetic.de_dictionary(), synthetic.DE_LETTERS, "de"
    else:
        model, model_cpu = _w2v_base(device, seed), _w2v_base("cpu", seed)
        dictionary, letters, lang = synthetic.w2v_dictionary(), synthetic.LETTERS, "en"
    tr = synthetic.Transcriber(seed, letters=letters)
    segs = tr.segments([{"start": seg_s * k, "end": seg_s * (k + 1)} for k in range(n_seg)])
    g = torch.Generator().manual_seed(seed)
    audio = torch.randn(int(seg_s * n_seg * 16000), generator=g) * 0.1
    meta = {"language": lang, "dictionary": dictionary, "type": "huggingface"}
    gpu = whisperx_amd.align([dict(s) for s in segs], model, meta, audio, device,
                             return_char_alignments=True)["segments"]
    cpu, _ = _cpu_reference_align(segs, model_cpu, dictionary, audio[None], lang=lang, chars=True)
    errs, n_words, n_diff, n_path = [], 0, 0, 0
    for a, b in zip(gpu, cpu):
        wa, wb = a["words"], b["words"]
        seg_diff = False
        for x, y in zip(wa, wb):
            for k in ("start", "end"):
                if k in x and k in y:
                    errs.append(abs(x[k] - y[k]) * 1000.0)
                    seg_diff |= x[k] != y[k]
            n_words += 1
        n_diff += int(seg_diff or len(wa) != len(wb))
        ca = [(c.get("start"), c.get("end")) for c in a.get("chars", [])]
        cb = [(c.get("start"), c.get("end")) for c in b.get("chars", [])]
        n_path += int(ca != cb)
    del model, model_cpu
    torch.cuda.empty_cache()
    return {"mae_ms": float(np.mean(errs)) if errs else None, "max_ms": float(np.max(errs)) if errs else None,
            "words": n_words, "segments": len(gpu), "segments_with_differing_times": n_diff,
            "segments_with_differing_token_paths": n_path, "frame_ms": 1000.0 * seg_s / ((seg_s * 16000 - 400) // 320 + 1),
            "model": ("wav2vec2-large-xlsr shape (24 x 1024, layer-norm feature encoder), V=40 DE, "
                      f"{n_seg} x {seg_s:.0f} s" if large else f"wav2vec2-base shape, V=32 EN, {n_seg} x {seg_s:.0f} s"),
            "vs": "reference CPU align() path (CPU forward + CPU DP), same weights and audio"}


def config5_inputs(device, n_seg=8, seed=5):
    """config5_leg's align() inputs: (segments, audio, large-xlsr-shaped model, metadata)."""
    from whisperx_amd import synthetic

    model = _w2v_large(device, seed)
    meta = {"language": "de", "dictionary": synthetic.de_dictionary(), "type": "huggingface"}
    tr = synthetic.Transcriber(seed, letters=synthetic.DE_LETTERS)
    segs = tr.segments([{"start": 60.0 * k, "end": 60.0 * (k + 1)} for k in range(n_seg)])
    g = torch.Generator().manual_seed(seed)
    audio = torch.randn(int(60 * n_seg * 16000), generator=g) * 0.1
    return segs, audio, model, meta


def config5_leg(device, n_seg=8, seed=5, cpu_budget_s=20.0, dp_steps=20):
    """BASELINE config 5: German wav2vec2-large-xlsr-shaped model (24 x 1024, layer-norm feature
    encoder, stable layer norm; random weights), V = 40, long-form 60 s segments (T = 2999).
    (a) align() end to end on the GPU over n_seg x 60 s: audio-s/s and ms per segment;
    (b) the fused DP alone on 64 x T=2999, V=40, N~U[850,950] with emissions resident in HBM:
        device time of back-to-back launches, algorithmic bytes, HBM fraction, and the PMC
        traffic of the committed rocprofv3 summary for the same kernel;
    (c) the reference-structured CPU align() (CPU forward + TorchPort DP + host aggregation) on
        one 60 s clip at every usable host thread, repeated for ~cpu_budget_s."""
    import whisperx_amd
    from whisperx_amd import _lib

    out = {}
    segs, audio, model, meta = config5_inputs(device, n_seg, seed)
    dictionary = meta["dictionary"]
    whisperx_amd.align([dict(x) for x in segs], model, meta, audio, device)  # warm-up: the timed call
    torch.cuda.synchronize()
    st0 = _dp_stats()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        res = whisperx_amd.align([dict(x) for x in segs], model, meta, audio, device)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    dt = float(np.median(ts))
    out["align"] = {"value": 60.0 * n_seg / dt, "unit": "audio-sec/s", "segments": n_seg, "segment_s": 60.0,
                    "ms_per_segment": 1000 * dt / n_seg, "words": len(res["word_segments"]),
                    "calls_ms": [1000 * t for t in ts],
                    "timing": "median of 3 calls after one untimed warm-up call of the same segments",
                    "dp": _recovered_since(st0)}
    del model
    torch.cuda.empty_cache()
    # (b) DP only
    rng = np.random.default_rng(55)
    ems, toks = make_batch(rng, 64, 2999, 40, 850, 950, device)
    b = _lib.Batch(ems, toks, [0] * len(ems), device=device)
    del ems
    plan = _lib.AlignPlan(b)
    _h, d = time_steps(plan, dp_steps, 3, False)
    launch_s = d / dp_steps
    B = algorithmic_bytes(b.Ts, b.Ns, 40)
    knames = _lib.align_dp_plan(b.S, b.min_N, b.max_N, 40)
    traffic, src = pmc_traffic(knames[0]) if knames else (None, None)
    out["dp_only"] = {"segments": b.S, "T": 2999, "V": 40, "N": [850, 950], "kernel": ";".join(knames),
                      "us_per_launch": launch_s * 1e6, "audio_sec_per_s": sum(b.Ts) * FRAME_S / launch_s,
                      "bytes_per_launch": B, "achieved_GBps": B / launch_s / 1e9,
                      "frac": B / launch_s / 1e9 / HBM_PEAK_GBPS, "traffic": traffic,
                      "traffic_ratio": (traffic / B) if traffic else None, "traffic_source": src,
                      "us_per_launch_events": time_steps.last_launch_s * 1e6,
                      "dp": _lib.status_summary(plan.status[: b.S])}
    del plan, b
    torch.cuda.empty_cache()
    # (c) CPU align() of the same shape
    thr = _host_threads()
    old = torch.get_num_threads()
    torch.set_num_threads(thr)
    try:
        mc = _w2v_large("cpu", seed)
        one = segs[:1]
        wav = audio[None, : 60 * 16000]
        _cpu_reference_align(one, mc, dictionary, wav, lang="de")  # warm-up
        n, tot = 0, [0.0, 0.0, 0.0]
        while sum(tot) < cpu_budget_s and n < 20:
            _, ph = _cpu_reference_align(one, mc, dictionary, wav, lang="de")
            tot = [a + c for a, c in zip(tot, ph)]
            n += 1
            log(f"bench: cfg5 cpu align clip {n}: {sum(ph):.2f} s")
        el = sum(tot)
        out["cpu_align"] = {"value": 60.0 * n / el, "unit": "audio-sec/s", "threads": thr, "clips": n,
                            "ms_per_clip": 1000 * el / n, "forward_ms": 1000 * tot[0] / n, "dp_ms": 1000 * tot[1] / n,
                            "aggregate_ms": 1000 * tot[2] / n, "cpu_model": _cpu_model(), "kind": "port",
                            "sample": "one 60 s DE clip (T=2999), random-weight large-xlsr shape, CPU forward + "
                                      "TorchPort DP + host aggregation"}
        del mc
    finally:
        torch.set_num_threads(old)
    out["gpu_over_cpu"] = out["align"]["value"] / out["cpu_align"]["value"]
    out["note"] = ("BASELINE configs[4] on one GPU (the 8-GPU curve is the driver's SCALE run); random weights, "
                   "synthetic audio and transcripts: timings only (parity: mae_e2e_cfg5)")
    return out


def _recovered_since(before):
    """Segments the legs' align() calls recomputed in-kernel after a lost split hand-off
    (WX_STATUS_RECOVERED), since `before` (a copy of alignment.DP_STATS)."""
    from whisperx_amd import alignment

    return {k: alignment.DP_STATS[k] - before[k] for k in before}


def _dp_stats():
    from whisperx_amd import alignment

    return dict(alignment.DP_STATS)


def _allreduce(vals, op):
    """All-reduce a few host numbers (fp64) over the process group: on the rank's GPU for
    RCCL, on the CPU for gloo."""
    t = torch.tensor(vals, dtype=torch.float64, device=_allreduce.dev)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX if op == "max" else torch.distributed.ReduceOp.SUM)
    return [float(x) for x in t.cpu().tolist()]


_allreduce.dev = torch.device("cpu")


def host_share_leg(k):
    """Child process of the N=1 bench (bench.py --host-share-leg K): rank 0 of a K-GPU node as the
    config-4 corpus run would make it — pinned with distributed.pin_rank(0, K) before any GPU
    call (its NUMA node's share of the host CPUs, 1/K of the threads), then its LPT shard of the
    10 h corpus — so that one GPU measures the host share a rank has at K GPUs.  Prints one
    JSON line."""
    from whisperx_amd import synthetic
    from whisperx_amd.distributed import pin_rank, shard_files

    pin = pin_rank(0, k)
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    res = corpus_config4(device, 0, k, False)
    durs = synthetic.corpus_durations(4)
    loads = [sum(durs[i] for i in s) for s in shard_files(durs, k)]
    shard_audio = loads[0]
    # strong-scaling prediction for K GPUs: every rank at rank 0's rate, the slowest LPT share
    rate = shard_audio / res["wall_s"]
    pred_wall = max(loads) / rate
    print(json.dumps({"ranks_modelled": k, "rank": 0, "cpus": len(pin["cpus"] or []), "threads": pin["threads"],
                      "cpu_set": _cpu_ranges(pin["cpus"]), "numa_node": pin["numa"],
                      "numa_source": pin["numa_source"], "numa_reason": pin["numa_reason"],
                      "shard_audio_sec": shard_audio, "files": res["files"],
                      "segments": res["segments"], "wall_s": res["wall_s"], "audio_sec_per_s": rate,
                      "predicted_node_audio_sec_per_s": float(sum(durs)) / pred_wall,
                      "predicted_node_wall_s": pred_wall,
                      "note": f"rank 0 of a {k}-GPU node on one GPU: pin_rank(0, {k}) host share, its LPT shard of "
                              f"the config-4 corpus; prediction = total audio / (largest shard / this rate)"}),
          flush=True)
    return 0


def _host_share(k, timeout=300):
    import subprocess

    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--host-share-leg", str(k)],
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"rc {r.returncode}: {r.stderr[-300:]}"}
    return json.loads(lines[-1])


def _spawn_ranks(args):
    """--gpus N > 1 without a torchrun environment: launch N ranks as a child torchrun and
    exit with its status.  The parent never touches the GPU (no HIP init before the child)."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--segments", type=int, default=64)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-scale", action="store_true")
    ap.add_argument("--no-corpus", action="store_true", help="skip the config-4 10 h corpus leg")
    ap.add_argument("--host-share-leg", type=int, default=0, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.host_share_leg:
        return host_share_leg(args.host_share_leg)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        log(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}; reporting n_gpus={world}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist_on = world > 1
    pin = None
    if dist_on:  # disjoint host CPUs per rank, before any GPU call
        from whisperx_amd.distributed import pin_rank

        pin = pin_rank(local_rank, int(os.environ.get("LOCAL_WORLD_SIZE", str(world))))
        log(f"bench[{rank}]: pinned to {len(pin['cpus'] or [])} CPUs, {pin['threads']} torch threads")
    # one GPU per rank (LOCAL_RANK); WX_DIST_BACKEND=gloo rehearses the multi-rank path on a
    # box with fewer GPUs than ranks (ranks then share GPUs; RCCL refuses that)
    backend = os.environ.get("WX_DIST_BACKEND", "nccl")
    n_dev = torch.cuda.device_count()
    gpu = local_rank % n_dev if (backend == "gloo" and n_dev) else local_rank
    torch.cuda.set_device(gpu)
    device = torch.device("cuda", gpu)
    if dist_on:
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=device)
        else:
            torch.distributed.init_process_group(backend)
    _allreduce.dev = device if backend == "nccl" else torch.device("cpu")
    ranks = None
    if dist_on:  # every rank's host share and device, for the driver's SCALE line (rank 0 prints)
        ranks = [None] * world
        torch.distributed.all_gather_object(ranks, {
            "rank": rank, "local_rank": local_rank, "device": gpu, "numa": pin["numa"],
            "numa_source": pin["numa_source"], "numa_reason": pin["numa_reason"], "threads": pin["threads"],
            "cpus": _cpu_ranges(pin["cpus"])})

    from whisperx_amd import _lib
    from whisperx_amd.distributed import broadcast_dictionary

    _lib.load()
    dictionary = {c.lower(): i for i, c in enumerate(W2V_VOCAB)} if rank == 0 else None
    dictionary = broadcast_dictionary(dictionary, _allreduce.dev if backend != "nccl" else device) if dist_on else dictionary
    V = len(dictionary)

    # ---- the config-2 batch (per rank), resident in HBM
    T = 1499
    rng = np.random.default_rng(1000 + rank)
    ems, toks = make_batch(rng, args.segments, T, V, 300, 500, device)
    batch = _lib.Batch(ems, toks, [0] * len(ems), device=device)
    plan = _lib.AlignPlan(batch)
    host_s, dev_s = time_steps(plan, args.steps, args.warmup, dist_on)
    step_s = max(host_s, dev_s) / args.steps
    step_s = _allreduce([step_s], "max")[0] if dist_on else step_s
    audio_per_step = float(sum(batch.Ts)) * FRAME_S * world  # seconds of audio aligned per step, all ranks
    value = audio_per_step / step_s
    log(f"bench[{rank}]: headline {step_s * 1e3:.4f} ms/step")
    corpus = None
    if not args.no_corpus:
        try:
            corpus = corpus_config4(device, rank, world, dist_on)
            log(f"bench[{rank}]: config4 {corpus['wall_s']:.1f} s")
        except Exception as e:  # never let the secondary leg hide the primary line
            corpus = {"error": repr(e)[:300]}

    out = None
    if rank == 0:
        B = algorithmic_bytes(batch.Ts, batch.Ns, V)
        # the kernel's time per launch: the device time of the K back-to-back timed launches (one
        # launch per step), not the per-launch event pairs, whose bracketing adds its own gaps
        launch_s = dev_s / args.steps
        achieved = B / launch_s / 1e9
        knames = _lib.align_dp_plan(batch.S, batch.min_N, batch.max_N, V)  # kernels this step launches
        kname = knames[0] if knames else "?"
        traffic, traffic_src = pmc_traffic(kname)
        out = {
            "metric": "aligned audio-sec/s + word-boundary MAE(ms) vs ref, 1/2/4/8 GPU",
            "value": value,
            "unit": "audio-sec/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": step_s * 1000.0,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": "cfg2: batch=64 x 30 s EN segments, T=1499, V=32, N~U[300,500]; "
                                   "fused HIP align DP (wx_align_dp) on HBM-resident emissions",
                       "global_batch": args.segments * world, "seq_len": T,
                       "parallelism": f"dp{world} (per-file sharding, RCCL vocab broadcast)"
                                      + (f"; host pinning: {pin['threads']} threads per rank on disjoint CPUs"
                                         if pin else "")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": kname + (" (the step's only launch)" if len(knames) == 1 else
                                            f" (+{len(knames) - 1} more launches)"),
                         "bytes_per_launch": B, "avg_launch_us": launch_s * 1e6,
                         "avg_launch_us_source": "device time of the timed back-to-back launches / steps",
                         "avg_launch_us_events": time_steps.last_launch_s * 1e6,
                         "traffic_ratio": (traffic / B) if traffic else None},
        }
        out["roofline"]["dp"] = _lib.status_summary(plan.status[: batch.S])
        # The latency roofline: a segment's T steps are a dependent chain, and one step of the
        # register-resident forward is 5 VALU instructions of one wave64 (4 cycles each: add,
        # DPP add, compare, max3, add-with-carry; tools/ubench/step*.hip measures ~20 cycles
        # alone), so no launch can beat T x 20 cycles at the 2.4 GHz peak engine clock.
        t_max = int(max(batch.Ts))
        floor_us = t_max * STEP_CYCLES / ENGINE_PEAK_GHZ / 1e3
        out["roofline"]["latency"] = {"bound": "dependent DP steps", "T": t_max, "cycles_per_step": STEP_CYCLES,
                                      "clock_GHz": ENGINE_PEAK_GHZ, "floor_us": floor_us,
                                      "achieved_us": launch_s * 1e6, "frac": floor_us / (launch_s * 1e6)}
        mae, ntok, nbad = mae_vs_oracle([e.cpu().numpy() for e in ems], toks, plan)
        out["mae_ms"] = mae
        out["mae_detail"] = {"tokens": ntok, "segments_with_path_mismatch": nbad, "vs": "CPU oracle, same emission"}
        extra = {}
        if ranks is not None:
            extra["ranks"] = {"world_size": world, "backend": "rccl" if backend == "nccl" else backend,
                              "per_rank": ranks}
        if corpus is not None:
            extra["config4_10h_corpus"] = corpus
        if not args.no_corpus:
            from whisperx_amd import synthetic
            from whisperx_amd.distributed import lpt_plan

            extra["lpt_plan"] = lpt_plan(synthetic.corpus_durations(4))
            if world == 1:
                log("bench: config-4 host-share leg (rank 0 of 8) ...")
                try:
                    extra["config4_host_share"] = _host_share(8)
                except Exception as e:  # never let the secondary leg hide the primary line
                    extra["config4_host_share"] = {"error": repr(e)[:300]}
        if not args.no_scale and world == 1:
            # saturated batch: enough segments in flight to fill the chip (roofline regime)
            rng2 = np.random.default_rng(77)
            n_big = 4096
            ems2, toks2 = make_batch(rng2, n_big, T, V, 300, 500, device)
            b2 = _lib.Batch(ems2, toks2, [0] * n_big, device=device)
            del ems2
            p2 = _lib.AlignPlan(b2)
            h2, d2 = time_steps(p2, 5, 2, False)
            B2 = algorithmic_bytes(b2.Ts, b2.Ns, V)
            log("bench: saturated T=1499 done")
            extra["saturated"] = {"segments": n_big, "ms_per_step": 1000 * d2 / 5,
                                  "audio_sec_per_s": sum(b2.Ts) * FRAME_S / (d2 / 5),
                                  "achieved_GBps": B2 / (d2 / 5) / 1e9,
                                  "frac": B2 / (d2 / 5) / 1e9 / HBM_PEAK_GBPS,
                                  "cells_per_s": float(sum(t_ * n_ for t_, n_ in zip(b2.Ts, b2.Ns))) / (d2 / 5),
                                  "dp": _lib.status_summary(p2.status[: b2.S])}
            del p2, b2
            torch.cuda.empty_cache()
            # the north star's roofline case: T=3000 x V=32 trellises (N ~ 900, 60 s segments)
            rng3 = np.random.default_rng(78)
            n3 = 2048
            ems3, toks3 = make_batch(rng3, n3, 2999, V, 850, 951, device)
            b3 = _lib.Batch(ems3, toks3, [0] * n3, device=device)
            del ems3
            p3 = _lib.AlignPlan(b3)
            h3, d3 = time_steps(p3, 3, 1, False)
            B3 = algorithmic_bytes(b3.Ts, b3.Ns, V)
            log("bench: saturated T=3000 done")
            k3 = _lib.align_dp_plan(b3.S, b3.min_N, b3.max_N, V)
            t3, t3src = pmc_traffic(k3[0]) if k3 else (None, None)
            extra["saturated_T3000"] = {"segments": n3, "ms_per_step": 1000 * d3 / 3,
                                        "kernel": ";".join(k3), "bytes_per_launch": B3,
                                        "traffic": t3, "traffic_ratio": (t3 / B3) if t3 else None,
                                        "traffic_source": t3src,
                                        "audio_sec_per_s": sum(b3.Ts) * FRAME_S / (d3 / 3),
                                        "achieved_GBps": B3 / (d3 / 3) / 1e9,
                                        "frac": B3 / (d3 / 3) / 1e9 / HBM_PEAK_GBPS,
                                        "cells_per_s": float(sum(t_ * n_ for t_, n_ in zip(b3.Ts, b3.Ns))) / (d3 / 3),
                                        "dp": _lib.status_summary(p3.status[: b3.S])}
            # get_trellis (materialised, wx_trellis) on the same T=3000 batch: the HBM-write-bound
            # kernel of the path (4 B per cell written)
            try:
                tr_flat, tr_offs = _lib.trellis(b3)
                tr_off_d = _lib._dev_i64(tr_offs, device)
                lib = _lib.load()

                def tr_run():
                    lib.wx_trellis(_lib._ptr(b3.em), _lib._ptr(b3.em_off_d), b3.V, _lib._ptr(b3.tok),
                                   _lib._ptr(b3.tok_off_d), _lib._ptr(b3.blank), b3.S, b3.max_N, _lib._ptr(tr_flat),
                                   _lib._ptr(tr_off_d), _lib._stream(device))
                tr_run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    tr_run()
                e1.record()
                torch.cuda.synchronize()
                dt = e0.elapsed_time(e1) / 1000.0 / 3
                Bt = sum(4 * t_ * V + 4 * n_ + 4 * (t_ + 1) * (n_ + 1) for t_, n_ in zip(b3.Ts, b3.Ns))
                extra["trellis_T3000"] = {"kernel": "wx_trellis (get_trellis, materialised fp32 [T+1,N+1])",
                                          "segments": n3, "ms_per_launch": 1000 * dt,
                                          "bytes_per_launch": Bt, "achieved_GBps": Bt / dt / 1e9,
                                          "frac": Bt / dt / 1e9 / HBM_PEAK_GBPS,
                                          "bytes_per_cell": 4, "bound": "hbm (writes)"}
                del tr_flat
            except Exception as e:  # never let the secondary leg hide the primary line
                extra["trellis_T3000"] = {"error": repr(e)[:200]}
            del p3, b3
            torch.cuda.empty_cache()
        if not args.no_cpu and world == 1:
            ems_cpu = [e.cpu() for e in ems]
            log("bench: cpu baselines ...")
            out["cpu_baseline"] = cpu_port_baseline(ems_cpu, toks)
            extra["cpu_c_oracle"] = c_oracle_baseline([e.numpy() for e in ems_cpu], toks)
            extra["host_cpu"] = {"os_cpu_count": os.cpu_count(), "usable_threads": _host_threads(),
                                 "model": _cpu_model()}
            try:
                extra["cpu_align_config1"] = {
                    "all_threads": cpu_align_baseline(_host_threads()),
                    "one_thread": cpu_align_baseline(1, budget_s=15.0),
                    "kind": "port", "model": "random-weight wav2vec2-base (WAV2VEC2_ASR_BASE_960H architecture)",
                    "sample": "config 1: one 30 s clip, T=1499, ~70 words, CPU forward + TorchPort DP + host "
                              "aggregation, repeated for ~15-20 s; all_threads = the cores this process may "
                              "use (sched_getaffinity, capped by OMP_NUM_THREADS), not os.cpu_count(): on a "
                              "shared box os.cpu_count() counts the whole machine and oversubscribes"}
            except Exception as e:
                extra["cpu_align_config1"] = {"error": repr(e)[:300]}
        if not args.no_e2e and world == 1:
            log("bench: e2e legs ...")
            try:
                extra["e2e_align"] = e2e_align(device)
            except Exception as e:  # never let the secondary leg hide the primary line
                extra["e2e_align"] = {"error": repr(e)[:200]}
            try:
                extra["binarize_1h"] = binarize_1h(device)
            except Exception as e:
                extra["binarize_1h"] = {"error": repr(e)[:300]}
            try:
                extra["vad_producer_1h"] = vad_producer_1h(device)
            except Exception as e:
                extra["vad_producer_1h"] = {"error": repr(e)[:300]}
            try:
                extra["e2e_config3_1h"] = e2e_config3(device)
            except Exception as e:
                extra["e2e_config3_1h"] = {"error": repr(e)[:200]}
            try:
                extra["e2e_config3_1h_from_waveform"] = e2e_config3_waveform(device)
            except Exception as e:
                extra["e2e_config3_1h_from_waveform"] = {"error": repr(e)[:300]}
            log("bench: emission-path MAE ...")
            try:
                me = mae_e2e(device)
                out["mae_e2e_ms"] = me["mae_ms"]
                extra["mae_e2e"] = me
            except Exception as e:
                extra["mae_e2e"] = {"error": repr(e)[:300]}
            log("bench: config 5 ...")
            try:
                extra["config5"] = config5_leg(device)
            except Exception as e:  # never let the secondary leg hide the primary line
                extra["config5"] = {"error": repr(e)[:300]}
            try:  # config 5: the layer-norm (large-xlsr) family, V = 40, 60 s segments
                m5 = mae_e2e(device, n_seg=2, seed=5, large=True, seg_s=60.0)
                out["mae_e2e_cfg5_ms"] = m5["mae_ms"]
                extra["mae_e2e_cfg5"] = m5
            except Exception as e:
                extra["mae_e2e_cfg5"] = {"error": repr(e)[:300]}
            ca = extra.get("cpu_align_config1", {}).get("all_threads", {})
            ea = extra.get("e2e_align", {})
            if "value" in ca and "value" in ea:
                extra["north_star_ratio"] = {
                    "gpu_align_audio_sec_per_s": ea["value"], "cpu_align_audio_sec_per_s": ca["value"],
                    "cpu_threads": ca["threads"], "ratio": ea["value"] / ca["value"], "target": 50.0,
                    "note": "align() end to end on 1 MI355X (GPU forward + fused DP) over the reference-structured "
                            "CPU align() on every usable host thread, same model architecture and clip length"}
        out["extra"] = extra
    if dist_on:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


def _host_threads():
    from whisperx_amd.distributed import thread_budget

    return thread_budget()


def _cpu_ranges(cpus):
    """[0, 1, 2, 5] -> "0-2,5" (None stays None)."""
    if cpus is None:
        return None
    cpus, out, i = sorted(cpus), [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(f"{cpus[i]}-{cpus[j]}" if j > i else f"{cpus[i]}")
        i = j + 1
    return ",".join(out)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == "__main__":
    main()
