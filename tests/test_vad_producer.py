"""VAD producer (vad.py:198-240): the PyanNet-shaped segmentation model, pyannote's sliding
windows and overlap-add geometry, and the wx_vad_aggregate kernel against the oracle
restatement of pyannote.audio 3.1.1 Inference.aggregate (pyannote itself is absent: parity
unpinned at the pyannote boundary; the kernel is pinned to the restatement bit for bit)."""
import math

import numpy as np
import pytest
import torch

from oracle import oracle


def test_oracle_aggregate_hand_case():
    # 3 windows of K=4 frames, 2 classes, starting at frames 0, 2, 3 (n_frames 8)
    sc = np.array([[[0.1, 0.3], [0.2, 0.1], [0.5, np.nan], [0.4, 0.4]],
                   [[0.9, 0.0], [0.1, 0.2], [np.nan, np.nan], [0.7, 0.6]],
                   [[0.2, 0.2], [0.3, 0.1], [0.6, 0.6], [0.8, 0.9]]], np.float32)
    out = oracle.vad_aggregate(sc, [0, 2, 3, 99][:3], 8, missing=-1.0)
    m = np.max(sc, axis=-1)  # per window frame; a NaN class makes the frame NaN (masked)
    exp = [m[0, 0], m[0, 1], (m[1, 0]) / 1, (m[0, 3] + m[1, 1] + m[2, 0]) / 3,
           (m[2, 1]) / 1, (m[1, 3] + m[2, 2]) / 2, m[2, 3], -1.0]
    # frame 2: window 0's value is NaN (masked), window 1 covers it with 0.9
    exp[2] = np.float32(m[1, 0])
    np.testing.assert_allclose(out, np.array(exp, np.float32), rtol=1e-6)
    assert out[7] == -1.0


def test_pyannet_geometry_and_windows():
    from whisperx_amd.vad_model import PyanNet, VoiceActivitySegmentation, closest_frame

    m = PyanNet()
    assert PyanNet.n_frames(80000) == 293
    assert round(m.frame_step * 16000) == 270 and round(m.frame_duration * 16000) == 991
    with torch.no_grad():
        y = m(torch.randn(2, 1, 80000))
    assert y.shape == (2, 293, 3) and float(y.min()) >= 0 and float(y.max()) <= 1
    v = VoiceActivitySegmentation.__new__(VoiceActivitySegmentation)
    v.duration, v.step = 5.0, 0.5
    assert v.windows(80000) == (1, False)
    assert v.windows(80000 + 8000) == (2, False)
    assert v.windows(80000 + 8001) == (2, True)
    assert v.windows(1000) == (0, True)
    # pyannote closest_frame: rint((t - start - d/2) / step)
    assert closest_frame(0.5 + 0.5 * m.frame_duration, 0.0, m.frame_duration, m.frame_step) == round(0.5 / m.frame_step)


@pytest.mark.gpu
def test_vad_aggregate_kernel_vs_oracle():
    from whisperx_amd import _lib

    rng = np.random.default_rng(5)
    for n_chunks, K, C in ((50, 293, 3), (7, 20, 1), (1, 5, 2)):
        sc = rng.random((n_chunks, K, C)).astype(np.float32)
        sc[rng.random(sc.shape) < 0.02] = np.nan
        sc[3 % n_chunks, :, :] = np.nan  # a fully masked window
        starts = np.cumsum(np.concatenate([[0], rng.integers(0, K // 3 + 1, n_chunks - 1)]))
        n_frames = int(starts[-1] + K + 3)  # a few frames no window covers
        got = _lib.vad_aggregate(torch.from_numpy(sc).cuda(), starts.tolist(), n_frames).cpu().numpy()
        exp = oracle.vad_aggregate(sc, starts, n_frames)
        assert np.array_equal(got, exp, equal_nan=True), (n_chunks, K, C)


@pytest.mark.gpu
def test_vad_producer_end_to_end_device_scores():
    """60 s of audio through the producer; its scores equal the oracle aggregation of its own
    window outputs, and merge_chunks on the device-resident scores equals merge_chunks on a
    host copy and the oracle Binarize + chunk merge."""
    from whisperx_amd.vad import SlidingWindowFeature, merge_chunks
    from whisperx_amd.vad_model import VoiceActivitySegmentation

    torch.manual_seed(0)
    vad = VoiceActivitySegmentation(device="cuda:0", batch_size=16)
    wav = torch.randn(1, 61 * 16000 + 123) * 0.1
    feat = vad({"waveform": wav, "sample_rate": 16000})
    assert feat.data.is_cuda and feat.data.shape[1] == 1
    cs = vad.chunk_scores(wav).cpu().numpy()
    n_full, has_last = vad.windows(wav.shape[1])
    assert cs.shape == (n_full + int(has_last), 293, 3)
    fd, fs = vad.model.frame_duration, vad.model.frame_step
    from whisperx_amd.vad_model import closest_frame
    starts = [closest_frame(c * 0.5 + 0.5 * fd, 0.0, fd, fs) for c in range(cs.shape[0])]
    exp = oracle.vad_aggregate(cs, starts, feat.data.shape[0])
    assert np.array_equal(feat.data[:, 0].cpu().numpy(), exp, equal_nan=True)
    # a random-weight model's scores hover near one value: binarise around their median
    med = float(np.nanmedian(exp))
    dev_chunks = merge_chunks(feat, 30, onset=med, offset=med)
    host = SlidingWindowFeature(feat.data.cpu().numpy(), feat.sliding_window)
    assert dev_chunks == merge_chunks(host, 30, onset=med, offset=med)
    sw = feat.sliding_window
    regions = oracle.binarize(exp, sw.start, sw.step, sw.duration, med, med, 30)
    ref = oracle.merge_chunks_regions(regions, 30)
    assert [(c["start"], c["end"]) for c in dev_chunks] == [(c["start"], c["end"]) for c in ref]


@pytest.mark.gpu
@pytest.mark.parametrize("B,L,C,do_abs,stride_pad", [(3, 7975, 80, True, 0), (5, 2654, 60, False, 4),
                                                      (2, 880, 60, False, 4), (1, 4, 8, True, 0), (4, 2, 4, False, 0)])
def test_sincnet_stage_vs_torch(B, L, C, do_abs, stride_pad):
    """wx_sincnet_stage against torch's |.| -> MaxPool1d(3, 3) -> InstanceNorm1d(affine) ->
    LeakyReLU on the same time-major input (fp32 reference of the same ops; statistics in
    fp64 here, fp32 in MIOpen: tolerance 2e-5), windows with a row-padded stride (the k = 5
    GEMM convs' output view), NaN propagation through the max-pool, L not a multiple of 3."""
    from whisperx_amd import _lib

    torch.manual_seed(L + C)
    full = torch.randn(B, L + stride_pad, C, device="cuda") * 3 + torch.randn(1, 1, C, device="cuda")
    x_tm = full[:, :L]
    if B > 1 and L > 30:
        x_tm[1, 10, 2] = float("nan")  # -> pooled row 3 channel 2 NaN -> that window/channel NaN
    norm = torch.nn.InstanceNorm1d(C, affine=True).cuda().eval()  # inference, as pyannote runs it
    with torch.no_grad():
        norm.weight.copy_(torch.randn(C) * 0.5 + 1)
        norm.bias.copy_(torch.randn(C) * 0.1)
    got = _lib.sincnet_stage(x_tm, do_abs, norm.weight, norm.bias, norm.eps)
    assert got.shape == (B, L // 3, C)
    if L < 3:  # no pooled row (torch's max_pool1d refuses the empty output)
        return
    with torch.no_grad():
        xc = x_tm.transpose(1, 2)
        pooled = torch.nn.functional.max_pool1d(xc.abs() if do_abs else xc, 3, 3)
        if pooled.shape[-1] > 1:
            normed = norm(pooled)
        else:  # (torch's instance_norm refuses one element; InstanceNorm1d's formula by hand)
            mean = pooled.mean(-1, keepdim=True)
            var = pooled.var(-1, unbiased=False, keepdim=True)
            normed = (pooled - mean) / torch.sqrt(var + norm.eps) * norm.weight[:, None] + norm.bias[:, None]
        ref = torch.nn.functional.leaky_relu(normed)
    torch.testing.assert_close(got.transpose(1, 2), ref, rtol=2e-5, atol=2e-5, equal_nan=True)


@pytest.mark.gpu
def test_sincnet_stage_ex_affine_overlapping_windows():
    """wx_sincnet_stage_ex reading overlapping windows of one shared time-major buffer (window
    stride 800 rows < L) with a per-window input affine x * scale[b] + shift[b, c] before |.|,
    against torch's ops on the materialised windows (fp32 tolerance)."""
    from whisperx_amd import _lib

    torch.manual_seed(7)
    B, L, C, fpw = 5, 2654, 80, 800
    G = torch.randn((B - 1) * fpw + L, C, device="cuda") * 2
    x = G.as_strided((B, L, C), (fpw * C, C, 1))
    scale = torch.rand(B, device="cuda") + 0.5
    shift = torch.randn(B, C, device="cuda")
    norm = torch.nn.InstanceNorm1d(C, affine=True).cuda().eval()
    with torch.no_grad():
        norm.weight.copy_(torch.randn(C) * 0.5 + 1)
        norm.bias.copy_(torch.randn(C) * 0.1)
        xa = x * scale[:, None, None] + shift[:, None, :]
        ref = torch.nn.functional.leaky_relu(norm(torch.nn.functional.max_pool1d(xa.abs().transpose(1, 2), 3, 3)))
    got = _lib.sincnet_stage(x, True, norm.weight, norm.bias, norm.eps, in_scale=scale, in_shift=shift)
    torch.testing.assert_close(got.transpose(1, 2), ref, rtol=2e-5, atol=2e-5)


@pytest.mark.gpu
def test_shared_sinc_filterbank_matches_per_window(monkeypatch):
    """chunk_scores with the sinc filterbank run once over the waveform (the windows' waveform
    InstanceNorm commuted into a per-window affine of the shared convolution) against one
    convolution per window (WX_NO_SHARED_SINC=1), both with the fused epilogues: the same
    scores up to the reassociation's float noise, the zero-padded last window included."""
    from whisperx_amd.vad_model import VoiceActivitySegmentation

    torch.manual_seed(2)
    vad = VoiceActivitySegmentation(device="cuda:0", batch_size=64)
    wav = torch.randn(1, 75 * 16000 + 1234) * 0.1 + 0.01
    monkeypatch.delenv("WX_NO_SHARED_SINC", raising=False)
    shared = vad.chunk_scores(wav)
    monkeypatch.setenv("WX_NO_SHARED_SINC", "1")
    per_window = vad.chunk_scores(wav)
    assert shared.shape == per_window.shape
    torch.testing.assert_close(shared, per_window, rtol=0, atol=2e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [251, 252, 261, 2551, 80000 + 7, 16000 * 75 + 1234])
def test_sinc_filterbank_kernel_vs_fp64_conv(n):
    """wx_sinc_filterbank (the shared-sinc route's stage-1 convolution: 80 filters of 251 taps,
    stride 10, taps zero-padded to 260, rows read in place) against an fp64 F.conv1d of the
    same span, fp32 tolerance; spans that end inside a block of 256 rows, in the padded taps,
    and a single row."""
    import torch.nn.functional as F

    from whisperx_amd import _lib

    g = torch.Generator().manual_seed(n)
    x = (torch.randn(n, generator=g) * 0.1).cuda()
    w = (torch.randn(80, 251, generator=g) * 0.05).cuda()
    wp = F.pad(w, (0, 9)).t().contiguous()
    got = _lib.sinc_filterbank(x, wp, 251, 10)
    ref = F.conv1d(x.double()[None, None], w.double()[:, None], stride=10)[0].t()
    assert got.shape == ref.shape == ((n - 251) // 10 + 1, 80)
    torch.testing.assert_close(got.double(), ref, rtol=1e-5, atol=2e-6)


@pytest.mark.gpu
def test_sincnet_fused_epilogue_matches_torch_ops(monkeypatch):
    """PyanNet's forward with the fused SincNet epilogues against the same forward through
    torch's ops (WX_NO_SINC_EPILOGUE=1), both on the GEMM route: scores within float noise, and
    merge_chunks of the aggregated scores identical."""
    from whisperx_amd.vad import merge_chunks
    from whisperx_amd.vad_model import VoiceActivitySegmentation

    torch.manual_seed(1)
    vad = VoiceActivitySegmentation(device="cuda:0", batch_size=64)
    wav = torch.randn(1, 90 * 16000 + 77) * 0.1
    monkeypatch.delenv("WX_NO_SINC_EPILOGUE", raising=False)
    fused = vad.chunk_scores(wav)
    feat_f = vad({"waveform": wav, "sample_rate": 16000})
    monkeypatch.setenv("WX_NO_SINC_EPILOGUE", "1")
    plain = vad.chunk_scores(wav)
    feat_p = vad({"waveform": wav, "sample_rate": 16000})
    diff = (fused - plain).abs().max().item()
    assert diff <= 2e-4  # (the shared filterbank convolution reassociates the window norm)
    # scores this close give the same chunks unless a frame sits on the threshold: binarise at
    # the middle of the widest gap between the sorted frame scores (5th to 95th percentile)
    vals = np.sort(feat_p.data[:, 0].cpu().numpy())
    vals = vals[np.isfinite(vals)]
    lo, hi = len(vals) // 20, 19 * len(vals) // 20
    i = lo + int(np.argmax(np.diff(vals[lo:hi + 1])))
    thr = float(0.5 * (vals[i] + vals[i + 1]))
    if vals[i + 1] - vals[i] > 4 * diff:  # (every frame on the same side of thr in both)
        assert merge_chunks(feat_f, 30, onset=thr, offset=thr) == merge_chunks(feat_p, 30, onset=thr, offset=thr)


@pytest.mark.gpu
@pytest.mark.parametrize("B,T,layers", [(37, 293, 2), (16, 1, 1), (3, 50, 2), (130, 293, 1)])
def test_lstm_kernel_vs_torch_lstm(B, T, layers):
    """wx_lstm_bidir_layer (PyanNet's bidirectional LSTM, one persistent launch per layer)
    through vad_model.lstm_forward against torch.nn.LSTM (fp32): batches that are not a
    multiple of the kernel's 16 sequences, a single step, both layer counts."""
    from whisperx_amd import vad_model

    torch.manual_seed(B * 1000 + T)
    lstm = torch.nn.LSTM(60, 128, num_layers=layers, bidirectional=True, batch_first=True).cuda().eval()
    x = torch.randn(B, T, 60, device="cuda")
    with torch.inference_mode():
        ref = lstm(x)[0]
        got = vad_model.lstm_forward(lstm, x)
    assert got.shape == ref.shape == (B, T, 256)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=2e-5)


@pytest.mark.gpu
def test_lstm_kernel_producer_scores_and_chunks(monkeypatch):
    """The VAD producer with the LSTM kernel against torch's LSTM (WX_NO_LSTM_KERNEL=1): window
    scores within float noise and identical merge_chunks (threshold in the widest score gap)."""
    from whisperx_amd.vad import merge_chunks
    from whisperx_amd.vad_model import VoiceActivitySegmentation

    torch.manual_seed(3)
    vad = VoiceActivitySegmentation(device="cuda:0", batch_size=64)
    wav = torch.randn(1, 75 * 16000 + 123) * 0.1
    monkeypatch.delenv("WX_NO_LSTM_KERNEL", raising=False)
    kern = vad.chunk_scores(wav)
    feat_k = vad({"waveform": wav, "sample_rate": 16000})
    monkeypatch.setenv("WX_NO_LSTM_KERNEL", "1")
    plain = vad.chunk_scores(wav)
    feat_p = vad({"waveform": wav, "sample_rate": 16000})
    diff = (kern - plain).abs().max().item()
    assert diff <= 1e-4
    vals = np.sort(feat_p.data[:, 0].cpu().numpy())
    vals = vals[np.isfinite(vals)]
    lo, hi = len(vals) // 20, 19 * len(vals) // 20
    i = lo + int(np.argmax(np.diff(vals[lo:hi + 1])))
    thr = float(0.5 * (vals[i] + vals[i + 1]))
    assert vals[i + 1] - vals[i] > 4 * diff
    assert merge_chunks(feat_k, 30, onset=thr, offset=thr) == merge_chunks(feat_p, 30, onset=thr, offset=thr)


@pytest.mark.gpu
@pytest.mark.parametrize("B,L,Cin,Cout", [(3, 2658, 80, 60), (5, 884, 60, 60), (2, 5, 80, 60), (1, 300, 8, 4),
                                         (7, 129, 64, 64)])
def test_conv_taps_kernel_vs_torch(B, L, Cin, Cout):
    """wx_conv1d_taps_tm (SincNet's k = 5 convolutions, every window in one launch) through
    vad_model.conv1d_batched against torch's fp32 conv1d: both PyanNet stage shapes, a single
    output frame, narrow channels, the 128-frame tile edge."""
    from whisperx_amd import vad_model

    torch.manual_seed(B * L + Cin)
    x_tm = torch.randn(B, L, Cin, device="cuda")
    w = torch.randn(Cout, Cin, 5, device="cuda") * 0.1
    b = torch.randn(Cout, device="cuda")
    with torch.inference_mode():
        ref = torch.nn.functional.conv1d(x_tm.transpose(1, 2), w, b)
        got = vad_model.conv1d_batched(x_tm.transpose(1, 2), w, b, 1)
    assert got.shape == ref.shape
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)
