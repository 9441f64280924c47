"""Emission producer kernels and routes (-m gpu): the time-major GroupNorm+GELU kernel
against torch's fp32 GroupNorm + GELU, the f32-MFMA attention against an fp64 attention, and
the prepared (GEMM-conv + fused-norm + wx attention) wav2vec2
forward against the stock PyTorch forward (fp32 reference of the same op; tolerance: the
log-probabilities' float noise, with identical frame argmax)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


@pytest.mark.parametrize("L,C,gelu", [(95999, 512, True), (1000, 64, False), (7, 8, True), (3, 512, True)])
def test_channel_norm_vs_torch_groupnorm(L, C, gelu):
    from whisperx_amd import _lib

    torch.manual_seed(L)
    x = (torch.randn(L, C, device="cuda") * 3 + torch.randn(1, C, device="cuda")).contiguous()
    g = torch.randn(C, device="cuda")
    b = torch.randn(C, device="cuda")
    gn = torch.nn.GroupNorm(C, C).cuda()
    with torch.no_grad():
        gn.weight.copy_(g)
        gn.bias.copy_(b)
        ref = gn(x.t().unsqueeze(0))[0].t()
        if gelu:
            ref = torch.nn.functional.gelu(ref)
    got = _lib.channel_norm(x, g, b, gn.eps, gelu)
    torch.testing.assert_close(got, ref, rtol=2e-5, atol=2e-5)
    inplace = x.clone()
    _lib.channel_norm(inplace, g, b, gn.eps, gelu, out=inplace)
    assert torch.equal(inplace, got)


@pytest.mark.parametrize("B,H,T", [(1, 12, 1), (1, 12, 31), (1, 12, 33), (1, 12, 400), (1, 12, 1499), (2, 16, 97)])
def test_attention_f32_vs_fp64(B, H, T):
    """wx_attention_f32 on transformers' q/k/v views of [B, T, H*64] projections against an
    fp64 softmax(q k^T / 8) v; fp32 tolerance (f32 MFMA, its own summation order)."""
    from whisperx_amd import _lib

    torch.manual_seed(T)
    proj = [torch.randn(B, T, H * 64, device="cuda") * 2 for _ in range(3)]
    q, k, v = (p.view(B, T, H, 64).transpose(1, 2) for p in proj)  # [B, H, T, 64] views
    got = _lib.attention_f32(q, k, v, 0.125)  # [B, T, H, 64]
    qd, kd, vd = (x.double() for x in (q, k, v))
    ref = torch.softmax(qd @ kd.transpose(-1, -2) * 0.125, -1) @ vd  # [B, H, T, 64]
    ref = ref.transpose(1, 2).float()
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=2e-5)


def test_attention_f32_csr_vs_fp64():
    """wx_attention_f32_csr on a ragged batch (segments of 1, 31, 33, 400 and 1,499 rows,
    including an empty one) against an fp64 attention within each segment."""
    from whisperx_amd import _lib

    torch.manual_seed(1)
    Ts = [31, 1, 0, 400, 33, 1499]
    R, H = sum(Ts), 12
    proj = [torch.randn(R, H * 64, device="cuda") * 2 for _ in range(3)]
    q, k, v = (p.view(R, H, 64) for p in proj)
    got = _lib.attention_f32_csr(q, k, v, Ts, 0.125)
    o = 0
    for t in Ts:
        qd, kd, vd = (x[o:o + t].transpose(0, 1).double() for x in (q, k, v))
        ref = (torch.softmax(qd @ kd.transpose(-1, -2) * 0.125, -1) @ vd).transpose(0, 1).float()
        torch.testing.assert_close(got[o:o + t], ref, rtol=1e-5, atol=2e-5)
        o += t


@pytest.mark.parametrize("stable", [False, True])
def test_batched_logits_vs_per_segment_forward_gpu(stable):
    """The batched emission forward (emission.batched_logits: concatenated rows, ragged
    attention) against each segment's own prepared forward on the GPU: log-probabilities within
    float noise, identical frame argmax."""
    from transformers import Wav2Vec2Config, Wav2Vec2ForCTC

    from whisperx_amd import emission

    torch.manual_seed(2)
    if stable:
        cfg = Wav2Vec2Config(vocab_size=40, num_hidden_layers=4, hidden_size=1024, num_attention_heads=16,
                             intermediate_size=4096, feat_extract_norm="layer", do_stable_layer_norm=True, conv_bias=True)
    else:
        cfg = Wav2Vec2Config(vocab_size=32)
    m = Wav2Vec2ForCTC(cfg).cuda().eval()
    emission.prepare_model(m)
    rng = np.random.default_rng(3)
    wavs = [torch.from_numpy(rng.standard_normal(n).astype(np.float32) * 0.1).cuda() for n in (480000, 400, 117000, 33333)]
    got = emission.batched_logits(m, wavs)
    for w, g in zip(wavs, got):
        with torch.inference_mode():
            ref = m(w.reshape(1, -1)).logits[0]
        assert g.shape == ref.shape
        lg, lr = torch.log_softmax(g, -1), torch.log_softmax(ref, -1)
        assert (lg - lr).abs().max().item() <= 5e-5
        assert torch.equal(lg.argmax(-1), lr.argmax(-1))


def _check_prepared_vs_stock(m, V, lengths, tol=5e-5):
    from whisperx_amd import emission

    rng = np.random.default_rng(0)
    worst = 0.0
    for n in lengths:
        x = torch.from_numpy(rng.standard_normal(n).astype(np.float32) * 0.1)[None].cuda()
        with torch.inference_mode():
            ref = torch.log_softmax(m(x).logits, -1)
            emission.prepare_model(m)
            got = torch.log_softmax(m(x).logits, -1)
            emission.restore_model(m)
        assert got.shape == ref.shape == (1, emission.n_frames(n, m), V)
        err = float((got - ref).abs().max())
        worst = max(worst, err)
        assert err < tol, f"{n} samples: max |prepared - stock| = {err}"
        assert torch.equal(got.argmax(-1), ref.argmax(-1)), f"{n} samples: frame argmax differs"
    return worst


def test_prepared_wav2vec2_forward_matches_stock():
    """Group-norm feature encoder (wav2vec2-base-960h, the torchaudio/HF English defaults)."""
    from transformers import Wav2Vec2Config, Wav2Vec2ForCTC

    torch.manual_seed(0)
    m = Wav2Vec2ForCTC(Wav2Vec2Config(vocab_size=32)).cuda().eval()
    _check_prepared_vs_stock(m, 32, (400, 7 * 16000 + 123, 30 * 16000))


def large_xlsr_config(V=40):
    """The layer-norm wav2vec2 family of the HF default alignment models (alignment.py:32-61:
    every DEFAULT_ALIGN_MODELS_HF entry but `vi` is a large-xlsr / xls-r checkpoint, and
    BASELINE config 5 names DE wav2vec2-large-xlsr): feat_extract_norm="layer" (a LayerNorm
    after every feature-encoder conv), stable layer norm, conv bias."""
    from transformers import Wav2Vec2Config

    return Wav2Vec2Config(vocab_size=V, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                          intermediate_size=4096, feat_extract_norm="layer", do_stable_layer_norm=True,
                          conv_bias=True)


def test_prepared_large_xlsr_forward_matches_stock():
    """The GEMM-route convolutions on the layer-norm family (no GroupNorm layer: every conv
    of the feature encoder takes the plain GEMM route, LayerNorm runs on its time-major
    output): 400 samples, 7.3 s and 60 s (config 5's T = 2999)."""
    from transformers import Wav2Vec2ForCTC

    torch.manual_seed(1)
    m = Wav2Vec2ForCTC(large_xlsr_config()).cuda().eval()
    assert m.config.feat_extract_norm == "layer"
    worst = _check_prepared_vs_stock(m, 40, (400, int(7.3 * 16000), 60 * 16000))
    print(f"large-xlsr prepared vs stock: max |dlogp| = {worst:.3g}")


@pytest.mark.parametrize("batched", [False, True])
def test_emissions_fan_out_fresh_parametrised_model(monkeypatch, batched):
    """the positional conv's weight_norm weight is cached; on a freshly
    built model the cache must exist before the forwards fan out over 8 streams, or the
    streams read it before it is computed.  Segment 0 is much longer than the others (its
    stream would still be building the weight when the others reach the positional conv).
    Every segment's emission must equal a single-stream forward of the same model (per-segment
    forwards: to 1e-6; batched forwards, whose GEMMs have other row counts: to float noise with
    identical frame argmax)."""
    from transformers import Wav2Vec2Config, Wav2Vec2ForCTC

    from whisperx_amd import alignment, emission

    if batched:
        monkeypatch.setenv("WX_EMISSION_BATCH", "8")
    else:
        monkeypatch.delenv("WX_EMISSION_BATCH", raising=False)
    torch.manual_seed(2)
    m = Wav2Vec2ForCTC(Wav2Vec2Config(vocab_size=32)).cuda().eval()
    pos = m.wav2vec2.encoder.pos_conv_embed.conv
    assert getattr(pos, "parametrizations", None) is not None and not hasattr(pos, "_wx_w_cache")
    g = torch.Generator().manual_seed(3)
    audio = (torch.randn(1, 80 * 16000, generator=g) * 0.1).cuda()
    wavs = [audio[:, : 60 * 16000]] + [audio[:, 16000 * k: 16000 * k + 16000 + 1234 * k] for k in range(1, 12)]
    csr = alignment._emissions(m, "huggingface", wavs, "cuda:0", n_streams=8)
    main = torch.cuda.current_stream()
    for st in csr.streams:
        main.wait_stream(st)
    torch.cuda.synchronize()
    with torch.inference_mode():
        for i, w in enumerate(wavs):
            ref = torch.log_softmax(m(w).logits, -1)[0]
            err = float((csr[i] - ref).abs().max())
            assert err <= (5e-5 if batched else 1e-6), f"segment {i}: fan-out emission differs from single-stream by {err}"
            assert torch.equal(csr[i].argmax(-1), ref.argmax(-1))
    emission.restore_model(m)
