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


@pytest.mark.parametrize("S,K,stride,bias,gelu", [(480000, 10, 5, False, True), (112123, 10, 5, True, True),
                                                  (400, 10, 5, False, False), (15, 10, 5, False, True),
                                                  (3001, 16, 3, True, True), (64, 1, 1, False, True)])
def test_conv0_channel_norm_vs_torch(S, K, stride, bias, gelu):
    """wx_conv0_channel_norm (the feature encoder's first layer in one pass) against torch's fp32
    Conv1d(1, 512, K, stride) -> GroupNorm(512, 512) -> GELU(erf), time-major: 30 s, 7 s, the
    400-sample minimum, two frames, other tap counts / strides, with and without a conv
    bias and the GELU."""
    from whisperx_amd import _lib

    torch.manual_seed(S)
    C = 512
    conv = torch.nn.Conv1d(1, C, K, stride=stride, bias=bias).cuda().eval()
    gn = torch.nn.GroupNorm(C, C).cuda().eval()
    with torch.no_grad():
        gn.weight.copy_(torch.randn(C) * 0.5 + 1)
        gn.bias.copy_(torch.randn(C) * 0.1)
    x = (torch.randn(S, device="cuda") * 0.1).contiguous()
    with torch.no_grad():
        ref = gn(conv(x[None, None]))
        if gelu:
            ref = torch.nn.functional.gelu(ref)
        ref = ref[0].t()  # [Lout, C]
        got = _lib.conv0_channel_norm(x, conv.weight, conv.bias, stride, gn.weight, gn.bias, gn.eps, gelu)
    assert got.shape == ref.shape
    torch.testing.assert_close(got, ref, rtol=5e-5, atol=5e-5)


@pytest.mark.parametrize("shape", [(1, 1499, 768), (2, 97, 1024), (1, 1, 768), (3, 5, 256), (1, 0, 512)])
def test_add_layernorm_vs_torch(shape):
    """wx_add_layernorm against torch's fp32 `layer_norm(a + b)` (the encoder layer's residual
    step; torch's Welford vs two passes here: fp32 tolerance), the sum output equal to a + b,
    and a row-strided operand (a column slice of a wider buffer)."""
    from whisperx_amd import _lib

    torch.manual_seed(sum(shape))
    D = shape[-1]
    wide = torch.randn(*shape[:-1], D + 8, device="cuda") * 2 + 0.5
    a = wide[..., 4:4 + D] if shape[1] else torch.randn(shape, device="cuda")
    b = torch.randn(shape, device="cuda")
    ln = torch.nn.LayerNorm(D).cuda()
    with torch.no_grad():
        ln.weight.copy_(torch.randn(D) * 0.3 + 1)
        ln.bias.copy_(torch.randn(D) * 0.1)
        ref = ln(a + b)
    y, s = _lib.add_layernorm(a, b, ln.weight, ln.bias, ln.eps, want_sum=True)
    assert y.shape == tuple(shape) and y.is_contiguous()
    torch.testing.assert_close(y, ref, rtol=2e-5, atol=2e-5)
    assert torch.equal(s, a + b)
    torch.testing.assert_close(_lib.add_layernorm(a, b, ln.weight, ln.bias, ln.eps), ref, rtol=2e-5, atol=2e-5)


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


@pytest.mark.parametrize("split", [0, 1, 2, 4])
def test_attention_f32_packed_vs_fp64(split):
    """wx_attention_f32_packed: ragged segments packed by rows (lengths 1499, 37, 1, 0, 500, 64,
    33, 2999, as transformers' views of one fused [rows, 3 x H x 64] q/k/v projection), each
    segment attending only to its own rows, against a per-segment fp64 attention; every
    wave split, and the automatic choice."""
    from whisperx_amd import _lib

    torch.manual_seed(11 + split)
    H = 12
    lengths = [1499, 37, 1, 0, 500, 64, 33, 2999]
    segs = _lib.PackedSegments(lengths)
    R = segs.rows
    qkv = torch.randn(1, R, 3 * H * 64, device="cuda") * 2
    q, k, v = (qkv[..., i * H * 64:(i + 1) * H * 64].view(1, R, H, 64).transpose(1, 2) for i in range(3))
    got = _lib.attention_f32_packed(q, k, v, 0.125, segs, split)  # [1, R, H, 64]
    assert got.shape == (1, R, H, 64)
    for a, b in zip(segs.offsets[:-1], segs.offsets[1:]):
        if b == a:
            continue
        qd, kd, vd = (x[:, :, a:b].double() for x in (q, k, v))
        ref = (torch.softmax(qd @ kd.transpose(-1, -2) * 0.125, -1) @ vd).transpose(1, 2).float()
        torch.testing.assert_close(got[:, a:b], ref, rtol=1e-5, atol=2e-5, msg=f"segment rows [{a}, {b})")


@pytest.mark.parametrize("D,residual", [(768, True), (768, False), (1024, True)])
def test_posconv_packed_vs_torch(D, residual):
    """wx_posconv_packed (the positional conv embedding of every packed segment in one launch:
    grouped K = 128 conv with each segment's own zero padding, last output dropped, erf GELU,
    optionally + h) against transformers' Wav2Vec2PositionalConvEmbedding on each segment
    alone, fp32 tolerance; ragged lengths around the 128-frame tile and the 64-frame padding."""
    from transformers import Wav2Vec2Config
    from transformers.models.wav2vec2.modeling_wav2vec2 import Wav2Vec2PositionalConvEmbedding

    from whisperx_amd import _lib, emission

    torch.manual_seed(D + residual)
    cfg = Wav2Vec2Config(hidden_size=D, num_attention_heads=D // 64)
    pce = Wav2Vec2PositionalConvEmbedding(cfg).cuda().eval()
    pc = emission._posconv_weights(pce)
    assert pc is not None
    lengths = [1499, 1, 63, 64, 65, 200, 0, 128, 129, 2999]
    segs = _lib.PackedSegments(lengths)
    h = torch.randn(1, segs.rows, D, device="cuda")
    got = _lib.posconv_packed(h, pc[0], pc[1], pc[2], pc[3], segs, residual=residual)
    with torch.no_grad():
        for a, b in zip(segs.offsets[:-1], segs.offsets[1:]):
            if b == a:
                continue
            ref = pce(h[:, a:b])
            if residual:
                ref = ref + h[:, a:b]
            torch.testing.assert_close(got[:, a:b], ref, rtol=1e-4, atol=1e-4, msg=f"segment rows [{a}, {b})")


def _packed_vs_per_segment(m, V, lengths, tol=5e-5):
    """emission.packed_logits over ragged waveforms against the stock per-segment forward."""
    from whisperx_amd import _lib, alignment, emission

    rng = np.random.default_rng(sum(lengths))
    wavs = [torch.from_numpy(rng.standard_normal(n).astype(np.float32) * 0.1)[None].cuda() for n in lengths]
    with torch.inference_mode():
        ref = [torch.log_softmax(m(w if w.shape[-1] >= 400 else torch.nn.functional.pad(w, (0, 400 - w.shape[-1]))).logits,
                                 -1)[0] for w in wavs]
    streams = [torch.cuda.Stream() for _ in range(3)]
    worst = 0.0
    # the packed route runs the unprepared model from its weights (no patched forward)
    assert emission.packed_supported(m) and not getattr(m, "_wx_gemm_conv", False)
    Ts = [emission.n_frames(n, m) for n in lengths]
    with torch.inference_mode():
        got = torch.log_softmax(emission.packed_logits(m, wavs, _lib.PackedSegments(Ts), streams), -1)
    torch.cuda.synchronize()
    # and through _emissions (pack ranges, CSR rows, events)
    csr = alignment._emissions(m, "huggingface", wavs, "cuda:0", n_streams=3)
    assert isinstance(csr, alignment._EmissionsCSR) and csr.groups, "the packed route was not taken"
    main = torch.cuda.current_stream()
    for st in csr.streams:
        main.wait_stream(st)
    torch.cuda.synchronize()
    assert not any("forward" in mod.__dict__ for mod in m.modules()), "the packed route patched the model"
    off = np.cumsum([0] + Ts)
    for i, r in enumerate(ref):
        g = got[off[i]: off[i + 1]]
        assert g.shape == r.shape, (i, g.shape, r.shape)
        err = float((g - r).abs().max())
        worst = max(worst, err)
        assert err <= tol, f"segment {i} ({lengths[i]} samples): max |packed - stock| = {err}"
        assert torch.equal(g.argmax(-1), r.argmax(-1)), f"segment {i}: frame argmax differs"
        # (_emissions packs differently — its last pack's quarter runs alone — so its GEMM
        # tiling, and only that, may differ)
        err2 = float((csr[i] - r).abs().max())
        assert err2 <= tol, f"segment {i}: max |_emissions - stock| = {err2}"
        assert torch.equal(csr[i].argmax(-1), r.argmax(-1)), f"segment {i}: _emissions frame argmax differs"
    return worst


@pytest.mark.parametrize("fe", ["packed", "per_segment"])
def test_packed_encoder_matches_stock_base(fe, monkeypatch):
    """The packed encoder (all segments' rows in one transformer pass, attention per segment)
    on wav2vec2-base: 30 s, a < 400-sample segment (padded like alignment.py:217-224), 7.3 s,
    the 400-sample minimum and 1 s — each segment's log-probabilities equal its own stock
    forward's to fp32 tolerance with identical frame argmax.  The feature encoder either packed
    too (one GEMM per tap over the aligned sample buffer) or run per segment."""
    from transformers import Wav2Vec2Config, Wav2Vec2ForCTC

    if fe == "per_segment":
        monkeypatch.setenv("WX_NO_PACKED_FE", "1")
    torch.manual_seed(21)
    m = Wav2Vec2ForCTC(Wav2Vec2Config(vocab_size=32)).cuda().eval()
    worst = _packed_vs_per_segment(m, 32, [30 * 16000, 250, int(7.3 * 16000), 400, 16000])
    print(f"base packed vs stock: max |dlogp| = {worst:.3g}")


def test_packed_encoder_matches_stock_large_xlsr():
    """The same on the stable-layer-norm / layer-norm-feature-encoder family (8 layers of
    large-xlsr's width to keep the test short)."""
    from transformers import Wav2Vec2ForCTC

    torch.manual_seed(22)
    cfg = large_xlsr_config()
    cfg.num_hidden_layers = 8
    m = Wav2Vec2ForCTC(cfg).cuda().eval()
    worst = _packed_vs_per_segment(m, 40, [int(12.5 * 16000), 16000 + 7, 60 * 16000])
    print(f"large-xlsr packed vs stock: max |dlogp| = {worst:.3g}")


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


def test_emissions_fan_out_fresh_parametrised_model():
    """the positional conv's weight_norm weight is cached; on a freshly
    built model the cache must exist before the forwards fan out over 8 streams, or the
    streams read it before it is computed.  Segment 0 is much longer than the others (its
    stream would still be building the weight when the others reach the positional conv).
    Every segment's emission must equal a single-stream forward of the same model (to 1e-6
    through the per-segment route; to fp32 tolerance through the packed encoder, whose GEMMs
    tile differently)."""
    from transformers import Wav2Vec2Config, Wav2Vec2ForCTC

    from whisperx_amd import alignment, emission

    torch.manual_seed(2)
    m = Wav2Vec2ForCTC(Wav2Vec2Config(vocab_size=32)).cuda().eval()
    pos = m.wav2vec2.encoder.pos_conv_embed.conv
    assert getattr(pos, "parametrizations", None) is not None and pos not in emission._W_CACHE
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
            tol = 5e-5 if emission.packed_supported(m) else 1e-6
            assert err <= tol, f"segment {i}: fan-out emission differs from single-stream by {err}"
            assert torch.equal(csr[i].argmax(-1), ref.argmax(-1))
    emission.restore_model(m)


# --------------------------------------------------------------- torchaudio-shaped models
class _TAConvBlock(torch.nn.Module):
    """torchaudio's ConvLayerBlock shape: conv -> optional norm -> F.gelu, lengths tracked."""

    def __init__(self, cin, cout, k, s, norm):
        super().__init__()
        self.kernel_size, self.stride = k, s
        self.conv = torch.nn.Conv1d(cin, cout, k, s, bias=False)
        self.layer_norm = norm

    def forward(self, x, length):
        x = self.conv(x)
        if self.layer_norm is not None:
            x = self.layer_norm(x)
        x = torch.nn.functional.gelu(x)
        if length is not None:
            length = torch.clamp(torch.div(length - self.kernel_size, self.stride, rounding_mode="floor") + 1, min=0)
        return x, length


class _TAPosConv(torch.nn.Module):
    """torchaudio's ConvolutionalPositionalEmbedding: grouped weight-normed conv (dim=2),
    padding k // 2, the last frame dropped for an even kernel, GELU."""

    def __init__(self, d, k, groups, parametrized):
        super().__init__()
        conv = torch.nn.Conv1d(d, d, k, padding=k // 2, groups=groups)
        if parametrized:
            conv = torch.nn.utils.parametrizations.weight_norm(conv, name="weight", dim=2)
        else:
            conv = torch.nn.utils.weight_norm(conv, name="weight", dim=2)  # the older hook form
        self.conv = conv
        self.num_remove = 1 if k % 2 == 0 else 0

    def forward(self, x):
        x = self.conv(x.transpose(-2, -1))
        if self.num_remove > 0:
            x = x[..., : -self.num_remove]
        return torch.nn.functional.gelu(x).transpose(-2, -1)


class _TAWav2Vec2(torch.nn.Module):
    """A torchaudio-bundle-shaped wav2vec2 (WAV2VEC2_ASR_BASE_960H layout at reduced depth):
    feature_extractor(ConvLayerBlocks) -> projection -> positional conv -> transformer layers
    -> aux head; forward(x, lengths) -> (emissions, lengths) as alignment.py:227-228 calls it."""

    def __init__(self, V=29, d=768, layers=2, parametrized=True):
        super().__init__()
        shapes = [(1, 512, 10, 5)] + [(512, 512, 3, 2)] * 4 + [(512, 512, 2, 2)] * 2
        self.feature_extractor = torch.nn.ModuleList(
            [_TAConvBlock(ci, co, k, s, torch.nn.GroupNorm(512, 512) if i == 0 else None)
             for i, (ci, co, k, s) in enumerate(shapes)])
        self.proj_norm = torch.nn.LayerNorm(512)
        self.proj = torch.nn.Linear(512, d)
        self.pos_conv = _TAPosConv(d, 128, 16, parametrized)
        self.norm = torch.nn.LayerNorm(d)
        self.layers = torch.nn.ModuleList(
            [torch.nn.TransformerEncoderLayer(d, 12, 3072, dropout=0.0, activation="gelu", batch_first=True)
             for _ in range(layers)])
        self.aux = torch.nn.Linear(d, V)

    def forward(self, x, lengths=None):
        x = x.unsqueeze(1)
        for blk in self.feature_extractor:
            x, lengths = blk(x, lengths)
        x = self.proj(self.proj_norm(x.transpose(1, 2)))
        x = self.norm(x + self.pos_conv(x))
        for layer in self.layers:
            x = layer(x)
        return self.aux(x), lengths


@pytest.mark.parametrize("parametrized", [True, False])
def test_torchaudio_shaped_model_prepared_vs_stock(parametrized):
    """alignment.py:227-228's torchaudio branch through the emission route: a stand-in with
    torchaudio's module layout (ConvLayerBlock convs, weight-norm positional conv in both the
    parametrisation and the older hook form, aux head, (emissions, lengths) output) gives the
    same log-probabilities as its unprepared forward (<= 5e-5, identical frame argmax), for a
    < 400-sample segment (padded, lengths passed) too.  torchaudio itself is absent here, so
    parity with the real bundles is unpinned."""
    from whisperx_amd import alignment, emission

    torch.manual_seed(5)
    m = _TAWav2Vec2(parametrized=parametrized).cuda().eval()
    g = torch.Generator().manual_seed(6)
    wavs = [(torch.randn(1, n, generator=g) * 0.1).cuda() for n in (30 * 16000, 123457, 300, 400)]
    with torch.inference_mode():
        ref = [torch.log_softmax(alignment._logits(m, "torchaudio", w, "cuda:0"), -1)[0] for w in wavs]
    with emission.prepared(m):
        csr = alignment._emissions(m, "torchaudio", wavs, "cuda:0", n_streams=4)
        assert isinstance(csr, alignment._EmissionsCSR), "the torchaudio branch left the packed emission route"
        main = torch.cuda.current_stream()
        for st in csr.streams:
            main.wait_stream(st)
        torch.cuda.synchronize()
        got = [csr[i].clone() for i in range(len(wavs))]
        assert any("forward" in mod.__dict__ for mod in m.modules()), "no convolution took the GEMM route"
    for i, (a, b) in enumerate(zip(got, ref)):
        assert a.shape == b.shape, (i, a.shape, b.shape)
        err = float((a - b).abs().max())
        assert err <= 5e-5, f"segment {i}: max |prepared - stock| = {err}"
        assert torch.equal(a.argmax(-1), b.argmax(-1)), f"segment {i}: frame argmax differs"
    # the caller's model is unchanged afterwards
    assert not any("forward" in mod.__dict__ or hasattr(mod, "_wx_w_cache") for mod in m.modules())


def test_align_leaves_callers_model_unchanged():
    """align() prepares the model for the call only (alignment.py:226-233 takes the caller's
    model and leaves it alone): afterwards no instance-level forwards, no cached weights, the
    original attention implementation, identical state_dict, and the stock forward's output."""
    from transformers import Wav2Vec2Config, Wav2Vec2ForCTC

    from whisperx_amd import align

    torch.manual_seed(7)
    m = Wav2Vec2ForCTC(Wav2Vec2Config(vocab_size=32, num_hidden_layers=2)).cuda().eval()
    attn0 = m.config._attn_implementation
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    x = (torch.randn(1, 5 * 16000, generator=torch.Generator().manual_seed(8)) * 0.1).cuda()
    with torch.inference_mode():
        y0 = m(x).logits.clone()
    letters = "abcdefghijklmnopqrstuvwxyz"
    dictionary = {c: i + 4 for i, c in enumerate(letters)}
    dictionary.update({"<pad>": 0, "|": 1})
    segs = [{"start": 0.0, "end": 2.5, "text": "hello world"}, {"start": 2.5, "end": 5.0, "text": "again here"}]
    out = align(segs, m, {"language": "en", "dictionary": dictionary, "type": "huggingface"}, x[0], "cuda:0")
    assert len(out["segments"]) == 2
    assert m.config._attn_implementation == attn0
    assert not any("forward" in mod.__dict__ or hasattr(mod, "_wx_w_cache") or hasattr(mod, "_wx_orig_forward")
                   for mod in m.modules())
    assert not hasattr(m, "_wx_gemm_conv") and not hasattr(m, "_wx_orig_attn")
    sd1 = m.state_dict()
    assert sd0.keys() == sd1.keys() and all(torch.equal(sd0[k], sd1[k]) for k in sd0)
    with torch.inference_mode():
        assert torch.equal(m(x).logits, y0)


@pytest.mark.gpu
def test_align_packed_value_error_redoes_call_on_prepared_route(monkeypatch):
    """When emission.packed_logits raises ValueError (a frame geometry n_frames does not
    predict), align() joins what the packs queued, enters emission.prepared() and redoes the
    emissions per segment: same words as the packed route (times within one 20 ms frame) and the
    caller's model unchanged afterwards."""
    from transformers import Wav2Vec2Config, Wav2Vec2ForCTC

    from whisperx_amd import align, emission

    torch.manual_seed(11)
    m = Wav2Vec2ForCTC(Wav2Vec2Config(vocab_size=32, num_hidden_layers=2)).cuda().eval()
    x = (torch.randn(1, 6 * 16000, generator=torch.Generator().manual_seed(12)) * 0.1).cuda()
    letters = "abcdefghijklmnopqrstuvwxyz"
    dictionary = {c: i + 4 for i, c in enumerate(letters)}
    dictionary.update({"<pad>": 0, "|": 1})
    meta = {"language": "en", "dictionary": dictionary, "type": "huggingface"}

    def segs():
        return [{"start": 0.0, "end": 2.0, "text": "hello world"},
                {"start": 2.0, "end": 4.5, "text": "again here"},
                {"start": 4.5, "end": 6.0, "text": "last one"}]

    assert emission.packed_supported(m)
    ref = align(segs(), m, meta, x[0], "cuda:0")
    calls = []

    def refuse(*a, **k):
        calls.append(1)
        raise ValueError("frame geometry")

    entered = []
    prepared = emission.prepared

    def spy(model):
        entered.append(model)
        return prepared(model)

    monkeypatch.setattr(emission, "packed_logits", refuse)
    monkeypatch.setattr(emission, "prepared", spy)
    got = align(segs(), m, meta, x[0], "cuda:0")
    assert calls, "the packed route was not taken"
    assert entered == [m], "the per-segment redo did not run on the prepared model"
    assert len(got["word_segments"]) == len(ref["word_segments"]) == 6
    for a, b in zip(got["word_segments"], ref["word_segments"]):
        assert a["word"] == b["word"]
        assert abs(a["start"] - b["start"]) <= 0.0201 and abs(a["end"] - b["end"]) <= 0.0201, (a, b)
    assert not any("forward" in mod.__dict__ or hasattr(mod, "_wx_w_cache") or hasattr(mod, "_wx_orig_forward")
                   for mod in m.modules())
    assert not hasattr(m, "_wx_gemm_conv") and not hasattr(m, "_wx_orig_attn")
