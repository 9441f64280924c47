"""Emission producer kernels and routes (-m gpu): the time-major GroupNorm+GELU kernel
against torch's fp32 GroupNorm + GELU, and the prepared (GEMM-conv + fused-norm) wav2vec2
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


def test_prepared_wav2vec2_forward_matches_stock():
    from transformers import Wav2Vec2Config, Wav2Vec2ForCTC

    from whisperx_amd import emission

    torch.manual_seed(0)
    m = Wav2Vec2ForCTC(Wav2Vec2Config(vocab_size=32)).cuda().eval()
    rng = np.random.default_rng(0)
    for n in (400, 7 * 16000 + 123, 30 * 16000):
        x = torch.from_numpy(rng.standard_normal(n).astype(np.float32) * 0.1)[None].cuda()
        with torch.inference_mode():
            ref = torch.log_softmax(m(x).logits, -1)
            emission.prepare_model(m)
            got = torch.log_softmax(m(x).logits, -1)
            emission.restore_model(m)
        assert got.shape == ref.shape == (1, emission.n_frames(n), 32)
        assert float((got - ref).abs().max()) < 5e-5
        assert torch.equal(got.argmax(-1), ref.argmax(-1))
