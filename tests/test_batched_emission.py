"""emission.batched_logits' host logic on the CPU: the ragged batched wav2vec2 forward (per
segment feature encoder and positional conv, row-wise ops over the concatenated frames,
per-segment attention) against each segment's own unpadded HF forward, for the post-norm
(wav2vec2-base) and the stable-layer-norm (large-xlsr) encoders.  The attention kernel itself
(wx_attention_f32_csr) is replaced by an fp32 torch attention here; it is tested on the GPU
(tests/test_gpu_emission.py)."""
import pytest
import torch


def _torch_attention_csr(q, k, v, Ts, scale):
    out, o = [], 0
    for t in Ts:
        qs, ks, vs = (x[o:o + t].transpose(0, 1) for x in (q, k, v))  # [H, t, 64]
        p = torch.softmax(qs @ ks.transpose(-1, -2) * scale, -1)
        out.append((p @ vs).transpose(0, 1))
        o += t
    return torch.cat(out, 0)


@pytest.mark.parametrize("stable", [False, True])
def test_batched_logits_match_per_segment_forward(monkeypatch, stable):
    from transformers import Wav2Vec2Config, Wav2Vec2ForCTC

    from whisperx_amd import _lib, emission

    monkeypatch.setattr(_lib, "attention_f32_csr", _torch_attention_csr)
    monkeypatch.setenv("WX_EMISSION_BATCH", "8")
    torch.manual_seed(0)
    if stable:
        cfg = Wav2Vec2Config(vocab_size=40, num_hidden_layers=2, hidden_size=256, num_attention_heads=4,
                             intermediate_size=512, feat_extract_norm="layer", do_stable_layer_norm=True, conv_bias=True)
    else:
        cfg = Wav2Vec2Config(vocab_size=32, num_hidden_layers=2, hidden_size=256, num_attention_heads=4,
                             intermediate_size=512)
    m = Wav2Vec2ForCTC(cfg).eval()
    assert emission.batchable(m)
    wavs = [torch.randn(n) * 0.1 for n in (16000, 400, 23456)]
    got = emission.batched_logits(m, wavs)
    with torch.no_grad():
        for w, g in zip(wavs, got):
            ref = m(w.reshape(1, -1)).logits[0]
            assert g.shape == ref.shape
            torch.testing.assert_close(g, ref, rtol=1e-4, atol=1e-5)
