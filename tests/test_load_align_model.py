"""load_align_model (alignment.py:64-97) on a locally saved random-weight Wav2Vec2ForCTC +
tokenizer directory: the offline Hugging Face branch (no hub access here or on the GPU box)."""
import json
import os

import pytest
import torch


def _save_local_model(d):
    from transformers import (Wav2Vec2Config, Wav2Vec2CTCTokenizer, Wav2Vec2FeatureExtractor, Wav2Vec2ForCTC,
                              Wav2Vec2Processor)

    from whisperx_amd.synthetic import W2V_VOCAB

    vocab = {c: i for i, c in enumerate(W2V_VOCAB)}
    with open(os.path.join(d, "vocab.json"), "w") as f:
        json.dump(vocab, f)
    tok = Wav2Vec2CTCTokenizer(os.path.join(d, "vocab.json"), unk_token="<unk>", pad_token="<pad>",
                               word_delimiter_token="|")
    fe = Wav2Vec2FeatureExtractor(feature_size=1, sampling_rate=16000, padding_value=0.0, do_normalize=True,
                                  return_attention_mask=False)
    Wav2Vec2Processor(feature_extractor=fe, tokenizer=tok).save_pretrained(d)
    torch.manual_seed(0)
    cfg = Wav2Vec2Config(vocab_size=len(vocab), hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                         intermediate_size=128, conv_dim=(32,) * 7, num_conv_pos_embeddings=16,
                         num_conv_pos_embedding_groups=2)
    Wav2Vec2ForCTC(cfg).save_pretrained(d)
    return vocab


def test_load_align_model_local_directory(tmp_path):
    from whisperx_amd import load_align_model

    vocab = _save_local_model(str(tmp_path))
    model, meta = load_align_model("en", "cpu", model_name=str(tmp_path))
    assert meta["language"] == "en" and meta["type"] == "huggingface"
    assert meta["dictionary"] == {c.lower(): i for c, i in vocab.items()}
    assert model.lm_head.out_features == len(vocab)
    with torch.inference_mode():
        lg = model(torch.zeros(1, 16000)).logits
    assert lg.shape == (1, 49, len(vocab))


def test_load_align_model_unknown_language_and_model(tmp_path, capsys):
    from whisperx_amd import load_align_model

    with pytest.raises(ValueError, match="No default align-model for language: xx"):
        load_align_model("xx", "cpu")
    with pytest.raises(ValueError, match="could not be found in huggingface"):
        load_align_model("en", "cpu", model_name=str(tmp_path / "missing"))
