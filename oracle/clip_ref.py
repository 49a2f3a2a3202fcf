"""CLIP text tower oracle -- TEST INFRASTRUCTURE ONLY (fp32, CPU).

transformers' own CLIPTextModel (the SD1.5 text encoder the reference's pipeline
loads, scripts/inference.py:30-33; modeling_clip.py CLIPTextTransformer) with the
product's seeded weights (clap2diffusion_amd.weights.synth_clip_text) loaded into
it, so the HIP TextEncoder and the oracle share one state dict.
"""
from __future__ import annotations

import torch

from clap2diffusion_amd import weights as W


def clip_text_model(seed: int = 0):
    from transformers import CLIPTextConfig, CLIPTextModel
    c = W.CLIP_TEXT_CFG
    cfg = CLIPTextConfig(vocab_size=c["vocab"], hidden_size=c["width"], intermediate_size=c["mlp"],
                         num_hidden_layers=c["layers"], num_attention_heads=c["heads"],
                         max_position_embeddings=c["max_len"], hidden_act="quick_gelu", projection_dim=768)
    m = CLIPTextModel(cfg).eval()
    sd = W.synth_clip_text(seed)
    have = set(m.state_dict().keys())
    if not any(k.startswith("text_model.") for k in have):   # transformers >= 5 drops the wrapper
        sd = {k[len("text_model."):]: v for k, v in sd.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected and all("position_ids" in k for k in missing), (missing, unexpected)
    return m


@torch.no_grad()
def encode(ids: torch.Tensor, seed: int = 0, model=None) -> torch.Tensor:
    """ids [N, 77] -> last_hidden_state [N, 77, 768] fp32."""
    m = model or clip_text_model(seed)
    return m(input_ids=ids.cpu()).last_hidden_state.float()
