"""CLIP ViT-L/14 text tower (SD1.5 encoder_hidden_states producer) — out of the
north-star scope: runs once per prompt in PyTorch-ROCm.

No tokenizer vocabulary or weights exist offline, so prompts map to fixed,
deterministic token-id lists (BOS, per-word ids from a stable hash, EOS, EOS
padding to 77 as in SD1.5) and the tower is randomly initialised from a seed
(the SD1.5 architecture: 12 layers, width 768, 12 heads, quick_gelu).
"""
from __future__ import annotations

import zlib

import torch

BOS, EOS, VOCAB, MAXLEN = 49406, 49407, 49408, 77


def prompt_to_ids(prompt: str) -> list[int]:
    ids = [BOS]
    for w in prompt.lower().replace(",", " ").split():
        ids.append(256 + zlib.crc32(w.encode()) % (VOCAB - 512))
    ids = ids[:MAXLEN - 1] + [EOS]
    return ids + [EOS] * (MAXLEN - len(ids))


def tokenize(prompts: list[str], device=None) -> torch.Tensor:
    return torch.tensor([prompt_to_ids(p) for p in prompts], dtype=torch.long, device=device)


class TextEncoder:
    def __init__(self, device, seed: int = 0, dtype=torch.float16):
        from transformers import CLIPTextConfig, CLIPTextModel
        cfg = CLIPTextConfig(vocab_size=VOCAB, hidden_size=768, intermediate_size=3072, num_hidden_layers=12,
                             num_attention_heads=12, max_position_embeddings=MAXLEN, hidden_act="quick_gelu",
                             projection_dim=768)
        with torch.random.fork_rng(devices=[]):
            torch.manual_seed(seed)
            self.model = CLIPTextModel(cfg).eval()
        self.model = self.model.to(device=device, dtype=dtype)
        self.device = device

    @torch.no_grad()
    def __call__(self, ids: torch.Tensor) -> torch.Tensor:
        """ids [N, 77] -> last_hidden_state [N, 77, 768] fp16."""
        return self.model(input_ids=ids.to(self.device)).last_hidden_state.to(torch.float16).contiguous()
