"""CLIP ViT-L/14 text tower (SD1.5 encoder_hidden_states producer)
on the HIP kernels: per layer LN kernel -> fused QKV GEMM -> causal short-sequence
attention (c2d_attention_small) -> out-proj GEMM + residual epilogue -> LN -> fc1 GEMM
with the quick_gelu epilogue -> fc2 GEMM + residual; final LN.  Semantics of
transformers CLIPTextModel (modeling_clip.py CLIPTextTransformer), which the SD1.5
pipeline the reference drives loads (scripts/inference.py:30-33).

No tokenizer vocabulary or weights exist offline, so prompts map to fixed,
deterministic token-id lists (BOS, per-word ids from a stable hash, EOS, EOS
padding to 77 as in SD1.5) and the tower is randomly initialised from a seed
(the SD1.5 architecture: 12 layers, width 768, 12 heads, quick_gelu).
"""
from __future__ import annotations

import zlib

import torch

from . import ops
from .layers import HLinear

BOS, EOS, VOCAB, MAXLEN = 49406, 49407, 49408, 77


def prompt_to_ids(prompt: str) -> list[int]:
    ids = [BOS]
    for w in prompt.lower().replace(",", " ").split():
        ids.append(256 + zlib.crc32(w.encode()) % (VOCAB - 512))
    ids = ids[:MAXLEN - 1] + [EOS]
    return ids + [EOS] * (MAXLEN - len(ids))


def tokenize(prompts: list[str], device=None) -> torch.Tensor:
    return torch.tensor([prompt_to_ids(p) for p in prompts], dtype=torch.long, device=device)


def clip_text_model(seed: int = 0):
    """The seeded random-init transformers CLIPTextModel (fp32, CPU): the weight source
    of TextEncoder and, in tests, its fp32 oracle."""
    from transformers import CLIPTextConfig, CLIPTextModel
    cfg = CLIPTextConfig(vocab_size=VOCAB, hidden_size=768, intermediate_size=3072, num_hidden_layers=12,
                         num_attention_heads=12, max_position_embeddings=MAXLEN, hidden_act="quick_gelu",
                         projection_dim=768)
    with torch.random.fork_rng(devices=[]):
        torch.manual_seed(seed)
        return CLIPTextModel(cfg).eval()


class TextEncoder:
    HEADS, D = 12, 64

    def __init__(self, device, seed: int = 0, model=None):
        m = model or clip_text_model(seed)
        m = getattr(m, "text_model", m)  # transformers < 5 wraps the tower
        dev = torch.device(device)
        self.device = dev
        f32 = lambda t: t.detach().float().contiguous().to(dev)  # noqa: E731
        self.tok = m.embeddings.token_embedding.weight.detach().half().to(dev)
        self.pos = m.embeddings.position_embedding.weight.detach().half().to(dev)
        self.layers = []
        for lyr in m.encoder.layers:
            a = lyr.self_attn
            qkv = HLinear(768, 2304)
            qkv.load(torch.cat([a.q_proj.weight, a.k_proj.weight, a.v_proj.weight]).detach(),
                     torch.cat([a.q_proj.bias, a.k_proj.bias, a.v_proj.bias]).detach())
            out, fc1, fc2 = HLinear(768, 768), HLinear(768, 3072), HLinear(3072, 768)
            out.load(a.out_proj.weight.detach(), a.out_proj.bias.detach())
            fc1.load(lyr.mlp.fc1.weight.detach(), lyr.mlp.fc1.bias.detach())
            fc2.load(lyr.mlp.fc2.weight.detach(), lyr.mlp.fc2.bias.detach())
            self.layers.append(dict(
                ln1=(f32(lyr.layer_norm1.weight), f32(lyr.layer_norm1.bias)),
                ln2=(f32(lyr.layer_norm2.weight), f32(lyr.layer_norm2.bias)),
                qkv=qkv.to(dev), out=out.to(dev), fc1=fc1.to(dev), fc2=fc2.to(dev)))
        self.lnf = (f32(m.final_layer_norm.weight), f32(m.final_layer_norm.bias))
        self.eps = m.final_layer_norm.eps

    @torch.no_grad()
    def __call__(self, ids: torch.Tensor) -> torch.Tensor:
        """ids [N, 77] -> last_hidden_state [N, 77, 768] fp16."""
        n, l = ids.shape
        x = (self.tok[ids.to(self.device)] + self.pos[:l]).reshape(n * l, 768).contiguous()
        c = 768
        for p in self.layers:
            h = ops.layer_norm(x, *p["ln1"], self.eps)
            qkv = p["qkv"](h)
            a = ops.attention_small(qkv[:, :c], qkv[:, c:2 * c], qkv[:, 2 * c:], n, self.HEADS, l, self.D,
                                    causal=True)
            x = p["out"](a, resid=x)
            h = ops.layer_norm(x, *p["ln2"], self.eps)
            x = p["fc2"](p["fc1"](h, act="quick_gelu"), resid=x)
        return ops.layer_norm(x, *self.lnf, self.eps).view(n, l, c)
