"""CLIP ViT-L/14 text tower (SD1.5 encoder_hidden_states producer)
on the HIP kernels: per layer LN kernel -> fused QKV GEMM -> causal short-sequence
attention (c2d_attention_small) -> out-proj GEMM + residual epilogue -> LN -> fc1 GEMM
with the quick_gelu epilogue -> fc2 GEMM + residual; final LN.  Semantics of
transformers CLIPTextModel (modeling_clip.py CLIPTextTransformer), which the SD1.5
pipeline the reference drives loads (scripts/inference.py:30-33).

Prompts become token ids through the SD1.5 folder's CLIP BPE tokenizer (tokenizer/vocab.json +
merges.txt; clap2diffusion_amd/tokenizer.py) when one is given (make_tokenizer); with no
vocabulary offline they map to fixed, deterministic token-id lists instead (BOS, per-word ids
from a stable hash, EOS, EOS padding to 77 as in SD1.5).  The tower loads a CLIPTextModel-keyed state dict,
by default the seeded recipe weights.synth_clip_text (the SD1.5 architecture:
12 layers, width 768, 12 heads, quick_gelu).  The product never imports
transformers; the tests load the same state dict into transformers'
CLIPTextModel as the fp32 oracle (oracle/clip_ref.py).
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
    """The offline fallback: hash ids (prompt_to_ids), [B, 77]."""
    return torch.tensor([prompt_to_ids(p) for p in prompts], dtype=torch.long, device=device)


def make_tokenizer(sd_model_path=None):
    """prompts, device -> [B, 77] token ids: the CLIP BPE tokenizer of an SD1.5 diffusers
    folder (its tokenizer/ subfolder, or the folder itself) when it holds vocab.json and
    merges.txt, else the hash-id fallback `tokenize`."""
    if sd_model_path is not None:
        from pathlib import Path
        from .tokenizer import CLIPBPETokenizer
        for d in (Path(sd_model_path) / "tokenizer", Path(sd_model_path)):
            if (d / "vocab.json").exists() and (d / "merges.txt").exists():
                return CLIPBPETokenizer.from_folder(d)
    return tokenize


class TextEncoder:
    HEADS, D = 12, 64

    def __init__(self, device, seed: int = 0, state_dict: dict | None = None):
        """Weights from a CLIPTextModel state dict (SD1.5 text_encoder keys, with or without
        the "text_model." prefix); default: the seeded recipe weights.synth_clip_text(seed)."""
        from .weights import synth_clip_text
        sd = state_dict if state_dict is not None else synth_clip_text(seed)
        sd = {(k[len("text_model."):] if k.startswith("text_model.") else k): v for k, v in sd.items()}
        dev = torch.device(device)
        self.device = dev
        f32 = lambda k: sd[k].detach().float().contiguous().to(dev)  # noqa: E731
        self.tok = sd["embeddings.token_embedding.weight"].detach().half().to(dev)
        self.pos = sd["embeddings.position_embedding.weight"].detach().half().to(dev)
        self.layers = []
        n_layers = 1 + max(int(k.split(".")[2]) for k in sd if k.startswith("encoder.layers."))
        for i in range(n_layers):
            b = f"encoder.layers.{i}."
            a = b + "self_attn."
            qkv = HLinear(768, 2304)
            qkv.load(torch.cat([sd[a + "q_proj.weight"], sd[a + "k_proj.weight"], sd[a + "v_proj.weight"]]).float(),
                     torch.cat([sd[a + "q_proj.bias"], sd[a + "k_proj.bias"], sd[a + "v_proj.bias"]]).float())
            out, fc1, fc2 = HLinear(768, 768), HLinear(768, 3072), HLinear(3072, 768)
            out.load(sd[a + "out_proj.weight"].float(), sd[a + "out_proj.bias"].float())
            fc1.load(sd[b + "mlp.fc1.weight"].float(), sd[b + "mlp.fc1.bias"].float())
            fc2.load(sd[b + "mlp.fc2.weight"].float(), sd[b + "mlp.fc2.bias"].float())
            self.layers.append(dict(
                ln1=(f32(b + "layer_norm1.weight"), f32(b + "layer_norm1.bias")),
                ln2=(f32(b + "layer_norm2.weight"), f32(b + "layer_norm2.bias")),
                qkv=qkv.to(dev), out=out.to(dev), fc1=fc1.to(dev), fc2=fc2.to(dev)))
        self.lnf = (f32("final_layer_norm.weight"), f32("final_layer_norm.bias"))
        self.eps = 1e-5   # CLIPTextConfig.layer_norm_eps

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
