"""Attention-processor plugin API on the HIP kernels.

Mirrors the reference plugin surface (models/audio_attention_processor.py):
  AudioAttnProcessor(level, audio_dim=768, hidden_dim=768, mode="add",
                     dropout=0.1, bottleneck_dim=64)              (:13-41)
  processor(attn, hidden_states, encoder_hidden_states=None,
            attention_mask=None, temb=None, scale=1.0, **cross_attention_kwargs)  (:43-52)
  AudioProcessorManager(unet): _create_level_mapping / setup_processors /
            get_audio_kwargs                                      (:148-267)
registered through unet.attn_processors / unet.set_attn_processor, audio passed
as cross_attention_kwargs={'audio': {'early'|'mid'|'late': [B, K, 768]}}.

Processors are nn.Modules with the reference parameter names (audio_proj.0,
audio_proj.3, alpha) so reference state dicts load unchanged.  Every processor
here accepts and ignores unknown kwargs, including on attn1.
The compute runs on libc2d_hip.so: fused-QKV / KV GEMMs, the flash attention
kernel, the out-projection with the block residual fused into its epilogue.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops


def _as_tokens(x: torch.Tensor):
    """[B, L, C] token matrix (fp16, contiguous) of the hidden states, and the map back to the
    caller's form: 4-D [B, C, H, W] input is viewed as [B, H*W, C] and the output transposed
    back (reference :67-70, :137-138); a non-fp16 input gets its output in its own dtype."""
    restore = None
    if x.dim() == 4:
        b, c, hh, ww = x.shape
        dt = x.dtype
        x = x.reshape(b, c, hh * ww).transpose(1, 2)

        def restore(o, b=b, c=c, hh=hh, ww=ww, dt=dt):
            return o.transpose(-1, -2).reshape(b, c, hh, ww).to(dt)
    elif x.dim() == 3:
        if x.dtype != torch.float16:
            dt = x.dtype

            def restore(o, dt=dt):
                return o.to(dt)
    else:
        raise ValueError(f"attention processors take [B, L, C] or [B, C, H, W] hidden states, got {tuple(x.shape)}")
    x = x.to(torch.float16)
    return (x if x.is_contiguous() else x.contiguous()), restore


def key_bias_of(attention_mask: Optional[torch.Tensor], batch: int, heads: int, lk: int,
                lq: int = 1) -> Optional[torch.Tensor]:
    """attention_mask (additive, as Attention.get_attention_scores adds it to q k^T * scale:
    reference :129) -> the score bias c2d_attention_fwd_mask takes, fp32 [B|1, H|1, Lq|1, lk].
    Accepted: what broadcasts to the [B*H, Lq, Lk] scores the reference's baddbmm forms --
    [lk], [Lq|1, lk], [B*H | 1, Lq|1, lk] -- plus the per-image forms [B, Lq|1, lk] (the UNet's
    encoder_attention_mask bias) and 4-D [B|1, H|1, Lq|1, lk]; masks varying over queries
    included.  Any other shape raises, as the reference's broadcasting would."""
    if attention_mask is None:
        return None
    m = attention_mask
    if m.shape[-1] != lk:
        raise ValueError(f"attention_mask last dim {m.shape[-1]} != number of keys {lk}")
    if m.dim() == 4:
        if m.shape[0] not in (1, batch) or m.shape[1] not in (1, heads) or m.shape[2] not in (1, lq):
            raise ValueError(f"4-D attention_mask {tuple(m.shape)} does not broadcast to [{batch}, {heads}, {lq}, {lk}]")
        return m.float()
    if m.dim() == 1:
        m = m.view(1, 1, lk)
    elif m.dim() == 2:
        m = m.view(1, m.shape[0], lk)
    if m.dim() != 3:
        raise ValueError(f"attention_mask of shape {tuple(attention_mask.shape)} is not supported")
    x, q = m.shape[0], m.shape[1]
    if q not in (1, lq):
        raise ValueError(f"attention_mask query dim {q} matches neither 1 nor Lq={lq}")
    if x == batch * heads and heads > 1:
        return m.reshape(batch, heads, q, lk).float()
    if x in (batch, 1):
        return m.reshape(x, 1, q, lk).float()
    raise ValueError(f"attention_mask batch dim {x} matches neither B*heads={batch * heads}, B={batch} nor 1")


class AttnProcessor(nn.Module):
    """Default processor (stock diffusers AttnProcessor semantics) on HIP.
    Self-attention uses the fused [to_q; to_k; to_v] weight of the layer."""

    fuses_residual = True

    def __call__(self, attn, hidden_states, encoder_hidden_states=None, attention_mask=None, temb=None,
                 scale: float = 1.0, _residual: Optional[torch.Tensor] = None, _qkv: Optional[torch.Tensor] = None,
                 _q: Optional[torch.Tensor] = None, **cross_attention_kwargs):
        """_qkv / _q: the self-attention's [B*L, 3*inner] / the cross-attention's [B*L, inner]
        projections already computed by the caller (BasicTransformerBlock: norm1 / norm2 folded into
        the GEMM); hidden_states then only gives the shape."""
        x, restore = _as_tokens(hidden_states)
        b, l, c = x.shape
        x2 = x.view(b * l, c)
        heads, d = attn.heads, attn.dim_head
        inner = heads * d
        if encoder_hidden_states is None:
            qkv = _qkv if _qkv is not None else ops.conv(x2, attn.w_qkv, attn.kpad_q, 3 * inner, ksize=1)
            if scale != 1.0:
                qkv[:, :inner].mul_(scale)
            o = ops.attention(qkv[:, :inner], qkv[:, inner:2 * inner], qkv[:, 2 * inner:], b, heads, l, l, d,
                              key_bias=key_bias_of(attention_mask, b, heads, l, l))
        else:
            cache = cross_attention_kwargs.get("context_kv")
            kv = cache.get(attn) if cache is not None else None
            if kv is None:
                kv = AttnProcessor.context_kv(self, attn, encoder_hidden_states)
            lk = kv.shape[0] // b
            q = _q if _q is not None else ops.conv(x2, attn.to_q.weight, attn.kpad_q, inner, ksize=1)
            if scale != 1.0:
                q.mul_(scale)
            o = ops.attention(q, kv[:, :inner], kv[:, inner:], b, heads, l, lk, d,
                              key_bias=key_bias_of(attention_mask, b, heads, lk, l))
        return _project_out(attn, o, b, l, c, _residual, restore)

    def context_kv(self, attn, encoder_hidden_states: torch.Tensor, audio: Optional[dict] = None,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """K|V = context @ [W_k; W_v]^T, [B*Lk, 2*inner] fp16 (loop-invariant across denoise steps)."""
        ehs, _ = _as_tokens(encoder_hidden_states.to(torch.float16))
        inner = attn.heads * attn.dim_head
        kv = ops.conv(ehs.reshape(-1, ehs.shape[-1]), attn.w_kv, attn.kpad_kv, 2 * inner, ksize=1, out=out)
        return kv


class AudioAttnProcessor(nn.Module):
    """Audio-injecting cross-attention processor (reference :13-145) on HIP.

    mode "add" (Add-FiLM, default):  ctx' = ctx + sigmoid(alpha) * mean_K(audio_proj(audio[level]))
    mode "concat": ctx' = cat(ctx, adaptive_avg_pool(audio_proj(audio[level]), <= 4 tokens))
    then q = to_q(h) * scale, k, v = to_k/to_v(ctx'), softmax(q k^T / sqrt(d)) v, to_out.

    Add-FiLM is evaluated by linearity without materialising ctx':
    K|V = ctx W_kv^T + [sigmoid(alpha) * pooled] W_kv^T, the second term entering
    the KV GEMM epilogue as a per-image row vector (the kernel's temb input).
    """

    fuses_residual = True

    def __init__(self, level: str, audio_dim: int = 768, hidden_dim: int = 768, mode: str = "add",
                 dropout: float = 0.1, bottleneck_dim: int = 64):
        super().__init__()
        self.level = level
        self.mode = mode
        self.audio_proj = nn.Sequential(
            nn.Linear(audio_dim, bottleneck_dim), nn.GELU(), nn.Dropout(dropout), nn.Linear(bottleneck_dim, hidden_dim))
        self.alpha = nn.Parameter(torch.zeros(1))
        self._packed = None
        self._packed_key = None

    def _pack(self, device):
        key = tuple((p.data_ptr(), p._version) for p in self.parameters()) + (str(device),)
        if self._packed_key != key:
            l1, l2 = self.audio_proj[0], self.audio_proj[3]
            w1, k1 = ops.pack_linear_weight(l1.weight.detach().float())
            w2, k2 = ops.pack_linear_weight(l2.weight.detach().float())
            self._packed = dict(w1=w1.to(device), k1=k1, b1=l1.bias.detach().float().to(device).contiguous(),
                                w2=w2.to(device), k2=k2, b2=l2.bias.detach().float().to(device).contiguous(),
                                n1=l1.out_features, n2=l2.out_features)
            self._packed_key = key
        return self._packed

    def project_audio(self, audio_tokens: torch.Tensor) -> torch.Tensor:
        """audio_proj (Linear, GELU, Dropout(eval), Linear) on the GEMM kernel -> [B, K, hidden] fp16."""
        pk = self._pack(audio_tokens.device)
        b, k, dim = audio_tokens.shape
        a = audio_tokens.reshape(b * k, dim).to(torch.float16).contiguous()
        a = ops.conv(a, pk["w1"], pk["k1"], pk["n1"], ksize=1, bias=pk["b1"], act="gelu")
        a = ops.conv(a, pk["w2"], pk["k2"], pk["n2"], ksize=1, bias=pk["b2"])
        return a.view(b, k, pk["n2"])

    def context_kv(self, attn, encoder_hidden_states: torch.Tensor, audio: Optional[dict] = None,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """K|V of the audio-injected context (reference :76-111 and :121-122), [B*Lk, 2*inner] fp16.

        Depends only on the context tokens, the audio tokens and the weights, never on
        the latent: the sampler computes it once per request (into `out`, so a
        captured graph keeps reading the same buffer) and hands it back through
        cross_attention_kwargs['context_kv'] on every denoise step."""
        ehs, _ = _as_tokens(encoder_hidden_states.to(torch.float16))
        b = ehs.shape[0]
        inner = attn.heads * attn.dim_head
        audio_tokens = audio[self.level] if (audio is not None and self.level in audio) else None
        kv_bias = None
        if audio_tokens is not None:
            if audio_tokens.shape[0] != b:
                if b % audio_tokens.shape[0]:
                    raise ValueError("audio batch must divide the UNet batch")
                audio_tokens = audio_tokens.repeat(b // audio_tokens.shape[0], 1, 1)
            proj = self.project_audio(audio_tokens)
            if self.mode == "add":
                pooled = ops.row_mean(proj.view(b * proj.shape[1], -1), b, proj.shape[1])   # [B, hidden] fp32
                gp = (torch.sigmoid(self.alpha.detach().float().to(pooled.device)) * pooled).to(torch.float16)
                kv_bias = ops.conv(gp, attn.w_kv, attn.kpad_kv, 2 * inner, ksize=1)           # [B, 2*inner]
            elif self.mode == "concat":
                if proj.shape[1] > 4:
                    proj = F.adaptive_avg_pool1d(proj.float().transpose(1, 2), 4).transpose(1, 2).to(torch.float16)
                ehs = torch.cat([ehs, proj.to(ehs.dtype)], dim=1).contiguous()
        lk = ehs.shape[1]
        ehs4 = ehs.view(b, 1, lk, ehs.shape[-1])
        if out is not None:
            out = out.view(b, 1, lk, 2 * inner)
        kv = ops.conv(ehs4, attn.w_kv, attn.kpad_kv, 2 * inner, ksize=1, temb=kv_bias, out=out)
        return kv.view(b * lk, 2 * inner)

    def __call__(self, attn, hidden_states, encoder_hidden_states=None, attention_mask=None, temb=None,
                 scale: float = 1.0, _residual: Optional[torch.Tensor] = None, _q: Optional[torch.Tensor] = None,
                 **cross_attention_kwargs):
        """_q: to_q(hidden_states) already computed by the caller (BasicTransformerBlock: norm2
        folded into the to_q GEMM); hidden_states then only gives the shape."""
        x, restore = _as_tokens(hidden_states)
        b, l, c = x.shape
        heads, d = attn.heads, attn.dim_head
        inner = heads * d
        ehs = encoder_hidden_states
        q = _q if _q is not None else ops.conv(x.view(b * l, c), attn.to_q.weight, attn.kpad_q, inner, ksize=1)
        if scale != 1.0:
            q.mul_(scale)
        if ehs is None:
            # reference :115-121: hidden_states = to_q(h) * scale, then encoder_hidden_states =
            # that projected query, so K / V = to_k / to_v(to_q(h) * scale); no audio injection
            # (the reference injects only when encoder_hidden_states is given, :86)
            if attn.to_k.in_features != inner:
                raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied ({b * l}x{inner} and "
                                   f"{attn.to_k.in_features}x{inner}): to_k of this layer does not take the "
                                   "projected query (reference :120)")
            kv = ops.conv(q, attn.w_kv, attn.kpad_kv, 2 * inner, ksize=1)
        else:
            cache = cross_attention_kwargs.get("context_kv")
            kv = cache.get(attn) if cache is not None else None
            if kv is None:
                kv = self.context_kv(attn, ehs, cross_attention_kwargs.get("audio", None))
        lk = kv.shape[0] // b
        o = ops.attention(q, kv[:, :inner], kv[:, inner:], b, heads, l, lk, d,
                          key_bias=key_bias_of(attention_mask, b, heads, lk, l))
        return _project_out(attn, o, b, l, c, _residual, restore)


def _project_out(attn, o, b, l, c, residual, restore):
    """to_out[0] (+ the block residual fused into its epilogue when the UNet passes it),
    back in the caller's layout / dtype."""
    out = attn.to_out[0](o, resid=None if residual is None else residual.reshape(b * l, c),
                         out=None if residual is None else residual.reshape(b * l, c))
    out = out.view(b, l, c)
    return out if restore is None else restore(out)


class AudioProcessorManager:
    """Maps the UNet's cross-attention processors to audio levels (reference :148-267)."""

    def __init__(self, unet):
        self.unet = unet
        self.processors = {}
        self.level_mapping = self._create_level_mapping()

    def _create_level_mapping(self) -> Dict[str, list]:
        mapping = {"early": [], "mid": [], "late": []}
        for name in self.unet.attn_processors.keys():
            if "attn1" in name:
                continue
            if "mid_block" in name:
                mapping["mid"].append(name)
            elif "down_blocks.0" in name or "down_blocks.1" in name:
                mapping["early"].append(name)
            elif "down_blocks.2" in name or "down_blocks.3" in name:
                mapping["late"].append(name)
            elif "up_blocks.0" in name or "up_blocks.1" in name:
                mapping["late"].append(name)
            elif "up_blocks.2" in name or "up_blocks.3" in name:
                mapping["mid"].append(name)
            else:
                mapping["mid"].append(name)
        return mapping

    def setup_processors(self, audio_dim: int = 768, hidden_dim: int = None, mode: str = "add",
                         dropout: float = 0.1, verbose: bool = True):
        if hidden_dim is None:
            for name in self.unet.attn_processors:
                if "attn2" in name:
                    hidden_dim = self.unet.get_submodule(name.rsplit(".", 1)[0]).to_k.in_features
                    break
            if hidden_dim is None:
                hidden_dim = 768
        new = dict(self.unet.attn_processors)
        for level, names in self.level_mapping.items():
            proc = AudioAttnProcessor(level=level, audio_dim=audio_dim, hidden_dim=hidden_dim, mode=mode,
                                      dropout=dropout)
            for name in names:
                new[name] = proc
        self.unet.set_attn_processor(new)
        self.processors = new
        if verbose:
            print("Setup audio processors:")
            for lv in ("early", "mid", "late"):
                print(f"  {lv.capitalize()} blocks: {len(self.level_mapping[lv])}")

    def level_processors(self) -> Dict[str, "AudioAttnProcessor"]:
        out = {}
        for level, names in self.level_mapping.items():
            if names and isinstance(self.processors.get(names[0]), AudioAttnProcessor):
                out[level] = self.processors[names[0]]
        return out

    def get_audio_kwargs(self, routed_tokens: Dict[str, torch.Tensor]) -> Dict:
        return {"audio": routed_tokens}
