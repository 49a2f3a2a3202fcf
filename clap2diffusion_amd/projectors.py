"""Audio projector modules with the reference's Python API and state-dict keys.

They run once per request (~0.3 GFLOP per sample), so
they stay PyTorch-ROCm modules; what matters here is API and checkpoint
compatibility with the reference:
  models/audio_adapter_v4.py       AudioAdapter (:264-301), AudioTokenGenerator (:13-119),
                                   AudioSelfAttention (:122-165)
  models/hierarchical_audio_v4.py  TemperatureScheduler (:20-76), SoftHierarchicalDecomposition (:79-238),
                                   AdaptiveHierarchyWeights (:241-290), LevelToUNetRouter (:293-369),
                                   CrossAttentionBlock (:375-414), AudioProjectionTransformer77 (:417-492),
                                   CrossHierarchyAttention (:495-591), ImprovedHierarchicalAudioEncoder (:594-772),
                                   HierarchicalAudioDecomposition (:776-882), HierarchicalAudioV4 (:885-932)
Module attribute names (hence state-dict keys, e.g. audio_projector_stage2.pth
'adapter_state_dict' and hierarchical_v4_final.pth, scripts/inference.py:44-59)
are identical to the reference.  Arithmetic is checked against goldens produced
by the reference modules themselves (tests/golden/projectors.npz).
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple, Union

import torch
import torch.nn as nn
import torch.nn.functional as F


def _heads_split(t: torch.Tensor, h: int) -> torch.Tensor:
    b, n, d = t.shape
    return t.view(b, n, h, d // h).transpose(1, 2)


def _heads_merge(t: torch.Tensor) -> torch.Tensor:
    b, h, n, d = t.shape
    return t.transpose(1, 2).reshape(b, n, h * d)


# ----------------------------------------------------------------- adapter (v4)
class AudioSelfAttention(nn.Module):
    def __init__(self, hidden_dim: int, num_heads: int, dropout: float = 0.1):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = hidden_dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.to_qkv = nn.Linear(hidden_dim, 3 * hidden_dim, bias=False)
        self.to_out = nn.Sequential(nn.Linear(hidden_dim, hidden_dim), nn.Dropout(dropout))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        q, k, v = (_heads_split(t, self.num_heads) for t in self.to_qkv(x).chunk(3, dim=-1))
        w = torch.softmax(q @ k.transpose(-1, -2) * self.scale, dim=-1)
        return self.to_out(_heads_merge(w @ v))


class AudioTokenGenerator(nn.Module):
    """CLAP [B, 512] -> [B, num_tokens, hidden] via learned queries attending to
    per-token keys/values generated from the embedding, then self-attention."""

    def __init__(self, audio_dim: int = 512, hidden_dim: int = 768, num_tokens: int = 16, num_layers: int = 4,
                 num_heads: int = 8, dropout: float = 0.1):
        super().__init__()
        self.num_tokens, self.hidden_dim = num_tokens, hidden_dim
        self.audio_queries = nn.Parameter(torch.randn(num_tokens, hidden_dim))
        self.pos_embed = nn.Parameter(torch.randn(num_tokens, hidden_dim))
        self.audio_to_kv = nn.Sequential(nn.Linear(audio_dim, 256), nn.GELU(), nn.Dropout(dropout),
                                         nn.Linear(256, 2 * hidden_dim * num_tokens))
        self.self_attn_layers = nn.ModuleList(
            [AudioSelfAttention(hidden_dim, num_heads, dropout) for _ in range(num_layers)])
        self.layer_norms = nn.ModuleList([nn.LayerNorm(hidden_dim) for _ in range(num_layers)])
        self.output_proj = nn.Sequential(nn.Linear(hidden_dim, hidden_dim), nn.LayerNorm(hidden_dim))
        nn.init.xavier_uniform_(self.audio_queries)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)

    def forward(self, audio_embedding: torch.Tensor) -> torch.Tensor:
        b = audio_embedding.shape[0]
        q = (self.audio_queries + self.pos_embed).unsqueeze(0).expand(b, -1, -1)
        kv = self.audio_to_kv(audio_embedding).view(b, self.num_tokens, 2, self.hidden_dim)
        k, v = kv[:, :, 0], kv[:, :, 1]
        w = torch.softmax(torch.bmm(q, k.transpose(1, 2)) * self.hidden_dim ** -0.5, dim=-1)
        tok = torch.bmm(w, v) + q
        for attn, norm in zip(self.self_attn_layers, self.layer_norms):
            tok = attn(norm(tok)) + tok
        return self.output_proj(tok)


class AudioAdapter(nn.Module):
    def __init__(self, audio_dim: int = 512, hidden_dim: int = 768, num_tokens: int = 16, num_layers: int = 4,
                 num_heads: int = 8, dropout: float = 0.1):
        super().__init__()
        self.token_generator = AudioTokenGenerator(audio_dim, hidden_dim, num_tokens, num_layers, num_heads, dropout)

    def forward(self, audio_embedding: torch.Tensor) -> torch.Tensor:
        return self.token_generator(audio_embedding)


# ----------------------------------------------------------------- hierarchy (v4)
class TemperatureScheduler:
    """Cosine / linear annealing of the decomposer temperature (T_max during warm-up).
    Unlike the reference, step() also returns the temperature it set."""

    def __init__(self, decomposer: nn.Module, T_max: float = 2.0, T_min: float = 0.5, total_steps: int = 5000,
                 warmup_steps: int = 200, mode: str = "cosine"):
        self.decomposer, self.T_max, self.T_min = decomposer, T_max, T_min
        self.total_steps, self.warmup_steps, self.mode = total_steps, warmup_steps, mode
        decomposer.set_temperature(T_max)

    def step(self, current_step: int) -> float:
        if current_step < self.warmup_steps:
            t = self.T_max
        elif current_step >= self.total_steps or self.total_steps <= self.warmup_steps:
            t = self.T_min
        else:
            frac = (current_step - self.warmup_steps) / (self.total_steps - self.warmup_steps)
            if self.mode == "cosine":
                t = self.T_min + 0.5 * (self.T_max - self.T_min) * (1.0 + math.cos(math.pi * frac))
            elif self.mode == "linear":
                t = self.T_max - (self.T_max - self.T_min) * frac
            else:
                raise ValueError(f"Unknown annealing mode: {self.mode}")
        self.decomposer.set_temperature(t)
        return max(t, 0.1)


class CrossHierarchyAttention(nn.Module):
    """Pre-norm transformer layer run in a bottleneck space with an outer residual."""

    def __init__(self, dim: int, num_heads: int = 4, dropout: float = 0.1, bottleneck_dim: int = 256,
                 mlp_ratio: float = 2.0):
        super().__init__()
        if bottleneck_dim % num_heads:
            raise ValueError(f"bottleneck_dim ({bottleneck_dim}) must be divisible by num_heads ({num_heads})")
        self.dim, self.bottleneck_dim, self.num_heads = dim, bottleneck_dim, num_heads
        self.head_dim = bottleneck_dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.input_proj = nn.Linear(dim, bottleneck_dim)
        self.norm1 = nn.LayerNorm(bottleneck_dim)
        self.qkv = nn.Linear(bottleneck_dim, 3 * bottleneck_dim, bias=True)
        self.attn_drop = nn.Dropout(dropout)
        self.proj = nn.Linear(bottleneck_dim, bottleneck_dim)
        self.proj_drop = nn.Dropout(dropout)
        self.norm2 = nn.LayerNorm(bottleneck_dim)
        hid = int(bottleneck_dim * mlp_ratio)
        self.mlp = nn.Sequential(nn.Linear(bottleneck_dim, hid), nn.GELU(), nn.Dropout(dropout),
                                 nn.Linear(hid, bottleneck_dim), nn.Dropout(dropout))
        self.output_proj = nn.Linear(bottleneck_dim, dim)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        b, n, _ = x.shape
        y = self.input_proj(x)
        qkv = self.qkv(self.norm1(y)).view(b, n, 3, self.num_heads, self.head_dim).permute(2, 0, 3, 1, 4)
        w = self.attn_drop(torch.softmax(qkv[0] @ qkv[1].transpose(-1, -2) * self.scale, dim=-1))
        y = y + self.proj_drop(self.proj((w @ qkv[2]).transpose(1, 2).reshape(b, n, self.bottleneck_dim)))
        y = y + self.mlp(self.norm2(y))
        return x + self.output_proj(y)


class SoftHierarchicalDecomposition(nn.Module):
    def __init__(self, audio_dim: int = 512, text_dim: int = 768, num_tokens: int = 10, num_levels: int = 3,
                 dropout: float = 0.1, initial_temperature: float = 2.0):
        super().__init__()
        self.audio_dim, self.text_dim = audio_dim, text_dim
        self.num_tokens, self.num_levels = num_tokens, num_levels
        self.shared_mlp = nn.Sequential(nn.Linear(audio_dim, 512), nn.GELU(), nn.LayerNorm(512), nn.Dropout(dropout),
                                        nn.Linear(512, text_dim))
        self.token_offsets = nn.Parameter(torch.randn(num_tokens, text_dim) * 0.02)
        self.level_anchors = nn.Parameter(torch.randn(num_levels, text_dim) * 0.02)
        self.gating_head = nn.Sequential(nn.Linear(text_dim, 10), nn.GELU(), nn.Linear(10, num_levels))
        self.register_buffer("temperature", torch.tensor(initial_temperature))
        self.register_buffer("level_prior", torch.tensor([5.0, 3.0, 2.0]) / 10.0)
        self.cross_hierarchy_attn = CrossHierarchyAttention(text_dim, num_heads=4, dropout=dropout,
                                                            bottleneck_dim=192, mlp_ratio=1.5)
        self.norm = nn.LayerNorm(text_dim)

    @torch.no_grad()
    def set_temperature(self, temperature: float) -> None:
        self.temperature.fill_(max(temperature, 0.1))

    def compute_assignments(self, tokens: torch.Tensor) -> torch.Tensor:
        sim = F.normalize(tokens, p=2, dim=-1) @ F.normalize(self.level_anchors, p=2, dim=-1).t()
        logits = 10.0 * sim + self.gating_head(tokens)
        return torch.softmax(logits / self.temperature, dim=-1)

    def tokens_and_assignments(self, audio_features: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """The forward's two tensors without the host-side info dict (no .item() sync:
        capturable into a hipGraph)."""
        tokens = self.shared_mlp(audio_features).unsqueeze(1) + self.token_offsets.unsqueeze(0)
        assign = self.compute_assignments(tokens)
        return self.norm(self.cross_hierarchy_attn(tokens)), assign

    def forward(self, audio_features: torch.Tensor, return_stats: bool = False) -> Tuple[torch.Tensor, Dict]:
        out, assign = self.tokens_and_assignments(audio_features)
        info = {"tokens": out, "assignments": assign, "temperature": self.temperature.item(),
                "level_anchors": self.level_anchors}
        if return_stats:
            with torch.no_grad():
                ent = -(assign * (assign + 1e-8).log()).sum(-1).mean()
                info["stats"] = {"avg_assignment": assign.mean(dim=(0, 1)), "entropy": ent.item(),
                                 "effective_levels": torch.exp(ent).item()}
        return out, info


class AdaptiveHierarchyWeights(nn.Module):
    def __init__(self, audio_dim: int = 512, hidden_dim: int = 6, num_levels: int = 3, use_audio_context: bool = True):
        super().__init__()
        self.num_levels, self.use_audio_context = num_levels, use_audio_context
        if use_audio_context:
            self.weight_network = nn.Sequential(nn.Linear(audio_dim, hidden_dim), nn.GELU(), nn.LayerNorm(hidden_dim),
                                                nn.Linear(hidden_dim, num_levels))
        else:
            self.weights = nn.Parameter(torch.tensor([0.5, 0.3, 0.2]))

    def forward(self, audio_features: torch.Tensor) -> torch.Tensor:
        if self.use_audio_context:
            return torch.softmax(self.weight_network(audio_features), dim=-1)
        return torch.softmax(self.weights, dim=0).unsqueeze(0).expand(audio_features.shape[0], -1)


class LevelToUNetRouter(nn.Module):
    LEVELS = ("early", "mid", "late")

    def __init__(self, num_levels: int = 3, text_dim: int = 768):
        super().__init__()
        self.num_levels, self.text_dim = num_levels, text_dim
        self.level_gates = nn.ParameterDict({k: nn.Parameter(torch.zeros(1)) for k in self.LEVELS})
        self.routing_matrix = nn.Parameter(torch.tensor([[0.1, 0.3, 0.6], [0.2, 0.6, 0.2], [0.6, 0.3, 0.1]]))

    def forward(self, tokens: torch.Tensor, assignments: torch.Tensor,
                hierarchy_weights: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        if hierarchy_weights is not None:
            assignments = assignments * hierarchy_weights.unsqueeze(1)
            assignments = assignments / (assignments.sum(dim=-1, keepdim=True) + 1e-8)
        routing = assignments @ torch.softmax(self.routing_matrix, dim=1)
        return {lv: tokens * routing[:, :, i:i + 1] * torch.sigmoid(self.level_gates[lv])
                for i, lv in enumerate(self.LEVELS)}


class CrossAttentionBlock(nn.Module):
    def __init__(self, d_model: int, num_heads: int, dropout: float = 0.1):
        super().__init__()
        self.ln_q = nn.LayerNorm(d_model)
        self.ln_kv = nn.LayerNorm(d_model)
        self.cross_attn = nn.MultiheadAttention(d_model, num_heads, dropout=dropout, batch_first=True)
        self.ffn = nn.Sequential(nn.LayerNorm(d_model), nn.Linear(d_model, 2 * d_model), nn.GELU(),
                                 nn.Dropout(dropout), nn.Linear(2 * d_model, d_model), nn.Dropout(dropout))

    def forward(self, queries: torch.Tensor, keys_values: torch.Tensor) -> torch.Tensor:
        kv = self.ln_kv(keys_values)
        queries = queries + self.cross_attn(self.ln_q(queries), kv, kv, need_weights=False)[0]
        return queries + self.ffn(queries)


class AudioProjectionTransformer77(nn.Module):
    """Perceiver-style decoder: 77 learned queries attend to the audio tokens."""

    def __init__(self, audio_dim: int = 768, clip_dim: int = 768, bottleneck_dim: int = 256, num_heads: int = 8,
                 num_layers: int = 4, dropout: float = 0.1) -> None:
        super().__init__()
        self.audio_dim, self.clip_dim, self.bottleneck_dim = audio_dim, clip_dim, bottleneck_dim
        self.audio_proj = nn.Linear(audio_dim, bottleneck_dim)
        self.queries = nn.Parameter(torch.randn(77, bottleneck_dim) * 0.02)
        self.query_pos = nn.Parameter(torch.zeros(77, bottleneck_dim))
        self.blocks = nn.ModuleList([CrossAttentionBlock(bottleneck_dim, num_heads, dropout)
                                     for _ in range(num_layers)])
        self.out_proj = nn.Linear(bottleneck_dim, clip_dim)
        self.out_norm = nn.LayerNorm(clip_dim)
        self.clip_pos_embed = nn.Parameter(torch.zeros(1, 77, clip_dim))
        nn.init.trunc_normal_(self.clip_pos_embed, std=0.02)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        feats = self.audio_proj(x)
        q = (self.queries + self.query_pos).unsqueeze(0).expand(x.shape[0], -1, -1)
        for blk in self.blocks:
            q = blk(q, feats)
        return self.out_norm(self.out_proj(q) + self.clip_pos_embed)


class HierarchicalAudioDecomposition(nn.Module):
    """Legacy rigid 5/3/2 foreground / background / ambience decomposition."""

    def __init__(self, audio_dim: int = 512, text_dim: int = 768, num_foreground: int = 5, num_background: int = 3,
                 num_ambience: int = 2, dropout: float = 0.1):
        super().__init__()
        self.audio_dim, self.text_dim = audio_dim, text_dim
        self.num_foreground, self.num_background, self.num_ambience = num_foreground, num_background, num_ambience
        self.total_tokens = num_foreground + num_background + num_ambience

        def head(hidden, n):
            return nn.Sequential(nn.Linear(audio_dim, hidden), nn.GELU(), nn.Dropout(dropout),
                                 nn.Linear(hidden, text_dim * n))

        self.foreground_proj = head(text_dim * 2, num_foreground)
        self.background_proj = head(text_dim, num_background)
        self.ambience_proj = head(text_dim // 2, num_ambience)
        self.hierarchy_weights = nn.Parameter(torch.tensor([0.5, 0.3, 0.2], dtype=torch.float32))
        self.layer_norm = nn.LayerNorm(text_dim)
        self.cross_hierarchy_attn = CrossHierarchyAttention(text_dim, num_heads=4, dropout=dropout, bottleneck_dim=192)

    def forward(self, audio_features: torch.Tensor, return_hierarchy: bool = False):
        b = audio_features.shape[0]
        w = torch.softmax(self.hierarchy_weights, dim=0)
        parts = {}
        for i, (name, proj, n) in enumerate((("foreground", self.foreground_proj, self.num_foreground),
                                             ("background", self.background_proj, self.num_background),
                                             ("ambience", self.ambience_proj, self.num_ambience))):
            parts[name] = proj(audio_features).view(b, n, self.text_dim) * w[i]
        tok = self.layer_norm(self.cross_hierarchy_attn(torch.cat(list(parts.values()), dim=1)))
        if return_hierarchy:
            return tok, dict(parts, weights=w, combined=tok)
        return tok


class ImprovedHierarchicalAudioEncoder(nn.Module):
    def __init__(self, audio_dim: int = 512, text_dim: int = 768, num_tokens: int = 10, num_levels: int = 3,
                 out_tokens: int = 77, dropout: float = 0.1, use_adaptive_weights: bool = True,
                 use_soft_decomposition: bool = True):
        super().__init__()
        self.use_soft_decomposition = use_soft_decomposition
        if use_soft_decomposition:
            self.decomposer = SoftHierarchicalDecomposition(audio_dim, text_dim, num_tokens, num_levels, dropout)
        else:
            self.decomposer = HierarchicalAudioDecomposition(audio_dim, text_dim, dropout=dropout)
        self.adaptive_weights = (AdaptiveHierarchyWeights(audio_dim, 6, num_levels, True)
                                 if use_adaptive_weights else None)
        self.router = LevelToUNetRouter(num_levels, text_dim)
        self.projector = AudioProjectionTransformer77(text_dim, text_dim, bottleneck_dim=256, num_heads=8,
                                                      num_layers=4)
        self.temperature_scheduler = None

    def compute_losses(self, assignments, tokens, hierarchy_weights=None) -> Dict[str, torch.Tensor]:
        ent = -(assignments * (assignments + 1e-8).log()).sum(dim=-1).mean()
        tn = F.normalize(tokens, p=2, dim=-1)
        gram = torch.bmm(tn, tn.transpose(1, 2))
        eye = torch.eye(tokens.shape[1], device=tokens.device).expand_as(gram)
        losses = {"entropy": ent, "orthogonality": F.mse_loss(gram, eye)}
        if self.use_soft_decomposition and hasattr(self.decomposer, "level_prior"):
            avg = assignments.mean(dim=1)
            prior = self.decomposer.level_prior.unsqueeze(0).expand_as(avg)
            losses["prior"] = F.kl_div(prior.log(), avg, reduction="batchmean")
        else:
            losses["prior"] = torch.tensor(0.0, device=tokens.device)
        return losses

    def routed_tokens(self, audio_features: torch.Tensor) -> Dict[str, torch.Tensor]:
        """forward(x, return_all=True)[1]["routed"] -- the level-keyed tokens the UNet's audio
        processors consume -- without the projector-77 head, the losses and the stats
        (no host syncs: capturable into a hipGraph).  Soft decomposition only."""
        tokens_10, assignments = self.decomposer.tokens_and_assignments(audio_features)
        hw = self.adaptive_weights(audio_features) if self.adaptive_weights is not None else None
        return self.router(tokens_10, assignments, hw)

    def forward(self, audio_features: torch.Tensor, return_all: bool = False
                ) -> Union[torch.Tensor, Tuple[torch.Tensor, Dict]]:
        if self.use_soft_decomposition:
            tokens_10, info_d = self.decomposer(audio_features, return_stats=True)
            assignments = info_d["assignments"]
        else:
            tokens_10 = self.decomposer(audio_features)
            assignments = torch.zeros(tokens_10.shape[0], tokens_10.shape[1], 3, device=tokens_10.device)
            info_d = {"temperature": 1.0}
        hw = self.adaptive_weights(audio_features) if self.adaptive_weights is not None else None
        routed = self.router(tokens_10, assignments, hw)
        tokens_77 = self.projector(tokens_10)
        if not return_all:
            return tokens_77
        return tokens_77, {
            "tokens_10": tokens_10, "tokens_77": tokens_77, "assignments": assignments, "routed": routed,
            "hierarchy_weights": hw, "losses": self.compute_losses(assignments, tokens_10, hw),
            "stats": info_d.get("stats", {}), "temperature": info_d["temperature"],
        }


class HierarchicalAudioV4(nn.Module):
    """Legacy stage-1 encoder: rigid decomposition + projection to 77 tokens."""

    def __init__(self, audio_dim: int = 512, text_dim: int = 768, num_foreground: int = 5, num_background: int = 3,
                 num_ambience: int = 2, out_tokens: int = 77, projector_layers: int = 4, projector_heads: int = 8,
                 projector_mlp_ratio: float = 4.0, dropout: float = 0.1) -> None:
        super().__init__()
        self.decomposer = HierarchicalAudioDecomposition(audio_dim, text_dim, num_foreground, num_background,
                                                         num_ambience, dropout)
        self.projector = AudioProjectionTransformer77(text_dim, text_dim, bottleneck_dim=256,
                                                      num_heads=projector_heads, num_layers=projector_layers,
                                                      dropout=dropout)

    def forward(self, clap_features: torch.Tensor, return_intermediate: bool = False):
        tokens10, hier = self.decomposer(clap_features, return_hierarchy=True)
        tokens77 = self.projector(tokens10)
        if return_intermediate:
            return tokens77, dict(hier, tokens10=tokens10)
        return tokens77


def normalize_tokens(audio_tokens: torch.Tensor, target_norm: float = 60.0) -> torch.Tensor:
    """'Norm 60' rescale (scripts/inference.py:92-99): mean per-token L2 norm -> target.
    The reference's `if raw_norm > 0` is a device-side select here (same values, no host
    sync, so the conditioning leg can be captured into a hipGraph)."""
    with torch.no_grad():
        raw = torch.norm(audio_tokens, dim=-1, keepdim=True).mean()
        scale = torch.where(raw > 0, target_norm / raw, torch.ones_like(raw))
        return audio_tokens * scale
