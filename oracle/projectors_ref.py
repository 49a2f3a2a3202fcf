"""fp32 CPU restatement of the audio projector path the sampler consumes (TEST ORACLE ONLY).

ImprovedHierarchicalAudioEncoder(clap)[1]["routed"] of the reference, written as plain tensor
functions over a state dict with the reference's key names, so the end-to-end oracle
(pipeline_ref) no longer runs the product's projector modules:
  models/hierarchical_audio_v4.py  SoftHierarchicalDecomposition.compute_assignments / forward
                                   (:154-238: shared MLP + token offsets, cosine-to-anchor +
                                   gating-head logits / temperature), CrossHierarchyAttention.forward
                                   (:550-591: bottleneck pre-norm attention + MLP, outer residual),
                                   AdaptiveHierarchyWeights.forward (:271-290), LevelToUNetRouter.forward
                                   (:325-369: weighted re-normalised assignments @ softmax(routing_matrix),
                                   sigmoid level gates), ImprovedHierarchicalAudioEncoder.forward (:713-772)
Pinned by tests/golden/projectors.npz (outputs of the reference modules themselves,
scripts/make_goldens.py): tests/test_golden_cpu.py::test_oracle_projector_matches_golden.
"""
from __future__ import annotations

import math

import torch

LEVELS = ("early", "mid", "late")


def projector_shapes(audio_dim: int = 512, text_dim: int = 768, num_tokens: int = 10, num_levels: int = 3,
                     bottleneck: int = 192, mlp_ratio: float = 1.5, gate_hidden: int = 6) -> dict:
    """State-dict keys / shapes of the routed-token path (the reference's names)."""
    d, c = "decomposer.", "decomposer.cross_hierarchy_attn."
    hid = int(bottleneck * mlp_ratio)
    s = {
        d + "shared_mlp.0.weight": (512, audio_dim), d + "shared_mlp.0.bias": (512,),
        d + "shared_mlp.2.weight": (512,), d + "shared_mlp.2.bias": (512,),
        d + "shared_mlp.4.weight": (text_dim, 512), d + "shared_mlp.4.bias": (text_dim,),
        d + "token_offsets": (num_tokens, text_dim), d + "level_anchors": (num_levels, text_dim),
        d + "gating_head.0.weight": (10, text_dim), d + "gating_head.0.bias": (10,),
        d + "gating_head.2.weight": (num_levels, 10), d + "gating_head.2.bias": (num_levels,),
        c + "input_proj.weight": (bottleneck, text_dim), c + "input_proj.bias": (bottleneck,),
        c + "norm1.weight": (bottleneck,), c + "norm1.bias": (bottleneck,),
        c + "qkv.weight": (3 * bottleneck, bottleneck), c + "qkv.bias": (3 * bottleneck,),
        c + "proj.weight": (bottleneck, bottleneck), c + "proj.bias": (bottleneck,),
        c + "norm2.weight": (bottleneck,), c + "norm2.bias": (bottleneck,),
        c + "mlp.0.weight": (hid, bottleneck), c + "mlp.0.bias": (hid,),
        c + "mlp.3.weight": (bottleneck, hid), c + "mlp.3.bias": (bottleneck,),
        c + "output_proj.weight": (text_dim, bottleneck), c + "output_proj.bias": (text_dim,),
        d + "norm.weight": (text_dim,), d + "norm.bias": (text_dim,),
        "adaptive_weights.weight_network.0.weight": (gate_hidden, audio_dim),
        "adaptive_weights.weight_network.0.bias": (gate_hidden,),
        "adaptive_weights.weight_network.2.weight": (gate_hidden,),
        "adaptive_weights.weight_network.2.bias": (gate_hidden,),
        "adaptive_weights.weight_network.3.weight": (num_levels, gate_hidden),
        "adaptive_weights.weight_network.3.bias": (num_levels,),
        "router.routing_matrix": (num_levels, num_levels),
    }
    for lv in LEVELS:
        s["router.level_gates." + lv] = (1,)
    return s


def _linear(x, sd, p):
    y = x @ sd[p + ".weight"].t()
    b = sd.get(p + ".bias")
    return y + b if b is not None else y


def _layer_norm(x, sd, p, eps=1e-5):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * sd[p + ".weight"] + sd[p + ".bias"]


def _gelu(x):   # nn.GELU(): the exact erf form
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def _l2_normalize(x, eps=1e-12):   # F.normalize(p=2, dim=-1)
    return x / x.norm(dim=-1, keepdim=True).clamp_min(eps)


def _cross_hierarchy_attention(x, sd, p, heads=4):
    b, n, _ = x.shape
    y = _linear(x, sd, p + "input_proj")
    bd = y.shape[-1]
    hd = bd // heads
    qkv = _linear(_layer_norm(y, sd, p + "norm1"), sd, p + "qkv").view(b, n, 3, heads, hd).permute(2, 0, 3, 1, 4)
    w = torch.softmax(qkv[0] @ qkv[1].transpose(-1, -2) * hd ** -0.5, dim=-1)
    y = y + _linear((w @ qkv[2]).transpose(1, 2).reshape(b, n, bd), sd, p + "proj")
    y = y + _linear(_gelu(_linear(_layer_norm(y, sd, p + "norm2"), sd, p + "mlp.0")), sd, p + "mlp.3")
    return x + _linear(y, sd, p + "output_proj")


@torch.no_grad()
def routed_tokens(clap: torch.Tensor, sd: dict, temperature: float = 2.0) -> dict:
    """clap [B, 512] fp32 -> {'tokens_10', 'assignments', 'hierarchy_weights', 'routed': {level: [B, 10, 768]}}
    (temperature: the decomposer's buffer, 2.0 = its initial value, max(T, 0.1) as set_temperature)."""
    d = "decomposer."
    h = _linear(clap, sd, d + "shared_mlp.0")
    h = _linear(_layer_norm(_gelu(h), sd, d + "shared_mlp.2"), sd, d + "shared_mlp.4")
    tokens = h[:, None, :] + sd[d + "token_offsets"][None]
    sim = _l2_normalize(tokens) @ _l2_normalize(sd[d + "level_anchors"]).t()
    gate = _linear(_gelu(_linear(tokens, sd, d + "gating_head.0")), sd, d + "gating_head.2")
    assign = torch.softmax((10.0 * sim + gate) / max(temperature, 0.1), dim=-1)
    tokens10 = _layer_norm(_cross_hierarchy_attention(tokens, sd, d + "cross_hierarchy_attn."), sd, d + "norm")
    a = "adaptive_weights.weight_network."
    hw = torch.softmax(_linear(_layer_norm(_gelu(_linear(clap, sd, a + "0")), sd, a + "2"), sd, a + "3"), dim=-1)
    wa = assign * hw[:, None, :]
    wa = wa / (wa.sum(dim=-1, keepdim=True) + 1e-8)
    routing = wa @ torch.softmax(sd["router.routing_matrix"], dim=1)
    routed = {lv: tokens10 * routing[:, :, i:i + 1] * torch.sigmoid(sd["router.level_gates." + lv])
              for i, lv in enumerate(LEVELS)}
    return {"tokens_10": tokens10, "assignments": assign, "hierarchy_weights": hw, "routed": routed}
