"""Generate the golden vectors in tests/golden/ from the REFERENCE's own code.

Run here (not on the GPU box, where /root/reference does not exist):
    PYTHONDONTWRITEBYTECODE=1 python scripts/make_goldens.py

  projectors.npz  reference models/hierarchical_audio_v4.py ImprovedHierarchicalAudioEncoder,
                  HierarchicalAudioV4 and models/audio_adapter_v4.py AudioAdapter (+ the Norm-60
                  rescale of scripts/inference.py:92-99) on synthetic weights (weights.synth_generic,
                  regenerated from seeds by the tests) and seeded CLAP embeddings.
  processor.npz   reference models/audio_attention_processor.py AudioAttnProcessor.__call__
                  (imported with a sys.modules stub for diffusers.models.attention_processor, which
                  the module only uses for type names at :10) driving a minimal restatement of the
                  diffusers Attention helpers it calls, at the four SD1.5 (C, heads*d) shapes, in
                  "add" and "concat" modes.
  processor_ext.npz  the same processor on the paths the SD1.5 pipeline does not take: the
                  self-attention branch (encoder_hidden_states=None: K / V from the projected
                  query, :115-121), 4-D [B, C, H, W] hidden states (:67-70, :137-138) and
                  attention masks passed to get_attention_scores (:129), including one that
                  varies over queries.
  htsat.npz       transformers ClapModel.get_audio_features (the call at
                  models/audio_encoder.py:171-174) on synthetic HTSAT weights and seeded mel input.
Only inputs and outputs are stored; weights are regenerated from their seeds.
"""
from __future__ import annotations

import sys
import types
from pathlib import Path

import numpy as np
import torch
import torch.nn as nn

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
REF = Path("/root/reference")
OUT = ROOT / "tests" / "golden"

from clap2diffusion_amd.weights import synth_generic, synth_htsat, synth_processor_weights  # noqa: E402


def load_reference():
    sys.path.insert(0, str(REF))
    stub = types.ModuleType("diffusers.models.attention_processor")
    stub.Attention = object
    stub.AttnProcessor = object
    for name in ("diffusers", "diffusers.models"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["diffusers.models.attention_processor"] = stub
    from models.audio_adapter_v4 import AudioAdapter
    from models.audio_attention_processor import AudioAttnProcessor
    from models.hierarchical_audio_v4 import HierarchicalAudioV4, ImprovedHierarchicalAudioEncoder
    return AudioAdapter, AudioAttnProcessor, HierarchicalAudioV4, ImprovedHierarchicalAudioEncoder


def fill(module: nn.Module, tag: str, seed: int = 0) -> None:
    sd = module.state_dict()
    shapes = {k: tuple(v.shape) for k, v in sd.items() if v.is_floating_point() and k not in
              ("decomposer.temperature", "decomposer.level_prior")}
    new = synth_generic(shapes, seed, tag)
    module.load_state_dict({**sd, **new})


class MiniAttention(nn.Module):
    """The diffusers-0.23.1 Attention surface the reference processor calls."""

    def __init__(self, c, ctx, heads, g):
        super().__init__()
        d = c // heads
        self.heads, self.scale = heads, d ** -0.5
        self.to_q = nn.Linear(c, c, bias=False)
        self.to_k = nn.Linear(ctx, c, bias=False)
        self.to_v = nn.Linear(ctx, c, bias=False)
        self.to_out = nn.ModuleList([nn.Linear(c, c), nn.Dropout(0.0)])
        for lin in (self.to_q, self.to_k, self.to_v, self.to_out[0]):
            lin.weight.data = torch.randn(lin.weight.shape, generator=g) / lin.weight.shape[1] ** 0.5
            if lin.bias is not None:
                lin.bias.data = 0.02 * torch.randn(lin.bias.shape, generator=g)
        self.spatial_norm = None
        self.norm_cross = False
        self.residual_connection = False
        self.rescale_output_factor = 1.0

    def head_to_batch_dim(self, t, out_dim=3):
        b, l, dim = t.shape
        return t.reshape(b, l, self.heads, dim // self.heads).permute(0, 2, 1, 3).reshape(b * self.heads, l, -1)

    def batch_to_head_dim(self, t):
        bh, l, d = t.shape
        return t.reshape(bh // self.heads, self.heads, l, d).permute(0, 2, 1, 3).reshape(bh // self.heads, l, -1)

    def get_attention_scores(self, q, k, mask=None):
        s = torch.baddbmm(torch.empty(q.shape[0], q.shape[1], k.shape[1]), q, k.transpose(-1, -2), beta=0,
                          alpha=self.scale)
        if mask is not None:   # diffusers 0.23.1: baddbmm(mask, q, k^T, beta=1, alpha=scale)
            s = torch.baddbmm(mask, q, k.transpose(-1, -2), beta=1, alpha=self.scale)
        return s.softmax(dim=-1)


def main():
    torch.manual_seed(0)
    AudioAdapter, AudioAttnProcessor, HierarchicalAudioV4, Improved = load_reference()
    OUT.mkdir(parents=True, exist_ok=True)

    # ---------------- projectors
    g = torch.Generator().manual_seed(1234)
    clap = torch.nn.functional.normalize(torch.randn(3, 512, generator=g), dim=-1)
    enc, ada, v4 = Improved(), AudioAdapter(), HierarchicalAudioV4()
    fill(enc, "improved.")
    fill(ada, "adapter.")
    fill(v4, "v4.")
    for m in (enc, ada, v4):
        m.eval()
    with torch.no_grad():
        t77, info = enc(clap, return_all=True)
        a16 = ada(clap)
        raw = torch.norm(a16, dim=-1, keepdim=True).mean()
        a16n = a16 * (60.0 / raw)
        v77, hier = v4(clap, return_intermediate=True)
    np.savez_compressed(OUT / "projectors.npz", clap=clap.numpy(), tokens_77=t77.numpy(),
                        tokens_10=info["tokens_10"].numpy(), assignments=info["assignments"].numpy(),
                        hierarchy_weights=info["hierarchy_weights"].numpy(),
                        routed_early=info["routed"]["early"].numpy(), routed_mid=info["routed"]["mid"].numpy(),
                        routed_late=info["routed"]["late"].numpy(),
                        loss_entropy=info["losses"]["entropy"].numpy(),
                        loss_orth=info["losses"]["orthogonality"].numpy(), loss_prior=info["losses"]["prior"].numpy(),
                        adapter=a16.numpy(), adapter_norm60=a16n.numpy(), v4_tokens_77=v77.numpy(),
                        v4_tokens_10=hier["tokens10"].numpy())

    # ---------------- processor
    gs = torch.Generator().manual_seed(99)
    ehs = torch.randn(2, 77, 768, generator=gs)
    audio = torch.randn(2, 10, 768, generator=gs)
    cases = {"ehs": ehs.numpy(), "audio": audio.numpy()}
    for ci, (c, lq) in enumerate(((320, 48), (640, 32), (1280, 16), (1280, 8))):
        gg = torch.Generator().manual_seed(100 + ci)
        attn = MiniAttention(c, 768, 8, gg).eval()
        h = torch.randn(2, lq, c, generator=gg)
        cases[f"c{c}_l{lq}_h"] = h.numpy()
        for mode in ("add", "concat"):
            proc = AudioAttnProcessor(level="mid", audio_dim=768, hidden_dim=768, mode=mode).eval()
            proc.load_state_dict(synth_processor_weights("mid", seed=ci))
            with torch.no_grad():
                out = proc(attn, h, encoder_hidden_states=ehs, audio={"mid": audio})
            cases[f"c{c}_l{lq}_{mode}_out"] = out.numpy()
    np.savez_compressed(OUT / "processor.npz", **cases)

    # ---------------- processor: self-attention branch, 4-D input, attention masks
    ext = {}
    for c, lq, seed in ((320, 48, 200), (640, 32, 201)):   # self-attention layers (to_k / to_v take C)
        gg = torch.Generator().manual_seed(seed)
        attn = MiniAttention(c, c, 8, gg).eval()
        h = torch.randn(2, lq, c, generator=gg)
        proc = AudioAttnProcessor(level="early", audio_dim=768, hidden_dim=768, mode="add").eval()
        proc.load_state_dict(synth_processor_weights("early", seed=seed))
        with torch.no_grad():
            out = proc(attn, h, encoder_hidden_states=None, audio={"early": audio})
        ext[f"self_c{c}_l{lq}_h"], ext[f"self_c{c}_l{lq}_out"] = h.numpy(), out.numpy()
    for c, hh, ww, seed in ((320, 6, 8, 210), (640, 4, 4, 211)):   # 4-D [B, C, H, W] cross-attention input
        gg = torch.Generator().manual_seed(seed)
        attn = MiniAttention(c, 768, 8, gg).eval()
        h4 = torch.randn(2, c, hh, ww, generator=gg)
        proc = AudioAttnProcessor(level="mid", audio_dim=768, hidden_dim=768, mode="add").eval()
        proc.load_state_dict(synth_processor_weights("mid", seed=seed))
        with torch.no_grad():
            out = proc(attn, h4, encoder_hidden_states=ehs, audio={"mid": audio})
        ext[f"nd4_c{c}_{hh}x{ww}_h"], ext[f"nd4_c{c}_{hh}x{ww}_out"] = h4.numpy(), out.numpy()
    for c, lq, form, seed in ((640, 32, "query", 220), (320, 48, "key", 221)):   # attention_mask forms
        gg = torch.Generator().manual_seed(seed)
        attn = MiniAttention(c, 768, 8, gg).eval()
        h = torch.randn(2, lq, c, generator=gg)
        if form == "query":   # [B*H, Lq, Lk], varies over queries
            mask = torch.randn(2 * 8, lq, 77, generator=gg) * 2.0
            mask = mask.masked_fill(torch.rand(2 * 8, lq, 77, generator=gg) < 0.3, -10000.0)
        else:                 # [B*H, 1, Lk] key padding (prepare_attention_mask's form)
            keep = torch.ones(2, 77)
            keep[0, 20:] = 0
            keep[1, 60:] = 0
            mask = ((1.0 - keep) * -10000.0).repeat_interleave(8, dim=0).unsqueeze(1)
        proc = AudioAttnProcessor(level="late", audio_dim=768, hidden_dim=768, mode="add").eval()
        proc.load_state_dict(synth_processor_weights("late", seed=seed))
        with torch.no_grad():
            out = proc(attn, h, encoder_hidden_states=ehs, attention_mask=mask, audio={"late": audio})
        ext[f"mask_{form}_c{c}_l{lq}_h"], ext[f"mask_{form}_c{c}_l{lq}_mask"] = h.numpy(), mask.numpy()
        ext[f"mask_{form}_c{c}_l{lq}_out"] = out.numpy()
    np.savez_compressed(OUT / "processor_ext.npz", **ext)

    # ---------------- HTSAT (transformers ClapModel, the reference's CLAP dependency)
    from transformers import ClapConfig, ClapModel
    model = ClapModel(ClapConfig()).eval()
    sd = model.state_dict()
    syn = synth_htsat(0)
    missing = [k for k in sd if (k.startswith("audio_model") or k.startswith("audio_projection"))
               and k not in syn and "relative_position_index" not in k and "num_batches_tracked" not in k]
    assert not missing, missing
    for k, v in syn.items():
        assert tuple(sd[k].shape) == tuple(v.shape), k
    model.load_state_dict({**sd, **syn})
    gm = torch.Generator().manual_seed(77)
    mel = torch.randn(2, 1, 1001, 64, generator=gm) * 2.0 - 4.0
    with torch.no_grad():
        emb = model.get_audio_features(input_features=mel).pooler_output
        pooled = model.audio_model(input_features=mel).pooler_output
    np.savez_compressed(OUT / "htsat.npz", mel=mel.numpy(), embedding=emb.numpy(), pooled=pooled.numpy())
    for f in sorted(OUT.glob("*.npz")):
        print(f.name, f.stat().st_size)


if __name__ == "__main__":
    main()
