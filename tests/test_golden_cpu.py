"""CPU tests: the oracle and the API-kept projector modules against golden
vectors produced by the reference's own code (scripts/make_goldens.py)."""
from pathlib import Path

import numpy as np
import pytest
import torch

from clap2diffusion_amd import projectors as P
from clap2diffusion_amd.weights import synth_generic, synth_htsat, synth_processor_weights
from oracle import unet_ref
from oracle.htsat_ref import htsat_forward

G = Path(__file__).resolve().parent / "golden"


def fill(module, tag):
    sd = module.state_dict()
    shapes = {k: tuple(v.shape) for k, v in sd.items() if v.is_floating_point() and k not in
              ("decomposer.temperature", "decomposer.level_prior")}
    module.load_state_dict({**sd, **synth_generic(shapes, 0, tag)})
    return module.eval()


def mini_attention_weights(c, seed, ctx=768):
    """Same draw order as scripts/make_goldens.py:MiniAttention (ctx = c: a self-attention layer)."""
    g = torch.Generator().manual_seed(seed)
    w = {}
    for name, (o, i, bias) in (("to_q", (c, c, False)), ("to_k", (c, ctx, False)), ("to_v", (c, ctx, False)),
                               ("to_out.0", (c, c, True))):
        w[name + ".weight"] = torch.randn((o, i), generator=g) / i ** 0.5
        if bias:
            w[name + ".bias"] = 0.02 * torch.randn((o,), generator=g)
    h_gen = g
    return w, h_gen


def test_projectors_match_reference():
    gd = np.load(G / "projectors.npz")
    clap = torch.from_numpy(gd["clap"])
    enc = fill(P.ImprovedHierarchicalAudioEncoder(), "improved.")
    ada = fill(P.AudioAdapter(), "adapter.")
    v4 = fill(P.HierarchicalAudioV4(), "v4.")
    with torch.no_grad():
        t77, info = enc(clap, return_all=True)
        a16 = ada(clap)
        v77, hier = v4(clap, return_intermediate=True)
    pairs = [(t77, "tokens_77"), (info["tokens_10"], "tokens_10"), (info["assignments"], "assignments"),
             (info["hierarchy_weights"], "hierarchy_weights"), (info["routed"]["early"], "routed_early"),
             (info["routed"]["mid"], "routed_mid"), (info["routed"]["late"], "routed_late"),
             (info["losses"]["entropy"], "loss_entropy"), (info["losses"]["orthogonality"], "loss_orth"),
             (info["losses"]["prior"], "loss_prior"), (a16, "adapter"),
             (P.normalize_tokens(a16, 60.0), "adapter_norm60"), (v77, "v4_tokens_77"),
             (hier["tokens10"], "v4_tokens_10")]
    for got, key in pairs:
        ref = torch.from_numpy(gd[key])
        assert torch.allclose(got, ref, atol=2e-5, rtol=1e-4), (key, (got - ref).abs().max().item())


def test_oracle_projector_matches_golden():
    """oracle/projectors_ref (plain tensor functions, no product module) against the
    reference-module goldens: the routed tokens the end-to-end oracle feeds its UNet."""
    from clap2diffusion_amd.weights import synth_generic
    from oracle.projectors_ref import projector_shapes, routed_tokens
    gd = np.load(G / "projectors.npz")
    sd = synth_generic(projector_shapes(), 0, "improved.")
    got = routed_tokens(torch.from_numpy(gd["clap"]), sd)
    pairs = [(got["tokens_10"], "tokens_10"), (got["assignments"], "assignments"),
             (got["hierarchy_weights"], "hierarchy_weights")] + \
            [(got["routed"][lv], "routed_" + lv) for lv in ("early", "mid", "late")]
    for t, key in pairs:
        ref = torch.from_numpy(gd[key])
        assert torch.allclose(t, ref, atol=2e-5, rtol=1e-4), (key, (t - ref).abs().max().item())


def test_projector_state_dict_keys_match_reference_layout():
    enc = P.ImprovedHierarchicalAudioEncoder()
    keys = set(enc.state_dict())
    for k in ("decomposer.shared_mlp.4.weight", "decomposer.cross_hierarchy_attn.mlp.3.bias",
              "router.level_gates.early", "projector.blocks.3.cross_attn.in_proj_weight",
              "adaptive_weights.weight_network.3.weight", "decomposer.temperature"):
        assert k in keys
    ada = P.AudioAdapter()
    assert "token_generator.audio_to_kv.3.weight" in ada.state_dict()
    assert "token_generator.self_attn_layers.3.to_qkv.weight" in ada.state_dict()


def test_temperature_scheduler():
    enc = P.ImprovedHierarchicalAudioEncoder()
    s = P.TemperatureScheduler(enc.decomposer, T_max=2.0, T_min=0.5, total_steps=2000)
    assert s.step(0) == 2.0 and s.step(100) == 2.0
    assert abs(s.step(2000) - 0.5) < 1e-9
    mid = s.step(1100)
    assert 0.5 < mid < 2.0 and abs(enc.decomposer.temperature.item() - mid) < 1e-6


@pytest.mark.parametrize("c,l", [(320, 48), (640, 32), (1280, 16), (1280, 8)])
@pytest.mark.parametrize("mode", ["add", "concat"])
def test_oracle_processor_matches_reference(c, l, mode):
    """oracle.unet_ref processor arithmetic vs the reference AudioAttnProcessor output."""
    gd = np.load(G / "processor.npz")
    ci = [(320, 48), (640, 32), (1280, 16), (1280, 8)].index((c, l))
    w, g = mini_attention_weights(c, 100 + ci)
    h = torch.from_numpy(gd[f"c{c}_l{l}_h"])
    ehs = torch.from_numpy(gd["ehs"])
    audio = torch.from_numpy(gd["audio"])
    pw = synth_processor_weights("mid", seed=ci)
    ref = unet_ref.UNetRef({f"x.{k}": v for k, v in w.items()}, processors={"mid": pw})
    if mode == "add":
        ctx = ref.audio_context("mid", ehs, {"mid": audio})
    else:
        a = torch.nn.functional.gelu(torch.nn.functional.linear(audio, pw["audio_proj.0.weight"], pw["audio_proj.0.bias"]))
        a = torch.nn.functional.linear(a, pw["audio_proj.3.weight"], pw["audio_proj.3.bias"])
        a = torch.nn.functional.adaptive_avg_pool1d(a.transpose(1, 2), 4).transpose(1, 2)
        ctx = torch.cat([ehs, a], dim=1)
    out = ref.attention("x", h, ctx)
    gold = torch.from_numpy(gd[f"c{c}_l{l}_{mode}_out"])
    assert torch.allclose(out, gold, atol=1e-5, rtol=1e-4), (out - gold).abs().max().item()


EXT_CASES = [("self_c320_l48", 320, 200, 320, "early"), ("self_c640_l32", 640, 201, 640, "early"),
             ("nd4_c320_6x8", 320, 210, 768, "mid"), ("nd4_c640_4x4", 640, 211, 768, "mid"),
             ("mask_query_c640_l32", 640, 220, 768, "late"), ("mask_key_c320_l48", 320, 221, 768, "late")]


@pytest.mark.parametrize("name,c,seed,ctx,level", EXT_CASES)
def test_oracle_processor_ext_matches_reference(name, c, seed, ctx, level):
    """oracle.unet_ref.processor_call vs the reference processor on its off-pipeline paths:
    encoder_hidden_states=None (K / V from the projected query), 4-D input, attention masks."""
    gd = np.load(G / "processor_ext.npz")
    w, _ = mini_attention_weights(c, seed, ctx)
    pw = synth_processor_weights(level, seed=seed)
    h = torch.from_numpy(gd[name + "_h"])
    mask = torch.from_numpy(gd[name + "_mask"]) if name + "_mask" in gd else None
    ehs = None if name.startswith("self") else torch.from_numpy(np.load(G / "processor.npz")["ehs"])
    audio = {level: torch.from_numpy(np.load(G / "processor.npz")["audio"])}
    out = unet_ref.processor_call(w, pw, h, ehs, audio, level, mask=mask)
    gold = torch.from_numpy(gd[name + "_out"])
    assert out.shape == gold.shape
    assert torch.allclose(out, gold, atol=1e-5, rtol=1e-4), (out - gold).abs().max().item()


def test_oracle_htsat_matches_transformers():
    gd = np.load(G / "htsat.npz")
    sd = synth_htsat(0)
    mel = torch.from_numpy(gd["mel"])
    with torch.no_grad():
        pooled = htsat_forward(sd, mel, return_pooled=True)
        emb = htsat_forward(sd, mel)
    assert torch.allclose(pooled, torch.from_numpy(gd["pooled"]), atol=1e-4, rtol=1e-4)
    assert torch.allclose(emb, torch.from_numpy(gd["embedding"]), atol=1e-5)


def test_level_mapping_oracle():
    assert unet_ref.level_of("down_blocks.1.attentions.0") == "early"
    assert unet_ref.level_of("down_blocks.2.attentions.1") == "late"
    assert unet_ref.level_of("up_blocks.1.attentions.2") == "late"
    assert unet_ref.level_of("up_blocks.3.attentions.0") == "mid"
    assert unet_ref.level_of("mid_block.attentions.0") == "mid"
