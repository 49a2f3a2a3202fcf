"""Checkpoint-key plumbing on the CPU: the seeded CLIP text weights carry exactly the
CLIPTextModel keys / shapes, and clap_encoder.pth in any of the forms the reference can
save (scripts/inference.py:38-41, models/audio_encoder.py:47) reduces to the HTSAT keys."""
import torch

from clap2diffusion_amd import weights as W


def test_clip_text_keys_match_transformers():
    from oracle.clip_ref import clip_text_model
    m = clip_text_model(0)
    ref = {k: tuple(v.shape) for k, v in m.state_dict().items() if "position_ids" not in k}
    ours = {k.removeprefix("text_model."): tuple(v) for k, v in W.clip_text_param_shapes().items()}
    assert ours == {k.removeprefix("text_model."): v for k, v in ref.items()}
    sd = W.synth_clip_text(0)
    assert torch.equal(sd["text_model.encoder.layers.3.mlp.fc1.weight"],
                       W.synth_clip_text(0)["text_model.encoder.layers.3.mlp.fc1.weight"])


def test_clap_checkpoint_forms(tmp_path):
    sd = W.synth_htsat(3)
    wrapped = {"clap_model." + k: v for k, v in sd.items()}
    wrapped["clap_model.text_model.embeddings.word_embeddings.weight"] = torch.zeros(4, 4)
    for ck in (sd, wrapped, {"state_dict": wrapped}, {"model_state_dict": sd}):
        p = tmp_path / "clap_encoder.pth"
        torch.save(ck, p)
        got = W.clap_audio_state_dict(torch.load(p, map_location="cpu", weights_only=True))
        assert set(got) == set(sd) and all(torch.equal(got[k], sd[k]) for k in sd)


def test_weights_files_and_sd15_folder(tmp_path):
    """diffusers-folder loading: safetensors and .bin files, the AutoencoderKL decoder half with
    the pre-0.14 attention names (query/key/value/proj_attn, 1x1-conv shaped) renamed."""
    from safetensors.torch import save_file
    g = torch.Generator().manual_seed(0)
    unet = {"conv_in.weight": torch.randn(320, 4, 3, 3, generator=g), "conv_in.bias": torch.randn(320, generator=g)}
    a = "decoder.mid_block.attentions.0."
    vae = {"encoder.conv_in.weight": torch.randn(2, 2), "quant_conv.weight": torch.randn(8, 8, 1, 1),
           "post_quant_conv.weight": torch.randn(4, 4, 1, 1), "post_quant_conv.bias": torch.randn(4),
           a + "query.weight": torch.randn(512, 512, generator=g), a + "query.bias": torch.randn(512),
           a + "proj_attn.weight": torch.randn(512, 512, 1, 1, generator=g), a + "group_norm.weight": torch.ones(512)}
    text = {"text_model.final_layer_norm.weight": torch.ones(768)}
    for sub, sd, name in (("unet", unet, "diffusion_pytorch_model.safetensors"),
                          ("vae", vae, "diffusion_pytorch_model.safetensors")):
        (tmp_path / sub).mkdir()
        save_file(sd, str(tmp_path / sub / name))
    (tmp_path / "text_encoder").mkdir()
    torch.save(text, tmp_path / "text_encoder" / "pytorch_model.bin")
    out = W.load_sd15_folder(tmp_path)
    assert set(out["unet"]) == set(unet) and torch.equal(out["unet"]["conv_in.weight"], unet["conv_in.weight"])
    assert set(out["vae"]) == {"post_quant_conv.weight", "post_quant_conv.bias", a + "to_q.weight", a + "to_q.bias",
                               a + "to_out.0.weight", a + "group_norm.weight"}
    assert out["vae"][a + "to_out.0.weight"].shape == (512, 512)
    assert torch.equal(out["vae"][a + "to_out.0.weight"], vae[a + "proj_attn.weight"][:, :, 0, 0])
    assert torch.equal(out["text_encoder"]["text_model.final_layer_norm.weight"], torch.ones(768))


def test_clap_weight_precedence(tmp_path):
    """An explicit --clap_model file wins over checkpoint_dir/clap_encoder.pth; an unrecognised
    clap_encoder.pth is reported and skipped (the reference carries on); neither -> seeded."""
    import pytest
    ck = tmp_path / "ck"
    ck.mkdir()
    explicit = tmp_path / "clap.pth"
    torch.save(W.synth_htsat(5), explicit)
    torch.save({"clap_model." + k: v for k, v in W.synth_htsat(6).items()}, ck / "clap_encoder.pth")
    sd, src = W.resolve_clap_weights(ck, explicit, seed=0)
    k = "audio_projection.linear1.weight" if "audio_projection.linear1.weight" in sd else next(iter(sd))
    assert torch.equal(sd[k], W.synth_htsat(5)[k]) and "--clap_model" in src
    sd, src = W.resolve_clap_weights(ck, None, seed=0)
    assert torch.equal(sd[k], W.synth_htsat(6)[k]) and src.endswith("clap_encoder.pth")
    torch.save({"something_else.weight": torch.zeros(3)}, ck / "clap_encoder.pth")
    with pytest.warns(UserWarning, match="no CLAP audio-tower keys"):
        sd, src = W.resolve_clap_weights(ck, None, seed=2)
    assert torch.equal(sd[k], W.synth_htsat(2)[k]) and "seeded" in src
    sd, src = W.resolve_clap_weights(tmp_path / "nowhere", None, seed=1)
    assert torch.equal(sd[k], W.synth_htsat(1)[k])


def test_processor_checkpoint_forms():
    """unet_adapter_final.pth forms -> per-level AudioAttnProcessor state dicts."""
    mapping = {"early": ["down_blocks.0.attentions.0.transformer_blocks.0.attn2.processor"],
               "mid": ["mid_block.attentions.0.transformer_blocks.0.attn2.processor"],
               "late": ["up_blocks.1.attentions.2.transformer_blocks.0.attn2.processor"]}
    per = {lv: W.synth_processor_weights(lv, seed=i) for i, lv in enumerate(("early", "mid", "late"))}
    forms = [per, {"state_dict": per},
             {f"{lv}.{k}": v for lv, sd in per.items() for k, v in sd.items()},
             {f"processors.{lv}.{k}": v for lv, sd in per.items() for k, v in sd.items()},
             {f"{mapping[lv][0]}.{k}": v for lv, sd in per.items() for k, v in sd.items()}]
    for ck in forms:
        got = W.processor_state_dicts(ck, mapping)
        assert set(got) == {"early", "mid", "late"}, list(ck)[:3]
        for lv in got:
            assert all(torch.equal(got[lv][k], per[lv][k]) for k in W.PROCESSOR_KEYS)
    one = W.processor_state_dicts(per["mid"], mapping)   # a single processor for every level
    assert set(one) == {"early", "mid", "late"} and torch.equal(one["early"]["alpha"], per["mid"]["alpha"])
    assert W.processor_state_dicts({"foo.weight": torch.zeros(2)}, mapping) == {}
