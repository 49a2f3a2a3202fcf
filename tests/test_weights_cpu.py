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
