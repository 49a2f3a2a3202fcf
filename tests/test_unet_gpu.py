"""One full UNet denoise call (HIP, fp16) against the fp32 CPU oracle on the
same synthetic SD1.5 weights, with the audio-injecting processors routed by
AudioProcessorManager.  Tolerance: eps rel-L2 <= 1e-2."""
import pytest
import torch

from clap2diffusion_amd.processor import AudioProcessorManager
from clap2diffusion_amd.unet import UNet2DConditionModel
from clap2diffusion_amd.weights import synth_processor_weights, synth_unet
from oracle.unet_ref import UNetRef

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def unet_pair(dev):
    torch.set_num_threads(min(16, torch.get_num_threads()))
    sd = synth_unet(seed=0)
    hip = UNet2DConditionModel().to(dev)
    hip.load_diffusers_state_dict(sd)
    mgr = AudioProcessorManager(hip)
    mgr.setup_processors(verbose=False)
    procs = {}
    for level, p in mgr.level_processors().items():
        w = synth_processor_weights(level, seed=0)
        p.audio_proj[0].weight.data.copy_(w["audio_proj.0.weight"])
        p.audio_proj[0].bias.data.copy_(w["audio_proj.0.bias"])
        p.audio_proj[3].weight.data.copy_(w["audio_proj.3.weight"])
        p.audio_proj[3].bias.data.copy_(w["audio_proj.3.bias"])
        p.alpha.data.copy_(w["alpha"])
        p.to(dev).eval()
        procs[level] = w
    ref = UNetRef(sd, processors=procs)
    return hip, ref, mgr


def rel_l2(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.parametrize("hw,t", [(16, 981), (32, 501), (64, 1), (96, 741)])   # 96: config c5 (768^2)
def test_unet_step_matches_oracle(dev, unet_pair, hw, t):
    hip, ref, mgr = unet_pair
    g = torch.Generator().manual_seed(hw)
    n = 2
    x = torch.randn(n, 4, hw, hw, generator=g)
    ehs = torch.randn(n, 77, 768, generator=g)
    audio = {lv: torch.randn(n, 10, 768, generator=g) * 0.5 for lv in ("early", "mid", "late")}
    with torch.no_grad():
        e_ref = ref(x, t, ehs, audio)
        e_hip = hip(x.to(dev), t, ehs.to(dev),
                    cross_attention_kwargs=mgr.get_audio_kwargs({k: v.to(dev) for k, v in audio.items()})).sample
    torch.cuda.synchronize()
    assert torch.isfinite(e_hip).all()
    err = rel_l2(e_hip, e_ref)
    assert err <= 1e-2, f"eps rel-L2 {err:.3e}"


def test_unet_without_audio_and_batch4(dev, unet_pair):
    hip, ref, mgr = unet_pair
    g = torch.Generator().manual_seed(7)
    x = torch.randn(4, 4, 16, 16, generator=g)
    ehs = torch.randn(4, 77, 768, generator=g)
    with torch.no_grad():
        e_ref = ref(x, 261, ehs, None)
        e_hip = hip(x.to(dev), 261, ehs.to(dev)).sample
    assert rel_l2(e_hip, e_ref) <= 1e-2


def test_attn_processor_names_and_levels(unet_pair):
    hip, _, mgr = unet_pair
    names = list(hip.attn_processors.keys())
    assert len(names) == 32
    assert len(mgr.level_mapping["early"]) == 4
    assert len(mgr.level_mapping["mid"]) == 7
    assert len(mgr.level_mapping["late"]) == 5
