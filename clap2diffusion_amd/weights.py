"""Deterministic synthetic weights in the checkpoint key
layouts the reference stack loads: diffusers-0.23.1 UNet2DConditionModel /
AutoencoderKL keys for SD1.5, transformers ClapModel keys for HTSAT.

No network and no checkpoints exist here, so every weight is drawn from a
per-tensor seeded generator (seed = f(base_seed, crc32(key))): the same key
gives the same tensor on every rank and in every process.  Scales are chosen
to keep activations O(1) through 50 DDIM steps; norm affines are non-trivial
(gamma ~ 1 + 0.1 N(0,1), beta ~ 0.1 N(0,1)) so the parity tests exercise them.
"""
from __future__ import annotations

import math
import zlib
from collections import OrderedDict

import torch

SD15_UNET = dict(
    in_channels=4, out_channels=4, block_out_channels=(320, 640, 1280, 1280), layers_per_block=2,
    cross_attention_dim=768, heads=8, norm_groups=32, norm_eps=1e-5, attn_blocks=(True, True, True, False),
)

SD15_VAE = dict(latent_channels=4, block_out_channels=(128, 256, 512, 512), layers_per_block=2, norm_groups=32,
                out_channels=3)


def unet_param_shapes(cfg: dict = SD15_UNET) -> "OrderedDict[str, tuple]":
    """diffusers UNet2DConditionModel state-dict keys -> shapes (SD1.5 topology)."""
    S: "OrderedDict[str, tuple]" = OrderedDict()
    ch = cfg["block_out_channels"]
    ctx = cfg["cross_attention_dim"]
    temb = ch[0] * 4

    def lin(p, i, o, bias=True):
        S[p + ".weight"] = (o, i)
        if bias:
            S[p + ".bias"] = (o,)

    def conv(p, i, o, k):
        S[p + ".weight"] = (o, i, k, k)
        S[p + ".bias"] = (o,)

    def norm(p, c):
        S[p + ".weight"] = (c,)
        S[p + ".bias"] = (c,)

    def resnet(p, i, o):
        norm(p + ".norm1", i)
        conv(p + ".conv1", i, o, 3)
        lin(p + ".time_emb_proj", temb, o)
        norm(p + ".norm2", o)
        conv(p + ".conv2", o, o, 3)
        if i != o:
            conv(p + ".conv_shortcut", i, o, 1)

    def transformer(p, c):
        norm(p + ".norm", c)
        conv(p + ".proj_in", c, c, 1)
        b = p + ".transformer_blocks.0"
        norm(b + ".norm1", c)
        for n in ("to_q", "to_k", "to_v"):
            lin(f"{b}.attn1.{n}", c, c, bias=False)
        lin(b + ".attn1.to_out.0", c, c)
        norm(b + ".norm2", c)
        lin(b + ".attn2.to_q", c, c, bias=False)
        lin(b + ".attn2.to_k", ctx, c, bias=False)
        lin(b + ".attn2.to_v", ctx, c, bias=False)
        lin(b + ".attn2.to_out.0", c, c)
        norm(b + ".norm3", c)
        lin(b + ".ff.net.0.proj", c, 8 * c)
        lin(b + ".ff.net.2", 4 * c, c)
        conv(p + ".proj_out", c, c, 1)

    lin("time_embedding.linear_1", ch[0], temb)
    lin("time_embedding.linear_2", temb, temb)
    conv("conv_in", cfg["in_channels"], ch[0], 3)
    out_c = ch[0]
    for i, c in enumerate(ch):
        in_c, out_c = out_c, c
        for j in range(cfg["layers_per_block"]):
            resnet(f"down_blocks.{i}.resnets.{j}", in_c if j == 0 else out_c, out_c)
            if cfg["attn_blocks"][i]:
                transformer(f"down_blocks.{i}.attentions.{j}", out_c)
        if i < len(ch) - 1:
            conv(f"down_blocks.{i}.downsamplers.0.conv", out_c, out_c, 3)
    resnet("mid_block.resnets.0", ch[-1], ch[-1])
    transformer("mid_block.attentions.0", ch[-1])
    resnet("mid_block.resnets.1", ch[-1], ch[-1])
    rev = list(reversed(ch))
    rev_attn = list(reversed(cfg["attn_blocks"]))
    out_c = rev[0]
    for i in range(len(rev)):
        prev_c, out_c = out_c, rev[i]
        in_c = rev[min(i + 1, len(rev) - 1)]
        n = cfg["layers_per_block"] + 1
        for j in range(n):
            skip = in_c if j == n - 1 else out_c
            r_in = prev_c if j == 0 else out_c
            resnet(f"up_blocks.{i}.resnets.{j}", r_in + skip, out_c)
            if rev_attn[i]:
                transformer(f"up_blocks.{i}.attentions.{j}", out_c)
        if i < len(rev) - 1:
            conv(f"up_blocks.{i}.upsamplers.0.conv", out_c, out_c, 3)
    norm("conv_norm_out", ch[0])
    conv("conv_out", ch[0], cfg["out_channels"], 3)
    return S


def vae_decoder_param_shapes(cfg: dict = SD15_VAE) -> "OrderedDict[str, tuple]":
    """diffusers AutoencoderKL decoder + post_quant_conv keys (SD1.5 topology)."""
    S: "OrderedDict[str, tuple]" = OrderedDict()
    ch = list(reversed(cfg["block_out_channels"]))

    def conv(p, i, o, k):
        S[p + ".weight"] = (o, i, k, k)
        S[p + ".bias"] = (o,)

    def norm(p, c):
        S[p + ".weight"] = (c,)
        S[p + ".bias"] = (c,)

    def resnet(p, i, o):
        norm(p + ".norm1", i)
        conv(p + ".conv1", i, o, 3)
        norm(p + ".norm2", o)
        conv(p + ".conv2", o, o, 3)
        if i != o:
            conv(p + ".conv_shortcut", i, o, 1)

    lc = cfg["latent_channels"]
    conv("post_quant_conv", lc, lc, 1)
    conv("decoder.conv_in", lc, ch[0], 3)
    resnet("decoder.mid_block.resnets.0", ch[0], ch[0])
    a = "decoder.mid_block.attentions.0"
    norm(a + ".group_norm", ch[0])
    for n in ("to_q", "to_k", "to_v", "to_out.0"):
        S[f"{a}.{n}.weight"] = (ch[0], ch[0])
        S[f"{a}.{n}.bias"] = (ch[0],)
    resnet("decoder.mid_block.resnets.1", ch[0], ch[0])
    out_c = ch[0]
    for i, c in enumerate(ch):
        prev, out_c = out_c, c
        for j in range(cfg["layers_per_block"] + 1):
            resnet(f"decoder.up_blocks.{i}.resnets.{j}", prev if j == 0 else out_c, out_c)
        if i < len(ch) - 1:
            conv(f"decoder.up_blocks.{i}.upsamplers.0.conv", out_c, out_c, 3)
    norm("decoder.conv_norm_out", ch[-1])
    conv("decoder.conv_out", ch[-1], cfg["out_channels"], 3)
    return S


def key_seed(base: int, key: str) -> int:
    return (base * 1000003 + zlib.crc32(key.encode())) % (2 ** 31 - 1)


def _init_one(key: str, shape: tuple, gen: torch.Generator, device) -> torch.Tensor:
    leaf = key.rsplit(".", 2)
    is_norm = any(s in key for s in ("norm", "group_norm")) and len(shape) == 1
    if is_norm and key.endswith(".weight"):
        return 1.0 + 0.1 * torch.randn(shape, generator=gen, device=device)
    if key.endswith(".bias"):
        return 0.02 * torch.randn(shape, generator=gen, device=device) if not is_norm else \
            0.1 * torch.randn(shape, generator=gen, device=device)
    if len(shape) == 4:  # conv: torch-default-like scale 1/sqrt(3 fan_in)
        fan_in = shape[1] * shape[2] * shape[3]
        std = 1.0 / math.sqrt(3.0 * fan_in)
        if key.startswith("conv_out") or key.endswith("decoder.conv_out.weight"):
            std *= 0.5
        return std * torch.randn(shape, generator=gen, device=device)
    if len(shape) == 2:  # linear: N(0, 0.02^2), attention/ff projections
        del leaf
        return 0.02 * torch.randn(shape, generator=gen, device=device)
    return torch.randn(shape, generator=gen, device=device)


def synth_state_dict(shapes: "OrderedDict[str, tuple]", seed: int = 0, device="cpu",
                     dtype=torch.float32) -> "OrderedDict[str, torch.Tensor]":
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    gen = torch.Generator(device=device)
    for k, shp in shapes.items():
        gen.manual_seed(key_seed(seed, k))
        sd[k] = _init_one(k, shp, gen, device).to(dtype)
    return sd


def synth_unet(seed: int = 0, device="cpu", dtype=torch.float32, cfg: dict = SD15_UNET):
    return synth_state_dict(unet_param_shapes(cfg), seed, device, dtype)


def synth_vae_decoder(seed: int = 0, device="cpu", dtype=torch.float32, cfg: dict = SD15_VAE):
    return synth_state_dict(vae_decoder_param_shapes(cfg), seed + 17, device, dtype)


def synth_processor_weights(level: str, seed: int = 0, audio_dim: int = 768, hidden_dim: int = 768,
                            bottleneck: int = 64) -> "OrderedDict[str, torch.Tensor]":
    """AudioAttnProcessor state dict (reference models/audio_attention_processor.py:33-41):
    audio_proj.0 Linear(audio_dim, 64), audio_proj.3 Linear(64, hidden_dim), alpha [1]."""
    shapes = OrderedDict([
        ("audio_proj.0.weight", (bottleneck, audio_dim)), ("audio_proj.0.bias", (bottleneck,)),
        ("audio_proj.3.weight", (hidden_dim, bottleneck)), ("audio_proj.3.bias", (hidden_dim,)),
    ])
    sd = OrderedDict()
    g = torch.Generator()
    for k, s in shapes.items():
        g.manual_seed(key_seed(seed, f"proc.{level}.{k}"))
        fan_in = s[1] if len(s) == 2 else s[0]
        sd[k] = torch.randn(s, generator=g) / math.sqrt(fan_in)
    g.manual_seed(key_seed(seed, f"proc.{level}.alpha"))
    sd["alpha"] = torch.randn(1, generator=g)
    return sd


def param_count(shapes) -> int:
    return sum(math.prod(s) for s in shapes.values())


# ------------------------------------------------------------------ HTSAT / generic
HTSAT_CFG = dict(depths=(2, 2, 6, 2), embed=96, heads=(4, 8, 16, 32), window=8, mlp_ratio=4, mel_bins=64,
                 hidden=768, proj_dim=512)


def htsat_param_shapes(cfg: dict = HTSAT_CFG) -> "OrderedDict[str, tuple]":
    """transformers ClapModel audio keys (htsat-unfused, enable_fusion False):
    audio_model.audio_encoder.* and audio_projection.* (modeling_clap.py:720-921)."""
    S: "OrderedDict[str, tuple]" = OrderedDict()
    e = "audio_model.audio_encoder."
    S[e + "patch_embed.proj.weight"] = (cfg["embed"], 1, 4, 4)
    S[e + "patch_embed.proj.bias"] = (cfg["embed"],)
    S[e + "patch_embed.norm.weight"] = (cfg["embed"],)
    S[e + "patch_embed.norm.bias"] = (cfg["embed"],)
    w = cfg["window"]
    for i, depth in enumerate(cfg["depths"]):
        dim = cfg["embed"] * 2 ** i
        for j in range(depth):
            b = f"{e}layers.{i}.blocks.{j}."
            S[b + "layernorm_before.weight"] = (dim,)
            S[b + "layernorm_before.bias"] = (dim,)
            S[b + "attention.self.relative_position_bias_table"] = ((2 * w - 1) ** 2, cfg["heads"][i])
            for n in ("query", "key", "value"):
                S[f"{b}attention.self.{n}.weight"] = (dim, dim)
                S[f"{b}attention.self.{n}.bias"] = (dim,)
            S[b + "attention.output.dense.weight"] = (dim, dim)
            S[b + "attention.output.dense.bias"] = (dim,)
            S[b + "layernorm_after.weight"] = (dim,)
            S[b + "layernorm_after.bias"] = (dim,)
            S[b + "intermediate.dense.weight"] = (cfg["mlp_ratio"] * dim, dim)
            S[b + "intermediate.dense.bias"] = (cfg["mlp_ratio"] * dim,)
            S[b + "output.dense.weight"] = (dim, cfg["mlp_ratio"] * dim)
            S[b + "output.dense.bias"] = (dim,)
        if i < len(cfg["depths"]) - 1:
            S[f"{e}layers.{i}.downsample.reduction.weight"] = (2 * dim, 4 * dim)
            S[f"{e}layers.{i}.downsample.norm.weight"] = (4 * dim,)
            S[f"{e}layers.{i}.downsample.norm.bias"] = (4 * dim,)
    for n in ("weight", "bias", "running_mean", "running_var"):
        S[f"{e}batch_norm.{n}"] = (cfg["mel_bins"],)
    S[e + "norm.weight"] = (cfg["hidden"],)
    S[e + "norm.bias"] = (cfg["hidden"],)
    S["audio_projection.linear1.weight"] = (cfg["proj_dim"], cfg["hidden"])
    S["audio_projection.linear1.bias"] = (cfg["proj_dim"],)
    S["audio_projection.linear2.weight"] = (cfg["proj_dim"], cfg["proj_dim"])
    S["audio_projection.linear2.bias"] = (cfg["proj_dim"],)
    return S


def synth_generic(shapes, seed: int = 0, tag: str = "", device="cpu") -> "OrderedDict[str, torch.Tensor]":
    """Name-pattern synthetic init for small modules (HTSAT, projectors)."""
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    g = torch.Generator(device=device)
    for k, s in shapes.items():
        s = tuple(s)
        g.manual_seed(key_seed(seed, tag + k))
        r = torch.randn(s, generator=g, device=device) if len(s) else torch.randn((), generator=g, device=device)
        leaf = k.rsplit(".", 1)[-1]
        normish = any(t in k for t in ("norm", "ln_", "layer_norms", "batch_norm")) or k.endswith("ffn.0.weight") \
            or k.endswith("ffn.0.bias") or k.endswith("shared_mlp.2.weight") or k.endswith("shared_mlp.2.bias") \
            or k.endswith("weight_network.2.weight") or k.endswith("weight_network.2.bias") \
            or k.endswith("output_proj.1.weight") or k.endswith("output_proj.1.bias")
        if leaf == "running_var":
            v = 0.5 + r.abs()
        elif leaf == "running_mean":
            v = 0.1 * r
        elif len(s) == 1 and normish and leaf == "weight":
            v = 1.0 + 0.1 * r
        elif len(s) == 1 and normish and leaf == "bias":
            v = 0.1 * r
        elif leaf in ("bias", "in_proj_bias"):
            v = 0.02 * r
        elif "relative_position_bias_table" in k:
            v = 0.5 * r
        elif len(s) >= 2 and (leaf in ("weight", "in_proj_weight")):
            v = r / math.sqrt(math.prod(s[1:]))
        else:
            v = 0.1 * r
        sd[k] = v
    return sd


def synth_htsat(seed: int = 0, device="cpu") -> "OrderedDict[str, torch.Tensor]":
    return synth_generic(htsat_param_shapes(), seed, "htsat.", device)


def clap_audio_state_dict(ck: dict) -> "OrderedDict[str, torch.Tensor]":
    """Audio-tower keys of a CLAP checkpoint, as HTSATEncoder.load_clap_state_dict takes
    them (audio_model.audio_encoder.*, audio_projection.*).  Accepts a ClapModel state dict,
    the reference's CLAPAudioEncoder state dict (models/audio_encoder.py:47: keys under
    "clap_model."), or either wrapped in {"state_dict" | "model_state_dict": ...} -- the
    forms a clap_encoder.pth (scripts/inference.py:38-41) can take."""
    for wrap in ("state_dict", "model_state_dict"):
        if isinstance(ck.get(wrap), dict):
            ck = ck[wrap]
    out: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    for k, v in ck.items():
        k2 = k[len("clap_model."):] if k.startswith("clap_model.") else k
        if k2.startswith("audio_model.") or k2.startswith("audio_projection."):
            out[k2] = v
    if not out:
        raise KeyError("no CLAP audio-tower keys (audio_model.* / audio_projection.*) in checkpoint")
    return out


PROCESSOR_KEYS = ("audio_proj.0.weight", "audio_proj.0.bias", "audio_proj.3.weight", "audio_proj.3.bias", "alpha")


def processor_state_dicts(ck: dict, level_mapping: dict) -> "dict[str, OrderedDict]":
    """Per-level AudioAttnProcessor state dicts (audio_proj.0/3 weight+bias, alpha) from a
    unet_adapter_final.pth (reference scripts/inference.py:61-65, app/gradio_app.py:39-46,
    scripts/train_stage3.py:78-81; the reference never writes the file, so every natural form
    is read):
      {"early"|"mid"|"late": {audio_proj..., alpha}}            per-level dicts
      {"<level>.audio_proj.0.weight", ...}                       flat, level-prefixed (any prefix
                                                                 ending in the level name)
      {"<processor name>.audio_proj.0.weight", ...}              keyed by unet.attn_processors
                                                                 names (diffusers AttnProcsLayers),
                                                                 e.g. down_blocks.0....attn2.processor.*
      {"audio_proj.0.weight", ...}                               one processor for every level
    optionally wrapped in {"state_dict" | "model_state_dict" | "processor_state_dict" |
    "unet_adapter_state_dict" | "processors": ...}.  level_mapping: AudioProcessorManager's
    {level: [processor names]}.  Returns {} when nothing is recognised."""
    for wrap in ("state_dict", "model_state_dict", "processor_state_dict", "unet_adapter_state_dict", "processors"):
        if isinstance(ck.get(wrap), dict):
            ck = ck[wrap]
    out: "dict[str, OrderedDict]" = {}
    if all(isinstance(ck.get(lv), dict) for lv in ("early", "mid", "late") if lv in ck) and \
            any(isinstance(ck.get(lv), dict) for lv in ("early", "mid", "late")):
        for lv in ("early", "mid", "late"):
            if isinstance(ck.get(lv), dict) and all(k in ck[lv] for k in PROCESSOR_KEYS):
                out[lv] = OrderedDict((k, ck[lv][k]) for k in PROCESSOR_KEYS)
        return out
    if all(k in ck for k in PROCESSOR_KEYS):
        return {lv: OrderedDict((k, ck[k]) for k in PROCESSOR_KEYS) for lv in ("early", "mid", "late")}
    name_level = {n.rsplit(".processor", 1)[0]: lv for lv, names in level_mapping.items() for n in names}
    for k, v in ck.items():
        for pk in PROCESSOR_KEYS:
            if not k.endswith("." + pk):
                continue
            prefix = k[: -len(pk) - 1]
            stem = prefix[: -len(".processor")] if prefix.endswith(".processor") else prefix
            lv = name_level.get(stem)
            if lv is None:
                last = prefix.rsplit(".", 1)[-1]
                lv = last if last in ("early", "mid", "late") else None
            if lv is not None:
                out.setdefault(lv, OrderedDict())[pk] = v
    return {lv: OrderedDict((k, sd[k]) for k in PROCESSOR_KEYS) for lv, sd in out.items()
            if all(k in sd for k in PROCESSOR_KEYS)}


def resolve_clap_weights(checkpoint_dir, clap_model_path=None, seed: int = 0):
    """(state dict, source) for the HTSAT tower, in the pipeline's order of precedence:
      1. an explicit clap_model_path (--clap_model: a ClapModel weights file or folder) -- what
         the user asked for wins;
      2. checkpoint_dir/clap_encoder.pth (reference scripts/inference.py:38-41, which only
         announces the file: it never loads or writes it, so its format is open) when it holds
         CLAP audio-tower keys in a clap_audio_state_dict form; a file without them is reported
         (warnings.warn) and skipped, as the reference carries on;
      3. the seeded synthetic recipe synth_htsat(seed)."""
    import warnings
    from pathlib import Path
    if clap_model_path:
        cp = Path(clap_model_path)
        cp = find_weights_file(cp, ("model", "pytorch_model")) if cp.is_dir() else cp
        return clap_audio_state_dict(load_weights_file(cp)), f"--clap_model {cp}"
    path = Path(checkpoint_dir) / "clap_encoder.pth"
    if path.exists():
        try:
            return clap_audio_state_dict(torch.load(path, map_location="cpu", weights_only=True)), str(path)
        except KeyError as e:
            warnings.warn(f"{path}: {e}; keeping the seeded CLAP weights")
    return synth_htsat(seed), f"seeded synthetic weights (seed {seed})"


# ------------------------------------------------------------------ checkpoint files
def load_weights_file(path) -> dict:
    """A state dict from a .safetensors file (safetensors loader) or a torch .bin / .pt /
    .pth file (torch.load with weights_only=True: nothing in the file is executed)."""
    path = str(path)
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    return torch.load(path, map_location="cpu", weights_only=True)


def find_weights_file(folder, stems=("diffusion_pytorch_model", "model", "pytorch_model")):
    """The first <stem>.safetensors / <stem>.bin present in a diffusers / transformers folder."""
    from pathlib import Path
    folder = Path(folder)
    for stem in stems:
        for ext in (".safetensors", ".bin"):
            f = folder / (stem + ext)
            if f.exists():
                return f
    raise FileNotFoundError(f"no {'/'.join(stems)}.safetensors|.bin under {folder}")


# diffusers < 0.14 VAE attention names (what the SD1.5 vae/ files carry) -> current ones
_VAE_OLD_ATTN = {"query": "to_q", "key": "to_k", "value": "to_v", "proj_attn": "to_out.0"}


def vae_decoder_state_dict(sd: dict) -> "OrderedDict[str, torch.Tensor]":
    """Decoder half of an AutoencoderKL state dict (decoder.*, post_quant_conv.*), with the
    old mid-block attention names renamed and their 1x1-conv weights flattened to Linear."""
    out: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    for k, v in sd.items():
        if not (k.startswith("decoder.") or k.startswith("post_quant_conv.")):
            continue
        parts = k.split(".")
        if "attentions" in parts and len(parts) >= 2 and parts[-2] in _VAE_OLD_ATTN:
            k = ".".join(parts[:-2] + [_VAE_OLD_ATTN[parts[-2]], parts[-1]])
            if v.dim() == 4:
                v = v[:, :, 0, 0]
        out[k] = v
    if "post_quant_conv.weight" not in out:
        raise KeyError("no AutoencoderKL decoder keys (decoder.* / post_quant_conv.*) in checkpoint")
    return out


def load_sd15_folder(folder) -> dict:
    """SD1.5 weights from a diffusers-format folder (unet/, vae/, text_encoder/, each a
    *.safetensors or *.bin): {"unet": ..., "vae": decoder keys, "text_encoder": ...}."""
    from pathlib import Path
    folder = Path(folder)
    return {"unet": load_weights_file(find_weights_file(folder / "unet")),
            "vae": vae_decoder_state_dict(load_weights_file(find_weights_file(folder / "vae"))),
            "text_encoder": load_weights_file(find_weights_file(folder / "text_encoder", ("model", "pytorch_model")))}


# ------------------------------------------------------------------ CLIP text tower
CLIP_TEXT_CFG = dict(vocab=49408, width=768, layers=12, heads=12, mlp=3072, max_len=77)


def clip_text_param_shapes(cfg: dict = CLIP_TEXT_CFG) -> "OrderedDict[str, tuple]":
    """CLIPTextModel keys of the SD1.5 text_encoder checkpoint (transformers 4.35
    layout, "text_model." prefix; modeling_clip.py CLIPTextTransformer)."""
    S: "OrderedDict[str, tuple]" = OrderedDict()
    t, w, f = "text_model.", cfg["width"], cfg["mlp"]
    S[t + "embeddings.token_embedding.weight"] = (cfg["vocab"], w)
    S[t + "embeddings.position_embedding.weight"] = (cfg["max_len"], w)
    for i in range(cfg["layers"]):
        b = f"{t}encoder.layers.{i}."
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            S[f"{b}self_attn.{n}.weight"] = (w, w)
            S[f"{b}self_attn.{n}.bias"] = (w,)
        S[b + "layer_norm1.weight"] = (w,)
        S[b + "layer_norm1.bias"] = (w,)
        S[b + "mlp.fc1.weight"] = (f, w)
        S[b + "mlp.fc1.bias"] = (f,)
        S[b + "mlp.fc2.weight"] = (w, f)
        S[b + "mlp.fc2.bias"] = (w,)
        S[b + "layer_norm2.weight"] = (w,)
        S[b + "layer_norm2.bias"] = (w,)
    S[t + "final_layer_norm.weight"] = (w,)
    S[t + "final_layer_norm.bias"] = (w,)
    return S


def synth_clip_text(seed: int = 0, device="cpu") -> "OrderedDict[str, torch.Tensor]":
    """Seeded CLIP text tower (Appendix B recipe): embeddings N(0, 0.02^2) (CLIP's own
    init scale), linears N(0, 1/fan_in), LayerNorm gamma 1 + 0.1 N, beta 0.1 N."""
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    g = torch.Generator(device=device)
    for k, shp in clip_text_param_shapes().items():
        g.manual_seed(key_seed(seed, "clip." + k))
        r = torch.randn(shp, generator=g, device=device)
        if "embedding" in k:
            v = 0.02 * r
        elif "layer_norm" in k:
            v = (1.0 + 0.1 * r) if k.endswith(".weight") else 0.1 * r
        elif k.endswith(".bias"):
            v = 0.02 * r
        else:
            v = r / math.sqrt(shp[1])
        sd[k] = v
    return sd


def fill_module(module, tag: str, seed: int = 0, keep=("decomposer.temperature", "decomposer.level_prior")):
    """Deterministically (re)initialise every floating tensor of a torch module by key."""
    sd = module.state_dict()
    shapes = {k: tuple(v.shape) for k, v in sd.items() if v.is_floating_point() and k not in keep}
    module.load_state_dict({**sd, **synth_generic(shapes, seed, tag)})
    return module
