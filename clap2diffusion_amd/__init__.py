"""clap2diffusion_amd — MI355X-native audio-conditioned SD1.5 sampling path.

Hot path (hand-written HIP for gfx950, C ABI in include/c2d.h): the UNet denoise
step (ResnetBlock2D, BasicTransformerBlock self-attention, the reference
AudioAttnProcessor cross-attention), the fused CFG+DDIM update and the CLAP
HTSAT audio tower.  Python keeps the reference API (AudioToImageInference,
AudioAttnProcessor / AudioProcessorManager, the audio projector modules).
"""
__version__ = "0.1.0"
