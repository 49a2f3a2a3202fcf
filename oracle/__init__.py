"""CPU oracle — TEST INFRASTRUCTURE ONLY.

An fp32 PyTorch-CPU restatement of the reference's sampling path, used by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker.  The product path (clap2diffusion_amd) never imports this package.

  unet_ref.py      SD1.5 UNet2DConditionModel forward (diffusers 0.23.1 semantics,
                   SURVEY.md Appendix A) with the reference AudioAttnProcessor
                   arithmetic (models/audio_attention_processor.py:62-145) in every
                   cross-attention, routed per AudioProcessorManager (:158-193).
  ddim_ref.py      DDIMScheduler (scaled_linear, leading spacing, steps_offset 1,
                   set_alpha_to_one False, eta 0) + classifier-free guidance loop.
  htsat_ref.py     transformers ClapAudioEncoder + ClapProjectionLayer forward
                   (modeling_clap.py:720-921, 1503-1536), called by the reference
                   at models/audio_encoder.py:171-174.
  vae_ref.py       AutoencoderKL decoder (SD1.5), next-row component.

Parity pinning: the processor / projector arithmetic is pinned by golden
vectors generated from the reference's own modules (tests/golden/, script
scripts/make_goldens.py) and the HTSAT restatement by goldens from the
transformers ClapModel the reference calls.  The UNet / DDIM / VAE parts are
restated from diffusers==0.23.1, which is absent from /root/reference and from
this image: parity for them is "unpinned by the reference" (SURVEY.md §8(c)).
"""
