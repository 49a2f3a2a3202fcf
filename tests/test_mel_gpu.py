"""HIP CLAP log-mel (c2d_clap_log_mel) vs the transformers golden and the float64 oracle.

Tolerance: fp32 FFT / mel sums vs float64; |dB error| <= 2e-2 everywhere (features
then pass a BatchNorm and a bicubic resize in the HTSAT stem).
"""
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from oracle.mel_ref import log_mel  # noqa: E402

pytestmark = pytest.mark.gpu
TOL_DB = 2e-2


def test_log_mel_matches_golden(dev):
    from clap2diffusion_amd.features import ClapLogMel
    from clap2diffusion_amd.pipeline import synthetic_thunder
    # exact, short (zero tail) and long (first second kept) clips, as the reference composes them
    g = np.load(ROOT / "tests" / "golden" / "mel.npz")
    fe = ClapLogMel(dev, max_length_s=1)
    for (s, n), ref in zip(g["recipe"], g["features"]):
        out = fe([synthetic_thunder(int(s), int(n) / 48_000)])[0].cpu().numpy()
        assert np.abs(out - ref).max() < TOL_DB


def test_log_mel_batch_full_length(dev):
    # configs' 10 s / 48 kHz clips, mixed lengths in one launch: exact, short clips zero-padded
    # to 10 s (models/audio_encoder.py:123-126), a 12 s clip truncated to its first 10 s (:127-129)
    from clap2diffusion_amd.features import ClapLogMel
    from clap2diffusion_amd.pipeline import synthetic_thunder
    clips = [synthetic_thunder(0, 10.0), synthetic_thunder(1, 3.3), synthetic_thunder(2, 0.05),
             synthetic_thunder(3, 12.0)]
    fe = ClapLogMel(dev)
    out = fe(clips).cpu().numpy()
    assert out.shape == (4, 1001, 64)
    for c, o in zip(clips, out):
        assert np.abs(o - log_mel(c)).max() < TOL_DB
    # short clip == its explicit zero-padded 10 s version
    pad = np.zeros(480_000, np.float32)
    pad[: clips[1].size] = clips[1]
    assert np.abs(out[1] - fe([pad]).cpu().numpy()[0]).max() == 0.0


def test_log_mel_device_lengths_clamped(dev):
    # from_device with lengths outside [1, max_len]: clamped on the device (no fault, no garbage)
    from clap2diffusion_amd.features import ClapLogMel
    from clap2diffusion_amd.pipeline import synthetic_thunder
    fe = ClapLogMel(dev, max_length_s=1)
    c = synthetic_thunder(4, 1.5)
    wave = torch.from_numpy(np.concatenate([c, c])).to(dev)
    offs = torch.tensor([0, c.size], dtype=torch.int64, device=dev)
    lens = torch.tensor([c.size, 0], dtype=torch.int32, device=dev)
    out = fe.from_device(wave, offs, lens).cpu().numpy()
    assert np.abs(out[0] - log_mel(c, max_len=48_000)).max() < TOL_DB
    assert np.all(np.abs(out[1] + 100.0) < 1e-4)


def test_log_mel_silence_floor(dev):
    from clap2diffusion_amd.features import ClapLogMel
    fe = ClapLogMel(dev, max_length_s=1)
    out = fe([np.zeros(48_000, np.float32)]).cpu()
    assert torch.all((out + 100.0).abs() < 1e-4)


def test_log_mel_empty_clip_is_silence(dev):
    # the reference zero-pads an empty clip to max_len samples (models/audio_encoder.py:123-126):
    # log-mel of silence (-100 dB), beside a real clip and alone
    from clap2diffusion_amd.features import ClapLogMel
    from oracle.mel_ref import log_mel
    fe = ClapLogMel(dev, max_length_s=1)
    c = np.random.RandomState(3).randn(30_000).astype(np.float32) * 0.1
    out = fe([np.zeros(0, np.float32), c]).cpu().numpy()
    assert np.all(np.abs(out[0] + 100.0) < 1e-4)
    assert np.abs(out[1] - log_mel(c, max_len=48_000)).max() < TOL_DB
    alone = fe([np.zeros(0, np.float32)]).cpu().numpy()
    assert np.all(np.abs(alone + 100.0) < 1e-4)
