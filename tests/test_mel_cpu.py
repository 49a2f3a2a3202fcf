"""CLAP log-mel oracle pinned against transformers' ClapFeatureExtractor (CPU)."""
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from oracle.mel_ref import log_mel, slaney_filters  # noqa: E402

GOLD = ROOT / "tests" / "golden" / "mel.npz"


def _clips(recipe):
    from clap2diffusion_amd.pipeline import synthetic_thunder
    return [synthetic_thunder(int(s), int(n) / 48_000) for s, n in recipe]


def test_oracle_matches_golden():
    g = np.load(GOLD)
    for c, off, ref in zip(_clips(g["recipe"]), g["crop"], g["features"]):
        if c.size > 48_000:
            c = c[off: off + 48_000]
        out = log_mel(c, max_len=48_000)
        assert out.shape == ref.shape
        assert np.abs(out - ref).max() < 1e-3


def test_filter_bank_matches_transformers():
    from transformers.audio_utils import mel_filter_bank
    from clap2diffusion_amd.features import slaney_mel_filters
    ref = mel_filter_bank(num_frequency_bins=513, num_mel_filters=64, min_frequency=0, max_frequency=14_000,
                          sampling_rate=48_000, norm="slaney", mel_scale="slaney")
    np.testing.assert_allclose(slaney_filters(513, 64, 0, 14_000, 48_000), ref, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(slaney_mel_filters(513, 64, 0, 14_000, 48_000), ref, rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("seconds", [10.0, 3.3])
def test_oracle_matches_transformers_full_length(seconds):
    from transformers import ClapFeatureExtractor
    from clap2diffusion_amd.pipeline import synthetic_thunder
    c = synthetic_thunder(7, seconds)
    ref = ClapFeatureExtractor(truncation="rand_trunc", padding="repeatpad")([c], sampling_rate=48_000,
                                                                            return_tensors="np")["input_features"][0, 0]
    out = log_mel(c)
    assert out.shape == (1001, 64)
    assert np.abs(out - ref).max() < 1e-3
