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
    # exact length, short (zero tail) and long (first second kept) clips
    g = np.load(GOLD)
    for c, ref in zip(_clips(g["recipe"]), g["features"]):
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


@pytest.mark.parametrize("seconds", [10.0, 3.3, 12.5])
def test_oracle_matches_transformers_full_length(seconds):
    # the reference zero-pads / truncates to 10 s (models/audio_encoder.py:121-129) before
    # ClapProcessor (:163-167): restated here inline, the extractor is transformers' own
    from transformers import ClapFeatureExtractor
    from clap2diffusion_amd.pipeline import synthetic_thunder
    c = synthetic_thunder(7, seconds)
    t = 480_000
    cp = np.pad(c, (0, t - len(c)), mode="constant") if len(c) < t else c[:t]
    ref = ClapFeatureExtractor(truncation="rand_trunc", padding="repeatpad")([cp], sampling_rate=48_000,
                                                                             return_tensors="np")["input_features"][0, 0]
    out = log_mel(c)
    assert out.shape == (1001, 64)
    assert np.abs(out - ref).max() < 1e-3


def test_preprocess_zero_pads_and_truncates():
    from oracle.mel_ref import preprocess
    x = np.arange(1, 6, dtype=np.float32)
    np.testing.assert_array_equal(preprocess(x, 8), [1, 2, 3, 4, 5, 0, 0, 0])
    np.testing.assert_array_equal(preprocess(x, 3), [1, 2, 3])
    st = np.stack([x, 3 * x], 1)  # [samples, channels] -> mono mean
    np.testing.assert_array_equal(preprocess(st, 5), 2 * x)


def test_product_crop_matches_reference_truncation():
    # host half of the product path: first max_len samples, no random offset, mono mean
    from clap2diffusion_amd.features import ClapLogMel
    fe = ClapLogMel.__new__(ClapLogMel)
    fe.max_len = 4
    x = np.arange(10, dtype=np.float32)
    np.random.seed(0)
    a = fe.crop([x, x[:2], np.stack([x, x], 1), np.zeros(0, np.float32)])
    np.testing.assert_array_equal(a[0], [0, 1, 2, 3])
    np.testing.assert_array_equal(a[1], [0, 1])
    np.testing.assert_array_equal(a[2], [0, 1, 2, 3])
    # an empty clip passes through (length 0): the kernel zero-pads it to max_len samples of
    # silence, as the reference's preprocess_audio zero-pads (models/audio_encoder.py:123-126)
    assert a[3].size == 0
