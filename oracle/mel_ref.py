"""CLAP log-mel oracle -- TEST INFRASTRUCTURE ONLY (float64 numpy).

Restates the reference's audio composition on ONE clip:
  preprocess(): CLAPAudioEncoder.preprocess_audio (models/audio_encoder.py:109-129):
    mono mean, zero-pad to max_len samples (np.pad mode "constant") or keep the first
    max_len;
  log_mel(): transformers ClapFeatureExtractor on that exact-length clip
    (feature_extraction_clap.py _get_input_mel -- at exact length neither repeat-pad
    nor the random crop fires -- and _np_extract_fbank_features ->
    audio_utils.spectrogram(window_function(1024, "hann") periodic, frame 1024, hop
    480, power 2, centre reflect pad, mel filters (Slaney scale + norm), log_mel "dB"
    = power_to_db: 10 log10(max(x, 1e-10)))), called by the reference through
    ClapProcessor at models/audio_encoder.py:163-167.
Pinned against transformers itself by tests/test_mel_cpu.py and the fixture
tests/golden/mel.npz (scripts/make_mel_golden.py).
"""
from __future__ import annotations

import numpy as np


def slaney_filters(n_bins: int, n_mels: int, fmin: float, fmax: float, sr: int) -> np.ndarray:
    def h2m(f):
        f = np.asarray(f, np.float64)
        return np.where(f >= 1000.0, 15.0 + np.log(np.maximum(f, 1e-30) / 1000.0) * 27.0 / np.log(6.4), 3.0 * f / 200.0)

    def m2h(m):
        return np.where(m >= 15.0, 1000.0 * np.exp(np.log(6.4) / 27.0 * (m - 15.0)), 200.0 * m / 3.0)

    hz = m2h(np.linspace(h2m(fmin), h2m(fmax), n_mels + 2))
    fft_f = np.linspace(0, sr // 2, n_bins)
    fb = np.zeros((n_bins, n_mels))
    for m in range(n_mels):  # plain triangle per filter (audio_utils._create_triangular_filter_bank)
        lo, c, hi = hz[m], hz[m + 1], hz[m + 2]
        up = (fft_f - lo) / (c - lo)
        down = (hi - fft_f) / (hi - c)
        fb[:, m] = np.maximum(0.0, np.minimum(up, down)) * 2.0 / (hi - lo)
    return fb


def preprocess(clip: np.ndarray, max_len: int = 480_000) -> np.ndarray:
    """models/audio_encoder.py:109-129: mono, then zero-pad / truncate to max_len."""
    x = np.asarray(clip, np.float64)
    if x.ndim > 1:
        x = x.mean(axis=-1)
    if x.size < max_len:
        return np.pad(x, (0, max_len - x.size), mode="constant")
    return x[:max_len]


def log_mel(clip: np.ndarray, max_len: int = 480_000, sr: int = 48_000, n_fft: int = 1024, hop: int = 480,
            n_mels: int = 64, fmin: float = 0.0, fmax: float = 14_000.0) -> np.ndarray:
    """clip (any length) -> preprocess -> [1 + max_len // hop, n_mels] float64 dB features."""
    w = preprocess(clip, max_len)
    w = np.pad(w, n_fft // 2, mode="reflect")
    win = np.hanning(n_fft + 1)[:-1]
    frames = 1 + (w.size - n_fft) // hop
    idx = np.arange(frames)[:, None] * hop + np.arange(n_fft)[None, :]
    spec = np.abs(np.fft.rfft(w[idx] * win, axis=1)) ** 2          # [frames, bins]
    mel = np.maximum(1e-10, spec @ slaney_filters(n_fft // 2 + 1, n_mels, fmin, fmax, sr))
    return 10.0 * np.log10(np.maximum(mel, 1e-10))
