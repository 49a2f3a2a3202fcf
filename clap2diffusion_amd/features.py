"""CLAP log-mel front end on the GPU (c2d_clap_log_mel).

Does the work of the reference's audio composition: CLAPAudioEncoder.preprocess_audio
(models/audio_encoder.py:121-129: zero-pad a clip to target_length x sample_rate =
480,000 samples, or keep its first 480,000) followed by transformers' ClapProcessor /
ClapFeatureExtractor on that exact-length clip (models/audio_encoder.py:163-167; at
exact length the extractor's repeat-pad and random crop never fire).  Waveforms in,
[B, 1001, 64] fp32 dB log-mel features out, on device, ready for the HTSAT tower.
The host only truncates (a view, no copy) and builds the constant tables once
(periodic Hann window, Slaney mel filter bank of audio_utils.mel_filter_bank); the
zero padding, STFT, power, mel projection and dB run in one HIP kernel; there is no
CPU fallback.
"""
from __future__ import annotations

import numpy as np
import torch

from . import torch_ops  # noqa: F401  (registers c2d::clap_log_mel)


def _hz_to_mel_slaney(f):
    f = np.asarray(f, dtype=np.float64)
    m = 3.0 * f / 200.0
    log = f >= 1000.0
    return np.where(log, 15.0 + np.log(np.maximum(f, 1e-30) / 1000.0) * (27.0 / np.log(6.4)), m)


def _mel_to_hz_slaney(m):
    m = np.asarray(m, dtype=np.float64)
    f = 200.0 * m / 3.0
    log = m >= 15.0
    return np.where(log, 1000.0 * np.exp((np.log(6.4) / 27.0) * (m - 15.0)), f)


def slaney_mel_filters(n_bins: int, n_mels: int, fmin: float, fmax: float, sr: int) -> np.ndarray:
    """[n_bins, n_mels] triangular filters, Slaney scale and area norm
    (transformers audio_utils.mel_filter_bank(norm="slaney", mel_scale="slaney"))."""
    mel_pts = np.linspace(_hz_to_mel_slaney(fmin), _hz_to_mel_slaney(fmax), n_mels + 2)
    hz = _mel_to_hz_slaney(mel_pts)
    fft_freqs = np.linspace(0, sr // 2, n_bins)
    diff = np.diff(hz)
    slopes = hz[None, :] - fft_freqs[:, None]
    down = -slopes[:, :-2] / diff[:-1]
    up = slopes[:, 2:] / diff[1:]
    fb = np.maximum(0.0, np.minimum(down, up))
    return fb * (2.0 / (hz[2:n_mels + 2] - hz[:n_mels]))[None, :]


class ClapLogMel:
    """Device-side preprocess_audio (zero-pad / truncate to max_length_s) + ClapFeatureExtractor."""

    def __init__(self, device, feature_size: int = 64, sampling_rate: int = 48_000, hop_length: int = 480,
                 max_length_s: int = 10, fft_window_size: int = 1024, frequency_min: float = 0.0,
                 frequency_max: float = 14_000.0):
        self.device = torch.device(device)
        self.n_mels, self.sr, self.hop, self.n_fft = feature_size, sampling_rate, hop_length, fft_window_size
        self.max_len = max_length_s * sampling_rate
        self.frames = 1 + self.max_len // hop_length
        n_bins = fft_window_size // 2 + 1
        fb = slaney_mel_filters(n_bins, feature_size, frequency_min, frequency_max, sampling_rate)  # [bins, mels]
        nz = fb > 0
        rng = np.stack([nz.argmax(0), n_bins - nz[::-1].argmax(0)], 1).astype(np.int32)
        rng[~nz.any(0)] = 0
        win = np.hanning(fft_window_size + 1)[:-1]                # periodic Hann (audio_utils.window_function)
        self.window = torch.from_numpy(win.astype(np.float32)).to(self.device)
        self.filters = torch.from_numpy(np.ascontiguousarray(fb.T).astype(np.float32)).to(self.device)
        self.filter_range = torch.from_numpy(rng).to(self.device)

    def crop(self, audios: list) -> list:
        """Host part of preprocess_audio (models/audio_encoder.py:109-129): mono (channel
        mean of a [samples, channels] array) and the first max_len samples of a longer
        clip; shorter clips are zero-padded by the kernel (lengths < max_len) -- an empty
        clip included, which becomes max_len samples of silence as the reference's zero-pad
        (:123-126) makes it (c2d_clap_log_mel: length 0 -> -100 dB)."""
        out = []
        for a in audios:
            a = np.asarray(a, dtype=np.float32)
            if a.ndim > 1:
                a = a.mean(axis=-1)
            a = a.reshape(-1)
            out.append(a[: self.max_len])
        return out

    def __call__(self, audios: list, out: torch.Tensor | None = None) -> torch.Tensor:
        clips = self.crop(audios)
        lengths = np.array([c.size for c in clips], dtype=np.int32)
        offsets = np.concatenate([[0], np.cumsum(lengths[:-1], dtype=np.int64)]).astype(np.int64)
        flat = np.concatenate(clips) if clips else np.zeros(0, np.float32)
        if flat.size == 0:   # every clip empty: a one-sample buffer nothing reads (all lengths 0)
            flat = np.zeros(1, np.float32)
        wave = torch.from_numpy(flat).to(self.device)
        return self.from_device(wave, torch.from_numpy(offsets).to(self.device),
                                torch.from_numpy(lengths).to(self.device), out)

    def from_device(self, wave: torch.Tensor, offsets: torch.Tensor, lengths: torch.Tensor,
                    out: torch.Tensor | None = None) -> torch.Tensor:
        """wave fp32 (clips concatenated), offsets int64 [B], lengths int32 [B], all on device
        -> features fp32 [B, frames, n_mels].  The kernel clamps each length to [0, max_len]:
        a longer clip keeps its first max_len samples, a shorter one is zero-padded."""
        b = offsets.numel()
        assert wave.dtype == torch.float32 and offsets.dtype == torch.int64 and lengths.dtype == torch.int32
        if out is None:
            out = torch.empty(b, self.frames, self.n_mels, device=self.device, dtype=torch.float32)
        assert out.shape == (b, self.frames, self.n_mels) and out.is_contiguous()
        torch.ops.c2d.clap_log_mel(wave, offsets, lengths, self.max_len, self.n_fft, self.hop, self.window,
                                   self.filters, self.filter_range, self.n_mels, out)
        return out


__all__ = ["ClapLogMel", "slaney_mel_filters"]
