"""WAV / AIFF / AIFC / Sun AU decoding of AudioToImageInference.load_audio (reference scripts/inference.py:73-79:
librosa.load(path, sr=48000, mono=True, duration=10), then peak normalisation).  librosa is
absent here, so the resampler's numerics are not pinned to it (scipy polyphase vs soxr); what
is checked: every RIFF/WAVE encoding the reader claims decodes to the samples written, channels
are averaged, duration is cut at the native rate before resampling, and a non-48 kHz file comes
out at 48 kHz with the tone where it was."""
import numpy as np
import pytest

from clap2diffusion_amd.pipeline import SR, AudioToImageInference, _read_wav


def write_wav(path, x, sr, fmt):
    """x: float [frames, ch] in [-1, 1)."""
    ch = x.shape[1]
    if fmt == "pcm8":
        body, tag, bits = np.clip(np.round(x * 128 + 128), 0, 255).astype(np.uint8).tobytes(), 1, 8
    elif fmt == "pcm16":
        body, tag, bits = np.round(x * 32767).astype("<i2").tobytes(), 1, 16
    elif fmt == "pcm24":
        v = np.round(x * (2 ** 23 - 1)).astype(np.int64).reshape(-1)
        v = np.where(v < 0, v + (1 << 24), v)
        body = np.stack([(v >> 0) & 255, (v >> 8) & 255, (v >> 16) & 255], 1).astype(np.uint8).tobytes()
        tag, bits = 1, 24
    elif fmt == "pcm32":
        body, tag, bits = np.round(x * (2 ** 31 - 1)).astype("<i4").tobytes(), 1, 32
    elif fmt == "f32":
        body, tag, bits = x.astype("<f4").tobytes(), 3, 32
    elif fmt == "f64ext":
        body, tag, bits = x.astype("<f8").tobytes(), 0xFFFE, 64
    ba = ch * bits // 8
    fmtc = (tag.to_bytes(2, "little") + ch.to_bytes(2, "little") + sr.to_bytes(4, "little") +
            (sr * ba).to_bytes(4, "little") + ba.to_bytes(2, "little") + bits.to_bytes(2, "little"))
    if tag == 0xFFFE:   # WAVE_FORMAT_EXTENSIBLE: cbSize, valid bits, channel mask, SubFormat GUID (float)
        fmtc += (22).to_bytes(2, "little") + bits.to_bytes(2, "little") + (0).to_bytes(4, "little") + \
            (3).to_bytes(2, "little") + bytes(14)
    chunks = b"fmt " + len(fmtc).to_bytes(4, "little") + fmtc
    chunks += b"LIST" + (3).to_bytes(4, "little") + b"abc\0"            # odd-sized chunk: pad byte
    chunks += b"data" + len(body).to_bytes(4, "little") + body
    path.write_bytes(b"RIFF" + (4 + len(chunks)).to_bytes(4, "little") + b"WAVE" + chunks)


@pytest.mark.parametrize("fmt,tol", [("pcm8", 1 / 64), ("pcm16", 1e-4), ("pcm24", 1e-6), ("pcm32", 1e-6),
                                     ("f32", 0.0), ("f64ext", 1e-7)])
def test_wav_encodings_decode(tmp_path, fmt, tol):
    rng = np.random.default_rng(3)
    x = (rng.uniform(-0.9, 0.9, size=(1000, 2))).astype(np.float32)
    p = tmp_path / f"a_{fmt}.wav"
    write_wav(p, x, 22050, fmt)
    y, sr = _read_wav(str(p))
    assert sr == 22050 and y.dtype == np.float32 and y.shape == (1000,)
    assert np.abs(y - x.mean(axis=1)).max() <= tol + 1e-7


def test_load_audio_resamples_and_cuts(tmp_path):
    sr = 44100
    t = np.arange(int(12.5 * sr)) / sr
    x = (0.5 * np.sin(2 * np.pi * 1000.0 * t))[:, None].astype(np.float32)
    p = tmp_path / "tone.wav"
    write_wav(p, x, sr, "pcm16")
    pipe = AudioToImageInference.__new__(AudioToImageInference)   # load_audio needs no model
    a = pipe.load_audio(str(p), duration=10)
    assert a.shape == (10 * SR,)
    assert abs(np.abs(a).max() - 1.0) < 1e-6                     # peak normalised
    spec = np.abs(np.fft.rfft(a[SR:3 * SR]))
    assert abs(np.argmax(spec) * SR / (2 * SR) - 1000.0) < 1.0   # the tone stays at 1 kHz


def test_non_wav_is_refused(tmp_path):
    p = tmp_path / "x.mp3"
    p.write_bytes(b"ID3\x03\x00" + bytes(100))
    with pytest.raises(ValueError, match="RIFF/WAVE"):
        _read_wav(str(p))


def _write_stdlib(mod, path, x, sr, width, comp=None):
    """AIFF / AIFC / Sun AU through the standard library's writers; x float [frames, ch]."""
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", DeprecationWarning)
        f = mod.open(str(path), "wb")
        f.setnchannels(x.shape[1])
        f.setframerate(sr)
        if comp is not None:
            f.setcomptype(*comp)
            f.setsampwidth(2)
            v = np.round(x * 32767).astype(np.int16)
            f.writeframes(v.astype("<i2" if comp[0] in (b"ULAW", "ULAW", b"ALAW") else ">i2").tobytes())
        else:
            if mod.__name__ == "sunau":
                f.setcomptype("NONE", "not compressed")   # sunau's writer defaults to u-law
            f.setsampwidth(width)
            scale = 2 ** (8 * width - 1)
            v = np.clip(np.round(x.astype(np.float64) * scale), -scale, scale - 1).astype(np.int64).reshape(-1)
            if width == 3:
                v = np.where(v < 0, v + (1 << 24), v)
                raw = np.stack([(v >> 16) & 255, (v >> 8) & 255, v & 255], 1).astype(np.uint8).tobytes()
            else:
                raw = v.astype({1: "i1", 2: ">i2", 4: ">i4"}[width]).tobytes()
            f.writeframes(raw)
        f.close()


@pytest.mark.parametrize("kind,width,comp,tol", [
    ("aiff", 1, None, 1 / 64), ("aiff", 2, None, 1e-4), ("aiff", 3, None, 1e-6), ("aiff", 4, None, 1e-6),
    ("aifc", 2, (b"ULAW", b""), 0.03),
    ("au", 1, None, 1 / 64), ("au", 2, None, 1e-4), ("au", 3, None, 1e-6), ("au", 4, None, 1e-6),
    ("au", 2, ("ULAW", "CCITT G.711 u-law"), 0.03),
])
def test_aiff_and_au_decode(tmp_path, kind, width, comp, tol):
    """reference scripts/inference.py:78 reads any container librosa does; this image has no
    decoder beyond the standard library, so load_audio takes WAV (above), AIFF / AIFC and Sun AU:
    every linear width and the u-law codec decode to the samples written, channels averaged."""
    import aifc
    import sunau
    from clap2diffusion_amd.pipeline import read_audio
    rng = np.random.default_rng(5)
    x = rng.uniform(-0.9, 0.9, size=(800, 2)).astype(np.float32)
    p = tmp_path / f"a.{kind}"
    if kind == "au" and width == 1:   # sunau writes 8-bit as u-law: linear 8-bit (encoding 2) by hand
        body = np.clip(np.round(x.astype(np.float64) * 128), -128, 127).astype(np.int8).tobytes()
        hdr = b".snd" + b"".join(v.to_bytes(4, "big") for v in (24, len(body), 2, 16000, 2))
        p.write_bytes(hdr + body)
    else:
        _write_stdlib(sunau if kind == "au" else aifc, p, x, 16000, width, comp)
    y, sr = read_audio(str(p))
    assert sr == 16000 and y.dtype == np.float32 and y.shape == (800,)
    assert np.abs(y - x.mean(axis=1)).max() <= tol + 1e-7
    y2, _ = read_audio(str(p), max_seconds=0.01)
    assert y2.shape == (160,) and np.array_equal(y2, y[:160])


def test_load_audio_reads_aiff_and_refuses_unknown(tmp_path):
    import aifc
    from clap2diffusion_amd.pipeline import read_audio
    sr = 44100
    t = np.arange(int(11 * sr)) / sr
    x = (0.5 * np.sin(2 * np.pi * 1000.0 * t))[:, None].astype(np.float32)
    p = tmp_path / "tone.aiff"
    _write_stdlib(aifc, p, x, sr, 2)
    pipe = AudioToImageInference.__new__(AudioToImageInference)
    a = pipe.load_audio(str(p), duration=10)
    assert a.shape == (10 * SR,) and abs(np.abs(a).max() - 1.0) < 1e-6
    spec = np.abs(np.fft.rfft(a[SR:3 * SR]))
    assert abs(np.argmax(spec) * SR / (2 * SR) - 1000.0) < 1.0
    q = tmp_path / "x.mp3"
    q.write_bytes(b"ID3\x03\x00" + bytes(100))
    with pytest.raises(ValueError, match="AIFF/AIFC or Sun AU"):
        read_audio(str(q))
