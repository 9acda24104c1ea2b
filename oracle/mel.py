"""ORACLE (test infrastructure only) — numpy restatement of the Whisper log-mel
front end the reference calls (HF ``WhisperFeatureExtractor.__call__`` with
``padding='max_length'``; call sites src/utils.py:186-187,
src/efficient_kws/dataset.py:949-954, src/data/dataset.py:332-339).

Third-party algorithm restated: transformers==4.37.2 (requirements.txt:21;
installed 5.15.0) ``feature_extraction_whisper._torch_extract_fbank_features``
and ``audio_utils.mel_filter_bank(norm='slaney', mel_scale='slaney')``:
zero-pad/truncate to 480000 samples, periodic Hann(400), hop 160,
``torch.stft(center=True, pad_mode='reflect')``, drop the last frame,
|X|^2, mel projection, log10(max(., 1e-10)), max(x, max(x) - 8), (x + 4) / 4.
Pinned by tests/golden/mel_{80,128}.npz.
"""
from __future__ import annotations

import numpy as np

N_FFT = 400
HOP = 160
N_SAMPLES = 480000
SR = 16000


def _hz_to_mel_slaney(f):
    f = np.asarray(f, np.float64)
    m = 3.0 * f / 200.0
    logstep = 27.0 / np.log(6.4)
    return np.where(f >= 1000.0, 15.0 + np.log(np.maximum(f, 1e-30) / 1000.0) * logstep, m)


def _mel_to_hz_slaney(m):
    m = np.asarray(m, np.float64)
    f = 200.0 * m / 3.0
    logstep = np.log(6.4) / 27.0
    return np.where(m >= 15.0, 1000.0 * np.exp(logstep * (m - 15.0)), f)


def mel_filters(n_mel: int, n_freq: int = N_FFT // 2 + 1, sr: int = SR, fmin=0.0, fmax=8000.0) -> np.ndarray:
    """audio_utils.mel_filter_bank(norm='slaney', mel_scale='slaney') -> [n_freq, n_mel]."""
    mels = np.linspace(_hz_to_mel_slaney(fmin), _hz_to_mel_slaney(fmax), n_mel + 2)
    ff = _mel_to_hz_slaney(mels)
    fft_freqs = np.linspace(0, sr // 2, n_freq)
    diff = np.diff(ff)
    slopes = ff[None, :] - fft_freqs[:, None]
    down = -slopes[:, :-2] / diff[:-1]
    up = slopes[:, 2:] / diff[1:]
    fb = np.maximum(0.0, np.minimum(down, up))
    enorm = 2.0 / (ff[2:n_mel + 2] - ff[:n_mel])
    return fb * enorm[None, :]


def pad_or_trim(pcm: np.ndarray) -> np.ndarray:
    x = np.zeros(N_SAMPLES, np.float32)
    n = min(N_SAMPLES, pcm.shape[0])
    x[:n] = pcm[:n]
    return x


def log_mel(pcm: np.ndarray, n_mel: int) -> np.ndarray:
    """[n_samples] float -> [n_mel, 3000] float32."""
    x = pad_or_trim(pcm).astype(np.float64)
    xp = np.pad(x, (N_FFT // 2, N_FFT // 2), mode="reflect")
    n_frames = 1 + (xp.shape[0] - N_FFT) // HOP               # 3001
    win = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(N_FFT) / N_FFT)   # periodic Hann
    idx = np.arange(N_FFT)[None, :] + HOP * np.arange(n_frames)[:, None]
    frames = xp[idx] * win[None, :]
    spec = np.fft.rfft(frames, axis=1)                          # [3001, 201]
    power = (spec.real ** 2 + spec.imag ** 2)[:-1]              # drop last frame -> [3000, 201]
    mel = mel_filters(n_mel).T @ power.T                        # [n_mel, 3000]
    log_spec = np.log10(np.maximum(mel, 1e-10))
    log_spec = np.maximum(log_spec, log_spec.max() - 8.0)
    return ((log_spec + 4.0) / 4.0).astype(np.float32)


def log_mel_long(pcm: np.ndarray, n_mel: int) -> np.ndarray:
    """Long-form features (the caller of PBAWhisper.generate on > 30 s audio, pba_whisper.py:343-475):
    ``WhisperFeatureExtractor(padding='longest', truncation=False)`` on one waveform -- no zero padding,
    reflect padding at the audio's own ends, n // 160 frames, the max - 8 floor over the whole audio.
    [n_samples] -> [n_mel, n_samples // 160] float32."""
    x = np.asarray(pcm, np.float64)
    xp = np.pad(x, (N_FFT // 2, N_FFT // 2), mode="reflect")
    n_frames = 1 + (xp.shape[0] - N_FFT) // HOP
    win = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(N_FFT) / N_FFT)
    out = np.empty((n_mel, n_frames - 1), np.float64)
    fb = mel_filters(n_mel).T
    for f0 in range(0, n_frames - 1, 4096):     # bounded memory for long audio
        f1 = min(n_frames - 1, f0 + 4096)
        idx = np.arange(N_FFT)[None, :] + HOP * np.arange(f0, f1)[:, None]
        spec = np.fft.rfft(xp[idx] * win[None, :], axis=1)
        out[:, f0:f1] = np.log10(np.maximum(fb @ (spec.real ** 2 + spec.imag ** 2).T, 1e-10))
    out = np.maximum(out, out.max() - 8.0)
    return ((out + 4.0) / 4.0).astype(np.float32)
