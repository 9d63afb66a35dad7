"""GPU Kaldi log-mel filterbank: the feature front of the reference's decode paths.

The reference turns audio into features with `torchaudio.compliance.kaldi.fbank`
(chunkformer_model.py:276-318 `_load_audio_and_extract_features`: pydub decode to 16 kHz mono
int16, then fbank(num_mel_bins=80, frame_length=25, frame_shift=10, dither=0.0, energy_floor=0.0,
sample_frequency=16000) on the int16-scale samples; dataset/processor.py:210-239 `compute_fbank`
is the same with window_type povey).  Here the same computation is one HIP kernel behind the
C-ABI (`cfm_fbank_*`, include/cfm.h; csrc/fbank.hip), and `fbank()` mirrors kaldi.fbank's
signature on device tensors.

Audio decoding: pydub / ffmpeg are absent, so `load_wav` reads 16-bit PCM WAV with the standard
library (channels averaged as pydub's set_channels(1) does, audioop.tomono with 0.5 / 0.5 and
floor); other sample rates are refused rather than resampled.
"""
from __future__ import annotations

import ctypes
import wave
from typing import Dict, Tuple

import numpy as np
import torch

from . import _lib

WINDOWS = {"povey": 0, "hamming": 1, "hanning": 2, "rectangular": 3, "blackman": 4}


class KaldiFbank:
    """One configured filterbank on one device (window, twiddles and mel filters resident)."""

    def __init__(self, device=None, num_mel_bins: int = 23, frame_length: float = 25.0, frame_shift: float = 10.0,
                 dither: float = 0.0, energy_floor: float = 1.0, sample_frequency: float = 16000.0,
                 window_type: str = "povey", low_freq: float = 20.0, high_freq: float = 0.0,
                 preemphasis_coefficient: float = 0.97, remove_dc_offset: bool = True, round_to_power_of_two: bool = True,
                 snip_edges: bool = True, use_energy: bool = False, use_log_fbank: bool = True,
                 blackman_coeff: float = 0.42):
        if not torch.cuda.is_available():
            raise RuntimeError("KaldiFbank needs a GPU (libcfm HIP kernels; there is no CPU fallback)")
        if window_type not in WINDOWS:
            raise ValueError(f"invalid window type {window_type}")
        if window_type == "blackman" and blackman_coeff != 0.42:
            raise AssertionError("blackman window: only blackman_coeff 0.42 is supported")
        del energy_floor   # only used with use_energy (unsupported, as in the reference's calls)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.num_mel_bins = int(num_mel_bins)
        c = _lib.CfmFbankConfig(float(sample_frequency), float(frame_length), float(frame_shift), int(num_mel_bins),
                                float(low_freq), float(high_freq), float(preemphasis_coefficient), float(dither),
                                int(remove_dc_offset), int(round_to_power_of_two), int(snip_edges), int(use_energy),
                                int(use_log_fbank), WINDOWS[window_type])
        h = ctypes.c_void_p()
        _lib.check(_lib.cfm_fbank_create(ctypes.byref(c), self.device.index or 0, ctypes.byref(h)))
        self._h = h
        import weakref
        self._finalizer = weakref.finalize(self, _lib.cfm_fbank_destroy, ctypes.c_void_p(h.value))

    def num_frames(self, num_samples: int) -> int:
        return int(_lib.cfm_fbank_num_frames(self._h, int(num_samples)))

    def __call__(self, waveform: torch.Tensor) -> torch.Tensor:
        """[frames, num_mel_bins] f32 on self.device from a 1-D (or [1, n]) waveform."""
        if waveform.dim() == 2 and waveform.shape[0] == 1:
            waveform = waveform[0]
        if waveform.dim() != 1:
            raise ValueError(f"fbank takes a mono waveform [n] or [1, n], got {tuple(waveform.shape)}")
        w = waveform.to(self.device, torch.float32).contiguous()
        nf = self.num_frames(w.numel())
        out = torch.empty(nf, self.num_mel_bins, device=self.device, dtype=torch.float32)
        if nf:
            st = torch.cuda.current_stream(self.device).cuda_stream
            _lib.check(_lib.cfm_fbank_compute(self._h, w.data_ptr(), w.numel(), out.data_ptr(), st))
        return out


_CACHE: Dict[tuple, KaldiFbank] = {}


def fbank(waveform: torch.Tensor, **kwargs) -> torch.Tensor:
    """torchaudio.compliance.kaldi.fbank(waveform, **kwargs) on the waveform's GPU (a CPU
    waveform is moved to the current device).  Filterbanks are cached per (device, kwargs)."""
    dev = waveform.device if waveform.is_cuda else torch.device("cuda", torch.cuda.current_device())
    key = (str(dev), tuple(sorted(kwargs.items())))
    fb = _CACHE.get(key)
    if fb is None:
        fb = _CACHE[key] = KaldiFbank(dev, **kwargs)
    return fb(waveform)


def load_wav(path: str) -> Tuple[np.ndarray, int]:
    """16-bit PCM WAV -> (int16-scale float32 mono samples, sample rate)."""
    with wave.open(path, "rb") as f:
        if f.getsampwidth() != 2:
            raise ValueError(f"{path}: only 16-bit PCM WAV is supported (pydub/ffmpeg are not available)")
        ch, sr, n = f.getnchannels(), f.getframerate(), f.getnframes()
        pcm = np.frombuffer(f.readframes(n), dtype="<i2").astype(np.float64)
    if ch > 1:   # audioop.tomono(data, 2, 0.5, 0.5) for stereo: floor(0.5 l + 0.5 r); n channels: the mean
        pcm = np.floor(pcm.reshape(-1, ch).mean(axis=1))
    return pcm.astype(np.float32), sr
