"""Kaldi fbank oracle (oracle/fbank_ref.py) invariants and the WAV reader, on the CPU.

torchaudio is absent, so the oracle's parity with torchaudio.compliance.kaldi.fbank is UNPINNED
(no reference fixture holds fbank outputs); these tests check the restatement's own properties.
The GPU kernel is compared with the oracle in tests/test_gpu_fbank.py."""
import math
import wave

import numpy as np
import pytest
import torch

from oracle import fbank_ref as ref

REF = dict(num_mel_bins=80, frame_length=25, frame_shift=10, dither=0.0, energy_floor=0.0, sample_frequency=16000)


@pytest.mark.parametrize("n,frames", [(0, 0), (399, 0), (400, 1), (559, 1), (560, 2), (16000, 98), (16399, 100)])
def test_frame_count(n, frames):
    assert ref.num_frames(n, 400, 160) == frames
    assert ref.fbank(torch.randn(n) * 1000, **REF).shape == (frames, 80)


def test_silence_is_log_eps():
    e = ref.fbank(torch.full((4000,), 123.0), **REF)   # a constant: removed with the frame mean
    assert torch.equal(e, torch.full_like(e, math.log(ref.EPS)))


def test_tone_lands_in_its_mel_bin():
    sr, f0 = 16000, 1000.0
    t = torch.arange(16000, dtype=torch.float64) / sr
    x = (8000 * torch.sin(2 * math.pi * f0 * t)).float()
    e = ref.fbank(x, **REF)
    m0, m1 = ref.mel_scale_scalar(20.0), ref.mel_scale_scalar(8000.0)
    centers = [700 * (math.exp((m0 + (b + 1) * (m1 - m0) / 81) / 1127.0) - 1) for b in range(80)]
    nearest = min(range(80), key=lambda b: abs(centers[b] - f0))
    assert abs(int(e.mean(0).argmax()) - nearest) <= 1


def test_mel_banks_are_triangles():
    mel = ref.get_mel_banks(80, 512, 16000.0, 20.0, 0.0)
    assert mel.shape == (80, 256)
    assert (mel >= 0).all() and (mel <= 1).all()
    assert ((mel > 0).sum(0) <= 2).all()               # every FFT bin feeds at most two filters
    for b in range(80):
        nz = torch.nonzero(mel[b]).flatten()
        assert len(nz) > 0 and (nz[1:] - nz[:-1] == 1).all()   # one contiguous range


def test_povey_window():
    w = ref.feature_window("povey", 400)
    assert w[0] == 0 and torch.allclose(w, w.flip(0), atol=1e-6) and abs(float(w.max()) - 1.0) < 1e-4


def test_load_wav_stereo_floor_average(tmp_path):
    from chunkformer_amd.fbank import load_wav
    pcm = np.array([[100, 201], [-3, -4], [32767, 32767]], dtype="<i2")
    p = str(tmp_path / "s.wav")
    with wave.open(p, "wb") as f:
        f.setnchannels(2)
        f.setsampwidth(2)
        f.setframerate(16000)
        f.writeframes(pcm.tobytes())
    x, sr = load_wav(p)
    assert sr == 16000 and x.tolist() == [150.0, -4.0, 32767.0]   # floor(0.5 l + 0.5 r), audioop.tomono
