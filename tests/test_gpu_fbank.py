"""GPU Kaldi fbank (cfm_fbank_compute through chunkformer_amd/fbank.py) against the CPU oracle
(oracle/fbank_ref.py, a restatement of torchaudio.compliance.kaldi.fbank; parity with torchaudio
itself is UNPINNED: torchaudio is absent and the reference holds no fbank fixtures).

Tolerance: max |gpu - oracle| <= 2e-3 on log-mel values of int16-scale audio (both f32; the FFT
and the filter sums add in different orders), exact log(eps) on silence, identical frame counts."""
import math
import wave

import numpy as np
import pytest
import torch

from oracle import fbank_ref as ref

pytestmark = pytest.mark.gpu
TOL = 2e-3
REF = dict(num_mel_bins=80, frame_length=25, frame_shift=10, dither=0.0, energy_floor=0.0, sample_frequency=16000)


@pytest.fixture(scope="module")
def fb():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from chunkformer_amd import fbank
    return fbank


def _speechlike(n, seed):
    g = torch.Generator().manual_seed(seed)
    t = torch.arange(n, dtype=torch.float64) / 16000
    x = 3000 * torch.randn(n, generator=g, dtype=torch.float64)
    for f0 in (180.0, 730.0, 2300.0):
        x += 4000 * torch.sin(2 * math.pi * f0 * t + float(torch.rand(1, generator=g)) * 6.28)
    env = 0.5 + 0.5 * torch.sin(2 * math.pi * 3.0 * t)          # syllable-rate envelope
    return torch.clamp(x * env, -32768, 32767).round().float()


@pytest.mark.parametrize("n", [0, 399, 400, 401, 559, 560, 16000, 48123])
def test_fbank_matches_oracle(fb, n):
    x = _speechlike(n, n)
    got = fb.fbank(x.cuda(), **REF).cpu()
    exp = ref.fbank(x, **REF)
    assert got.shape == exp.shape
    if n >= 400:
        err = (got - exp).abs().max().item()
        assert err <= TOL, err


@pytest.mark.parametrize("window_type", ["povey", "hamming", "hanning", "rectangular", "blackman"])
@pytest.mark.parametrize("bins,sr,length", [(23, 16000, 25.0), (80, 8000, 25.0), (40, 16000, 32.0)])
def test_fbank_options(fb, window_type, bins, sr, length):
    x = _speechlike(20000, bins + sr)
    kw = dict(num_mel_bins=bins, frame_length=length, frame_shift=10, dither=0.0, sample_frequency=sr,
              window_type=window_type)
    got = fb.fbank(x.cuda(), **kw).cpu()
    exp = ref.fbank(x, **kw)
    assert got.shape == exp.shape
    assert (got - exp).abs().max().item() <= TOL


@pytest.mark.parametrize("shift_ms,length_ms,offset", [(10.0, 25.0, 1), (10.0625, 25.0, 0), (10.0, 25.0625, 0),
                                                       (10.0625, 31.9375, 3)])
def test_fbank_odd_shift_length_and_unaligned_samples(fb, shift_ms, length_ms, offset):
    """Odd frame shift / odd frame length (161 / 401 / 511 samples) and a waveform that does not
    start 8-B aligned: the scalar sample loads and the partial last pair of the N = 512 kernel."""
    x = _speechlike(30000 + offset, 11)
    kw = dict(num_mel_bins=80, frame_length=length_ms, frame_shift=shift_ms, dither=0.0, sample_frequency=16000)
    xd = x.cuda()[offset:]
    got = fb.fbank(xd, **kw).cpu()
    exp = ref.fbank(x[offset:], **kw)
    assert got.shape == exp.shape
    assert (got - exp).abs().max().item() <= TOL


@pytest.mark.parametrize("remove_dc,preemph,use_log", [(False, 0.97, True), (True, 0.0, True), (True, 0.97, False)])
def test_fbank_switches(fb, remove_dc, preemph, use_log):
    x = _speechlike(24000, 5)
    kw = dict(REF, remove_dc_offset=remove_dc, preemphasis_coefficient=preemph, use_log_fbank=use_log)
    got = fb.fbank(x.cuda(), **kw).cpu()
    exp = ref.fbank(x, **kw)
    assert got.shape == exp.shape
    if use_log:
        assert (got - exp).abs().max().item() <= TOL
    else:   # linear mel energies: relative to each value (2e-3 in log = 0.2% relative)
        assert ((got - exp).abs() / exp.abs().clamp_min(1e-3)).max().item() <= TOL


def test_fbank_silence_and_dc(fb):
    x = torch.cat([torch.zeros(8000), torch.full((8000,), -77.0)])
    got, exp = fb.fbank(x.cuda(), **REF).cpu(), ref.fbank(x, **REF)
    flat = [i for i in range(got.shape[0]) if i * 160 + 400 <= 8000 or i * 160 >= 8000]   # frames off the step
    assert abs(got[flat] - math.log(ref.EPS)).max().item() <= 1e-6   # floor at log(eps)
    assert torch.equal(exp[flat], torch.full_like(exp[flat], math.log(ref.EPS)))
    assert (got - exp).abs().max().item() <= TOL


def test_fbank_long_audio_property(fb):
    """10 minutes: frame count and the statistics of every frame against the oracle (sampled)."""
    n = 600 * 16000 + 123
    x = _speechlike(n, 5)
    got = fb.fbank(x.cuda(), **REF)
    assert got.shape == (1 + (n - 400) // 160, 80)
    idx = torch.linspace(0, got.shape[0] - 1, 200).long()
    for i in idx.tolist()[::20]:
        s = i * 160
        exp = ref.fbank(x[s: s + 400], **REF)
        assert (got[i].cpu() - exp[0]).abs().max().item() <= TOL


def test_wav_path_decode_matches_feature_decode(fb, tmp_path):
    """model.batch_decode on a .wav path (GPU fbank) == batch_decode on oracle features."""
    from chunkformer_amd.config import SMALL
    from chunkformer_amd.model import ChunkFormerModel
    from chunkformer_amd.weights import synthetic_state_dict
    x = _speechlike(16000 * 7 + 55, 11)
    p = str(tmp_path / "a.wav")
    with wave.open(p, "wb") as f:
        f.setnchannels(1)
        f.setsampwidth(2)
        f.setframerate(16000)
        f.writeframes(x.numpy().astype("<i2").tobytes())
    m = ChunkFormerModel(SMALL, synthetic_state_dict(SMALL, 3), dtype="fp32", device="cuda:0")
    feats_gpu = m.extract_features(x)
    feats_ref = ref.fbank(x, **REF)
    assert (feats_gpu.cpu() - feats_ref).abs().max().item() <= TOL
    a = m.batch_decode([p], 16, 32, 32)[0]
    b = m.batch_decode([feats_ref], 16, 32, 32)[0]
    agree = (a == b).float().mean().item()
    assert a.shape == b.shape and agree >= 0.99, agree
    with pytest.raises(ValueError):
        m.extract_features(x, sample_rate=8000)
