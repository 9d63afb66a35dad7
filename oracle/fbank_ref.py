"""CPU oracle of the Kaldi log-mel filterbank -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this module, as the
checker; the product path (chunkformer_amd/fbank.py -> libcfm cfm_fbank_compute) never does.

The reference computes features with torchaudio.compliance.kaldi.fbank
(chunkformer_model.py:306-314: num_mel_bins 80, frame_length 25, frame_shift 10, dither 0.0,
energy_floor 0.0, sample_frequency 16000, on int16-scale pydub samples; dataset/processor.py:
210-239 the same with the povey window on wav * 2**15).  torchaudio (pinned `torchaudio>=2.5.1`,
reference pyproject.toml:28) is a third-party dependency that is NOT vendored under
/root/reference and NOT installed here, so this module restates its published algorithm
(torchaudio/compliance/kaldi.py: fbank, _get_waveform_and_window_properties, _get_strided,
_get_window, _feature_window_function, get_mel_banks, mel_scale) step for step in torch float32 on
the CPU.  PARITY UNPINNED: no fixture or output of torchaudio itself exists in the reference or
in this image to pin it against; the tests check the restatement's own invariants (frame count,
a tone's energy in its mel bin, silence at log(eps), window / filter shapes) and the GPU kernel
against this restatement.
"""
import math

import torch

EPS = torch.finfo(torch.float).eps   # kaldi.py _get_epsilon


def _next_power_of_2(x: int) -> int:
    return 1 if x == 0 else 2 ** (x - 1).bit_length()


def mel_scale_scalar(freq: float) -> float:
    return 1127.0 * math.log(1.0 + freq / 700.0)


def mel_scale(freq: torch.Tensor) -> torch.Tensor:
    return 1127.0 * (1.0 + freq / 700.0).log()


def feature_window(window_type: str, window_size: int, blackman_coeff: float = 0.42) -> torch.Tensor:
    """_feature_window_function (float32)"""
    if window_type == "hanning":
        return torch.hann_window(window_size, periodic=False)
    if window_type == "hamming":
        return torch.hamming_window(window_size, periodic=False, alpha=0.54, beta=0.46)
    if window_type == "povey":
        return torch.hann_window(window_size, periodic=False).pow(0.85)
    if window_type == "rectangular":
        return torch.ones(window_size)
    if window_type == "blackman":
        a = 2 * math.pi / (window_size - 1)
        n = torch.arange(window_size, dtype=torch.float32)
        return blackman_coeff - 0.5 * torch.cos(a * n) + (0.5 - blackman_coeff) * torch.cos(2 * a * n)
    raise ValueError(f"invalid window type {window_type}")


def get_mel_banks(num_bins: int, window_length_padded: int, sample_freq: float, low_freq: float,
                  high_freq: float) -> torch.Tensor:
    """get_mel_banks with vtln_warp_factor = 1: [num_bins, window_length_padded / 2]"""
    num_fft_bins = window_length_padded // 2
    nyquist = 0.5 * sample_freq
    if high_freq <= 0.0:
        high_freq += nyquist
    fft_bin_width = sample_freq / window_length_padded
    mel_low, mel_high = mel_scale_scalar(low_freq), mel_scale_scalar(high_freq)
    delta = (mel_high - mel_low) / (num_bins + 1)
    b = torch.arange(num_bins).unsqueeze(1)
    left = mel_low + b * delta
    center = mel_low + (b + 1.0) * delta
    right = mel_low + (b + 2.0) * delta
    mel = mel_scale(fft_bin_width * torch.arange(num_fft_bins)).unsqueeze(0)
    up = (mel - left) / (center - left)
    down = (right - mel) / (right - center)
    return torch.max(torch.zeros(1), torch.min(up, down))


def num_frames(num_samples: int, window_size: int, window_shift: int) -> int:
    """_get_strided, snip_edges=True"""
    return 0 if num_samples < window_size else 1 + (num_samples - window_size) // window_shift


def fbank(waveform: torch.Tensor, num_mel_bins: int = 23, frame_length: float = 25.0, frame_shift: float = 10.0,
          dither: float = 0.0, energy_floor: float = 1.0, sample_frequency: float = 16000.0,
          window_type: str = "povey", low_freq: float = 20.0, high_freq: float = 0.0,
          preemphasis_coefficient: float = 0.97, remove_dc_offset: bool = True, use_log_fbank: bool = True,
          round_to_power_of_two: bool = True, blackman_coeff: float = 0.42) -> torch.Tensor:
    """kaldi.fbank on a 1-D (or [1, n]) float waveform, CPU float32: [frames, num_mel_bins].
    dither must be 0 (the reference's value); energy_floor only matters with use_energy (off)."""
    assert dither == 0.0
    x = waveform.reshape(-1).float().cpu()
    window_shift = int(sample_frequency * frame_shift * 0.001)
    window_size = int(sample_frequency * frame_length * 0.001)
    padded = _next_power_of_2(window_size) if round_to_power_of_two else window_size
    nf = num_frames(x.numel(), window_size, window_shift)
    if nf == 0:
        return torch.empty(0, num_mel_bins)
    frames = x.as_strided((nf, window_size), (window_shift, 1))
    if remove_dc_offset:
        frames = frames - torch.mean(frames, dim=1).unsqueeze(1)
    if preemphasis_coefficient != 0.0:
        off = torch.nn.functional.pad(frames.unsqueeze(0), (1, 0), mode="replicate").squeeze(0)
        frames = frames - preemphasis_coefficient * off[:, :-1]
    frames = frames * feature_window(window_type, window_size, blackman_coeff).unsqueeze(0)
    if padded != window_size:
        frames = torch.nn.functional.pad(frames.unsqueeze(0), (0, padded - window_size), mode="constant",
                                         value=0).squeeze(0)
    spectrum = torch.fft.rfft(frames).abs().pow(2.0)
    mel = get_mel_banks(num_mel_bins, padded, sample_frequency, low_freq, high_freq)
    mel = torch.nn.functional.pad(mel, (0, 1), mode="constant", value=0)
    e = torch.mm(spectrum, mel.T)
    if use_log_fbank:
        e = torch.max(e, torch.tensor(EPS)).log()
    return e
