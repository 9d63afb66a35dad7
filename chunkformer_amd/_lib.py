"""ctypes binding of libcfm.so (include/cfm.h).

The library is the product: there is no Python/CPU fallback.  If the shared
object is missing this module raises at import time, and every encoder call
goes through it.  torch is imported first so that libcfm's libamdhip64.so.7
dependency resolves to the HIP runtime torch already loaded (one runtime per
process).
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before libcfm)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CFM_LIB", os.path.join(HERE, "_build", "libcfm.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(f"libcfm.so not found at {LIB_PATH}: run `python -m chunkformer_amd.build` "
                      "(the HIP extension is required; there is no CPU fallback)")

lib = ctypes.CDLL(LIB_PATH)

P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
SZ = ctypes.c_size_t
PI32 = ctypes.POINTER(ctypes.c_int32)
PI64 = ctypes.POINTER(ctypes.c_int64)

CFM_OK, CFM_ERR_VALUE, CFM_ERR_ASSERT, CFM_ERR_RUNTIME = 0, 1, 2, 3
DTYPE_F32, DTYPE_BF16, DTYPE_F16 = 0, 1, 2
PLAN_HEADER = 16
PLAN_REC = 8


class CfmConfig(ctypes.Structure):
    _fields_ = [("input_dim", I32), ("d_model", I32), ("n_heads", I32), ("ffn_dim", I32), ("num_blocks", I32),
                ("kernel_size", I32), ("vocab", I32), ("norm_eps", ctypes.c_float), ("has_cmvn", I32),
                ("compute_dtype", I32)]


class CfmTensorView(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", P), ("numel", I64)]


def _sig(name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


cfm_version = _sig("cfm_version", ctypes.c_char_p)
cfm_last_error = _sig("cfm_last_error", ctypes.c_char_p)
cfm_model_create = _sig("cfm_model_create", I32, ctypes.POINTER(CfmConfig), ctypes.POINTER(CfmTensorView), I32, I32,
                        ctypes.POINTER(P))
cfm_model_destroy = _sig("cfm_model_destroy", None, P)
cfm_model_set_option = _sig("cfm_model_set_option", I32, P, ctypes.c_char_p, I64)
cfm_plan_masked = _sig("cfm_plan_masked", I32, P, P, I32, I32, I32, I32, P, P, PI32, P, PI64)
cfm_plan_masked_ex = _sig("cfm_plan_masked_ex", I32, P, P, P, I32, I32, I32, I32, P, P, PI32, P, PI64)
cfm_plan_padded = _sig("cfm_plan_padded", I32, P, I32, I32, I32, I32, I32, PI32, P, PI64)
cfm_plan_stream = _sig("cfm_plan_stream", I32, I32, I32, I32, I32, I32, PI32, P, PI64)
cfm_workspace_bytes_stream = _sig("cfm_workspace_bytes_stream", SZ, P, I32, I32, I32, I32)
cfm_encode_stream = _sig("cfm_encode_stream", I32, P, P, I32, P, P, P, P, P, P, P, P, SZ, P)
cfm_workspace_bytes_masked = _sig("cfm_workspace_bytes_masked", SZ, P, I32, I32, I32, I32)
cfm_workspace_bytes_padded = _sig("cfm_workspace_bytes_padded", SZ, P, I32, I32, I32, I32, I32)
cfm_encode_masked = _sig("cfm_encode_masked", I32, P, P, P, P, P, P, I32, P, P, P, P, SZ, P)
cfm_encode_padded = _sig("cfm_encode_padded", I32, P, P, P, P, P, P, SZ, P)
cfm_encode_masked_utts = _sig("cfm_encode_masked_utts", I32, P, P, P, P, P, P, I32, P, P, P, P, SZ, P)
cfm_encode_masked_stages = _sig("cfm_encode_masked_stages", I32, P, P, P, P, P, P, I32, P, P, P, P, SZ, I32, I32, P)
cfm_masks_from_plan = _sig("cfm_masks_from_plan", I32, P, P, P, P, P)
cfm_profile_read = _sig("cfm_profile_read", I32, P, P, P, P, I32)
cfm_ctc_workspace_bytes = _sig("cfm_ctc_workspace_bytes", SZ, P, I32)
cfm_ctc_logprobs = _sig("cfm_ctc_logprobs", I32, P, P, I32, P, P, P, SZ, P)
cfm_ctc_ids_workspace_bytes = _sig("cfm_ctc_ids_workspace_bytes", SZ, P, I32)
cfm_ctc_ids = _sig("cfm_ctc_ids", I32, P, P, I32, P, P, SZ, P)
cfm_ctc_collapse = _sig("cfm_ctc_collapse", I32, P, P, P, I32, I32, I32, P, P, P, P, P, P)
# Kaldi fbank (include/cfm.h)
class CfmFbankConfig(ctypes.Structure):
    _fields_ = [("sample_frequency", ctypes.c_float), ("frame_length_ms", ctypes.c_float),
                ("frame_shift_ms", ctypes.c_float), ("num_mel_bins", I32), ("low_freq", ctypes.c_float),
                ("high_freq", ctypes.c_float), ("preemphasis_coefficient", ctypes.c_float), ("dither", ctypes.c_float),
                ("remove_dc_offset", I32), ("round_to_power_of_two", I32), ("snip_edges", I32), ("use_energy", I32),
                ("use_log_fbank", I32), ("window_type", I32)]


cfm_fbank_create = _sig("cfm_fbank_create", I32, ctypes.POINTER(CfmFbankConfig), I32, ctypes.POINTER(P))
cfm_fbank_destroy = _sig("cfm_fbank_destroy", None, P)
cfm_fbank_num_frames = _sig("cfm_fbank_num_frames", I64, P, I64)
cfm_fbank_compute = _sig("cfm_fbank_compute", I32, P, P, I64, P, P)
# RNN-T greedy search (include/cfm.h)
class CfmRnntConfig(ctypes.Structure):
    _fields_ = [("vocab", I32), ("enc_dim", I32), ("embed_size", I32), ("hidden", I32), ("num_layers", I32),
                ("pred_out", I32), ("join_dim", I32), ("blank", I32)]


cfm_rnnt_create = _sig("cfm_rnnt_create", I32, ctypes.POINTER(CfmRnntConfig), ctypes.POINTER(CfmTensorView), I32, I32,
                       ctypes.POINTER(P))
cfm_rnnt_destroy = _sig("cfm_rnnt_destroy", None, P)
cfm_rnnt_workspace_bytes = _sig("cfm_rnnt_workspace_bytes", SZ, P, I32)
cfm_rnnt_greedy = _sig("cfm_rnnt_greedy", I32, P, P, I32, P, P, I32, I32, P, P, SZ, P)
cfm_rnnt_greedy_ex = _sig("cfm_rnnt_greedy_ex", I32, P, P, I32, P, P, I32, I32, P, P, SZ, I32, P)
CFM_RNNT_ONE_WORKGROUP = 1
cfm_rnnt_set_option = _sig("cfm_rnnt_set_option", I32, P, ctypes.c_char_p, I64)
cfm_rnnt_grid_blocks = _sig("cfm_rnnt_grid_blocks", I32, P, I32)
cfm_rnnt_error = _sig("cfm_rnnt_error", I32, P, P, I32)
# include/cfm_ops.h
cfm_op_gemm = _sig("cfm_op_gemm", I32, I32, I32, I32, P, I32, P, I32, I32, I32, I32, P, ctypes.c_float, P, I32, I32, P,
                   I32, P, I32, P, I32, P)
EXPORTED_OPS = ["cfm_op_gemm"]

EXPORTED = ["cfm_version", "cfm_last_error", "cfm_model_create", "cfm_model_destroy", "cfm_model_set_option",
            "cfm_plan_masked", "cfm_plan_masked_ex", "cfm_plan_padded", "cfm_workspace_bytes_masked", "cfm_workspace_bytes_padded",
            "cfm_encode_masked", "cfm_encode_masked_utts", "cfm_encode_masked_stages", "cfm_encode_padded", "cfm_masks_from_plan", "cfm_profile_read", "cfm_ctc_workspace_bytes",
            "cfm_ctc_logprobs", "cfm_ctc_ids_workspace_bytes", "cfm_ctc_ids", "cfm_ctc_collapse",
            "cfm_plan_stream", "cfm_workspace_bytes_stream", "cfm_encode_stream",
            "cfm_fbank_create", "cfm_fbank_destroy", "cfm_fbank_num_frames", "cfm_fbank_compute",
            "cfm_rnnt_create", "cfm_rnnt_destroy", "cfm_rnnt_workspace_bytes", "cfm_rnnt_greedy",
            "cfm_rnnt_greedy_ex", "cfm_rnnt_set_option", "cfm_rnnt_grid_blocks", "cfm_rnnt_error"]


def profile_read(h):
    """{kernel class: (total_ms, launches)} accumulated by the in-stream event profiler."""
    cap = 32
    names = (ctypes.c_char_p * cap)()
    ms = (ctypes.c_double * cap)()
    n = (ctypes.c_int64 * cap)()
    k = cfm_profile_read(h, ctypes.cast(names, P), ctypes.cast(ms, P), ctypes.cast(n, P), cap)
    return {names[i].decode(): (ms[i], n[i]) for i in range(min(k, cap))}


PROFILE_CLASSES = ["frontend_conv0_dw", "frontend_pw_gemm", "frontend_dw2", "pos_gemm", "layernorm", "ffn_w1_gemm",
                   "ffn_w2_gemm", "qkv_gemm", "chunk_attention", "out_proj_gemm", "pw1_glu_gemm", "conv_dw_ln_silu",
                   "pw2_gemm", "cache_copy", "ctc"]


def check(status: int) -> None:
    """Map a cfm_status to the reference's exception types (include/cfm.h)."""
    if status == CFM_OK:
        return
    msg = (cfm_last_error() or b"").decode(errors="replace")
    if status == CFM_ERR_VALUE:
        raise ValueError(msg)
    if status == CFM_ERR_ASSERT:
        raise AssertionError(msg)
    raise RuntimeError(msg)


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def plan_masked(lens, offsets, C: int, L: int, R: int, mask_lens=None):
    """Host planner (no GPU): returns (plan int32 CPU tensor, n_chunks list, out_lens list).
    lens: feature rows per utterance; mask_lens: xs_origin_lens when it differs (None = lens)."""
    B = len(lens)
    lens_t = torch.tensor([int(x) for x in lens], dtype=torch.int32)
    ml_t = torch.tensor([int(x) for x in mask_lens], dtype=torch.int32) if mask_lens is not None else None
    offs_t = torch.tensor([int(x) for x in offsets], dtype=torch.int32) if offsets is not None else None
    nch = torch.zeros(B, dtype=torch.int32)
    olen = torch.zeros(B, dtype=torch.int32)
    total = I32(0)
    n = I64(0)
    check(cfm_plan_masked_ex(lens_t.data_ptr(), ptr(ml_t), ptr(offs_t), B, C, L, R, nch.data_ptr(), olen.data_ptr(),
                             ctypes.byref(total), None, ctypes.byref(n)))
    plan = torch.zeros(n.value, dtype=torch.int32)
    check(cfm_plan_masked_ex(lens_t.data_ptr(), ptr(ml_t), ptr(offs_t), B, C, L, R, None, None, ctypes.byref(total),
                             plan.data_ptr(), ctypes.byref(n)))
    return plan, nch.tolist(), olen.tolist()


def plan_stream(T: int, C: int, L: int, R: int, offset: int):
    """Host planner of one forward_chunk step (no GPU): returns (plan int32 CPU tensor, T')."""
    tout = I32(0)
    n = I64(0)
    check(cfm_plan_stream(int(T), int(C), int(L), int(R), int(offset), ctypes.byref(tout), None, ctypes.byref(n)))
    plan = torch.zeros(n.value, dtype=torch.int32)
    check(cfm_plan_stream(int(T), int(C), int(L), int(R), int(offset), ctypes.byref(tout), plan.data_ptr(),
                          ctypes.byref(n)))
    return plan, tout.value


def plan_padded(lens, T: int, C: int, L: int, R: int):
    B = len(lens)
    lens_t = torch.tensor([int(x) for x in lens], dtype=torch.int32)
    tout = I32(0)
    n = I64(0)
    check(cfm_plan_padded(lens_t.data_ptr(), B, T, C, L, R, ctypes.byref(tout), None, ctypes.byref(n)))
    plan = torch.zeros(n.value, dtype=torch.int32)
    check(cfm_plan_padded(lens_t.data_ptr(), B, T, C, L, R, ctypes.byref(tout), plan.data_ptr(), ctypes.byref(n)))
    return plan, tout.value
