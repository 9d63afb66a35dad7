"""Encoder configuration for the ChunkFormer masked-chunk encoder.

Mirrors the `encoder_conf` keys the reference reads in
`chunkformer/modules/encoder.py:36-70` (ChunkFormerEncoder.__init__) and the
CTC `output_dim` read in `chunkformer/utils/init_model.py:73-76`.  Only the
configuration subset shipped by the reference checkpoints is supported
(dw_striding front-end, chunk_rel_pos, chunk_rel_seflattn, layer_norm conv
norm, dynamic_conv, swish, macaron, cnn module, pre-norm); anything else raises
AssertionError exactly like `encoder.py:94-96`.
"""
from __future__ import annotations

from dataclasses import dataclass, asdict
from typing import Any, Dict, Optional


@dataclass
class EncoderConfig:
    input_dim: int = 80          # fbank bins (encoder.py:38 input_size)
    d_model: int = 512           # output_size
    n_heads: int = 8             # attention_heads
    ffn_dim: int = 2048          # linear_units
    num_blocks: int = 12
    kernel_size: int = 15        # cnn_module_kernel
    vocab: int = 5000            # ctc output_dim (0 = encoder only)
    norm_eps: float = 1e-5
    cmvn: bool = True            # global_cmvn present

    @property
    def head_dim(self) -> int:
        return self.d_model // self.n_heads

    @property
    def conv_lorder(self) -> int:
        return self.kernel_size // 2

    def validate(self) -> None:
        assert self.d_model % self.n_heads == 0
        assert self.head_dim in (64, 128), "HIP attention kernels are built for head_dim 64 or 128"
        assert self.d_model % 64 == 0 and self.ffn_dim % 64 == 0
        assert self.kernel_size == 15, "conv module kernel is built for k=15"
        assert self.input_dim == 80, "front-end kernel is built for 80 mel bins"

    def to_dict(self) -> Dict[str, Any]:
        return asdict(self)

    @classmethod
    def from_encoder_conf(cls, encoder_conf: Dict[str, Any], input_dim: int = 80,
                          output_dim: int = 0, cmvn: bool = False) -> "EncoderConfig":
        """Build from a reference YAML `encoder_conf` dict (init_model.py:85-87)."""
        ec = dict(encoder_conf)
        assert ec.get("input_layer", "dw_striding") == "dw_striding"
        assert ec.get("pos_enc_layer_type", "chunk_rel_pos") == "chunk_rel_pos"
        assert ec.get("selfattention_layer_type", "chunk_rel_seflattn") == "chunk_rel_seflattn"
        assert ec.get("cnn_module_norm", "batch_norm") == "layer_norm"
        assert ec.get("dynamic_conv", False) is True
        assert ec.get("activation_type", "swish") == "swish"
        assert ec.get("macaron_style", True) and ec.get("use_cnn_module", True)
        assert ec.get("normalize_before", True) and not ec.get("causal", False)
        assert ec.get("layer_norm_type", "layer_norm") == "layer_norm"
        return cls(input_dim=input_dim, d_model=ec.get("output_size", 256),
                   n_heads=ec.get("attention_heads", 4), ffn_dim=ec.get("linear_units", 2048),
                   num_blocks=ec.get("num_blocks", 6), kernel_size=ec.get("cnn_module_kernel", 15),
                   vocab=output_dim, norm_eps=ec.get("norm_eps", 1e-5), cmvn=cmvn)


# chunkformer-large (BASELINE.json configs[1]): 12 layers, d=512, 8 heads, ff 2048, V=5000 (paper BPE)
LARGE = EncoderConfig()
# the reference's shipped d=512 recipe family: 4 heads -> head_dim 128
# (examples/asr/rnnt/conf/chunkformer-rnnt-large-vie.yaml:5-6)
LARGE_4H = EncoderConfig(n_heads=4)
# the reference's shipped small recipes (examples/asr/ctc/conf/chunkformer-ctc-small-libri-100h.yaml:5-8,
# rnnt small, libri-960h): d=256, 4 heads (head_dim 64), ff 2048, 12 blocks, bpe1024 vocabulary
SMALL256 = EncoderConfig(d_model=256, n_heads=4, ffn_dim=2048, num_blocks=12, vocab=1024)
# small config used for the committed golden fixtures (tests/golden)
SMALL = EncoderConfig(d_model=128, n_heads=2, ffn_dim=256, num_blocks=2, vocab=48)
