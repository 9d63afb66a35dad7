"""GPU: the on-disk checkpoint loader end to end.

A directory in the reference layout (chunkformer_model.py:146-205) is written from the seeded
4-head d=512 weights of tests/golden/large_4h.npz -- config.yaml (the large vie recipe's
encoder_conf, examples/asr/rnnt/conf/chunkformer-rnnt-large-vie.yaml), global_cmvn as JSON
stats (utils/cmvn.py:23-45), pytorch_model.bin (torch.save of plain tensors), vocab.txt -- then
ChunkFormerModel.from_pretrained -> batch_decode must return the strings the reference's own
model_utils.get_output produced from the reference's CTC ids (tests/golden/text.json)."""
import json
import os

import numpy as np
import pytest
import torch
import yaml

pytestmark = pytest.mark.gpu

ENCODER_CONF = {"output_size": 512, "attention_heads": 4, "linear_units": 2048, "num_blocks": 12,
                "dropout_rate": 0.1, "positional_dropout_rate": 0.1, "attention_dropout_rate": 0.1,
                "input_layer": "dw_striding", "normalize_before": True, "cnn_module_kernel": 15,
                "use_cnn_module": True, "activation_type": "swish", "pos_enc_layer_type": "chunk_rel_pos",
                "selfattention_layer_type": "chunk_rel_seflattn", "cnn_module_norm": "layer_norm",
                "dynamic_conv": True}


def write_checkpoint_dir(path, sd, cfg, with_cmvn_buffers: bool, cmvn_key: bool = True):
    from chunkformer_amd.weights import synthetic_vocab
    conf = {"encoder": "chunkformer", "encoder_conf": ENCODER_CONF, "input_dim": 80, "output_dim": cfg.vocab,
            "model": "asr_model", "ctc_conf": {"ctc_blank_id": 0}}
    if cmvn_key:   # the reference enables CMVN from the global_cmvn FILE alone (chunkformer_model.py:153-160)
        conf.update(cmvn="global_cmvn", cmvn_conf={"cmvn_file": "global_cmvn", "is_json_cmvn": True})
    with open(os.path.join(path, "config.yaml"), "w") as f:
        yaml.safe_dump(conf, f)
    # stats whose (mean, istd) reproduce the seeded CMVN tensors (up to f32 rounding)
    cnt = 1000.0
    mean = sd["encoder.global_cmvn.mean"].double()
    istd = sd["encoder.global_cmvn.istd"].double()
    var = 1.0 / istd ** 2
    stats = {"mean_stat": (mean * cnt).tolist(), "var_stat": ((var + mean ** 2) * cnt).tolist(), "frame_num": cnt}
    with open(os.path.join(path, "global_cmvn"), "w") as f:
        json.dump(stats, f)
    ckpt = {k: v for k, v in sd.items() if with_cmvn_buffers or "global_cmvn" not in k}
    torch.save(ckpt, os.path.join(path, "pytorch_model.bin"))
    with open(os.path.join(path, "vocab.txt"), "w", encoding="utf8") as f:
        for i, tok in synthetic_vocab(cfg.vocab).items():
            f.write(f"{tok} {i}\n")


@pytest.mark.parametrize("with_cmvn_buffers,cmvn_key", [(True, True), (False, True), (False, False)])
def test_from_pretrained_batch_decode(tmp_path, golden_dir, with_cmvn_buffers, cmvn_key):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from chunkformer_amd.config import LARGE_4H
    from chunkformer_amd.model import ChunkFormerModel
    from chunkformer_amd.weights import synthetic_features, synthetic_state_dict
    g = np.load(os.path.join(golden_dir, "large_4h.npz"))
    with open(os.path.join(golden_dir, "text.json"), encoding="utf8") as f:
        text = json.load(f)
    sd = synthetic_state_dict(LARGE_4H, int(g["seed"]))
    write_checkpoint_dir(str(tmp_path), sd, LARGE_4H, with_cmvn_buffers, cmvn_key)
    m = ChunkFormerModel.from_pretrained(str(tmp_path), dtype="fp32")
    assert m.config.cmvn
    assert m.config.n_heads == 4 and m.config.head_dim == 128 and m.config.vocab == LARGE_4H.vocab
    assert m.char_dict is not None and m.char_dict[0] == "<blank>"
    xs = synthetic_features(g["lens"].tolist(), int(g["feat_seed"]))
    out = m.batch_decode(xs, 64, 128, 128)
    assert out == text["large_4h_decode"]
    # endless_decode on the first utterance returns the reference's timestamp items format
    items = m.endless_decode(xs[0], 64, 128, 128, total_batch_duration=1800, return_timestamps=True)
    assert isinstance(items, list) and all(set(it) == {"decode", "start", "end"} for it in items)
    assert "".join(it["decode"] for it in items).replace(" ", "") == text["large_4h_decode"][0].replace(" ", "")
