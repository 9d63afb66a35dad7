"""RNN-T consumer of the encoder: the greedy search the reference runs for `model: transducer`
checkpoints (chunkformer_model.py:439-448 endless_decode, 533-543 batch_decode) on top of the
encoder hot path, as one persistent HIP kernel (csrc/rnnt.hip, cfm_rnnt_* in include/cfm.h).

  optimized_search      transducer/search/greedy_search.py:6-74   -> RNNTGreedy.optimized_search
  batch_greedy_search   transducer/search/greedy_search.py:78-92  -> RNNTGreedy.batch_greedy_search

Supported predictor / joint: the reference's shipped recipe
(examples/asr/rnnt/conf/chunkformer-rnnt-large-vie.yaml): `predictor: rnn` with rnn_type lstm
(transducer/predictor.py:66-208), `joint: transducer_joint` with prejoin_linear, no
postjoin_linear, joint_mode add, tanh, no HAT (transducer/joint.py:10-111); blank id 0
(init_model.py:125-128).  Anything else raises AssertionError like the reference's asserts.
The predictor and joint run in f32 whatever the encoder's compute dtype.
"""
from __future__ import annotations

import ctypes
import math
import weakref
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch

from . import _lib


@dataclass
class RNNTConfig:
    vocab: int = 1024           # output_dim (bpe 1024 in the vie recipe)
    enc_dim: int = 512          # joint_conf.enc_output_size
    embed_size: int = 256       # predictor_conf.embed_size
    hidden: int = 512           # predictor_conf.hidden_size
    num_layers: int = 2         # predictor_conf.num_layers
    pred_out: int = 512         # predictor_conf.output_size (= joint_conf.pred_output_size)
    join_dim: int = 512         # joint_conf.join_dim
    blank: int = 0

    @classmethod
    def from_conf(cls, conf: dict, vocab: int, enc_dim: int) -> "RNNTConfig":
        """From a reference config.yaml (init_model.py:118-135)."""
        assert conf.get("predictor", "rnn") == "rnn", "only predictor: rnn is supported"
        pc = dict(conf.get("predictor_conf") or {})
        jc = dict(conf.get("joint_conf") or {})
        assert conf.get("joint", "transducer_joint") == "transducer_joint"
        assert pc.get("rnn_type", "lstm") == "lstm", "only rnn_type lstm is supported"
        assert pc.get("bias", True), "predictor without bias is not supported"
        assert jc.get("prejoin_linear", True) and not jc.get("postjoin_linear", False)
        assert jc.get("joint_mode", "add") == "add" and jc.get("activation", "tanh") == "tanh"
        assert not jc.get("hat_joint", False)
        c = cls(vocab=int(vocab), enc_dim=int(jc.get("enc_output_size", enc_dim)),
                embed_size=int(pc["embed_size"]), hidden=int(pc["hidden_size"]), num_layers=int(pc["num_layers"]),
                pred_out=int(pc["output_size"]), join_dim=int(jc["join_dim"]))
        assert int(jc.get("pred_output_size", c.pred_out)) == c.pred_out
        return c

    def validate(self) -> None:
        for v in (self.embed_size, self.hidden, self.pred_out, self.join_dim, self.enc_dim):
            assert v % 4 == 0 and 0 < v <= 1024, "predictor / joint widths must be multiples of 4, <= 1024"
        assert self.num_layers >= 1 and self.vocab > 1


def schema(c: RNNTConfig) -> List[Tuple[str, Tuple[int, ...]]]:
    """(name, shape) of every predictor / joint tensor, keys as in the reference Transducer."""
    H = c.hidden
    out = [("predictor.embed.weight", (c.vocab, c.embed_size))]
    for l in range(c.num_layers):
        inp = c.embed_size if l == 0 else H
        out += [(f"predictor.rnn.weight_ih_l{l}", (4 * H, inp)), (f"predictor.rnn.weight_hh_l{l}", (4 * H, H)),
                (f"predictor.rnn.bias_ih_l{l}", (4 * H,)), (f"predictor.rnn.bias_hh_l{l}", (4 * H,))]
    out += [("predictor.projection.weight", (c.pred_out, H)), ("predictor.projection.bias", (c.pred_out,)),
            ("joint.enc_ffn.weight", (c.join_dim, c.enc_dim)), ("joint.enc_ffn.bias", (c.join_dim,)),
            ("joint.pred_ffn.weight", (c.join_dim, c.pred_out)), ("joint.pred_ffn.bias", (c.join_dim,)),
            ("joint.ffn_out.weight", (c.vocab, c.join_dim)), ("joint.ffn_out.bias", (c.vocab,))]
    return out


def synthetic_transducer_state_dict(c: RNNTConfig, seed: int = 0, blank_bias: float = 3.72, joint_scale: float = 4.0,
                                    enc_scale: float = 2.0, pred_scale: float = 6.0
                                    ) -> "OrderedDict[str, torch.Tensor]":
    """Seeded weights with the reference modules' default init magnitudes (Embedding N(0,1), LSTM
    U(+-1/sqrt(hidden)), Linear U(+-1/sqrt(fan_in))), then shaped like a trained joint: ffn_out
    scaled by `joint_scale`, enc_ffn by `enc_scale` and pred_ffn by `pred_scale` (peakier logits
    that depend on both the frame and the predictor state) and `blank_bias` added to the blank
    logit's bias.  With the defaults greedy search over the golden encoder outputs mixes blank
    frames, frames with a few tokens ended by a blank and frames that hit the n_steps cap (a
    default-init joint has nearly state- and frame-independent logits: all blank or all tokens)."""
    g = torch.Generator().manual_seed(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    shapes = dict(schema(c))
    for name, shape in schema(c):
        if name == "predictor.embed.weight":
            t = torch.randn(shape, generator=g)
        elif name.startswith("predictor.rnn."):
            a = 1.0 / math.sqrt(c.hidden)
            t = (torch.rand(shape, generator=g) * 2 - 1) * a
        else:
            fan = shapes[name[: -len("bias")] + "weight"][1] if name.endswith("bias") else shape[1]
            t = (torch.rand(shape, generator=g) * 2 - 1) / math.sqrt(fan)
        sd[name] = t.contiguous()
    sd["joint.ffn_out.weight"] *= joint_scale
    sd["joint.enc_ffn.weight"] *= enc_scale
    sd["joint.pred_ffn.weight"] *= pred_scale
    sd["joint.ffn_out.bias"][c.blank] += blank_bias
    return sd


def with_emission_memory(sd: Dict[str, torch.Tensor], c: RNNTConfig, frame_dirs: torch.Tensor,
                         frame_bias: torch.Tensor, tokens: List[int], forget: float = 0.3, write: float = 0.5,
                         suppress: float = 40.0, token_gain: float = 4.0, blank_logit: float = 2.0,
                         rest_scale: float = 0.1) -> "OrderedDict[str, torch.Tensor]":
    """Reshape seeded transducer weights so greedy search behaves like a trained transducer: a frame
    emits the few tokens it carries, one per step, then blank.  Test-fixture recipe
    (tests/golden/gen_golden.py gen_rnnt_memory); every tensor keeps its reference shape.

    * token k (tokens[k], k < K) has joint unit 1 + k: enc_ffn row = frame_dirs[k], bias
      frame_bias[k], so its logit token_gain * tanh(frame_dirs[k] . x + frame_bias[k] - memory_k)
      depends on the frame;
    * the predictor keeps a decaying memory of each emitted token: LSTM layer 0 unit k writes
      `write` when its input is tokens[k] (one-hot embedding column k) and every unit keeps `forget`
      of its cell per predictor step; layer 1 unit k and projection row k pass it through, and
      pred_ffn row 1 + k subtracts suppress x memory_k — a token just emitted is off for the next
      few steps, so the frame moves on to its next token or to blank;
    * blank's logit is the constant `blank_logit`; the seeded rows of the remaining joint units
      are scaled by `rest_scale` (small frame- and state-dependent perturbations) and every other
      token has bias -8."""
    sd = OrderedDict((k, v.clone()) for k, v in sd.items())
    K, H = len(tokens), c.hidden
    assert K + 1 <= min(c.join_dim, H, c.embed_size, c.pred_out)
    big = 10.0
    emb = sd["predictor.embed.weight"]
    emb[:, :K] = 0.0
    for k, t in enumerate(tokens):
        emb[t, k] = 1.0
    for layer in range(c.num_layers):
        wih, whh = sd[f"predictor.rnn.weight_ih_l{layer}"], sd[f"predictor.rnn.weight_hh_l{layer}"]
        bih, bhh = sd[f"predictor.rnn.bias_ih_l{layer}"], sd[f"predictor.rnn.bias_hh_l{layer}"]
        for k in range(K):
            gi, gf, gg, go = k, H + k, 2 * H + k, 3 * H + k     # gate rows i, f, g, o of unit k
            for r in (gi, gf, gg, go):
                wih[r].zero_()
                whh[r].zero_()
                bhh[r] = 0.0
            bih[go] = big
            if layer == 0:        # i: open on tokens[k] only; f: keep `forget`; g: write `write`
                wih[gi, k] = 2 * big
                bih[gi] = -big
                bih[gf] = math.log(forget / (1 - forget))
                bih[gg] = math.atanh(write)
            else:                 # pass-through of the layer below's unit k
                bih[gi] = big
                bih[gf] = -big
                wih[gg, k] = 1.0
                bih[gg] = 0.0
    proj_w, proj_b = sd["predictor.projection.weight"], sd["predictor.projection.bias"]
    proj_w[:K].zero_()
    proj_b[:K] = 0.0
    for k in range(K):
        proj_w[k, k] = 1.0
    ew, eb = sd["joint.enc_ffn.weight"], sd["joint.enc_ffn.bias"]
    pw, pb = sd["joint.pred_ffn.weight"], sd["joint.pred_ffn.bias"]
    ow, ob = sd["joint.ffn_out.weight"], sd["joint.ffn_out.bias"]
    ow *= rest_scale
    ob.fill_(-8.0)
    ob[c.blank] = blank_logit
    for u in range(K + 1):
        ew[u].zero_()
        eb[u] = 0.0
        pw[u].zero_()
        pb[u] = 0.0
        ow[:, u] = 0.0
    for k, t in enumerate(tokens):
        u = 1 + k
        ew[u] = frame_dirs[k].to(ew.dtype)
        eb[u] = float(frame_bias[k])
        pw[u, k] = -suppress
        ow[t, u] = token_gain
        ob[t] = 0.0
    return sd


class RNNTGreedy:
    """The transducer greedy search on libcfm (cfm_rnnt_*): predictor LSTM + joint + argmax loop in
    one persistent kernel — one workgroup per utterance for batches, `grid_blocks` workgroups per
    utterance with grid barriers between the predictor / joint phases for a few long utterances
    (endless_decode's B = 1) — the predictor evaluated once per emitted
    token and the joint evaluated over blocks of frames at a time (exact: frames before the first
    non-blank of a block see the same predictor state as in the sequential loop)."""

    def __init__(self, cfg: RNNTConfig, state_dict: Dict[str, torch.Tensor], device):
        cfg.validate()
        self.cfg = cfg
        self.device = torch.device(device)
        for name, shape in schema(cfg):
            if name not in state_dict:
                raise KeyError(f"missing weight {name}")
            if tuple(state_dict[name].shape) != tuple(shape):
                raise ValueError(f"weight {name}: shape {tuple(state_dict[name].shape)} != {shape}")
        c = _lib.CfmRnntConfig(cfg.vocab, cfg.enc_dim, cfg.embed_size, cfg.hidden, cfg.num_layers, cfg.pred_out,
                               cfg.join_dim, cfg.blank)
        names = [n for n, _ in schema(cfg)]
        keep = []
        views = (_lib.CfmTensorView * len(names))()
        for i, k in enumerate(names):
            t = state_dict[k].detach().to("cpu", torch.float32).contiguous()
            keep.append(t)
            views[i] = _lib.CfmTensorView(k.encode(), t.data_ptr(), t.numel())
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(_lib.cfm_rnnt_create(ctypes.byref(c), views, len(names), self.device.index or 0,
                                            ctypes.byref(h)))
        self._h = h
        self.grid_fallbacks = 0   # searches the multi-CU kernel left early (barrier timeout), rerun on one workgroup
        self._finalizer = weakref.finalize(self, _lib.cfm_rnnt_destroy, ctypes.c_void_p(h.value))

    def set_option(self, key: str, value: int) -> None:
        """cfm_rnnt_set_option: "grid_blocks" = workgroups per utterance of the multi-CU search
        (0 = one workgroup per utterance always)."""
        _lib.check(_lib.cfm_rnnt_set_option(self._h, key.encode(), int(value)))

    def grid_blocks(self, B: int) -> int:
        """Workgroups per utterance a search over B utterances runs with (0: one-workgroup kernel)."""
        return int(_lib.cfm_rnnt_grid_blocks(self._h, int(B)))

    @torch.no_grad()
    def greedy_packed(self, enc: torch.Tensor, row_start, row_len, n_steps: int = 64) -> torch.Tensor:
        """Greedy search over utterances b = rows [row_start[b], row_start[b] + row_len[b]) of
        enc [rows, enc_dim]; returns the dense decisions [rows, n_steps] int32 (0 = blank), row t of
        an utterance holding the tokens emitted at its frame t in step order (greedy_search.py:23-72
        output[:, t * n_steps + step], sos removed)."""
        enc = enc.reshape(-1, self.cfg.enc_dim).to(self.device, torch.float32).contiguous()
        rows = enc.shape[0]
        B = len(row_start)
        rs = torch.tensor([int(v) for v in row_start], dtype=torch.int32)
        rl = torch.tensor([int(v) for v in row_len], dtype=torch.int32)
        if B and (int((rs + rl).max()) > rows or int(rs.min()) < 0 or int(rl.min()) < 0):
            raise ValueError("utterance row ranges exceed the encoder rows")
        if n_steps < 1:
            raise ValueError("n_steps must be >= 1")
        out = torch.zeros(max(rows, 1), n_steps, dtype=torch.int32, device=self.device)
        if rows == 0 or B == 0:
            return out[:rows]
        nbytes = int(_lib.cfm_rnnt_workspace_bytes(self._h, rows))
        ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.device)
        rs_d, rl_d = rs.to(self.device), rl.to(self.device)
        _lib.check(_lib.cfm_rnnt_greedy(self._h, enc.data_ptr(), rows, rs_d.data_ptr(), rl_d.data_ptr(), B,
                                        int(n_steps), out.data_ptr(), ws.data_ptr(), nbytes,
                                        torch.cuda.current_stream(self.device).cuda_stream))
        self._keep = (rs_d, rl_d, ws)   # alive until the stream consumed them
        G = self.grid_blocks(B)
        if G:
            # the multi-CU search stops early if a grid barrier timed out (its workgroups were not all resident:
            # CUs held by another stream's kernels): never return that partial result, run the search again
            # on the one-workgroup kernel, which needs no co-residency (a per-call flag: the handle's options and
            # grid weight image stay as they are, so no device sync and no other caller is disturbed)
            torch.cuda.current_stream(self.device).synchronize()
            if int(_lib.cfm_rnnt_error(self._h, ws.data_ptr(), rows)) != 0:
                self.grid_fallbacks += 1
                out.zero_()
                _lib.check(_lib.cfm_rnnt_greedy_ex(self._h, enc.data_ptr(), rows, rs_d.data_ptr(), rl_d.data_ptr(),
                                                   B, int(n_steps), out.data_ptr(), ws.data_ptr(), nbytes,
                                                   _lib.CFM_RNNT_ONE_WORKGROUP,
                                                   torch.cuda.current_stream(self.device).cuda_stream))
        return out

    @torch.no_grad()
    def optimized_search(self, encoder_out: torch.Tensor, encoder_out_lens: torch.Tensor,
                         n_steps: int = 64) -> torch.Tensor:
        """greedy_search.py:6-74: encoder_out [B, T, E], lens [B] -> [B, T * n_steps] int64."""
        B, T, E = encoder_out.shape
        lens = [min(int(v), T) for v in encoder_out_lens.tolist()]
        dense = self.greedy_packed(encoder_out.reshape(B * T, E), [b * T for b in range(B)], lens, n_steps)
        return dense.view(B, T * n_steps).long()

    @torch.no_grad()
    def batch_greedy_search(self, encoder_out: torch.Tensor, encoder_out_lens: torch.Tensor,
                            n_steps: int = 64) -> List[List[int]]:
        """greedy_search.py:78-92: the non-blank decisions of every utterance, in order."""
        out = self.optimized_search(encoder_out, encoder_out_lens, n_steps)
        return [row[row != self.cfg.blank].tolist() for row in out]
