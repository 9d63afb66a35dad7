"""CPU restatement of the reference's transducer greedy search -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this module; the
product path (chunkformer_amd.transducer -> libcfm.so cfm_rnnt_greedy) never does.

Restates, with torch fp32 CPU ops as plain arithmetic:
  * RNNPredictor.forward_step (transducer/predictor.py:193-208): embed -> (dropout = identity in
    eval) -> nn.LSTM one step (gate order i, f, g, o) -> projection;
  * TransducerJoint.forward (transducer/joint.py:74-111) with prejoin_linear, joint_mode add,
    tanh, ffn_out;
  * optimized_search (transducer/search/greedy_search.py:6-74): per frame up to n_steps
    decisions; a decision is argmax(log_softmax(joint)); a non-blank decision becomes the next
    predictor input and commits the predictor's new LSTM state; a blank ends the frame.
Batch elements are independent in the reference (masks select rows), so each utterance runs alone.
Pinned against the reference itself by tests/golden/rnnt.npz (gen_golden.py gen_rnnt).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch


def predictor_step(sd: Dict[str, torch.Tensor], num_layers: int, tok: int, h: List[torch.Tensor],
                   c: List[torch.Tensor]) -> Tuple[torch.Tensor, List[torch.Tensor], List[torch.Tensor]]:
    """predictor.py:193-208 for one utterance: returns (projection output [P], new h, new c)."""
    x = sd["predictor.embed.weight"][tok]
    hn, cn = [], []
    for l in range(num_layers):
        g = (sd[f"predictor.rnn.weight_ih_l{l}"] @ x + sd[f"predictor.rnn.bias_ih_l{l}"]
             + sd[f"predictor.rnn.weight_hh_l{l}"] @ h[l] + sd[f"predictor.rnn.bias_hh_l{l}"])
        i, f, gg, o = g.chunk(4)
        c_new = torch.sigmoid(f) * c[l] + torch.sigmoid(i) * torch.tanh(gg)
        h_new = torch.sigmoid(o) * torch.tanh(c_new)
        hn.append(h_new)
        cn.append(c_new)
        x = h_new
    p = sd["predictor.projection.weight"] @ x + sd["predictor.projection.bias"]
    return p, hn, cn


def joint_logp(sd: Dict[str, torch.Tensor], enc_t: torch.Tensor, p: torch.Tensor) -> torch.Tensor:
    """joint.py:74-111 (prejoin, add, tanh, ffn_out) + log_softmax (greedy_search.py:51-52)."""
    e = sd["joint.enc_ffn.weight"] @ enc_t + sd["joint.enc_ffn.bias"]
    q = sd["joint.pred_ffn.weight"] @ p + sd["joint.pred_ffn.bias"]
    z = torch.tanh(e + q)
    return torch.log_softmax(sd["joint.ffn_out.weight"] @ z + sd["joint.ffn_out.bias"], dim=-1)


@torch.no_grad()
def greedy_one(sd: Dict[str, torch.Tensor], num_layers: int, hidden: int, enc: torch.Tensor, n_steps: int = 64,
               blank: int = 0) -> Tuple[torch.Tensor, float]:
    """One utterance enc [T, E] -> (decisions [T, n_steps] int64, smallest top-2 log-prob margin
    over every decision taken)."""
    sd = {k: v.float() for k, v in sd.items()}
    T = enc.shape[0]
    out = torch.zeros(T, n_steps, dtype=torch.int64)
    tok = blank
    h = [torch.zeros(hidden) for _ in range(num_layers)]
    c = [torch.zeros(hidden) for _ in range(num_layers)]
    margin = float("inf")
    for t in range(T):
        for step in range(n_steps):
            if step > 0 and out[t, step - 1] == blank:
                break
            p, hn, cn = predictor_step(sd, num_layers, tok, h, c)
            lp = joint_logp(sd, enc[t].float(), p)
            top = torch.topk(lp, 2).values
            margin = min(margin, float(top[0] - top[1]))
            k = int(lp.argmax())
            out[t, step] = k
            if k != blank:
                tok, h, c = k, hn, cn
    return out, margin


def optimized_search(sd, num_layers: int, hidden: int, encoder_out: torch.Tensor, encoder_out_lens,
                     n_steps: int = 64, blank: int = 0) -> Tuple[torch.Tensor, float]:
    """greedy_search.py:6-74 over [B, T, E]: -> ([B, T * n_steps] int64, smallest margin)."""
    B, T, _ = encoder_out.shape
    res = torch.zeros(B, T, n_steps, dtype=torch.int64)
    margin = float("inf")
    for b in range(B):
        n = min(int(encoder_out_lens[b]), T)
        o, m = greedy_one(sd, num_layers, hidden, encoder_out[b, :n], n_steps, blank)
        res[b, :n] = o
        margin = min(margin, m)
    return res.reshape(B, T * n_steps), margin
