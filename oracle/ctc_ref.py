"""ORACLE — test infrastructure only, never the product path.

Pure-Python restatement of the reference's CTC post-processing (ishine/chunkformer,
chunkformer/utils/model_utils.py), the checker for libcfm's `cfm_ctc_collapse`:

  remove_duplicates_and_blank   model_utils.py:23-32
  gen_ctc_peak_time             model_utils.py:49-58
  segments_with_timestamps      model_utils.py:174-221 (get_output_with_timestamps, before the
                                tokens -> text step: per sentence the de-duplicated non-blank tokens
                                and the start / end frame indices in 80 ms units)

Only `tests/` may import this module.
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple


def remove_duplicates_and_blank(hyp: Sequence[int], blank_id: int = 0) -> List[int]:
    """model_utils.py:23-32: keep the first frame of every run of equal ids, drop blanks."""
    out: List[int] = []
    cur = 0
    while cur < len(hyp):
        if hyp[cur] != blank_id:
            out.append(int(hyp[cur]))
        prev = cur
        while cur < len(hyp) and hyp[cur] == hyp[prev]:
            cur += 1
    return out


def gen_ctc_peak_time(hyp: Sequence[int], blank_id: int = 0) -> List[int]:
    """model_utils.py:49-58: frame index of every kept token."""
    times: List[int] = []
    cur = 0
    while cur < len(hyp):
        if hyp[cur] != blank_id:
            times.append(cur)
        prev = cur
        while cur < len(hyp) and hyp[cur] == hyp[prev]:
            cur += 1
    return times


def segments_with_timestamps(tokens: Sequence[int], max_silence: float) -> List[Tuple[List[int], int, int]]:
    """model_utils.py:174-221 for one utterance of frame ids (one id per 80 ms frame):
    returns [(deduplicated non-blank tokens, start frame, end frame), ...] -- the reference's
    {"decode", "start", "end"} items before class2str and milliseconds_to_hhmmssms."""
    start = end = prev_end = -1
    silence = 0
    per_time: List[int] = []
    items: List[Tuple[List[int], int, int]] = []
    t = -1
    for t in range(len(tokens)):
        v = int(tokens[t])
        if v == 0:
            silence += 1
        else:
            if start == -1 and end == -1:
                start = max(math.ceil((t + prev_end) / 2), t - 2) if prev_end != -1 else max(t - 2, 0)
            silence = 0
            per_time.append(v)
        if silence == max_silence and start != -1:
            end = prev_end = t
            items.append((remove_duplicates_and_blank(per_time), start, end))
            per_time, start, end, silence = [], -1, -1, 0
    if start != -1 and end == -1 and per_time:
        items.append((remove_duplicates_and_blank(per_time), start, t))
    return items
