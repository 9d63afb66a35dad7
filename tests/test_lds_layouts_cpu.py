"""LDS layout invariants of the ring attention kernel's rel_shift scratch (chunkformer_amd/csrc/attention.hip,
`skew_slot` / `skew_half`), checked on the CPU against the banking model of MI355X_MICROARCH.md §LDS: the 16-lane
groups of ds_write_b64 and the 32-lane groups of ds_read_b32 / ds_read2_b32 take one LDS cycle when their dwords hit
distinct banks ((a/4) mod 32).  The permuted row order is what removed the read side's 2-way conflicts (DESIGN §5,
round 6); a table edit that breaks the property fails here, without a GPU."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "chunkformer_amd", "csrc", "attention.hip")
RD_PITCH = 52   # ATTN_RD_PITCH (bf16 elements per scratch row)


def _slot_table():
    src = open(SRC).read()
    m = re.search(r"return \(int\)\(\((0x[0-9a-f]+)ull >> \(4 \* fr\)\) & 15u\)", src)
    assert m, "skew_slot table not found"
    word = int(m.group(1), 16)
    return [(word >> (4 * fr)) & 15 for fr in range(16)]


def _write_cycles(slot):
    """ds_write_b64 of band subtile pt (3 per half): lanes (fr, g) write elements slot[fr]*P + 16pt + 4g .. +3."""
    cyc = 0
    for pt in range(3):
        for g in range(4):   # 4 groups of 16 contiguous lanes (g = lane >> 4)
            banks = {}
            for fr in range(16):
                d = (2 * (slot[fr] * RD_PITCH + 16 * pt + 4 * g)) // 4
                for k in range(2):
                    banks.setdefault((d + k) % 32, set()).add(d + k)
            cyc += max(len(v) for v in banks.values())
    return cyc


def _read_cycles(slot):
    """the read-side shear: 3 dwords from the 4-B aligned address at or below element slot*P + 15 - fr + 16 st2 + 4g."""
    cyc = 0
    for st2 in range(2):
        for acc in range(3):            # ds_read2_b32 (2 accesses) + ds_read_b32
            for half in range(2):       # 32-lane groups
                banks = {}
                for lane in range(32 * half, 32 * half + 32):
                    fr, g = lane & 15, lane >> 4
                    al = (2 * (slot[fr] * RD_PITCH + 15 - fr + 16 * st2 + 4 * g)) & ~3
                    d = al // 4 + acc
                    banks.setdefault(d % 32, set()).add(d)
                cyc += max(len(v) for v in banks.values())
    return cyc


def test_skew_slot_table_is_a_permutation():
    assert sorted(_slot_table()) == list(range(16))


def test_skew_scratch_conflict_free_with_the_permutation():
    slot = _slot_table()
    assert _write_cycles(slot) == 3 * 4            # one cycle per 16-lane group
    assert _read_cycles(slot) == 2 * 3 * 2         # one cycle per 32-lane group


def test_query_order_is_two_way_on_the_read_side():
    # the round-6 first pass (rows in query order): writes conflict-free, reads 2-way -- what the table fixes
    ident = list(range(16))
    assert _write_cycles(ident) == 12
    assert _read_cycles(ident) == 24


@pytest.mark.parametrize("fr", range(16))
def test_rows_stay_inside_the_scratch(fr):
    # the farthest element a lane touches: its row start + the read window (15 - fr + 16 + 12 + 6 elements)
    slot = _slot_table()
    last = slot[fr] * RD_PITCH + (15 - fr) + 16 + 12 + 6
    assert last <= 16 * RD_PITCH + 8   # SCR_ELEMS = 16 * RD_PITCH + 8
