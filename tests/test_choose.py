"""CPU: which k blocks a decode uses when more are at hand (sec_decode_choose).

storb's validator fetches every data and parity piece of a chunk
(/root/reference/storb/validator/validator.py:1556-1604, 1631) and the reference decodes from the
first k in piece order (storb/util/piece.py:189-191).  Any k distinct blocks of an MDS code give
the same bytes, so the library picks the cheapest k: every present primary, then parity rows from
as few of the decode kernels' 16-row groups as possible.  Host logic only (no GPU); the oracle
checks that decoding from the chosen blocks returns the chunk."""

import random

import pytest

from oracle import cfec
from storb_amd.engine import choose_blocks


def _sn(pick, sharenums):
    return [sharenums[i] for i in pick]


def test_all_primaries_present_takes_only_primaries():
    sn = list(range(96))
    random.Random(1).shuffle(sn)
    pick = choose_blocks(64, 96, sn)
    assert sorted(_sn(pick, sn)) == list(range(64))
    assert _sn(pick, sn) == sorted(_sn(pick, sn))  # ascending sharenum order


def test_one_group_preferred_over_lowest_rows():
    # zfec(64,96): 10 data blocks lost; parity group 0 (rows 64..79) lost 8 rows, group 1 complete
    lost = set(range(0, 40, 4))
    sn = [j for j in range(64) if j not in lost] + [64 + r for r in range(16) if r % 2] + list(range(80, 96))
    got = _sn(choose_blocks(64, 96, sn), sn)
    assert [s for s in got if s >= 64] == list(range(80, 90))  # group 1, lowest rows first
    # the reference's first k would mix both groups
    assert sorted(sn)[:64][-10:] != list(range(80, 90))


def test_lowest_group_holding_e_rows_lowest_rows():
    lost = {3, 17, 41}
    sn = [j for j in range(96) if j not in lost and j != 65]
    got = _sn(choose_blocks(64, 96, sn), sn)
    assert [s for s in got if s >= 64] == [64, 66, 67]


def test_more_than_one_group_needed_fewest_groups_most_rows_first():
    rng = random.Random(3)
    lost = set(rng.sample(range(64), 20))  # e = 20 > 16: both groups
    par = [64 + r for r in range(16) if r not in (0, 1, 2, 3, 4, 5)] + list(range(80, 96))  # 10 + 16 present
    sn = [j for j in range(64) if j not in lost] + par
    rng.shuffle(sn)
    got = _sn(choose_blocks(64, 96, sn), sn)
    rows = sorted(s for s in got if s >= 64)
    # the fuller group whole, then the other's lowest present rows
    assert rows == [70, 71, 72, 73] + list(range(80, 96))


def test_duplicates_and_out_of_range_skipped_and_too_few():
    sn = [0, 0, 1, 7, -1, 5, 1, 2]  # zfec(4,6): distinct valid = {0, 1, 2, 5}
    pick = choose_blocks(4, 6, sn)
    assert _sn(pick, sn) == [0, 1, 2, 5] and pick == [0, 2, 7, 5]  # first occurrences
    assert choose_blocks(4, 6, [0, 0, 1, 5, 9]) is None


def test_shapes_without_bit_sliced_kernels_take_lowest_parity_rows():
    sn = [1, 4, 5, 3, 2, 0]  # zfec(3,6), every block present
    assert sorted(_sn(choose_blocks(3, 6, sn), sn)) == [0, 1, 2]
    sn = [5, 4, 3, 2]  # zfec(3,6) without 0 and 1
    assert _sn(choose_blocks(3, 6, sn), sn) == [2, 3, 4]


@pytest.mark.parametrize("k,m", [(4, 6), (10, 14), (16, 24), (32, 48), (64, 96), (8, 11)])
def test_random_losses_decode_to_the_chunk(k, m):
    """Random 10-30 % of the m blocks lost (parity rows included): the chosen k are distinct,
    valid, include every present primary, and the oracle decodes them to the chunk."""
    rng = random.Random(k * 1000 + m)
    for trial in range(6):
        n = rng.randrange(k * k + 1, 3000 * k)
        data = rng.randbytes(n)
        blocks = cfec.easy_encode(data, k, m)
        B = len(blocks[0])
        frac = rng.uniform(0.1, 0.3)
        present = [j for j in range(m) if rng.random() > frac]
        if len(present) < k:
            continue
        rng.shuffle(present)
        pick = choose_blocks(k, m, present)
        chosen = [present[i] for i in pick]
        assert len(set(chosen)) == k and all(0 <= s < m for s in chosen)
        assert {s for s in present if s < k} <= set(chosen)
        assert cfec.easy_decode([blocks[s] for s in chosen], chosen, k * B - n, k, m) == data
