"""CPU: the LDS piece swizzle of the halo-staged weight gradient (csrc/wgrad3h.hip, w3_swz) is free of bank
conflicts for every read the kernel issues.

k_wgrad3h keeps its input halo (128-B pixel rows: 8 pieces of 16 B) and its dY block (384-B pixel rows: 24 pieces)
as unswizzled pixel rows with piece' = piece ^ f(row), f(row) = bit 1 of row | bit 3 of row << 2.  Its MFMA operands
come from ds_read_b64_tr_b16: lane 4q + p of a 16-lane group reads 8 B at row r0 + q (and r0 + 4 + q), piece
L + 2 (p / 2), half p % 2; a half-wave is two such groups at rows r0 and r0 + 8 (the two 8-pixel k groups of a
16x16x32 step).  The kernel header claims the 32 lanes of a half-wave then touch 64 distinct 4-B banks for every
start row and every piece pair the kernel uses; this test re-checks the claim exhaustively against the same
model (64 banks x 4 B, one half-wave per cycle).
"""
import pytest


def w3_swz(row: int) -> int:  # csrc/wgrad3h.hip
    return ((row >> 1) & 1) | (((row >> 3) & 1) << 2)


def worst_conflict(row_units: int, piece_pairs) -> int:
    worst = 0
    for r0 in range(64):
        for L in piece_pairs:
            for second in (0, 4):
                banks = []
                for g in (0, 1):
                    for q in range(4):
                        row = r0 + 8 * g + second + q
                        for p in range(4):
                            lp = L + 2 * (p >> 1)
                            unit = row * row_units + (lp ^ w3_swz(row))
                            b0 = (unit * 16 + 8 * (p & 1)) // 4
                            banks += [b0 % 64, (b0 + 1) % 64]
                worst = max(worst, max(banks.count(b) for b in set(banks)))
    return worst


@pytest.mark.parametrize("name,row_units,pairs", [
    ("halo (32 channels, 128 B per pixel)", 8, [0, 1, 4, 5]),                                # hi / lo of each 16-ch half
    ("dY (96 channels, 384 B per pixel)", 24, [4 * m + h for m in range(6) for h in (0, 1)]),  # 6 blocks of 16
])
def test_wgrad3h_tr_reads_conflict_free(name, row_units, pairs):
    assert worst_conflict(row_units, pairs) == 1, name


def test_swizzle_stays_in_row():
    # the XOR only permutes pieces inside their aligned group of 8, so a 24-piece dY row never spills
    for row in range(256):
        for piece in range(24):
            assert (piece ^ w3_swz(row)) // 8 == piece // 8
