"""Known answers for the primary-ray pixel order: mrt.pixel_table
(csrc/host/raygen.cpp, the reference's PixelTable::recalculate, PixelTable.cc:93-156)
against indices derived by hand and against an independent restatement written as a
sort, not as the reference's loop:

  * the bulk (the largest multiple-of-8 rectangle) is cut into 8x8 blocks, visited in
    Morton order of the block coordinates (x bit in the even positions), and each block's
    64 pixels in Morton order of (x, y) inside the block;
  * then the horizontal stripe below the bulk, column by column (x outer, y inner);
  * then the vertical stripe right of the bulk, corner included, row by row.

The device ray generator takes the same table (mrt.raygen.DeviceRayGen), so the GPU's
primary rays follow this order too (tests/test_gpu_raygen.py)."""
import numpy as np
import pytest

import mrt


def morton2(x, y, bits=16):
    """x bits in the even positions, y bits in the odd ones."""
    k = 0
    for b in range(bits):
        k |= ((x >> b) & 1) << (2 * b) | ((y >> b) & 1) << (2 * b + 1)
    return k


def restated(w, h):
    """index -> pixel, by sorting the pixels on their keys."""
    bw, bh = w & ~7, h & ~7
    bulk = [(morton2(x >> 3, y >> 3), morton2(x & 7, y & 7), y * w + x) for y in range(bh) for x in range(bw)]
    order = [p for _, _, p in sorted(bulk)]
    order += [py * w + px for px in range(bw) for py in range(bh, h)]
    order += [py * w + px for py in range(h) for px in range(bw, w)]
    return np.array(order, np.int32)


# (index, pixel) pairs worked out by hand from PixelTable.cc:93-156
HAND = {
    (16, 16): [(0, 0), (1, 1), (2, 16), (3, 17), (4, 2), (5, 3), (6, 18), (8, 32), (16, 4), (63, 7 * 16 + 7),
               (64, 8), (65, 9), (66, 24), (127, 7 * 16 + 15), (128, 8 * 16), (191, 15 * 16 + 7),
               (192, 8 * 16 + 8), (255, 255)],
    (20, 13): [(0, 0), (1, 1), (2, 20), (63, 7 * 20 + 7), (64, 8), (127, 7 * 20 + 15),
               (128, 8 * 20 + 0), (129, 9 * 20 + 0), (132, 12 * 20 + 0), (133, 8 * 20 + 1), (207, 12 * 20 + 15),
               (208, 16), (209, 17), (211, 19), (212, 20 + 16), (259, 12 * 20 + 19)],
}


@pytest.mark.parametrize("w,h", sorted(HAND))
def test_hand_derived_indices(w, h):
    table = mrt.pixel_table(w, h)
    assert len(table) == w * h
    for idx, pix in HAND[(w, h)]:
        assert table[idx] == pix, f"{w}x{h}: index {idx} -> pixel {table[idx]}, hand-derived {pix}"


@pytest.mark.parametrize("w,h", [(16, 16), (20, 13), (8, 8), (7, 5), (1, 1), (24, 17), (64, 48), (640, 480),
                                 (33, 9)])
def test_equals_the_sorted_restatement_and_is_a_permutation(w, h):
    table = mrt.pixel_table(w, h)
    assert np.array_equal(np.sort(table), np.arange(w * h, dtype=np.int32))
    assert np.array_equal(table, restated(w, h))
