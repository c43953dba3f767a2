"""Board builders shared by the oracle (CPU) and HIP (GPU) parity tests."""
import numpy as np


def mask_boards():
    """Boards realising all 16 legal masks: a terminal board with 1-2 holes / equal pairs, plus
    one empty edge row/column for the four single-direction masks."""
    T = np.array([1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 1], np.uint8)
    out = []
    for i in range(16):
        b = T.copy(); b[i] = 0; out.append(b)
        for j in range(16):
            b2 = b.copy(); b2[j] = 0; out.append(b2)
            b3 = T.copy(); b3[j] = T[i]; out.append(b3)
    for cells in ([0, 1, 2, 3], [12, 13, 14, 15], [0, 4, 8, 12], [3, 7, 11, 15]):
        b = T.copy(); b[cells] = 0; out.append(b)
    return out


def boards_for_masks(masks, legal_mask):
    """One board per row whose legal mask (computed by legal_mask) is masks[row]."""
    by_mask = {}
    for b in mask_boards():
        by_mask.setdefault(legal_mask(b), b)
    assert len(by_mask) == 16
    return np.stack([by_mask[int(m)] for m in masks])
