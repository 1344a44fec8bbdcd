"""Host-side conversion between cell arrays and the packed board layout.

Layout (include/gol.h): row y, cell x = bit (x % 32) of 32-bit word (x / 32),
LSB first; words per row = ceil(width / 32); bits past the width are zero.
"""
from __future__ import annotations

import numpy as np


def words_per_row(width: int) -> int:
    return (width + 31) // 32


def pack(cells: np.ndarray) -> np.ndarray:
    """uint8/bool [H][W] -> uint32 [H][ceil(W/32)]."""
    c = np.asarray(cells, dtype=np.uint8) & 1
    H, W = c.shape
    ww = words_per_row(W)
    padded = np.zeros((H, ww * 32), dtype=np.uint8)
    padded[:, :W] = c
    return np.packbits(padded, axis=1, bitorder="little").view("<u4").astype(np.uint32)


def unpack(packed: np.ndarray, width: int) -> np.ndarray:
    """uint32 [H][>=ceil(W/32)] -> uint8 [H][W]."""
    p = np.ascontiguousarray(np.asarray(packed, dtype=np.uint32)[:, :words_per_row(width)])
    bits = np.unpackbits(p.astype("<u4").view(np.uint8), axis=1, bitorder="little")
    return bits[:, :width].astype(np.uint8)
