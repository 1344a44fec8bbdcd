"""The opt-in quad layout's hash in the oracle (CPU): with GOL_LAYOUT=quads a
torus whose rows hold whole quads of words is hashed over quad-interleaved
device words -- column 128g + 4b + j in bit b of word 4g + j, keys
A(y, c mod 4) B(c div 4) (DESIGN.md sections 3 and 5).  The C restatement
(oracle_quad_word built bit by bit) and the numpy one (np_device_words) must
agree; boards whose rows hold no whole quad hash exactly as without it."""
import numpy as np
import pytest

from oracle import oracle as O


@pytest.fixture
def quads(monkeypatch):
    monkeypatch.setenv("GOL_LAYOUT", "quads")


def test_quad_layout_rule(quads):
    assert [O.device_ilv(32 * w) for w in (1, 2, 3, 4, 6, 8, 12, 130)] == [1, 2, 1, 4, 2, 4, 4, 2]
    assert O.device_ilv(128, O.REF_CLIPPED) == 1
    assert all(O.device_ilv(32 * w) == O.np_ilv(32 * w) for w in range(1, 40))


@pytest.mark.parametrize("W", [128, 256, 32 * 12, 4096, 32 * 6, 32 * 7])
def test_quad_hash_c_equals_numpy(quads, W):
    b = O.seed_packed(W, 37, W + 1)
    assert O.hash_packed(b, W, row0=11) == O.np_hash(b, W, row0=11)


def test_quad_words_bit_by_bit(quads):
    W = 512
    b = O.seed_packed(W, 3, 9)
    dw = O.np_device_words(b, W)
    for c in range(16):
        expect = 0
        for bit in range(32):
            col = 128 * (c // 4) + 4 * bit + c % 4
            expect |= int((b[1, col // 32] >> (col % 32)) & 1) << bit
        assert int(dw[1, c]) == expect
        row = np.ascontiguousarray(b[1])
        assert O.lib().oracle_quad_word(row[c - c % 4:].ctypes.data_as(O._u32p), c % 4) == expect


def test_quad_hash_differs_from_pair_hash_only_on_quad_boards(monkeypatch):
    b = O.seed_packed(4096, 8, 3)
    pairs = O.hash_packed(b, 4096)
    monkeypatch.setenv("GOL_LAYOUT", "quads")
    assert O.hash_packed(b, 4096) != pairs
    b6 = O.seed_packed(32 * 6, 8, 3)
    monkeypatch.delenv("GOL_LAYOUT")
    p6 = O.hash_packed(b6, 32 * 6)
    monkeypatch.setenv("GOL_LAYOUT", "quads")
    assert O.hash_packed(b6, 32 * 6) == p6  # 6 words: pairs either way
