"""ops.FragMask on CPU: the unpacker and the row slicing agree with a direct transcription of
the kernel's fragment-order layout (gemm_tile.hpp frag_mask_offset + the register-direct
epilogue's byte / bit order). The GPU tests check the kernels against the same unpacker."""
import pytest
import torch

from docker_dist_nn_amd import ops
from docker_dist_nn_amd.ops.kernels import FRAG_WAVES


def pack(bits: torch.Tensor, tiles) -> torch.Tensor:
    """bool [M][N] -> fragment-order bytes, element by element as the epilogue stores them."""
    M, N = bits.shape
    bm, bn = tiles
    WM, WN = FRAG_WAVES[tiles]
    FM, SN = bm // WM // 16, bn // WN
    FN = SN // 16
    NB = FM * FN // 2
    tm_n, tn_n = -(-M // bm), -(-N // bn)
    out = torch.zeros(tm_n * tn_n * bm * bn // 8, dtype=torch.uint8)
    for tm in range(tm_n):
        for tn in range(tn_n):
            for wm in range(WM):
                for wn in range(WN):
                    for lane in range(64):
                        off = (((tm * tn_n + tn) * (WM * WN) + wm * WN + wn) * 64 + lane) * NB
                        frow, fg = lane & 15, lane >> 4
                        for jj in range(FN // 2):
                            for i in range(FM):
                                row = tm * bm + wm * 16 * FM + frow + 16 * i
                                col = tn * bn + wn * SN + 16 * (fg & 1) + 8 * (fg >> 1) + 32 * jj
                                b = 0
                                for e in range(8):
                                    if row < M and col + e < N and bits[row, col + e]:
                                        b |= 1 << e
                                out[off + jj * FM + i] = b
    return out


@pytest.mark.parametrize("tiles", [(128, 64), (128, 128), (256, 128)])
def test_frag_mask_unpack_and_rows(tiles):
    gen = torch.Generator().manual_seed(tiles[0] + tiles[1])
    M, N = 2 * tiles[0] + 64, tiles[1] + 48  # partial tiles in both dimensions
    bits = torch.rand(M, N, generator=gen) > 0.5
    fm = ops.FragMask(pack(bits, tiles), tiles, M, N)
    assert fm.buf.numel() == ops.FragMask.nbytes(M, N, tiles)
    assert torch.equal(fm.bits(), bits)
    sub = fm[slice(tiles[0], M)]  # a micro-batch starting on a row-tile boundary
    assert sub.m == M - tiles[0] and torch.equal(sub.bits(), bits[tiles[0]:])
    with pytest.raises(ValueError, match="tile boundary"):
        fm[slice(16, M)]


def test_frag_mask_alloc_rejects_unsupported_tile():
    with pytest.raises(ValueError):
        ops.FragMask.alloc(256, 64, (64, 64), "cpu")
