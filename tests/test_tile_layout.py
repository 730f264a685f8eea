"""CPU emulation of K1t's LDS address math (csrc/kernels/conv_tile3x3.hip), for both instances (64 and 128 input
channels): every 16-B chunk the patch and weight-stage writes place is read back by exactly the MFMA lane and step
that needs it, with no two chunks sharing an LDS slot and every offset inside its region. The arithmetic below is
the kernel's, line for line; a change to one must change the other."""
import numpy as np
import pytest

P_W = 34


def swz(row, c, m):  # the kernel's swz<M>
    return (c ^ (((row >> 1) & 7) if m == 8 else (row & 15))) << 4


def _cfg(cin):
    th = 8 if cin == 64 else 4
    return th, (th + 2) * P_W, cin // 8, cin * 2


@pytest.mark.parametrize("cin", [64, 128])
def test_patch_writes_and_fragment_reads_agree(cin):
    th, p_slots, nch, slot_b = _cfg(cin)
    lds = np.full(p_slots * slot_b // 16, -1, dtype=np.int64)  # one entry per 16-B chunk: the (slot, c) it holds
    for e in range(p_slots * nch):  # the store loop
        slot, c = divmod(e, nch)
        off = slot * slot_b + swz(slot, c, nch)
        assert 0 <= off < p_slots * slot_b and off % 16 == 0
        assert lds[off // 16] == -1, "two chunks in one LDS slot"
        lds[off // 16] = slot * nch + c
    assert (lds >= 0).all()
    fpw, halves = th // 2, cin // 64
    for wave in range(4):
        for lane in range(64):
            g4 = lane >> 4
            for f in range(fpw):
                sbase = ((th // 4) * wave + (f >> 1)) * P_W + 16 * (f & 1) + (lane & 15)
                r, col = (th // 4) * wave + (f >> 1), 16 * (f & 1) + (lane & 15)  # output pixel in the tile
                assert r < th and col < 32
                for tap in range(9):
                    kh, kw = divmod(tap, 3)
                    for half in range(halves):
                        for s in range(2):
                            chunk = 8 * half + 4 * s + g4
                            slot = sbase + kh * P_W + kw
                            off = slot * slot_b + swz(slot, chunk, nch)
                            got_slot, got_c = divmod(int(lds[off // 16]), nch)
                            # input pixel (r + kh - 1, col + kw - 1) of the tile = patch (r + kh, col + kw)
                            assert got_slot == (r + kh) * P_W + (col + kw)
                            # channels 64 half + 32 s + 8 (lane / 16): the MFMA B-operand k-block of this lane
                            assert 8 * got_c == 64 * half + 32 * s + 8 * g4


def test_weight_stage_writes_and_reads_agree():
    lds = np.full(64 * 128 // 16, -1, dtype=np.int64)
    for tid in range(256):
        for e in range(2):
            idx = tid + 256 * e
            n, c = idx >> 3, idx & 7
            off = n * 128 + swz(n, c, 8)
            assert lds[off // 16] == -1
            lds[off // 16] = n * 8 + c
    assert (lds >= 0).all()
    for lane in range(64):
        for j in range(4):
            for s in range(2):
                n = 16 * j + (lane & 15)
                wc = 4 * s + (lane >> 4)
                got = int(lds[(n * 128 + swz(n, wc, 8)) // 16])
                assert got == n * 8 + wc  # row n (output channel), input channels 8 wc .. 8 wc + 7 of the stage


@pytest.mark.parametrize("cin", [64, 128])
def test_fragment_reads_are_bank_conflict_free(cin):
    """ds_read_b128 serves 16 lanes per pass; the 16 pixels of a fragment row must cover all 64 banks once (16 B =
    4 banks each)."""
    th, p_slots, nch, slot_b = _cfg(cin)
    for wave in range(4):
        for f in range(th // 2):
            for tap in range(9):
                kh, kw = divmod(tap, 3)
                for g4 in range(4):
                    chunk = 4 * (tap % 2) + g4
                    banks = set()
                    for l16 in range(16):
                        slot = ((th // 4) * wave + (f >> 1)) * P_W + 16 * (f & 1) + l16 + kh * P_W + kw
                        off = slot * slot_b + swz(slot, chunk, nch)
                        banks.add((off // 16) % 16)
                    assert len(banks) == 16


def test_weight_reads_are_bank_conflict_free():
    for j in range(4):
        for wc in range(8):
            banks = {((n * 128 + swz(n, wc, 8)) // 16) % 16 for n in range(16 * j, 16 * j + 16)}
            assert len(banks) == 16
