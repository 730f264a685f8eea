"""CPU emulation of K1t's LDS address math (csrc/kernels/conv_tile3x3.hip), for both instances (64 and 128 input
channels; 128 runs each tile as two 64-channel k-slices through the same patch layout): every 16-B chunk the patch and
weight-stage writes place is read back by exactly the MFMA lane and step that needs it, with no two chunks sharing an
LDS slot and every offset inside its region. The arithmetic below is the kernel's, line for line; a change to one
must change the other."""
import numpy as np
import pytest

P_W = 34
NCH, SLOT_B = 8, 128               # 64-channel pixel slots (16-B chunks)
TH = 8                             # TileCfg<*, 64>: 8 x 32 tiles; TileCfg<*, 128>: 4 x 32 (tests below take th)
P_SLOTS = (TH + 2) * P_W


def swz(row, c):  # the kernel's swz<8>
    return (c ^ (row & 6)) << 4


# ds_read_b128 lane groups (one LDS cycle each; MI355X_MICROARCH.md, LDS): NOT 16 contiguous lanes
B128_GROUPS = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
B128_GROUPS += [[lane + 32 for lane in g] for g in B128_GROUPS]


@pytest.mark.parametrize("cin,cout", [(64, 64), (128, 64), (64, 128), (128, 128), (256, 128)])
def test_patch_writes_and_fragment_reads_agree(cin, cout):
    TH = 8 if cout == 64 else 4
    P_SLOTS = (TH + 2) * P_W
    fpw, ks_n = TH // 2, cin // 64
    for ks in range(ks_n):  # each k-slice refills the same patch buffer from input channels 64 ks .. 64 ks + 63
        lds = np.full(P_SLOTS * SLOT_B // 16, -1, dtype=np.int64)  # per 16-B chunk: the (slot, c) it holds
        for e in range(P_SLOTS * NCH):  # store_patch
            slot, c = divmod(e, NCH)
            off = slot * SLOT_B + swz(slot, c)
            assert 0 <= off < P_SLOTS * SLOT_B and off % 16 == 0
            assert lds[off // 16] == -1, "two chunks in one LDS slot"
            lds[off // 16] = slot * NCH + c
        assert (lds >= 0).all()
        for wave in range(4):
            for lane in range(64):
                g4 = lane >> 4
                for f in range(fpw):
                    sbase = ((TH // 4) * wave + (f >> 1)) * P_W + 16 * (f & 1) + (lane & 15)
                    r, col = (TH // 4) * wave + (f >> 1), 16 * (f & 1) + (lane & 15)  # output pixel in the tile
                    assert r < TH and col < 32
                    for tap in range(9):
                        kh, kw = divmod(tap, 3)
                        for s in range(2):
                            wc = 4 * s + g4
                            slot = sbase + kh * P_W + kw
                            got_slot, got_c = divmod(int(lds[(slot * SLOT_B + swz(slot, wc)) // 16]), NCH)
                            # input pixel (r + kh - 1, col + kw - 1) of the tile = patch (r + kh, col + kw)
                            assert got_slot == (r + kh) * P_W + (col + kw)
                            # input channel 64 ks + 8 got_c = the MFMA B-operand k-block of this lane and step; the
                            # weight stage (tap, ks) holds the same columns (test below)
                            assert 64 * ks + 8 * got_c == 64 * ks + 32 * s + 8 * g4


@pytest.mark.parametrize("cin,cout", [(64, 64), (128, 64), (64, 128), (128, 128), (256, 128)])
def test_weight_stage_writes_and_reads_agree(cin, cout):
    kpad = 9 * cin
    for tap in range(9):
        for ks in range(cin // 64):
            lds = np.full(cout * 128 // 16, -1, dtype=np.int64)  # per 16-B chunk: the packed-weight element it holds
            for tid in range(256):  # load_w(tap, ks) + store_w: rows tid / 8 + 32 e (e < cout / 32), chunk tid % 8
                n, c = tid >> 3, tid & 7
                col = tap * cin + ks * 64 + 8 * c
                assert col + 8 <= kpad
                for row in range(n, cout, 32):
                    off = row * 128 + swz(row, c)
                    assert lds[off // 16] == -1
                    lds[off // 16] = row * kpad + col
            assert (lds >= 0).all()
            for lane in range(64):
                for j in range(cout // 16):
                    for s in range(2):
                        n = 16 * j + (lane & 15)
                        wc = 4 * s + (lane >> 4)
                        got = int(lds[(n * 128 + swz(n, wc)) // 16])
                        # output channel n, input channels 64 ks + 8 wc .. + 7 of tap `tap` (K = (kh, kw, c))
                        assert got == n * kpad + tap * cin + 64 * ks + 8 * wc


@pytest.mark.parametrize("TH", [8, 4])
def test_fragment_reads_are_bank_conflict_free(TH):
    """Every ds_read_b128 lane group of a fragment read (lane l: pixel l % 16 at chunk 4 s + l / 16) hits 16 distinct
    16-B bank groups ((a / 4) % 64 over 4 banks each), for every tap offset of the window."""
    for wave in range(4):
        for f in range(TH // 2):
            for tap in range(9):
                kh, kw = divmod(tap, 3)
                for s in range(2):
                    for g in B128_GROUPS:
                        banks = set()
                        for lane in g:
                            slot = ((TH // 4) * wave + (f >> 1)) * P_W + 16 * (f & 1) + (lane & 15) + kh * P_W + kw
                            off = slot * SLOT_B + swz(slot, 4 * s + (lane >> 4))
                            banks.add((off // 16) % 16)
                        assert len(banks) == 16


def test_weight_reads_are_bank_conflict_free():
    for j in range(8):
        for s in range(2):
            for g in B128_GROUPS:
                banks = set()
                for lane in g:
                    n = 16 * j + (lane & 15)
                    banks.add(((n * 128 + swz(n, 4 * s + (lane >> 4))) // 16) % 16)
                assert len(banks) == 16


def test_old_key_conflicts_with_the_real_lane_groups():
    """The previous key, (row >> 1) & 7, is conflict-free for contiguous 16-lane groups but not for the real ones
    (the 16-18 % SQ_LDS_BANK_CONFLICT of profiles/r4h_unet/pmc_by_kernel.txt)."""
    old = lambda row, c: (c ^ ((row >> 1) & 7)) << 4  # noqa: E731
    extra = 0
    for start in range(16):
        for s in range(2):
            for g in B128_GROUPS:
                banks = [((start + (lane & 15)) * SLOT_B + old(start + (lane & 15), 4 * s + (lane >> 4))) // 16 % 16
                         for lane in g]
                extra += 16 - len(set(banks))
    assert extra > 0


def test_patch_and_weight_stores_are_bank_conflict_free():
    """ds_write_b128: 8 groups of 8 contiguous lanes, bank (a / 4) % 32; 8 lanes write one row's 8 chunks."""
    for row0 in range(0, 128, 1):
        offs = [(row0 * 128 + swz(row0, c)) // 16 % 8 for c in range(8)]
        assert sorted(offs) == list(range(8))


@pytest.mark.parametrize("H,W", [(8, 32), (16, 64), (64, 96), (512, 512)])
def test_ups_coarse_block_covers_every_fine_pixel(H, W):
    """K1t UPS (the 128 -> 64 instance's second k-slice = bilinear 2x upsample of a coarse [H/2, W/2] tensor): the
    coarse block of a tile (CR x CC slots from (h0/2 - 1, w0/2 - 1), loads clamped into the tensor) holds every
    source pixel of the upsample formula (upsample2x_kernel) for every in-image fine pixel of the tile's patch."""
    th, tw, pw = 8, 32, 34
    cr_n, cc_n = th // 2 + 2, tw // 2 + 3
    hc, wc = H // 2, W // 2
    for h0 in range(0, H, th):
        for w0 in range(0, W, tw):
            cy0, cx0 = h0 // 2 - 1, w0 // 2 - 1
            # what each coarse slot holds (the kernel's clamped load)
            held = {(r, c): (min(max(cy0 + r, 0), hc - 1), min(max(cx0 + c, 0), wc - 1))
                    for r in range(cr_n) for c in range(cc_n)}
            for pr in range(th + 2):
                for pc in range(pw):
                    ih, iw = h0 - 1 + pr, w0 - 1 + pc
                    if not (0 <= ih < H and 0 <= iw < W):
                        continue
                    sy, sx = max((ih + 0.5) * 0.5 - 0.5, 0.0), max((iw + 0.5) * 0.5 - 0.5, 0.0)
                    y0, x0 = int(sy), int(sx)
                    y1, x1 = min(y0 + 1, hc - 1), min(x0 + 1, wc - 1)
                    for yy in (y0, y1):
                        for xx in (x0, x1):
                            r, c = yy - cy0, xx - cx0
                            assert 0 <= r < cr_n and 0 <= c < cc_n, (h0, w0, ih, iw, r, c)
                            assert held[(r, c)] == (yy, xx)


@pytest.mark.parametrize("cin,cout", [(64, 64), (128, 64), (64, 128), (256, 128)])
def test_weight_stage_lds_dma_matches_the_reads(cin, cout):
    """WDMA (weights by global_load_lds_dwordx4, 16 B per lane at base + 16 lane): wave w's instruction i fills rows
    (NWV w + i) * 8 .. + 7 with the per-lane SOURCE chunk (lane % 8) ^ (row & 6). Every LDS chunk is written once and
    holds what the MFMA fragment read of swz<8> expects."""
    nwv, kpad = cout // 32, 9 * cin
    for tap in (0, 4, 8):
        for ks in range(cin // 64):
            lds = {}
            for wave in range(4):
                for i in range(nwv):
                    base = (nwv * wave + i) * 1024
                    for lane in range(64):
                        r = (nwv * wave + i) * 8 + (lane >> 3)
                        c = (lane & 7) ^ (r & 6)
                        col = tap * cin + ks * 64 + 8 * c
                        assert r < cout and col + 8 <= kpad
                        off = base + 16 * lane
                        assert off not in lds
                        lds[off] = r * kpad + col
            assert len(lds) == cout * 8
            for lane in range(64):
                for j in range(cout // 16):
                    for s in range(2):
                        n = 16 * j + (lane & 15)
                        wc = 4 * s + (lane >> 4)
                        assert lds[n * 128 + swz(n, wc)] == n * kpad + tap * cin + 64 * ks + 8 * wc
