"""The descriptor's owner-slot bin bytes (csrc/descriptor.hip, finish()).

A sample's 8 trilinear corners (dr, dc, do) land in interior bins
(Rm + dr, Cm + dc, O0 + do) of the reference's 6 x 6 x 10 histogram
(src/sift.cpp:654-672); corner k = dr*4 + dc*2 + do goes to owner slot
k ^ odd, odd = the parity bits of (Rm, Cm, O0).  The kernel builds the eight
bin bytes directly in slot order from two 6-entry byte tables looked up with
v_perm_b32 and an arithmetic O part; corners outside the interior rows /
columns carry +0.0, so their byte only has to name some interior bin.  These
tests restate v_perm_b32 and check that construction against the direct
formula for every base corner the kernel can see (Rm, Cm in [-1, 3],
O0 in [0, 7]), and the one-instruction histogram address.  No GPU needed.
"""

D = 4   # SIFT_DESCR_WIDTH
NB = 8  # SIFT_DESCR_HIST_BINS


def v_perm_b32(src0, src1, sel):
    """V_PERM_B32: byte i of the result = byte sel.byte[i] of {src0:src1}
    (selector 0-3 -> src1, 4-7 -> src0, 12 -> 0x00, 13-15 -> 0xff)."""
    b = [(src1 >> (8 * i)) & 0xFF for i in range(4)] + [(src0 >> (8 * i)) & 0xFF for i in range(4)]
    out = 0
    for i in range(4):
        s = (sel >> (8 * i)) & 0xFF
        if s < 8:
            v = b[s]
        elif s == 12:
            v = 0x00
        elif s >= 13:
            v = 0xFF
        else:  # 8-11: sign bits, unused here
            raise AssertionError("selector 8-11 not used by the kernel")
        out |= v << (8 * i)
    return out


def qidx(R, C, O):
    """Interior bin (R, C in [0, 4), O in [0, 10)) -> (parity slot, index within the class)."""
    return ((R & 1) << 2) | ((C & 1) << 1) | (O & 1), (R >> 1) * 10 + (C >> 1) * 5 + (O >> 1)


def kernel_slot_bytes(Rm, Cm, O0):
    x, y = (Rm + 1) & 0xFFFFFFFF, (Cm + 1) & 0xFFFFFFFF
    selR1 = v_perm_b32(0, x, 0)
    selR0 = (selR1 + 0x01010101) & 0xFFFFFFFF
    selC = (v_perm_b32(0, y, 0) + 0x00000101) & 0xFFFFFFFF
    po = O0 & 1
    o4 = (v_perm_b32(0, O0 >> 1, 0) + (po | (po << 16))) & 0xFFFFFFFF
    c4 = (v_perm_b32(0x00000505, 0x05000000, selC) + o4) & 0xFFFFFFFF
    w0 = (v_perm_b32(0x00000A0A, 0x0A000000, selR0) + c4) & 0xFFFFFFFF
    w1 = (v_perm_b32(0x00000A0A, 0x0A000000, selR1) + c4) & 0xFFFFFFFF
    return [(w0 >> (8 * i)) & 0xFF for i in range(4)] + [(w1 >> (8 * i)) & 0xFF for i in range(4)]


def test_slot_bytes_name_each_interior_corners_bin():
    seen = 0
    for Rm in range(-1, D):
        for Cm in range(-1, D):
            for O0 in range(NB):
                odd = ((Rm & 1) << 2) | ((Cm & 1) << 1) | (O0 & 1)
                got = kernel_slot_bytes(Rm, Cm, O0)
                for k in range(8):
                    dr, dc, do = k >> 2, (k >> 1) & 1, k & 1
                    R, C, O = Rm + dr, Cm + dc, O0 + do
                    s = k ^ odd
                    assert 0 <= got[s] < 20, (Rm, Cm, O0, s, got[s])  # always an interior bin row
                    if 0 <= R < D and 0 <= C < D:
                        owner, q = qidx(R, C, O)
                        assert owner == s  # the slot k ^ odd is the corner's parity class
                        assert got[s] == q, (Rm, Cm, O0, k, got[s], q)
                        seen += 1
    assert seen > 0


def test_histogram_address_is_one_perm():
    # byte address qidx * 256 + lane * 4: byte 0 <- lane * 4, byte 1 <- bin byte j of the word
    for lane in (0, 1, 17, 63):
        for word in (0x13020100, 0x00130a05, 0x0f0e0d0c):
            for j in range(4):
                sel = 0x0C0C0004 | (j << 8)
                q = (word >> (8 * j)) & 0xFF
                assert v_perm_b32(lane << 2, word, sel) == q * 256 + lane * 4
