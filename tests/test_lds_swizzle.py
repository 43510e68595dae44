"""Exhaustive check of the LDS XOR swizzles used by the conv kernels
(csrc/kernels/conv_glds.hip swz_r): every ds_read_b128 lane group of a
16x16x32 fragment read must touch 16 distinct 16-byte bank slots, and the
swizzle must be a permutation of each row's chunks (so the DMA source
permutation and the read permutation are the same involution)."""

# ds_read_b128 lane groups (MI355X_MICROARCH.md §LDS)
GROUPS = [
    list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
    list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
    list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
    list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64)),
]


def swz(row, cpr):
    if cpr == 8:
        return (row >> 1) & 7
    q = (row >> 2) & 3
    return (0x78 >> (2 * q)) & 3


def slot(row, chunk, cpr):
    addr = row * cpr * 16 + ((chunk ^ swz(row, cpr)) << 4)
    return (addr // 16) % 16          # 16-byte slot within the 256-byte bank row


def test_groups_cover_all_lanes():
    assert sorted(sum(GROUPS, [])) == list(range(64))


def test_fragment_reads_conflict_free():
    for cpr in (4, 8):                 # 64-byte and 128-byte rows
        for base in range(0, 256, 16):  # any 16-row fragment of the tile
            for kk in range(cpr // 4):  # 32-wide K substeps
                for g in GROUPS:
                    slots = [slot(base + (l & 15), (l >> 4) + 4 * kk, cpr) for l in g]
                    assert len(set(slots)) == 16, (cpr, base, kk, slots)


def test_swizzle_is_row_permutation():
    for cpr in (4, 8):
        for row in range(64):
            assert sorted(c ^ swz(row, cpr) for c in range(cpr)) == list(range(cpr))


def test_naive_xor_would_conflict():
    # the plain (row >> 2) & 3 XOR for 64-byte rows is NOT conflict free
    def bad(row, chunk):
        return ((row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4)) // 16) % 16

    g = GROUPS[0]
    assert len({bad(l & 15, l >> 4) for l in g}) < 16
