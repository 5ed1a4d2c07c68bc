"""CPU: the LDS images of the score kernels are bank-conflict-free for their MFMA fragment
reads (ds_read_b128), using the CDNA4 lane grouping of MI355X_MICROARCH.md §LDS:
a wave64 ds_read_b128 is serviced in 4 groups of 16 lanes, one LDS cycle per group when its
16 lanes touch 16 distinct 16-byte bank quads (bank = (addr / 4) mod 64)."""
import pytest

B128_GROUPS = [
    list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
    list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
    list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
    list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64)),
]


def conflict_cycles(addrs):
    """LDS cycles of one ds_read_b128 wave-instruction (4 = conflict-free)."""
    cyc = 0
    for grp in B128_GROUPS:
        per_quad = {}
        for l in grp:
            a = addrs[l]
            q = (a // 16) % 16          # 16-byte quad among the 64 banks
            per_quad.setdefault(q, set()).add(a)
        cyc += max(len(v) for v in per_quad.values())
    return cyc


def v3_slot(chunk, row):
    f = (0x1320 >> (((row >> 2) & 3) * 4)) & 3
    return chunk ^ f


def test_b128_groups_partition_the_wave():
    assert sorted(sum(B128_GROUPS, [])) == list(range(64))


@pytest.mark.parametrize("base_row", [0, 16, 112, 208, 240])
def test_v3_64byte_rows_conflict_free(base_row):
    # fragment read of MFMA 16x16x32: lane l -> row base + (l & 15), chunk l >> 4 (16 B each)
    addrs = [(base_row + (l & 15)) * 64 + v3_slot(l >> 4, l & 15) * 16 for l in range(64)]
    assert conflict_cycles(addrs) == 4


def test_v3_unswizzled_would_conflict():
    addrs = [((l & 15)) * 64 + (l >> 4) * 16 for l in range(64)]
    assert conflict_cycles(addrs) > 4


def test_v3_dma_lane_map_is_the_inverse_of_the_read_map():
    # DMA piece: lane L writes LDS bytes [16L, 16L+16) = row L >> 2, slot L & 3, and fetches
    # source chunk (L & 3) ^ f((L >> 4) & 3); the fragment read of (row, chunk) must find it.
    for L in range(64):
        row, slot = L >> 2, L & 3
        chunk = slot ^ ((0x1320 >> (((L >> 4) & 3) * 4)) & 3)
        assert v3_slot(chunk, row) == slot


@pytest.mark.parametrize("kk", [0, 1])
def test_v1_v2_128byte_rows_conflict_free(kk):
    # 128-B rows, slot = chunk ^ (row & 7); kk selects k-half (chunks 0-3 or 4-7)
    addrs = []
    for l in range(64):
        r, c = l & 15, (l >> 4) + 4 * kk
        addrs.append(r * 128 + ((c ^ (r & 7)) << 4))
    assert conflict_cycles(addrs) == 4
