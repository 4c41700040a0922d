"""The pointers every trace call rebuilds, round-tripped on the device (include/rt_diag.h
rt_selftest_tables). Round 4's first build of tables() (path_f64.h) rebuilt the compact-table pointer
from two readfirstlane halves and let the builtin's int result sign-extend the low word into the high
word: an illegal address whenever hipMalloc placed the table at a low word with bit 31 set, so the fault
came and went with the allocation (profiles/r04_ab.log). Here fabricated addresses with that bit set
(never dereferenced) pin the reconstruction deterministically, together with the kernarg views the
megakernels read their DevScene / RenderArgs through (megakernel_common.h: offsets 0 and 248). The
reference's trace call reads the scene's tables on every ray (scene.rs:272-289)."""
import pytest

PTRS = [
    0x00007FFF80001000,  # bit 31 of the low word set, non-zero high word (the faulting shape)
    0x0000000180000000,
    0x00007F00FFFFFF00,
    0x00007F0012345678,  # bit 31 clear
    0x0000000000001000,
    0xFFFFFFFF80000040,
]
M64 = (1 << 64) - 1


@pytest.mark.gpu
def test_table_pointer_round_trip_is_exact(rt, gpu_scenes):
    got = rt.selftest_tables(PTRS)
    for p, (k_tab, v_tab, sext, k_ctab, k_slot, k_tail) in zip(PTRS, got):
        assert k_tab == p, f"tables() via the kernarg view: {k_tab:#x} != {p:#x}"
        assert v_tab == p, f"tables() of the by-value argument: {v_tab:#x} != {p:#x}"
        assert k_ctab == p and k_slot == (p + 16) & M64 and k_tail == (p + 32) & M64, "kernarg offsets 0 / 248"


@pytest.mark.gpu
def test_round4_sign_extending_form_is_caught(rt, gpu_scenes):
    """The same check on the round-4 form (tables_form<true>, compiled only into this diagnostic): it
    must come out wrong for exactly the addresses whose low word has bit 31 set, so the round trip above
    would fail on a build that reintroduced it."""
    got = rt.selftest_tables(PTRS)
    for p, row in zip(PTRS, got):
        want = p | 0xFFFFFFFF00000000 if p & 0x80000000 else p
        assert row[2] == want, f"{p:#x}: {row[2]:#x}"
        assert (row[2] != p) == bool(p & 0x80000000) or p >> 32 == 0xFFFFFFFF
