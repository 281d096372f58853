"""The GEMM round / split-tail planner under CUs taken by collectives
(VERDICT r3 #4): the Python mirror and the C planner agree, and telling the
planner about k reserved CUs never plans more rounds than ignoring them.

Runs on the CPU: ``mxk_gemm_split_plan`` is host arithmetic in the kernel
library (loaded, never launched)."""
import ctypes
import itertools

import pytest

from mxk8s.ops import _lib, gemm

pytestmark = pytest.mark.skipif(not _lib.kernels_available(), reason="kernel library not built")

# Llama-3-8B step GEMMs at 16k tokens: output tiles (M/256 * N/256) and K
STEP = {
    "wqkv fwd": (64 * 24, 4096), "wo fwd": (64 * 16, 4096), "w13 fwd": (64 * 112, 4096),
    "w2 fwd": (64 * 16, 14336), "lm_head fwd": (64 * 501, 4096),
    "w2 dgrad": (64 * 56, 4096), "wqkv wgrad": (24 * 16, 16384), "w2 wgrad": (16 * 56, 16384),
}


@pytest.mark.parametrize("nwg,K,cus", list(itertools.product(
    [1, 64, 255, 256, 257, 384, 448, 1024, 1536, 3584, 7168, 32064],
    [512, 1024, 4096, 14336, 16384], [256, 240, 224, 192, 128])))
def test_c_and_python_plans_agree(nwg, K, cus):
    q = ctypes.c_long(0)
    tail = _lib.lib().mxk_gemm_split_plan(nwg, K, cus, ctypes.byref(q))
    assert (q.value, tail) == gemm.split_plan(nwg, K, cus)


@pytest.mark.parametrize("k", [16, 32, 64])
@pytest.mark.parametrize("name", sorted(STEP))
def test_reserved_cus_never_plans_more_rounds(name, k):
    """Planning for 256 - k CUs (what is free beside RCCL) against planning
    for 256 while only 256 - k are free: the first is never worse, and the
    planned rounds stay within one half-round of the ideal nwg / (256 - k)."""
    nwg, K = STEP[name]
    free = 256 - k

    def actual(plan_cus):
        whole, tail = gemm.split_plan(nwg, K, plan_cus)
        # what runs: `whole` tiles then 2 * tail half-depth workgroups, all
        # on `free` CUs
        r = -(-whole // free)
        if tail:
            r += 0.5 * -(-2 * tail // free)
        return r

    aware, blind = actual(free), actual(256)
    assert aware <= blind, (aware, blind)
    assert aware <= nwg / free + 0.5 + 1e-9, (aware, nwg / free)


def test_set_reserved_cus_roundtrip():
    L = _lib.lib()
    try:
        gemm.set_reserved_cus(32)
        assert L.mxk_gemm_reserved_cus() == 32
        gemm.set_reserved_cus(-5)
        assert L.mxk_gemm_reserved_cus() == 0
    finally:
        gemm.set_reserved_cus(0)


# ---- staggered rounds (schedule 54) ----------------------------------------
def _simulate(T, sx, cus, dur):
    """Greedy in-order dispatch per XCD (workgroup b on XCD b % 8, the next
    one to the first free CU): finish time of the grid, and the times at
    which tiles end (C stores)."""
    import heapq
    cx = cus // 8
    free = [[0.0] * cx for _ in range(8)]
    for q in free:
        heapq.heapify(q)
    end, stores = 0.0, []
    for b in range(T + 8 * sx):
        _, part, _ = gemm.stagger_part(b, T, sx)
        t0 = heapq.heappop(free[b & 7])
        t1 = t0 + (dur if part == 0 else dur / 2)
        heapq.heappush(free[b & 7], t1)
        end = max(end, t1)
        if part != 1:
            stores.append(t1)
    return end, stores


@pytest.mark.parametrize("T,K", [(1024, 8192), (4096, 16384), (64 * 112, 4096), (64 * 56, 4096),
                                 (64 * 24, 4096), (64 * 16, 4096), (256, 8192), (1000, 4096)])
@pytest.mark.parametrize("cus", [256, 240, 192])
def test_stagger_plan_and_parts(T, K, cus):
    sx = gemm.stagger_plan(T, K, cus)
    assert sx == _lib.lib().mxk_gemm_stagger_plan(T, K, cus)
    if T % 8 or T // 8 < 2 * (cus // 8):
        assert sx == 0
        return
    assert sx == cus // 16
    out = (ctypes.c_int * 3)()
    whole, first, second = {}, {}, {}
    for b in range(T + 8 * sx):
        p = gemm.stagger_part(b, T, sx)
        _lib.lib().mxk_gemm_stagger_part(b, T, sx, out)
        assert tuple(out) == p
        v, part, slot = p
        assert v % 8 == b % 8                      # the tile map keeps the XCD
        {0: whole, 1: first, 2: second}[part].setdefault(v, []).append((b, slot))
    # every tile exactly once: whole, or a first and a second half
    assert set(whole) | set(first) == set(range(T))
    assert not set(whole) & set(first) and set(first) == set(second)
    assert all(len(v) == 1 for d in (whole, first, second) for v in d.values())
    slots = sorted(first[v][0][1] for v in first)
    assert slots == list(range(8 * sx))
    for v in first:
        (bp, sp), (bc, sc) = first[v][0], second[v][0]
        assert sp == sc and bp < bc and bp % 8 == bc % 8   # producer dispatched first, same XCD
    # whole rounds stay whole (ideal makespan) and the stores no longer
    # coincide: half of them fall half a tile out of phase
    cx = cus // 8
    if (T // 8) % cx == 0:
        end, stores = _simulate(T, sx, cus, 1.0)
        assert end == pytest.approx(T / 8 / cx)
        frac = [t % 1.0 for t in stores]
        assert sum(abs(f - 0.5) < 1e-9 for f in frac) >= len(stores) // 2 - 8 * sx


def test_set_exclusive_roundtrip():
    try:
        gemm.set_exclusive(True)
        assert gemm.exclusive()
        gemm.set_exclusive(False)
        assert not gemm.exclusive()
    finally:
        gemm.set_exclusive(False)


@pytest.mark.parametrize("T,cus", [(1024, 256), (4096, 256), (64 * 56, 256), (1024, 192)])
def test_stagger_by_xcd_parts(T, cus):
    """Schedule 57: every tile once (whole, or two halves on one XCD of 4-7,
    producer dispatched first); XCDs 0-3 and 4-7 finish together and store
    half a tile apart."""
    cx = cus // 8
    out = (ctypes.c_int * 3)()
    seen = {}
    for b in range(T + 8 * cx):
        p = gemm.stagger_part_xcd(b, T, cx)
        _lib.lib().mxk_gemm_stagger_part_xcd(b, T, cx, out)
        assert tuple(out) == p
        v, part, slot = p
        if part < 0:
            assert b & 7 < 4
            continue
        assert v % 8 == b % 8
        seen.setdefault(v, []).append((part, b, slot))
    assert set(seen) == set(range(T))
    for v, ps in seen.items():
        kinds = sorted(p for p, _, _ in ps)
        assert kinds in ([0], [1, 2])
        if kinds == [1, 2]:
            (p1, b1, s1), (p2, b2, s2) = sorted(ps)
            assert v % 8 >= 4 and s1 == s2 and b1 < b2 and b1 % 8 == b2 % 8
    # dispatch simulation (unit tile time): both XCD groups end at T / 8 / cx,
    # and group 4-7 stores half a tile out of phase with group 0-3
    import heapq
    free = [[0.0] * cx for _ in range(8)]
    ends = {0: [], 1: []}
    for b in range(T + 8 * cx):
        v, part, _ = gemm.stagger_part_xcd(b, T, cx)
        if part < 0:
            continue
        q = free[b & 7]
        t0 = heapq.heappop(q)
        t1 = t0 + (1.0 if part == 0 else 0.5)
        heapq.heappush(q, t1)
        if part != 1:
            ends[(b & 7) >= 4].append(t1)
    if (T // 8) % cx == 0:
        assert max(ends[0]) == pytest.approx(T / 8 / cx) == max(ends[1])
        assert all(abs(t % 1.0) < 1e-9 for t in ends[0])
        assert sum(abs(t % 1.0 - 0.5) < 1e-9 for t in ends[1]) >= len(ends[1]) - 2 * 4 * cx
