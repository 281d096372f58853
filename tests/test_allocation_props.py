"""Property tests (hypothesis) of the preferred-allocation policy in libmxnode
(native/libmxnode/alloc.cc), the core of the device plugin's
GetPreferredAllocation ("no double allocation, NUMA
preference, all ids valid")."""
import pytest
from hypothesis import given, settings, strategies as st

from mxk8s.native import node


@st.composite
def topo_request(draw):
    n = draw(st.integers(1, 8))
    numa = draw(st.lists(st.integers(0, 1), min_size=n, max_size=n))
    hive = [draw(st.sampled_from([0, 0xA1, 0xB2]))] * n if draw(st.booleans()) else \
        draw(st.lists(st.sampled_from([0xA1, 0xB2]), min_size=n, max_size=n))
    full_mesh = draw(st.booleans())
    adj = [[int(i != j and (full_mesh or hive[i] == hive[j])) for j in range(n)] for i in range(n)]
    available = sorted(draw(st.sets(st.integers(0, n - 1), min_size=1)))
    size = draw(st.integers(1, len(available)))
    must = sorted(draw(st.sets(st.sampled_from(available), max_size=size)))
    return numa, hive, adj, available, must, size


@settings(max_examples=300, deadline=None)
@given(topo_request())
def test_allocation_invariants(req):
    numa, hive, adj, available, must, size = req
    out = node.preferred_allocation_topo(numa, hive, adj, available, must, size)
    assert len(out) == size
    assert len(set(out)) == size                       # no device handed out twice
    assert set(out) <= set(available)                  # only available ids
    assert set(must) <= set(out)                       # kubelet's must-include honoured
    assert out == sorted(out)
    assert out == node.preferred_allocation_topo(numa, hive, adj, available, must, size)  # deterministic


@settings(max_examples=200, deadline=None)
@given(topo_request())
def test_allocation_prefers_one_hive_then_one_numa_node(req):
    numa, hive, adj, available, must, size = req
    out = node.preferred_allocation_topo(numa, hive, adj, available, must, size)
    hives_must = {hive[i] for i in must}
    fits_one_hive = any(
        {hive[i] for i in must} <= {h} and sum(1 for i in available if hive[i] == h) >= size
        for h in set(hive[i] for i in available))
    if fits_one_hive and len(hives_must) <= 1:
        assert len({hive[i] for i in out}) == 1
        h = hive[out[0]]
        # among devices of that hive, a single NUMA node wins when it can hold the request
        cand = [i for i in available if hive[i] == h]
        for z in (0, 1):
            pool = [i for i in cand if numa[i] == z]
            if len(pool) >= size and all(numa[i] == z for i in must) and all(hive[i] == h for i in must):
                assert len({numa[i] for i in out}) == 1
                break


@pytest.mark.parametrize("available,must,size", [
    ([0, 1], [], 3),           # more than available
    ([0, 1], [2], 1),          # must-include not available
    ([0, 1, 2], [0, 1], 1),    # must-include larger than size
])
def test_allocation_rejects_invalid(available, must, size):
    numa = [0] * 4
    hive = [0] * 4
    adj = [[int(i != j) for j in range(4)] for i in range(4)]
    with pytest.raises(ValueError):
        node.preferred_allocation_topo(numa, hive, adj, available, must, size)
