"""CPU-side plan of the node agent's multi-GPU probe (which xGMI links get read)."""

from odh_kubeflow_amd.ops.gpu import ring_pairs


def test_ring_pairs():
    assert ring_pairs([3]) == []
    assert ring_pairs([2, 2]) == []  # duplicates collapse
    assert ring_pairs([0, 1]) == [(1, 0), (0, 1)]  # both directions of the one link
    assert ring_pairs([0, 1, 2, 3]) == [(1, 0), (2, 1), (3, 2), (0, 3)]
    pairs = ring_pairs(list(range(8)))
    assert len(pairs) == 8 and {s for _, s in pairs} == set(range(8)) and {r for r, _ in pairs} == set(range(8))
    assert all(r != s for r, s in pairs)
