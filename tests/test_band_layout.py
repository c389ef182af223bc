"""Host logic of the band kernel (CPU): a ring's cycle order (ops.band_layout) and the band check
(ops.band_of) on the reference's ring topologies and on graphs that are not rings."""
import numpy as np

from conftest import load_golden
from niidmix import ops
from niidmix.topology import MixCSR, mh_csr


def _csr(name):
    g = load_golden(name)
    return MixCSR(g["row_ptr"], g["col"], g["val"]).validate()


def test_ring_cycle_order_is_banded():
    for name in ("ring100_p257", "nonfinite_ring8_p16"):
        csr = _csr(name)
        assert ops.band_of(csr, 3) is None or csr.n <= 3      # rank order: not banded
        perm = ops.band_layout(csr)
        assert perm is not None and sorted(perm.tolist()) == list(range(csr.n))
        rel = csr.relabel(perm)
        assert ops.band_of(rel, 3) == 1
        # relabel keeps every row's operand order and weights (stored at the permuted row)
        for i in range(csr.n):
            a, b = csr.row_ptr[i], csr.row_ptr[i + 1]
            c, d = rel.row_ptr[perm[i]], rel.row_ptr[perm[i] + 1]
            assert list(perm[csr.col[a:b]]) == list(rel.col[c:d])
            assert np.array_equal(csr.val[a:b].view(np.uint32), rel.val[c:d].view(np.uint32))


def test_not_a_ring():
    for name in ("grid49_p20", "expander64_p48", "dcliques300_fc_p37", "n2_ring_linear7850"):
        assert ops.band_layout(_csr(name)) is None, name
    # two disjoint triangles: every node has two neighbours but there are two cycles
    edges = {0: [1, 2], 1: [2, 0], 2: [0, 1], 3: [4, 5], 4: [5, 3], 5: [3, 4]}
    assert ops.band_layout(mh_csr(6, edges)) is None


def test_band_of_lattice_and_wrap():
    n = 11
    edges = {i: [(i + 2) % n, (i - 1) % n, (i + 1) % n, (i - 2) % n] for i in range(n)}
    csr = mh_csr(n, edges)
    assert ops.band_of(csr, 5) == 2 and ops.band_of(csr, 3) is None
    ring = mh_csr(3, {0: [1, 2], 1: [2, 0], 2: [0, 1]})
    assert ops.band_of(ring, 3) == 1
