"""The benchmark's D-Cliques generator restatement (niidmix.generate) reproduces the topologies the
reference generators produced (golden fixtures): same cliques, same edge lists in the same order,
same MH weights bit for bit."""
import numpy as np
import pytest

from conftest import load_golden
from niidmix import generate


@pytest.mark.parametrize("name,n,size,inter", [
    ("dcliques1000_fc_p64", 1000, 100, "fully-connected"),
    ("dcliques1000_smallworld_p16", 1000, 100, "smallworld"),
    ("dcliques1000_ring_p16", 1000, 100, "ring"),
    ("dcliques300_fc_p37", 300, 30, "fully-connected"),
    ("dcliques200_fractal_rm5_p40", 200, 20, "fractal"),
])
def test_matches_reference_generator(name, n, size, inter):
    g = load_golden(name)
    csr, cliques = generate.dcliques_csr(n, size, inter, seed=1337,
                                         remove=5 if "_rm5" in name else 0)
    assert cliques == g["cliques"]
    np.testing.assert_array_equal(csr.row_ptr, g["row_ptr"])
    np.testing.assert_array_equal(csr.col, g["col"])
    assert np.array_equal(csr.val.view(np.uint32), g["val"].view(np.uint32))


def test_random_graph_matches_reference():
    """random_graph.create + compute_weights (random_graph.py:10-51), restated sparse: the same edge
    lists and MH weights, bit for bit, as the reference-run fixture (topology-seed 1, 5
    neighbours)."""
    g = load_golden("randomgraph50_p24")
    csr, edges = generate.random_graph_csr(50, 5, 1)
    np.testing.assert_array_equal(csr.row_ptr, g["row_ptr"])
    np.testing.assert_array_equal(csr.col, g["col"])
    assert np.array_equal(csr.val.view(np.uint32), g["val"].view(np.uint32))


def _digest_cases():
    import json
    import os
    from conftest import GOLDEN
    path = os.path.join(GOLDEN, "dcliques_digests.json")
    with open(path) as f:
        return sorted(json.load(f)["cases"].items())


@pytest.mark.parametrize("name,want", _digest_cases())
def test_configs4_topology_matches_reference_digest(name, want):
    """BASELINE configs[4] at full size: niidmix.generate.dcliques_csr builds, at 10 000 nodes (and
    the weak N=8 line's 8 000, and 10 000 under smallworld), the same cliques, the same edge lists
    in the same order and the same fp32 MH weights as the REFERENCE generator
    (random_cliques.py:18-37, interclique.py:57-75 / :81-119, weights.py:3-32), compared through
    SHA-256 digests the reference run left (tests/golden/make_digests.py)."""
    import sys
    import os
    from conftest import GOLDEN
    sys.path.insert(0, GOLDEN)
    from topo_digest import digest
    csr, cliques = generate.dcliques_csr(want["n"], want["clique_size"], want["interclique"],
                                         seed=want["seed"])
    got = digest(cliques, csr.edges(), csr.row_ptr, csr.val)
    for key in ("n", "nnz", "cliques", "edges", "row_ptr", "val"):
        assert got[key] == want[key], (name, key)
