"""Topology boundary (host logic, CPU): topology.json reader, CSR in the reference's operand order,
Metropolis-Hastings builder, sparse companion format."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden_cases, load_golden
from niidmix import topology as T

JSON_CASES = sorted(f[:-len(".topology.json")] for f in os.listdir(GOLDEN) if f.endswith(".topology.json"))


@pytest.mark.parametrize("name", JSON_CASES)
def test_reader_and_csr_match_reference_loader(name):
    """load_file mirrors setup.topology.load; to_csr reproduces the operand order and weights the
    reference's d_sgd.average used when the golden vectors were produced."""
    topo = T.load_file(os.path.join(GOLDEN, name + ".topology.json"))
    assert topo["weights"].dtype == torch.float32
    assert all(isinstance(k, int) for k in topo["edges"])
    csr = T.to_csr(topo)
    g = load_golden(name)
    np.testing.assert_array_equal(csr.row_ptr, g["row_ptr"])
    np.testing.assert_array_equal(csr.col, g["col"])
    assert np.array_equal(csr.val.view(np.uint32), g["val"].view(np.uint32))


@pytest.mark.parametrize("name", golden_cases())
def test_mh_builder_bitwise(name):
    """mh_csr (sparse, no dense JSON) == compute_weights' fp32 values bit for bit, incl. the
    diagonal 1 - sum(row) reduction (weights.py:15-25)."""
    g = load_golden(name)
    n = len(g["row_ptr"]) - 1
    edges = {i: g["col"][g["row_ptr"][i] + 1:g["row_ptr"][i + 1]].tolist() for i in range(n)}
    csr = T.mh_csr(n, edges)
    np.testing.assert_array_equal(csr.col, g["col"])
    assert np.array_equal(csr.val.view(np.uint32), g["val"].view(np.uint32)), name


def test_dense_mh_matches_sparse():
    g = load_golden("dcliques300_fc_p37")
    n = len(g["row_ptr"]) - 1
    edges = {i: g["col"][g["row_ptr"][i] + 1:g["row_ptr"][i + 1]].tolist() for i in range(n)}
    W = T.metropolis_hastings(n, edges)
    csr = T.to_csr({"edges": edges, "weights": W})
    assert np.array_equal(csr.val.view(np.uint32), g["val"].view(np.uint32))


def test_sparse_companion_roundtrip(tmp_path):
    g = load_golden("dcliques200_fractal_rm5_p40")
    csr = T.MixCSR(g["row_ptr"], g["col"], g["val"]).validate()
    T.save_csr(str(tmp_path / "topology.csr.npz"), csr, g["cliques"])
    topo = T.load(str(tmp_path))
    back = T.to_csr(topo)
    np.testing.assert_array_equal(back.col, csr.col)
    np.testing.assert_array_equal(back.val, csr.val)
    assert topo["cliques"] == g["cliques"]
    assert topo["edges"][0] == csr.edges()[0]


def test_validation_errors():
    with pytest.raises(ValueError, match="self"):
        T.MixCSR(np.array([0, 2]), np.array([1, 0], np.int32), np.ones(2, np.float32)).validate()
    with pytest.raises(KeyError):
        T.to_csr({"edges": {0: [1]}, "weights": torch.eye(2)})


def test_load_missing(tmp_path):
    with pytest.raises(FileNotFoundError):
        T.load(str(tmp_path))


def _rundir(tmp_path, n, seed, classes=10):
    import json
    (tmp_path / "nodes.json").write_text(json.dumps([{"rank": r} for r in range(n)]))
    (tmp_path / "params.json").write_text(json.dumps({"meta": {"seed": seed, "log": "WARNING"},
                                                      "dataset": {"nb-classes": classes}}))
    return str(tmp_path)


def test_sparse_topology_cli_dcliques(tmp_path):
    """python -m niidmix.sparse_topology d-cliques writes topology.csr.npz holding exactly the
    reference generator's topology (cliques, edge order, MH weights bit for bit) and the same
    params.json 'topology' section as random_cliques.py; niidmix.topology.load reads it back."""
    import json
    from niidmix import sparse_topology, topology
    rd = _rundir(tmp_path, 300, 1337)
    sparse_topology.main(["d-cliques", "--rundir", rd, "--max-clique-size", "30"])
    t = topology.load(rd)
    g = load_golden("dcliques300_fc_p37")
    csr = topology.to_csr(t)
    np.testing.assert_array_equal(csr.row_ptr, g["row_ptr"])
    np.testing.assert_array_equal(csr.col, g["col"])
    assert np.array_equal(csr.val.view(np.uint32), g["val"].view(np.uint32))
    assert t["cliques"] == g["cliques"]
    sec = json.loads((tmp_path / "params.json").read_text())["topology"]
    assert sec == {"name": "d-cliques/random-cliques", "weights": "metropolis-hasting",
                   "interclique-topology": "fully-connected", "max-clique-size": 30,
                   "remove-clique-edges": 0}


def test_sparse_topology_cli_random_graph(tmp_path):
    from niidmix import sparse_topology, topology
    rd = _rundir(tmp_path, 50, 1)
    sparse_topology.main(["random-graph", "--rundir", rd, "--nb-neighbours", "5"])
    csr = topology.to_csr(topology.load(rd))
    g = load_golden("randomgraph50_p24")
    np.testing.assert_array_equal(csr.col, g["col"])
    assert np.array_equal(csr.val.view(np.uint32), g["val"].view(np.uint32))


def test_randomized_topology_sparse_and_dense_files(tmp_path, monkeypatch):
    """--randomize's per-round graph (d_sgd.py:223-234) built sparse: topology.csr.npz every round,
    the reference's dense topology.json too below NIIDMIX_DENSE_JSON_MAX nodes; both load to the
    same CSR, and the loader takes the newer file."""
    import os
    import time
    from niidmix import d_sgd, generate, topology
    rd = str(tmp_path)
    nodes = [{"rank": r} for r in range(60)]
    params = {"topology": {"name": "random-graph", "nb-neighbours": 6, "topology-seed": 8,
                           "weights": "metropolis-hasting", "randomize": True}}
    t = d_sgd.randomized_topology(nodes, params, rd)
    ref, _ = generate.random_graph_csr(60, 6, 8)
    assert np.array_equal(topology.to_csr(t).val, ref.val)
    # the weights the reference's randomized round leaves in state['topology'] (d_sgd.py:233)
    assert isinstance(t["weights"], torch.Tensor) and t["weights"].shape == (60, 60)
    dense = topology.to_csr(topology.load_file(os.path.join(rd, "topology.json")))
    np.testing.assert_array_equal(dense.col, ref.col)
    assert np.array_equal(dense.val.view(np.uint32), ref.val.view(np.uint32))
    monkeypatch.setattr(d_sgd, "DENSE_JSON_MAX", 10)
    time.sleep(0.01)
    params["topology"]["topology-seed"] = 9
    t9 = d_sgd.randomized_topology(nodes, params, rd)       # above the cap: a SPARSE topology.json
    assert t9["weights"].numel() == 0
    want = generate.random_graph_csr(60, 6, 9)[0]
    for loaded in (topology.load(rd), topology.load_file(os.path.join(rd, "topology.json"))):
        got = topology.to_csr(loaded)                        # the JSON never lags the graph
        np.testing.assert_array_equal(got.col, want.col)
        assert np.array_equal(got.val.view(np.uint32), want.val.view(np.uint32))


def test_sparse_rundir_reads_with_reference_loader(tmp_path):
    """niidmix.sparse_topology writes a topology.json the reference's own loader reads unchanged
    (run.py:92-93 -> setup.topology.load, topology/__init__.py:4-12): the committed fixture is what
    that loader returned for this very file (tests/golden/make_sparse_load.py).  The restated
    loader (load_file) returns the same, and the plugin's to_csr turns it into the reference's
    dense-W operator bit for bit (MH weights rebuilt from the edges, or the companion CSR)."""
    import json
    from niidmix import sparse_topology, topology
    rd = _rundir(tmp_path, 300, 1337)
    sparse_topology.main(["d-cliques", "--rundir", rd, "--max-clique-size", "30"])
    text = (tmp_path / "topology.json").read_text()
    assert json.loads(text) == json.loads(open(os.path.join(GOLDEN, "sparse_dcliques300.written.json")).read())
    ref = json.loads(open(os.path.join(GOLDEN, "sparse_dcliques300.refload.json")).read())
    t = topology.load_file(str(tmp_path / "topology.json"))
    w = t["weights"]
    assert [type(w).__name__, str(w.dtype), list(w.shape)] == \
        [ref["weights_type"], ref["weights_dtype"], ref["weights_shape"]]
    assert {str(k): v for k, v in t["edges"].items()} == ref["edges"]
    assert all(isinstance(k, int) for k in t["edges"]) and ref["edge_key_types"] == ["int"]
    assert t["cliques"] == ref["cliques"] and sorted(t) == ref["keys"]
    g = load_golden("dcliques300_fc_p37")                   # the reference's dense-W round
    for topo in (t, topology.load(rd)):
        csr = topology.to_csr(topo)
        np.testing.assert_array_equal(csr.row_ptr, g["row_ptr"])
        np.testing.assert_array_equal(csr.col, g["col"])
        assert np.array_equal(csr.val.view(np.uint32), g["val"].view(np.uint32))
    assert "csr" in topology.load(rd) and "csr" not in t


def test_sparse_weights_errors():
    with pytest.raises(ValueError, match="weights-kind"):
        T.to_csr({"edges": {0: [1], 1: [0]}, "weights": torch.tensor([])})
    with pytest.raises(ValueError, match="every rank"):
        T.to_csr({"edges": {0: [2], 2: [0]}, "weights": [], "weights-kind": T.SPARSE_KIND})
    assert T.to_csr({"edges": {}, "weights": torch.tensor([])}).n == 0


def test_stale_companion_csr_is_ignored(tmp_path):
    """A sparse topology.json whose companion CSR has the same N but other edges (an interrupted
    write_sparse / --randomize writes the CSR first) does not get the CSR attached: to_csr then
    rebuilds the MH weights from the edges it does list."""
    from niidmix import generate
    csr_a, edges_a = generate.random_graph_csr(60, 4, 11)
    csr_b, _ = generate.random_graph_csr(60, 4, 12)
    T.write_sparse(str(tmp_path), csr_a, edges_a)
    assert "csr" in T.load(str(tmp_path))
    T.save_csr(str(tmp_path / "topology.csr.npz"), csr_b)        # stale companion, same N
    topo = T.load(str(tmp_path))
    assert "csr" not in topo
    back = T.to_csr(topo)
    np.testing.assert_array_equal(back.col, csr_a.col)
    assert np.array_equal(back.val.view(np.uint32), csr_a.val.view(np.uint32))


def test_mh_diag_large_n_matches_dense_row_sum():
    """At N >= 32768 ATen reduces a 1-D row over several threads; mh_csr then reduces every dense
    row on its own (ROWSUM_BATCH_MAX), as the reference's W[i, :].sum() (weights.py:25)."""
    n = T.ROWSUM_BATCH_MAX + 7232                                    # 40 000
    rng = np.random.default_rng(3)
    edges = {i: set() for i in range(n)}
    for i in range(n):
        for j in rng.integers(0, n, 3):
            if j != i:
                edges[i].add(int(j))
                edges[int(j)].add(i)
    edges = {i: sorted(e) for i, e in edges.items()}
    csr = T.mh_csr(n, edges)
    deg = [len(edges[i]) for i in range(n)]
    for i in (0, 1, n // 2, n - 1):
        row = torch.zeros(n)
        for j in edges[i]:
            row[j] = 1. / (max(deg[i], deg[j]) + 1)
        want = (1. - row.sum()).numpy()
        assert csr.val[csr.row_ptr[i]].view(np.uint32) == np.float32(want).view(np.uint32), i
