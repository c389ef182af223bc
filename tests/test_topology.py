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
