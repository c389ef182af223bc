"""The CPU oracle (oracle/) against the golden vectors produced by running the reference
(tests/golden/make_golden.py).  This pins the oracle before it is trusted as the GPU checker."""
import numpy as np
import pytest

from conftest import golden_cases, load_golden


@pytest.mark.parametrize("name", golden_cases())
def test_c_oracle_bitwise(name, oracle_mod):
    g = load_golden(name)
    y = oracle_mod.mix_exact_c(g["x"], g["row_ptr"], g["col"], g["val"])
    assert oracle_mod.bitwise_equal(y, g["y"]), name


@pytest.mark.parametrize("name", [n for n in golden_cases() if not n.startswith("dcliques1000")])
def test_numpy_oracle_bitwise(name, oracle_mod):
    g = load_golden(name)
    y = oracle_mod.mix_exact_np(g["x"], g["row_ptr"], g["col"], g["val"])
    assert oracle_mod.bitwise_equal(y, g["y"]), name


def test_c_oracle_column_windows(oracle_mod):
    """Columns are independent: any window of the oracle equals the same window of the full run
    (the basis of full-size parity on sampled windows)."""
    g = load_golden("dcliques1000_fc_p64")
    full = g["y"]
    for c0, c1 in [(0, 1), (5, 17), (60, 64)]:
        y = oracle_mod.mix_exact_c(g["x"], g["row_ptr"], g["col"], g["val"], cols=(c0, c1))
        assert oracle_mod.bitwise_equal(y[:, c0:c1], full[:, c0:c1])


def test_uniform_average(oracle_mod):
    d = np.load(__import__("conftest").GOLDEN + "/uniform_avg_k7_p100.npz")
    assert oracle_mod.bitwise_equal(oracle_mod.mean_rows_np(d["x"]), d["y"][0])
    assert oracle_mod.bitwise_equal(oracle_mod.mean_rows_c(d["x"]), d["y"][0])


def test_fma_variant_is_not_bitwise(oracle_mod):
    """Sanity of the bar: a fused/reassociated evaluation does NOT reproduce the reference bits, so
    bit-exact parity is a real check (FMA variant mismatches ~77% of elements)."""
    g = load_golden("dcliques1000_fc_p64")
    n = len(g["row_ptr"]) - 1
    W = np.zeros((n, n), np.float64)
    dst = np.repeat(np.arange(n), np.diff(g["row_ptr"]))
    W[g["col"], dst] = g["val"]
    y64 = (W.T @ g["x"].astype(np.float64)).astype(np.float32)
    assert not oracle_mod.bitwise_equal(y64, g["y"])
    bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
    ok, worst = oracle_mod.check_tolerance(y64, g["y"], bound, rtol=1e-5)
    assert ok, worst


def test_reference_loop_restatement(oracle_mod):
    """The CPU-baseline restatement of the reference loop (oracle.reference_loop_average) reproduces
    the golden outputs bit for bit, multi-tensor model included."""
    import json
    import torch
    for name in ["ring100_p257", "n2_ring_linear7850", "nonfinite_ring8_p16", "dcliques300_fc_p37"]:
        g = load_golden(name)
        shapes = [tuple(s) for s in json.loads(str(g["shapes_json"]))]
        n = len(g["row_ptr"]) - 1
        W = torch.zeros(n, n)
        edges = {}
        for i in range(n):
            b, e = g["row_ptr"][i], g["row_ptr"][i + 1]
            edges[i] = g["col"][b + 1:e].tolist()
            W[g["col"][b:e], i] = torch.from_numpy(g["val"][b:e])
        nodes = []
        for i in range(n):
            m = torch.nn.Module()
            m.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.zeros(s)) for s in shapes])
            off = 0
            with torch.no_grad():
                for p in m.parameters():
                    k = p.numel()
                    p.copy_(torch.from_numpy(g["x"][i, off:off + k].copy()).view_as(p))
                    off += k
            nodes.append({"rank": i, "model": m})
        oracle_mod.reference_loop_average(nodes, {"weights": W, "edges": edges})
        y = np.stack([torch.cat([p.detach().reshape(-1) for p in nd["model"].parameters()]).numpy()
                      for nd in nodes])
        assert oracle_mod.bitwise_equal(y, g["y"]), name


def test_logger_round_fixture(oracle_mod):
    """tests/golden/logger_round_dcliques300_p520 (make_golden.py --logger: one reference mixing
    round, then the reference Logger's consensus event and setup.model.average over all nodes, a
    subset and node 0): the oracle reproduces the round bitwise, the uniform averages bitwise
    (mean_rows_np / mix_exact_np AVERAGE_ONLY over the subset rows), and the event's statistics
    from the mixed rows in fp64 within 1e-6 relative."""
    import statistics
    g = load_golden("logger_round_dcliques300_p520")
    y = oracle_mod.mix_exact_c(g["x"], g["row_ptr"], g["col"], g["val"])
    assert oracle_mod.bitwise_equal(y, g["y"])
    assert oracle_mod.bitwise_equal(oracle_mod.mean_rows_np(g["y"]), g["center_all"])
    sub = g["subset"]
    k = len(sub)
    w = np.full(k, np.float32(1.0 / k), np.float32)
    c = oracle_mod.mix_exact_np(g["y"], np.asarray([0, k]), sub.astype(np.int32), w,
                                average_only=True)[0]
    assert oracle_mod.bitwise_equal(c, g["center_subset"])
    assert oracle_mod.bitwise_equal(g["y"][0] * np.float32(0) + np.float32(1) * g["y"][0],
                                    g["center_node0"])
    center = g["center_all"].astype(np.float64)
    d = np.sqrt(((g["y"].astype(np.float64) - center) ** 2).sum(1)).tolist()
    got = [statistics.mean(d), statistics.stdev(d), max(d), min(d),
           float(np.sqrt((center ** 2).sum()))]
    np.testing.assert_allclose(got, g["stats"], rtol=1e-6)
