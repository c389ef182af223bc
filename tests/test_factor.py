"""Clique factorisation (host logic, CPU): the plan reproduces the loaded W exactly and the
factored formula reproduces the reference outputs; rejections fall back to generic kernels."""
import numpy as np
import pytest

from conftest import golden_cases, load_golden
from niidmix.factor import build_clique_plan
from niidmix.topology import MixCSR


def _csr(g):
    return MixCSR(g["row_ptr"], g["col"], g["val"]).validate()


@pytest.mark.parametrize("name", golden_cases("dcliques"))
def test_plan_reproduces_w(name):
    g = load_golden(name)
    csr = _csr(g)
    plan, why = build_clique_plan(csr, g["cliques"])
    assert plan is not None, why
    W = csr.dense().astype(np.float64)
    We = plan.effective_weights()
    # exact except the fp32 rounding of a_i = W_ii - c and of in-clique corrections
    assert np.max(np.abs(W - We)) <= 4e-9
    assert np.array_equal(W != 0, np.abs(We) > 1e-12)


@pytest.mark.parametrize("name", golden_cases("dcliques"))
def test_factored_formula_matches_reference(name, oracle_mod):
    """The factored formula plus the kernels' non-finite guard (every non-finite factored output is
    recomputed from the node's CSR row, include/niidmix.h) reproduces the reference, inf/NaN
    pattern included; without the guard the non-finite fixtures leak NaN along removed / absent
    edges."""
    g = load_golden(name)
    plan, _ = build_clique_plan(_csr(g), g["cliques"])
    with np.errstate(all="ignore"):
        y = plan.apply_np(g["x"]).astype(np.float32)
        bad = ~np.isfinite(y)
        if bad.any():
            y = np.where(bad, oracle_mod.mix_exact_c(g["x"], g["row_ptr"], g["col"], g["val"]), y)
    bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
    ok, worst = oracle_mod.check_tolerance(y, g["y"], bound, rtol=1e-6)
    assert ok, worst


def test_cancelling_corrections_counted():
    """Removed clique edges are corrected by -c_g terms (cancelling): counted, so Mixer's auto
    choice avoids the factored kernel there; the headline topology has none."""
    g = load_golden("dcliques1000_fc_p64")
    assert build_clique_plan(_csr(g), g["cliques"])[0].n_cancel == 0
    g = load_golden("dcliques200_fractal_rm5_p40")
    assert build_clique_plan(_csr(g), g["cliques"])[0].n_cancel > 0


def test_headline_structure():
    """1000-node d-cliques (reference generator, seed 1337): 10 cliques of 100, two degree classes
    (99 and 100), 90 inter-clique residual terms, 9 per clique."""
    g = load_golden("dcliques1000_fc_p64")
    plan, _ = build_clique_plan(_csr(g), g["cliques"])
    assert plan.n_cliques == 10 and plan.max_clique == 100 and plan.n_groups == 2
    assert plan.n_res == 90 and plan.max_clique_res == 9


def test_rejections():
    g = load_golden("dcliques300_fc_p37")
    csr = _csr(g)
    assert build_clique_plan(csr, None)[0] is None
    assert build_clique_plan(csr, g["cliques"][:-1])[0] is None            # not a partition
    assert build_clique_plan(csr, g["cliques"], max_clique=16)[0] is None  # clique too large
    ring = load_golden("ring100_p257")
    cl = [[i] for i in range(100)]                                         # singletons: all residual
    plan, why = build_clique_plan(_csr(ring), cl, max_res_per_node=1.0)
    assert plan is None and "residual" in why
