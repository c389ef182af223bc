"""Merged-order row tiles (niidmix.tile, host side of k_mix_tile) on CPU: every row's operand
sequence in the plan is exactly its CSR row (the reference's self-then-edges order), and the numpy
model of the kernel reproduces the reference's golden outputs bit for bit."""
import numpy as np
import pytest

from conftest import golden_cases, load_golden


def _csr(g):
    from niidmix.topology import MixCSR
    return MixCSR(g["row_ptr"].astype(np.int64), g["col"].astype(np.int32),
                  g["val"].astype(np.float32))


@pytest.mark.parametrize("rt", [8, 16, 32])
@pytest.mark.parametrize("name", golden_cases())
def test_plan_rows_are_csr_rows(name, rt):
    from niidmix import tile
    g = load_golden(name)
    csr = _csr(g)
    plan, why = tile.build_tile_plan(csr, g.get("cliques"), rt)
    assert plan is not None, why
    rows = plan.row_lists()
    assert sorted(rows) == list(range(csr.n))
    for i in range(csr.n):
        b, e = csr.row_ptr[i], csr.row_ptr[i + 1]
        want = list(zip(csr.col[b:e].tolist(), csr.val[b:e].tolist()))
        got = [(c, float(w)) for c, w in rows[i]]
        assert got == [(int(c), float(np.float32(w))) for c, w in want], i
    full = (1 << rt) - 1
    for t in range(plan.n_sub):
        used = plan.sub_rows[t * rt:(t + 1) * rt] >= 0
        pad = full & ~int(sum(1 << r for r in range(rt) if used[r]))
        m = plan.pos_mask[plan.sub_ptr[t]:plan.sub_ptr[t + 1]].astype(np.int64)
        assert np.all((m & pad) == pad)          # unused slots always "take" (never stored)
        assert np.all((m & ~pad & full) != 0)    # no empty position


@pytest.mark.filterwarnings("ignore::RuntimeWarning")
@pytest.mark.parametrize("name", golden_cases())
def test_numpy_model_bitwise_vs_golden(name, oracle_mod):
    from niidmix import tile
    g = load_golden(name)
    plan, _ = tile.build_tile_plan(_csr(g), g.get("cliques"), 16)
    assert oracle_mod.bitwise_equal(tile.apply_np(plan, g["x"]), g["y"]), name


def test_dcliques_density():
    """The reference's d-cliques edge lists are set-iteration orders that disagree across rows; the
    LCS-guided merge must still keep the tiles dense (a greedy majority merge gave 0.48)."""
    from niidmix import tile
    for name in ["dcliques1000_fc_p64", "dcliques1000_ring_p16", "dcliques1000_smallworld_p16"]:
        g = load_golden(name)
        plan, _ = tile.build_tile_plan(_csr(g), g.get("cliques"), 16)
        assert plan.density > 0.8, (name, plan.density)


def test_supersequence_random_conflicts():
    from niidmix.tile import _supersequence
    rng = np.random.default_rng(0)
    for _ in range(200):
        base = rng.permutation(40).tolist()
        seqs = []
        for _ in range(int(rng.integers(1, 9))):
            s = [v for v in base if rng.random() < 0.9]
            for _ in range(int(rng.integers(0, 4))):          # local swaps: conflicting orders
                if len(s) > 1:
                    i = int(rng.integers(0, len(s) - 1))
                    s[i], s[i + 1] = s[i + 1], s[i]
            seqs.append(s)
        M = _supersequence(seqs)
        for s in seqs:
            it = iter(M)
            assert all(v in it for v in s)                   # s is a subsequence of M
        assert len(M) <= sum(len(s) for s in seqs)


def test_bad_inputs():
    from niidmix import tile
    g = load_golden("ring100_p257")
    assert tile.build_tile_plan(_csr(g), None, 12)[0] is None
    assert tile.build_tile_plan(_csr(g), [[0, 1]], 16)[0] is None     # not a partition


@pytest.mark.parametrize("rt", [8, 16, 32])
@pytest.mark.parametrize("name", ["dcliques1000_fc_p64", "dcliques1000_smallworld_p16",
                                  "dcliques200_fractal_rm5_p40", "dcliques300_fc_p37"])
def test_lds_plan_slots(name, rt):
    """LDS plan: every position / tile row slot names, in its group's staged list, the row the
    global tile plan names; lists are distinct and within the LDS budget; the uniform flag is kept
    and holds (all rt weights of a flagged position equal)."""
    from niidmix import tile
    g = load_golden(name)
    csr = _csr(g).validate()
    lp, why = tile.build_tile_lds_plan(csr, g["cliques"], rt)
    if lp is None:
        pytest.skip(why)
    tp = lp.tile
    mask = tile.POS_UNIFORM - 1
    assert lp.max_src <= tile.LDS_MAX_SRC and lp.max_tiles <= tile.LDS_MAX_WAVES[rt]
    for gi in range(lp.n_grp):
        srcs = lp.grp_src_rows[lp.grp_src_ptr[gi]:lp.grp_src_ptr[gi + 1]]
        assert len(np.unique(srcs)) == len(srcs)
        t0, t1 = lp.grp_tile_ptr[gi], lp.grp_tile_ptr[gi + 1]
        for k in range(tp.sub_ptr[t0], tp.sub_ptr[t1]):
            assert srcs[lp.pos_slot[k] & mask] == (tp.pos_src[k] & mask)
            assert (lp.pos_slot[k] & tile.POS_UNIFORM) == (tp.pos_src[k] & tile.POS_UNIFORM)
            if tp.pos_src[k] & tile.POS_UNIFORM:
                w = tp.pos_w[k * rt:(k + 1) * rt]
                assert np.all(w.view(np.uint32) == w[0].view(np.uint32))
        for k in range(t0 * rt, t1 * rt):
            if tp.sub_rows[k] >= 0:
                assert srcs[lp.sub_slot[k]] == tp.sub_rows[k]


def test_uniform_positions_dominate_dcliques():
    """Degree-class ordering inside a clique makes almost every position uniform-weight on the
    headline topology (the exact kernel then forms one product per position)."""
    from niidmix import tile
    g = load_golden("dcliques1000_fc_p64")
    csr = _csr(g).validate()
    tp, _ = tile.build_tile_plan(csr, g["cliques"], 16)
    frac = np.mean((tp.pos_src & tile.POS_UNIFORM) != 0)
    assert frac > 0.95, frac


def test_lds_plan_runs_dcliques():
    """rt-16 LDS plan on the headline topology: full-height tiles (7 per clique, no pad slot),
    rows in the clique's list order so that most 4-position groups are taken by every row, and
    slots numbered in list order so that most consecutive positions read consecutive slots."""
    from niidmix import tile
    g = load_golden("dcliques1000_fc_p64")
    csr = _csr(g).validate()
    lp, why = tile.build_tile_lds_plan(csr, g["cliques"], 16)
    assert lp is not None, why
    tp = lp.tile
    assert lp.max_tiles == 7 and tp.n_sub == 70
    full = (1 << 16) - 1
    groups = every_row = consecutive = pairs = 0
    for t in range(tp.n_sub):
        b, e = int(tp.sub_ptr[t]), int(tp.sub_ptr[t + 1])
        n = int(np.sum(tp.sub_rows[t * 16:(t + 1) * 16] >= 0))
        rows = (1 << n) - 1
        taken = [(int(tp.pos_mask[k]) & rows) == rows for k in range(b, e)]
        for j in range(0, (e - b) & ~3, 4):
            groups += 1
            every_row += all(taken[j:j + 4])
        slots = lp.pos_slot[b:e] & (tile.POS_UNIFORM - 1)
        consecutive += int(np.sum(np.diff(slots) == 1))
        pairs += len(slots) - 1
    assert every_row / groups > 0.7, every_row / groups
    assert consecutive / pairs > 0.8, consecutive / pairs


def _lds16(g, csr):
    from niidmix import tile
    cl = g.get("cliques")
    if not cl:
        span = 16 * tile.LDS_MAX_WAVES[16]
        cl = [list(range(s, min(s + span, csr.n))) for s in range(0, csr.n, span)]
    lp, why = tile.build_tile_lds_plan(csr, cl, 16)
    return lp, why


def _assert_rows_are_csr(rows, csr):
    assert sorted(rows) == list(range(csr.n))
    for i in range(csr.n):
        b, e = csr.row_ptr[i], csr.row_ptr[i + 1]
        want = [(int(c), float(np.float32(w))) for c, w in zip(csr.col[b:e], csr.val[b:e])]
        assert [(int(c), float(w)) for c, w in rows[i]] == want, i


@pytest.mark.parametrize("name", golden_cases())
def test_segments_apply_csr_rows(name):
    """The segment walker's view of an RT-16 LDS plan (runs + masked entries) gives every row
    exactly its CSR row, in order (k_mix_tile_lds's segment loop, niidmix.tile.build_tile_segments)."""
    from niidmix import tile
    g = load_golden(name)
    csr = _csr(g)
    lp, why = _lds16(g, csr)
    if lp is None:
        pytest.skip(why)
    ts = tile.build_tile_segments(lp)
    assert ts is not None and ts.seg.shape[1] == tile.SEG_WORDS
    _assert_rows_are_csr(tile.segments_row_lists(lp, ts), csr)


@pytest.mark.parametrize("cap", [8, 16])
@pytest.mark.parametrize("name", golden_cases("dcliques"))
def test_register_rows_apply_csr_rows(name, cap):
    """Plans with register rows (build_tile_lds_plan(remote_regs=True, rem_cap)): the walker's
    view -- runs, masked entries, masked entries reading a register row -- still gives every row
    its CSR row in order; at most `cap` register rows per tile, each read by one tile only, none
    of them staged; rem_regs says how many the kernel must load."""
    from niidmix import tile
    g = load_golden(name)
    csr = _csr(g)
    lp, why = tile.build_tile_lds_plan(csr, g["cliques"], 16, remote_regs=True, rem_cap=cap)
    if lp is None:
        pytest.skip(why)
    if lp.rem_rows is None:
        pytest.skip("no source qualifies for a register row")
    regs = lp.rem_rows.reshape(-1, tile.REM_MAX)
    per_tile = (regs >= 0).sum(1)
    assert per_tile.max() <= cap
    assert lp.rem_regs == (8 if per_tile.max() <= 8 else 16)
    gtp, gsp = lp.grp_tile_ptr, lp.grp_src_ptr
    for gi in range(lp.n_grp):
        in_regs = regs[gtp[gi]:gtp[gi + 1]]
        in_regs = in_regs[in_regs >= 0]
        assert len(np.unique(in_regs)) == len(in_regs)          # one tile, one register each
        assert not set(in_regs.tolist()) & set(lp.grp_src_rows[gsp[gi]:gsp[gi + 1]].tolist())
    ts = tile.build_tile_segments(lp)
    assert ts is not None
    _assert_rows_are_csr(tile.segments_row_lists(lp, ts), csr)


def test_balanced_tile_rows_dcliques():
    """balanced_tile_rows: a 100-row clique cuts into 7 full-height tiles (4k - 1 waves: one SIMD a
    wave short), so the rule picks the tallest height that cuts 8; the plan then has 8 tiles per
    clique, none taller than that height, and the segment walker's view still gives every row
    its CSR row in order (with and without register rows)."""
    from niidmix import tile
    g = load_golden("dcliques1000_fc_p64")
    csr = _csr(g).validate()
    r = tile.balanced_tile_rows(csr, g["cliques"], 16)
    assert 8 < r < 16
    for remote in (False, True):
        lp, why = tile.build_tile_lds_plan(csr, g["cliques"], 16, remote_regs=remote, tile_rows=r)
        assert lp is not None, why
        assert lp.max_tiles == 8 and lp.tile.n_sub == 80
        assert int((lp.tile.sub_rows.reshape(-1, 16) >= 0).sum(1).max()) <= r
        _assert_rows_are_csr(tile.segments_row_lists(lp, tile.build_tile_segments(lp)), csr)
    # already a multiple of 4 (or not rt 16): unchanged
    assert tile.balanced_tile_rows(csr, [c[:64] for c in g["cliques"]] +
                                   [c[64:] for c in g["cliques"]], 16) == 16
    assert tile.balanced_tile_rows(csr, g["cliques"], 8) == 8
    # a height that would cut more tiles than a block may have (8 rows: 13): full-height tiles
    lp, why = tile.build_tile_lds_plan(csr, g["cliques"], 16, tile_rows=8)
    assert lp is not None and lp.max_tiles == 7, why


def test_rem_two_phase_eligibility():
    """rem_two_phase: d-cliques plans with more than 8 register rows per tile read rows 0..7 before
    any of 8..15 (rem_rows lists them in first-use order, one masked entry each); a plan whose
    segments read a low row after a high one is refused; plans without register rows too."""
    import copy
    from niidmix import tile
    from niidmix.generate import dcliques_csr
    csr, cl = dcliques_csr(2000, 100, "fully-connected", 1337)
    lp, why = tile.build_tile_lds_plan(csr, cl, 16, remote_regs=True)
    assert lp is not None, why
    assert lp.rem_regs == 16 and int((lp.rem_rows.reshape(-1, 16) >= 0).sum(1).max()) > 8
    ts = tile.build_tile_segments(lp)
    assert tile.rem_two_phase(lp, ts)
    _assert_rows_are_csr(tile.segments_row_lists(lp, ts), csr)
    # swap the register indices 0 and 8 in the words of one tile that has both: 0 is then read last
    w0 = ts.seg[:, 0].astype(np.int64)
    remote = ((w0 & tile.SEG_HARD) != 0) & ((w0 & tile.SEG_REMOTE) != 0)
    for t in range(lp.tile.n_sub):
        b, e = int(ts.seg_ptr[t]), int(ts.seg_ptr[t + 1])
        idx = {int(w0[k] & tile.SEG_SLOT): k for k in range(b, e) if remote[k]}
        if 0 in idx and 8 in idx:
            bad = copy.copy(ts)
            bad.seg = ts.seg.copy()
            bad.seg[idx[0], 0] = (bad.seg[idx[0], 0] & ~tile.SEG_SLOT) | 8
            bad.seg[idx[8], 0] = (bad.seg[idx[8], 0] & ~tile.SEG_SLOT) | 0
            assert not tile.rem_two_phase(lp, bad)
            break
    else:
        raise AssertionError("no tile with register rows 0 and 8")
    lp0, _ = tile.build_tile_lds_plan(csr, cl, 16)
    assert not tile.rem_two_phase(lp0, tile.build_tile_segments(lp0))


def test_register_rows_cap_argument():
    from niidmix import tile
    g = load_golden("dcliques1000_fc_p64")
    with pytest.raises(ValueError):
        tile.build_tile_lds_plan(_csr(g), g["cliques"], 16, remote_regs=True, rem_cap=12)


@pytest.mark.parametrize("name", golden_cases())
def test_mfma_positions_apply_csr_rows(name):
    """The MFMA path's position lists (one entry per weight class, 4-entry groups) give every row
    exactly its CSR row, in order; padding entries take no row."""
    from niidmix import tile
    g = load_golden(name)
    csr = _csr(g)
    lp, why = _lds16(g, csr)
    if lp is None:
        pytest.skip(why)
    tm = tile.build_tile_mfma_positions(lp)
    assert tm is not None
    assert np.all(np.diff(tm.mf_ptr) % 4 == 0)
    assert np.all(tm.mf[:, 2].view(np.uint32) < (1 << 16))
    _assert_rows_are_csr(tile.mfma_row_lists(lp, tm), csr)


def test_mfma_positions_dcliques_headline_shape():
    """1000-node d-cliques (the headline): ~100 positions per 16-row tile, so the MFMA path issues
    ~26 groups of 4 positions per tile."""
    from niidmix import tile
    from niidmix.generate import dcliques_csr
    csr, cl = dcliques_csr(1000, 100, "fully-connected", 1337)
    lp, _ = tile.build_tile_lds_plan(csr, cl, 16)
    tm = tile.build_tile_mfma_positions(lp)
    per_tile = np.diff(tm.mf_ptr)
    assert per_tile.max() <= 112 and per_tile.mean() < 106
    _assert_rows_are_csr(tile.mfma_row_lists(lp, tm), csr)
