"""The C-ABI library builds for gfx950, loads, and exports every symbol include/niidmix.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import os
import re

from conftest import REPO


def _declared_symbols():
    text = open(os.path.join(REPO, "include", "niidmix.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int64_t|int|const char \*|void \*|void)\s*(niidmix_\w+)\s*\(",
                                 text, re.M)))


def test_header_declares_expected_api():
    syms = _declared_symbols()
    for s in ["niidmix_abi_version", "niidmix_last_error", "niidmix_mix_csr_f32",
              "niidmix_mix_clique_f32", "niidmix_mix_dense_f32", "niidmix_mean_rows_f32",
              "niidmix_mix_tile_lds_f32", "niidmix_grad_segment_mean_f32", "niidmix_hbm_alloc",
              "niidmix_hbm_free"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    from niidmix import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for s in _declared_symbols():
        assert hasattr(lib, s), s
    assert set(_lib.SIGNATURES) == set(_declared_symbols())
    assert _lib.lib.niidmix_abi_version() == _lib.ABI_VERSION


def test_library_is_gfx950_code_object():
    from niidmix import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_argument_errors_without_gpu():
    """Validation happens before any HIP call, so errors are reported on a CPU-only host too."""
    from niidmix import _lib
    L = _lib.lib
    rc = L.niidmix_mix_csr_f32(None, 4, None, 4, 1, 4, None, None, None, 0, None)
    assert rc == _lib.EINVAL and b"null" in L.niidmix_last_error()
    rc = L.niidmix_mix_csr_f32(16, 4, 16, 4, 1, 4, 8, 8, 8, 0, None)
    assert rc == _lib.EALIAS
    rc = L.niidmix_mix_csr_f32(16, 4, 1024, 4, 1, 4, 8, 8, 8, 16, None)
    assert rc == _lib.EINVAL        # unknown mode
    rc = L.niidmix_mix_csr_f32(16, 4, 1024, 4, 1, 4, 8, 8, 8, 2 | 8, None)
    assert rc == _lib.EINVAL        # AVERAGE_ONLY and MEAN are exclusive
    rc = L.niidmix_mix_csr_f32(16, 2, 1024, 4, 1, 4, 8, 8, 8, 0, None)
    assert rc == _lib.EINVAL        # ld < p
    assert L.niidmix_mix_csr_f32(16, 4, 1024, 4, 0, 4, 8, 8, 8, 0, None) == _lib.OK  # empty
    plan = _lib.CliquePlanC(1, 4, 5, 4, 0, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8)
    rc = L.niidmix_mix_clique_f32(16, 4, 1024, 4, 4, ctypes.byref(plan), None)
    assert rc == _lib.EUNSUPPORTED   # n_groups 5
    plan = _lib.CliquePlanC(1, 300, 2, 300, -1, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8)
    rc = L.niidmix_mix_clique_f32(16, 4, 1 << 24, 4, 4, ctypes.byref(plan), None)
    assert rc == _lib.EINVAL         # negative max_clique_res
    plan = _lib.CliquePlanC(1, 4, 1, 4, 0, 8, 8, 8, 8, 8, 8, 8, 8, None, 8, 8)
    rc = L.niidmix_mix_clique_f32(16, 4, 1024, 4, 4, ctypes.byref(plan), None)
    assert rc == _lib.EINVAL         # the CSR (non-finite guard) is required
    # partial overlap of x and y over the member rows (Jacobi): 4 rows of ld 8 floats
    plan = _lib.CliquePlanC(1, 4, 1, 4, 0, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8)
    base = 1 << 20
    rc = L.niidmix_mix_clique_f32(base, 8, base + 4 * 20, 8, 8, ctypes.byref(plan), None)
    assert rc == _lib.EALIAS         # y starts inside x's 3rd row
    rc = L.niidmix_mix_clique_blocked_f32(base, base + 4 * 1024 * 2, 8, 1024, 1024, 8192, 8192,
                                          ctypes.byref(plan), None)
    assert rc == _lib.EALIAS         # y inside x's member rows of block 0
    rc = L.niidmix_mix_csr_f32(base + 4 * 20, 8, base, 8, 4, 8, 8, 8, 8, 0, None)
    assert rc == _lib.EALIAS         # x starts inside y
    rc = L.niidmix_mix_dense_f32(16, 4, 1024, 4, 4, 4, 8, None, 8, 8, None)
    assert rc == _lib.EINVAL         # dense: the CSR (non-finite guard) is required
    # ABI 5: the bf16x6 dense GEMM and its W split
    assert L.niidmix_dense_split_elems(1000) == 3 * 1024 * 1008
    assert L.niidmix_dense_split_elems(0) == 0
    rc = L.niidmix_mix_dense_bf16x6_f32(16, 4, 1024, 4, 4, 4, 16, None, 8, 8, None)
    assert rc == _lib.EINVAL         # the CSR (non-finite guard) is required
    rc = L.niidmix_mix_dense_bf16x6_f32(16, 4, 1024, 4, 4, 4, 8, 8, 8, 8, None)
    assert rc == _lib.EUNSUPPORTED   # split W must be 16-B aligned
    rc = L.niidmix_mix_dense_bf16x6_f32(base, 8, base + 4 * 20, 8, 4, 8, 1 << 24, 8, 8, 8, None)
    assert rc == _lib.EALIAS
    rc = L.niidmix_dense_split_w(4096, 4, 4096 + 16, None)
    assert rc == _lib.EALIAS         # w and its split overlap
    # the bf16x6 GEMM's 32-bit offsets -- 16 rows of ld_x (ld_x >= 2^25) or a split
    # W of 2^31 B (n = 19 000) -- are refused, never launched (niidmix.ops.b6_fits avoids them)
    ld = 1 << 25
    rc = L.niidmix_mix_dense_bf16x6_f32(base, ld, base + 4 * 4 * ld, ld, 4, 8, 1 << 24, 8, 8, 8, None)
    assert rc == _lib.EUNSUPPORTED
    rc = L.niidmix_mix_dense_bf16x6_f32(base, 8, base + 4 * 8 * 19000, 8, 19000, 8, 1 << 24, 8, 8, 8,
                                        None)
    assert rc == _lib.EUNSUPPORTED
    tp = _lib.TilePlanC(1, 12, 0, 8, 8, 8, 8, 8, 8)
    rc = L.niidmix_mix_tile_f32(16, 4, 1024, 4, 1, 4, ctypes.byref(tp), 0, None)
    assert rc == _lib.EUNSUPPORTED   # tile height 12
    tp = _lib.TilePlanC(1, 16, 0, None, 8, 8, 8, 8, 8)
    rc = L.niidmix_mix_tile_f32(16, 4, 1024, 4, 1, 4, ctypes.byref(tp), 0, None)
    assert rc == _lib.EINVAL         # null sub_ptr
    tp = _lib.TilePlanC(1, 16, 0, 8, 8, 8, 8, 8, 8)
    assert L.niidmix_mix_tile_f32(16, 4, 1024, 4, 1, 4, ctypes.byref(tp), 9, None) == _lib.EINVAL
    assert L.niidmix_mix_tile_f32(16, 4, 16, 4, 1, 4, ctypes.byref(tp), 0, None) == _lib.EALIAS
    # ABI 3: partial overlaps are caught over the full [n_rows, ld] extents (4 rows of ld 8)
    assert L.niidmix_mix_tile_f32(base, 8, base + 4 * 20, 8, 4, 8, ctypes.byref(tp), 0, None) == _lib.EALIAS
    lp = _lib.TileLdsPlanC(1, 16, 1, 8, 1, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8)   # seg*/mf* NULL
    assert L.niidmix_mix_tile_lds_f32(base, 8, base + 4 * 20, 8, 4, 8, ctypes.byref(lp), 0, None) == _lib.EALIAS
    G = L.niidmix_grad_segment_mean_f32
    assert G(None, 4, 16, 4, 1, 4, 1, 8, 8, None) == _lib.EINVAL
    assert G(16, 4, 16, 4, 1, 4, 1, 8, 8, None) == _lib.EALIAS
    assert G(16, 2, 1024, 4, 1, 4, 1, 8, 8, None) == _lib.EINVAL
    assert G(16, 4, 1024, 4, 1, 4, 0, 8, 8, None) == _lib.OK
    assert G(base, 8, base + 4 * 20, 8, 4, 8, 1, 8, 8, None) == _lib.EALIAS   # partial overlap
    B = L.niidmix_grad_segment_mean_blocked_f32
    assert B(None, 1024, 1, 4, 1024, 1024, 4096, 4096, 1, 8, 8, None) == _lib.EINVAL    # null
    assert B(16, 1024, 1, 4, 1024, 1000, 4096, 4096, 1, 8, 8, None) == _lib.EINVAL      # block_cols
    assert B(16, 1024, 1, 4, 1024, 1024, 512, 4096, 1, 8, 8, None) == _lib.EINVAL       # stride
    assert B(16, 16, 1, 4, 1024, 1024, 4096, 4096, 1, 8, 8, None) == _lib.EALIAS
    assert B(16, 1 << 30, 1, 6, 1024, 1024, 4096, 4096, 1, 8, 8, None) == _lib.EUNSUPPORTED  # p % 4
    assert B(16, 1024, 1, 4, 1024, 1024, 4096, 4096, 0, 8, 8, None) == _lib.OK         # empty
    # y with a LARGER block stride than g: g's 2 blocks at base + 8 KB, y's block 1 at base + 12 KB
    assert B(base + 8192, base, 1, 2048, 1024, 1024, 1024, 3072, 1, 8, 8, None) == _lib.EALIAS
    U = L.niidmix_update_rows_f32
    assert U(None, 4, 1024, 4, 1, 4, 8, None) == _lib.EINVAL
    assert U(base, 8, 1 << 30, 8, 4, 8, base + 4 * 20, None) == _lib.EALIAS   # avg inside x
    assert U(base, 8, base + 4 * 20, 8, 4, 8, 1 << 30, None) == _lib.EALIAS   # partial x / y overlap
    assert U(base, 8, base, 8, 0, 8, 8, None) == _lib.OK                       # no rows
    rc = L.niidmix_copy2d_async(None, 4, None, 4, 4, 1, 0, None)
    assert rc == _lib.EINVAL
    assert L.niidmix_stream_copy_f32(16, 1024, 6, None) == _lib.EUNSUPPORTED   # n % 4
    assert L.niidmix_stream_copy_f32(16, 32, 8, None) == _lib.EALIAS
    assert L.niidmix_stream_copy_f32(None, 32, 8, None) == _lib.EINVAL
    assert L.niidmix_stream_copy_f32(16, 1024, 0, None) == _lib.OK
    h = ctypes.c_void_p()
    assert L.niidmix_sharded_create(0, None, ctypes.byref(h)) == _lib.EINVAL and not h.value
    assert L.niidmix_sharded_destroy(None) == _lib.OK
    assert L.niidmix_mix_sharded_f32(None, None, 4, 0) == _lib.EINVAL
    E = L.niidmix_mix_ell_f32
    assert E(16, 4, 1024, 4, 1, 4, 9, 8, 8, 8, 0, None) == _lib.EUNSUPPORTED            # width 9
    assert E(16, 4, 1024, 4, 1, 4, 4, 8, 8, 8, 0, None) == _lib.EINVAL                  # unpadded width
    assert E(16, 4, 16, 4, 1, 4, 3, 8, 8, 8, 0, None) == _lib.EALIAS
    assert E(None, 4, 1024, 4, 1, 4, 3, 8, 8, 8, 0, None) == _lib.EINVAL
    S = L.niidmix_mix_strip_f32
    assert S(16, 64, 1 << 30, 64, 2, 64, 4, 8, 8, 8, 0, None) == _lib.EUNSUPPORTED     # ELL width 4
    assert S(16, 64, 1 << 30, 64, 257, 64, 3, 8, 8, 8, 0, None) == _lib.EUNSUPPORTED   # > 256 rows
    assert S(16, 64, 16 + 4 * 64, 64, 2, 64, 3, 8, 8, 8, 0, None) == _lib.EALIAS       # y = x's row 1
    assert S(None, 64, 1 << 30, 64, 2, 64, 3, 8, 8, 8, 0, None) == _lib.EINVAL
    assert S(16, 32, 1 << 30, 64, 2, 64, 3, 8, 8, 8, 0, None) == _lib.EINVAL          # ld_x < p
    assert S(18, 64, 1 << 30, 64, 2, 64, 3, 8, 8, 8, 0, None) == _lib.EUNSUPPORTED     # x not 4-B aligned
    assert S(16, 64, 1 << 30, 64, 2, 64, 3, 8, 8, 8, 16, None) == _lib.EINVAL         # unknown mode
    assert S(16, 64, 1 << 30, 64, 0, 64, 3, 8, 8, 8, 0, None) == _lib.OK              # no rows


def test_kernel_for_respects_bf16x6_limits():
    """Mixer.kernel_for('fast') picks the bf16x6 GEMM ('dense') for a dense W only
    within its limits (niidmix.ops.b6_fits: split W and 16 rows of the slab under 2^31 B), else the
    fp32 MFMA GEMM ('dense-f32'), which has none.  Host arithmetic only."""
    import numpy as np
    import torch
    from niidmix import ops
    n = 64
    w = np.random.default_rng(0).random((n, n)).astype(np.float32)
    w /= w.sum(0, keepdims=True)
    rp = np.arange(n + 1, dtype=np.int64) * n
    col = np.concatenate([[i] + [j for j in range(n) if j != i] for i in range(n)]).astype(np.int32)
    m = ops.Mixer(csr=ops.csr_from_numpy(rp, col, w[col, np.repeat(np.arange(n), n)]), device="cpu")
    assert m.kernel_for("fast") == "dense"
    ok = torch.empty_strided((2, 8), ((1 << 25) - 64, 1), device="meta")
    wide = torch.empty_strided((2, 8), (1 << 25, 1), device="meta")
    assert m.kernel_for("fast", ok) == "dense"
    assert m.kernel_for("fast", wide) == "dense-f32"
    assert m.kernel_for("fast", ok, wide) == "dense"        # y is addressed in 64 bits
    assert ops.b6_fits(18000) and not ops.b6_fits(19000)
