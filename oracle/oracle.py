"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the mixing hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker (or the timed CPU baseline), never as the thing measured or shipped.  The
product path (non-iid-topology-simulator_amd/niidmix) never imports it and fails loudly without its
HIP library.

Parity pinning: the reference is pure Python, so there is nothing to compile into oracle/_ref.
Instead the reference itself was run in the development container (tests/golden/make_golden.py,
committed) to produce tests/golden/*.npz; tests/test_oracle_golden.py checks every function below
bit for bit against those vectors.

Contents
  mix_exact_np        numpy restatement of d_sgd.average (d_sgd.py:96-116) over a CSR of W^T in the
                      reference's order; small sizes only.
  mix_exact_c         the same in C (oracle/mix_oracle.c, OpenMP), on any row/column window.
  mean_rows_np/_c     setup.model.average(models) with weights=None (model/__init__.py:15-25).
  grad_mean_np/_c     average_gradients + update_gradients (d_sgd.py:19-27,37-45) over a CSR whose
                      row r lists the nodes whose gradients node r averages (--clique-gradient,
                      --unbiased-gradient; d_sgd.py:47-94).
  reference_loop_average   a faithful restatement of the reference's module-level loop (per-node
                      deepcopy, mul_(0), add_(w*p), then update_models), used as the CPU baseline
                      ("kind": "port") in bench.py.
  condition_bound / check_tolerance   the condition-aware fast-mode tolerance.
"""
import copy
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
C_LIB_PATH = os.path.join(HERE, "build", "libmixoracle.so")


# ------------------------------------------------------------------------------------------------
# numpy restatement (small sizes)
def mix_exact_np(x, row_ptr, col, val, average_only=False):
    """y_i = fl(z + acc), z = x_self*0, acc = z then acc = fl(acc + fl(w*x_j)) in CSR order.

    d_sgd.py:105-110 builds the operand list [self] + edges[rank] with weights W[.,rank];
    model/__init__.py:19-24 starts from deepcopy(self)*0 and add_(w*p) per model; d_sgd.py:33-34
    (update_models) then writes p*0 + new.
    """
    x = np.asarray(x, np.float32)
    n = len(row_ptr) - 1
    y = np.empty((n, x.shape[1]), np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        for r in range(n):
            b, e = int(row_ptr[r]), int(row_ptr[r + 1])
            if b == e:
                y[r] = 0.0
                continue
            z = x[col[b]] * np.float32(0.0)
            acc = z.copy()
            for k in range(b, e):
                acc = acc + np.float32(val[k]) * x[col[k]]
            y[r] = acc if average_only else z + acc
    return y


def grad_mean_np(g, row_ptr, col):
    """acc = zeros_like (+0); acc.add_(g_j) in row order; div_(len) (true fp32 division, not a
    reciprocal multiply); then the target grad is zero_() + add_(mean) -> +0 + mean
    (d_sgd.py:19-27 average_gradients, d_sgd.py:37-45 update_gradients).  Empty rows -> +0."""
    g = np.asarray(g, np.float32)
    n = len(row_ptr) - 1
    y = np.empty((n, g.shape[1]), np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        for r in range(n):
            b, e = int(row_ptr[r]), int(row_ptr[r + 1])
            acc = np.zeros(g.shape[1], np.float32)
            for k in range(b, e):
                acc = acc + g[col[k]]
            y[r] = np.float32(0.0) + acc / np.float32(max(e - b, 1))
    return y


def mean_rows_np(x):
    """setup.model.average(models) with weights=None: w = float(1./K) applied in fp32."""
    x = np.asarray(x, np.float32)
    w = np.float32(1.0 / x.shape[0])
    with np.errstate(invalid="ignore", over="ignore"):
        acc = x[0] * np.float32(0.0)
        for k in range(x.shape[0]):
            acc = acc + w * x[k]
    return acc


# ------------------------------------------------------------------------------------------------
# C restatement
_c = None


def c_lib(build=True):
    global _c
    if _c is not None:
        return _c
    if not os.path.exists(C_LIB_PATH) and build:
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    lib = ctypes.CDLL(C_LIB_PATH)
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    lib.oracle_mix_csr_f32.argtypes = [vp, i64, vp, i64, i64, i64, i64, i64, vp, vp, vp, ctypes.c_int]
    lib.oracle_mix_csr_f32.restype = None
    lib.oracle_mean_rows_f32.argtypes = [vp, i64, i64, i64, vp]
    lib.oracle_mean_rows_f32.restype = None
    lib.oracle_grad_mean_f32.argtypes = [vp, i64, vp, i64, i64, i64, i64, i64, vp, vp]
    lib.oracle_grad_mean_f32.restype = None
    _c = lib
    return lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def mix_exact_c(x, row_ptr, col, val, rows=None, cols=None, average_only=False, out=None):
    """C oracle on output rows [r0, r1) and columns [c0, c1) (columns are independent)."""
    lib = c_lib()
    x = np.ascontiguousarray(x, np.float32)
    row_ptr = np.ascontiguousarray(row_ptr, np.int64)
    col = np.ascontiguousarray(col, np.int32)
    val = np.ascontiguousarray(val, np.float32)
    n = len(row_ptr) - 1
    r0, r1 = rows if rows is not None else (0, n)
    c0, c1 = cols if cols is not None else (0, x.shape[1])
    if out is None:
        out = np.zeros((n, x.shape[1]), np.float32)
    lib.oracle_mix_csr_f32(_ptr(x), x.shape[1], _ptr(out), out.shape[1], r0, r1, c0, c1,
                           _ptr(row_ptr), _ptr(col), _ptr(val), int(bool(average_only)))
    return out


def grad_mean_c(g, row_ptr, col, rows=None, cols=None, out=None):
    """C restatement of grad_mean_np on output rows [r0, r1) and columns [c0, c1)."""
    lib = c_lib()
    g = np.ascontiguousarray(g, np.float32)
    row_ptr = np.ascontiguousarray(row_ptr, np.int64)
    col = np.ascontiguousarray(col, np.int32)
    n = len(row_ptr) - 1
    r0, r1 = rows if rows is not None else (0, n)
    c0, c1 = cols if cols is not None else (0, g.shape[1])
    if out is None:
        out = np.zeros((n, g.shape[1]), np.float32)
    lib.oracle_grad_mean_f32(_ptr(g), g.shape[1], _ptr(out), out.shape[1], r0, r1, c0, c1,
                             _ptr(row_ptr), _ptr(col))
    return out


def mean_rows_c(x):
    lib = c_lib()
    x = np.ascontiguousarray(x, np.float32)
    mean = np.empty(x.shape[1], np.float32)
    lib.oracle_mean_rows_f32(_ptr(x), x.shape[1], x.shape[0], x.shape[1], _ptr(mean))
    return mean


# ------------------------------------------------------------------------------------------------
# comparisons
def bitwise_equal(a, b):
    """Bit equality, except that any NaN equals any NaN (x86 and gfx950 produce different default
    NaN payloads/signs for inf*0; the reference only guarantees NaN-ness)."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    if a.shape != b.shape:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    return np.array_equal(a.view(np.uint32)[~na], b.view(np.uint32)[~nb])


def condition_bound(x, row_ptr, col, val, cols=None):
    """(|W|^T |X|) per output element: the scale for the fast-mode tolerance:
    elementwise relative error is ill-posed under cancellation, so fast kernels are checked with
    |y - y_ref| <= rtol * (|W|^T |X|)_ij."""
    ax = np.abs(np.asarray(x, np.float32))
    av = np.abs(np.asarray(val, np.float32))
    return mix_exact_c(ax, row_ptr, col, av, cols=cols, average_only=True)


def check_tolerance(y, y_ref, bound, rtol=1e-5, cols=None):
    """True iff every finite element satisfies |y - y_ref| <= rtol*bound (+ the fp32 subnormal
    floor) and non-finite elements agree in kind.  Returns (ok, worst_ratio)."""
    y = np.asarray(y, np.float32)
    y_ref = np.asarray(y_ref, np.float32)
    if cols is not None:
        y, y_ref, bound = y[:, cols[0]:cols[1]], y_ref[:, cols[0]:cols[1]], bound[:, cols[0]:cols[1]]
    fin = np.isfinite(y_ref)
    if not np.array_equal(np.isnan(y), np.isnan(y_ref)):
        return False, float("inf")
    inf_ref = np.isinf(y_ref)
    if not np.array_equal(y[inf_ref], y_ref[inf_ref]):
        return False, float("inf")
    d = np.abs(y[fin].astype(np.float64) - y_ref[fin].astype(np.float64))
    lim = rtol * bound[fin].astype(np.float64) + 1e-38
    ratio = float(np.max(d / lim)) if d.size else 0.0
    return ratio <= 1.0, ratio * rtol


# ------------------------------------------------------------------------------------------------
# faithful restatement of the reference loop (CPU baseline, "kind": "port")
def reference_loop_average(nodes, topology):
    """d_sgd.average (d_sgd.py:96-116) as the reference runs it: for every node, deepcopy its model,
    zero it with mul_(0), add_(w*p) for self then every neighbour (W[., rank], edges order), and only
    after all averages exist, update_models (p.mul_(0.); p.add_(new)).  torch CPU, no changes."""
    import torch
    W = topology["weights"]
    edges = topology["edges"]
    with torch.no_grad():
        results = {}
        for nd in nodes:
            r = nd["rank"]
            group = [nd["model"]] + [nodes[s]["model"] for s in edges[r]]
            coeffs = [W[r, r]] + [W[s, r] for s in edges[r]]
            center = copy.deepcopy(group[0])
            for cp in center.parameters():
                cp.mul_(0)
            for mdl, w in zip(group, coeffs):
                for cp, mp in zip(center.parameters(), mdl.parameters()):
                    cp.add_(w * mp)
            results[r] = center
        for nd in nodes:
            for mp, newp in zip(nd["model"].parameters(), results[nd["rank"]].parameters()):
                mp.mul_(0.)
                mp.add_(newp)


def reference_loop_clique_gradient(nodes, cliques):
    """d_sgd.gradient with --clique-gradient and no removed edges (d_sgd.py:56-65) as the
    reference runs it, minus the optimizer steps: per clique, average_gradients (zeros_like, add_
    every member's grad, div_(len), d_sgd.py:19-27) then update_gradients on every member
    (grad.zero_(); grad.add_(mean), d_sgd.py:37-45).  torch CPU; the CPU baseline of
    bench.py --workload grad-clique."""
    import torch
    with torch.no_grad():
        for clique in cliques:
            models = [nodes[r]["model"] for r in clique]
            acc = [torch.zeros_like(q.grad.data) for q in models[0].parameters()]
            for mdl in models:
                for a, q in zip(acc, mdl.parameters()):
                    a.add_(q.grad.data)
            for a in acc:
                a.div_(len(models))
            for mdl in models:
                for a, q in zip(acc, mdl.parameters()):
                    q.grad.data.zero_()
                    q.grad.data.add_(a)
