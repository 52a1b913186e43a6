"""Shared parity helpers for the tests.

Tolerance: the north star asks for 1e-10 relative agreement with the reference CPU solver.
Components that are sums of cancelling terms (e.g. the density row of the viscous flux, -sum(J_s),
which is zero up to the 1e-11 Stefan-Maxwell solver tolerance) are compared relative to the
magnitude of the array block they belong to, so the bound used everywhere is
    |a - b| <= RTOL * max(|b|, FLOOR * scale)
with scale = max |b| over the compared block and FLOOR a small per-call constant.
"""
import numpy as np

RTOL = 1e-10


def rel_err(a, b, floor=1e-6, scale=None):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if scale is None:
        scale = np.max(np.abs(b)) if b.size else 1.0
    den = np.maximum(np.abs(b), floor * scale)
    den = np.where(den == 0.0, 1.0, den)
    return float(np.max(np.abs(a - b) / den)) if a.size else 0.0


def assert_close(a, b, rtol=RTOL, floor=1e-6, scale=None, what=""):
    e = rel_err(a, b, floor, scale)
    assert e <= rtol, f"{what}: max rel err {e:.3e} > {rtol:.1e}"
    return e


def per_column_close(a, b, rtol=RTOL, floor=1e-6, what=""):
    """Compare column-wise (last axis = variable), each column scaled by its own max."""
    a = np.asarray(a).reshape(-1, np.asarray(a).shape[-1])
    b = np.asarray(b).reshape(-1, np.asarray(b).shape[-1])
    worst = 0.0
    for v in range(b.shape[1]):
        worst = max(worst, assert_close(a[:, v], b[:, v], rtol, floor, what=f"{what}[var {v}]"))
    return worst


def species_close(U, Uo, nDim, rtol=RTOL, rho_floor=1e-8, what=""):
    """Species partial densities compared elementwise: |a - b| <= rtol * max(|b|, rho_floor * rho_i) at every point
    i, with rho_i the point's density (column 0 of U). A minor species at 1e-6 of its column's max is held to rtol
    of its own value, not of the column max (per_column_close). Returns the worst relative error."""
    U, Uo = np.asarray(U, dtype=np.float64), np.asarray(Uo, dtype=np.float64)
    rho = np.abs(Uo[:, 0])
    b = Uo[:, nDim + 2:]
    den = np.maximum(np.abs(b), rho_floor * rho[:, None])
    den = np.where(den == 0.0, 1.0, den)
    e = np.abs(U[:, nDim + 2:] - b) / den
    worst = float(e.max()) if e.size else 0.0
    if worst > rtol:
        i, s = np.unravel_index(int(np.argmax(e)), e.shape)
        raise AssertionError(f"{what}: species {s} at point {i}: rel err {worst:.3e} > {rtol:.1e} "
                             f"({U[i, nDim + 2 + s]!r} vs {b[i, s]!r}, rho {rho[i]!r})")
    return worst
