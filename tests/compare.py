"""Column-tolerance comparator with the semantics of the reference's
tests/difffloat.py:53-128 (which crashes under numpy 2): per column
an absolute tolerance, a relative tolerance on |a-b|/|a+b|, and a limit
below which (|a|+|b| < limit) the relative test is skipped; both tolerances
get the reference's 1.1 slack."""
from __future__ import annotations

from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / "golden"


def load_tolerance(name: str):
    path = GOLDEN / name
    header = path.read_text().splitlines()[0].lstrip("#").split()
    data = np.loadtxt(path)
    return header, data[0], data[1], data[2]


def compare_columns(a: np.ndarray, b: np.ndarray, abs_tol, rel_tol, lim_tol, names=None):
    """a, b: (n, ncol). Returns a list of violation strings (empty = pass)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape
    errs = []
    absd = np.abs(a - b)
    s = np.abs(a + b)
    rel = np.where(s > 0, absd / np.where(s > 0, s, 1), 0.0)
    for j in range(a.shape[1]):
        bad_abs = absd[:, j] > 1.1 * abs_tol[j]
        check_rel = (np.abs(a[:, j]) + np.abs(b[:, j])) >= lim_tol[j]
        bad_rel = check_rel & (rel[:, j] > 1.1 * rel_tol[j])
        for i in np.nonzero(bad_abs | bad_rel)[0][:5]:
            nm = names[j] if names else j
            errs.append(f"row {i} col {nm}: a={a[i, j]:.7e} b={b[i, j]:.7e} "
                        f"abs={absd[i, j]:.3e} rel={rel[i, j]:.3e}")
    return errs


def rel_err(a, b, floor):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.abs(a - b) / np.maximum(np.abs(b), floor)
