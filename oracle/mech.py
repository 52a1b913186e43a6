"""Mechanism / property-table reader for the ORACLE (test infrastructure only).

CPU restatement of the reference library's setup path, so that golden vectors and the oracle
are fed the exact tables the reference builds:
  * file list + mixture file  Common/src/Framework/reacting_model_library.cpp:925-1019, 1520-1586
  * chemistry file            :1024-1157 (units, CGS -> SI conversion :1122-1132, Ta / R_cal :1209-1210,
                              product exponents of reversible reactions :1113-1120)
  * reaction-string parser    Common/src/Tools/utility.cpp:12-86 (Parse_Terms)
  * backward-rate extra line  reacting_model_library.cpp:1218-1260
  * thermo / transport tables :1311-1453, spline second derivatives Common/src/Tools/spline.cpp:10-58
    (called with yp1 = ypn = 0.0, i.e. CLAMPED zero-slope ends, not natural)
Constants: Common/include/Framework/physical_chemical_library.hpp:571-579.
"""
from __future__ import annotations

import os
import string

import numpy as np

NA = 6.02214129 * 1.0e23
KB = 1.3806488 * 1.0e-23
R_UNGAS = NA * KB * 1.0e3          # J/(kmol K)
R_UNGAS_SCAL = 1.9858775           # cal/(mol K)
R_UNGAS_ATM = 1.0e-3 * 0.082057338  # m3 atm/(mol K)

# property order in the table block
PROPS = ("cp", "h", "s", "mu", "kappa")


def _valid(line):
    return bool(line) and line[0] not in string.punctuation


def _lines(path):
    with open(path) as f:
        for raw in f:
            line = raw.rstrip("\n").rstrip("\r")
            if line == "STOP":
                return
            if _valid(line):
                yield line


def set_spline(x, y, yp1=0.0, ypn=0.0):
    """Spline second derivatives, same recurrence and boundary handling as spline.cpp:10-58."""
    n = len(x)
    u = np.zeros(n)
    y2 = np.zeros(n)
    if yp1 > 0.99e30:
        y2[0] = 0.0
    else:
        y2[0] = -0.5
        u[0] = (3.0 / (x[1] - x[0])) * ((y[1] - y[0]) / (x[1] - x[0]) - yp1)
    for i in range(2, n):
        sig = (x[i - 1] - x[i - 2]) / (x[i] - x[i - 2])
        p = sig * y2[i - 2] + 2.0
        y2[i - 1] = (sig - 1.0) / p
        u[i - 1] = (y[i] - y[i - 1]) / (x[i] - x[i - 1]) - (y[i - 1] - y[i - 2]) / (x[i - 1] - x[i - 2])
        u[i - 1] = (6.0 * u[i - 1] / (x[i] - x[i - 2]) - sig * u[i - 2]) / p
    if ypn > 0.99e30:
        qn = un = 0.0
    else:
        qn = 0.5
        un = (3.0 / (x[n - 1] - x[n - 2])) * (ypn - (y[n - 1] - y[n - 2]) / (x[n - 1] - x[n - 2]))
    y2[n - 1] = (un - qn * u[n - 2]) / (qn * y2[n - 2] + 1.0)
    for k in range(n - 1, 0, -1):
        y2[k - 1] = y2[k - 1] * y2[k] + u[k - 1]
    return y2


def _parse_terms(text, r, is_rev, is_reac, names, stoich, exp_reac, exp_prod):
    """utility.cpp:12-86, iterative form of the recursive parser."""
    line = text
    while True:
        size = len(line)
        idx = 0
        while not (line[idx].isdigit() or line[idx].isalpha()):
            idx += 1
        coeff = ""
        while line[idx].isdigit() or line[idx] in string.punctuation:
            coeff += line[idx]
            idx += 1
        symbol = ""
        while True:
            while idx < size and (line[idx].isalpha() or line[idx].isdigit()):
                symbol += line[idx]
                idx += 1
            if not (idx < size and line[idx] not in string.punctuation and not line[idx].isspace() and line[idx] != "+"):
                break
        s = names[symbol]
        coefficient = float(coeff) if coeff else 1.0
        stoich[s, r] += coefficient
        exp_coeff = ""
        if idx < size and line[idx] in string.punctuation:
            idx += 1
            while idx < size and (line[idx].isdigit() or line[idx] in string.punctuation):
                exp_coeff += line[idx]
                idx += 1
        if exp_coeff:
            e = float(exp_coeff)
            if is_reac:
                exp_reac[r, s] += e
            elif is_rev:
                exp_prod[r, s] += e
        elif is_reac:
            exp_reac[r, s] += stoich[s, r]
        if idx == size:
            return
        sub = line[idx + 1:]
        if not sub:
            return
        line = sub


def load_mechanism(base_dir, list_file):
    files = list(_lines(os.path.join(base_dir, list_file)))
    # --- mixture
    mix = list(_lines(os.path.join(base_dir, files[0])))
    ns = int(mix[0].split()[0])
    names, mm, hf, dv = {}, [], [], []
    for k, line in enumerate(mix[1:1 + ns]):
        t = line.split()
        names[t[0]] = k
        mm.append(float(t[1]))
        hf.append(float(t[2]))
        dv.append(float(t[3]))
    mm = np.array(mm)
    has_chem = len(files) == 2 * ns + 2
    nr = 0
    out = {}
    if has_chem:
        chem = list(_lines(os.path.join(base_dir, files[1])))
        nr = int(chem[0].split()[0])
        cgs = chem[1].split()[0] == "CGS"
        sr = np.zeros((ns, nr)); sp = np.zeros((ns, nr))
        er = np.zeros((nr, ns)); ep = np.zeros((nr, ns))
        A = np.zeros(nr); beta = np.zeros(nr); Ta = np.zeros(nr)
        Ab = np.zeros(nr); betab = np.zeros(nr); Tab = np.zeros(nr)
        rev = np.zeros(nr, dtype=np.int64); hasb = np.zeros(nr, dtype=np.int64)
        n_line = 2
        r = -1
        for line in chem[2:]:
            if n_line % 2 == 0 and n_line < 2 * nr + 1:
                r += 1
                is_rev = "<" in line
                rev[r] = int(is_rev)
                major = line.index(">")
                if is_rev:
                    reac_side = line[:line.index("<")]
                else:
                    reac_side = line[:line.index("=")]
                prod_side = line[major + 1:]
                _parse_terms(reac_side, r, is_rev, True, names, sr, er, ep)
                _parse_terms(prod_side, r, is_rev, False, names, sp, er, ep)
            elif n_line % 2 == 1 and n_line < 2 * nr + 2:
                t = line.split()
                A[r], beta[r] = float(t[0]), float(t[1])
                Ta[r] = float(t[2]) / R_UNGAS_SCAL if cgs else float(t[2])
            else:
                key = "Available Backward Rate reaction"
                if key in line:
                    rest = line[32:]
                    rr = int(rest.split(":")[0]) - 1
                    t = rest[3:].split()
                    hasb[rr] = 1
                    Ab[rr], betab[rr] = float(t[0]), float(t[1])
                    Tab[rr] = float(t[2]) / R_UNGAS_SCAL if cgs else float(t[2])
                for key, mat in (("Extra Forward terms reaction", er), ("Extra Backward terms reaction", ep)):
                    if key in line:
                        raise NotImplementedError("extra exponent terms are not used by the shipped mechanisms")
            n_line += 1
        for rr in range(nr):
            if rev[rr] and not hasb[rr]:
                ep[rr, :] = er[rr, :] + sp[:, rr] - sr[:, rr]
        if cgs:
            for rr in range(nr):
                A[rr] *= 10.0 ** (6.0 * (1.0 - er[rr].sum()))
                if hasb[rr]:
                    Ab[rr] *= 10.0 ** (6.0 * (1.0 - ep[rr].sum()))
        out.update(stoich_reac=sr, stoich_prod=sp, exp_reac=er, exp_prod=ep, A=A, beta=beta, Ta=Ta,
                   A_back=Ab, beta_back=betab, Ta_back=Tab, reversible=rev, has_backward=hasb)
    else:  # no chemistry file (the flat plate's air): zero reactions
        z = np.zeros(0)
        out.update(stoich_reac=np.zeros((ns, 0)), stoich_prod=np.zeros((ns, 0)), exp_reac=np.zeros((0, ns)),
                   exp_prod=np.zeros((0, ns)), A=z, beta=z, Ta=z, A_back=z, beta_back=z, Ta_back=z,
                   reversible=np.zeros(0, dtype=np.int64), has_backward=np.zeros(0, dtype=np.int64))
    # --- per-species tables (transport file then thermo file for each species)
    off = 0 if has_chem else 1
    tabs = {}
    for s in range(ns):
        for kind, fname in (("transp", files[2 * s + 2 - off]), ("thermo", files[2 * s + 3 - off])):
            ls = list(_lines(os.path.join(base_dir, fname)))
            sp_idx = names[ls[0]]
            data = np.array([[float(v) for v in l.split()] for l in ls[1:]])
            if kind == "transp":
                tabs[(sp_idx, "mu")] = (data[:, 0], data[:, 1])
                tabs[(sp_idx, "kappa")] = (data[:, 0], data[:, 2])
            else:
                tabs[(sp_idx, "cp")] = (data[:, 0], data[:, 1])
                tabs[(sp_idx, "h")] = (data[:, 0], data[:, 2])
                tabs[(sp_idx, "s")] = (data[:, 0], data[:, 3])
    ntab = len(tabs[(0, "cp")][0])
    tx = np.zeros((len(PROPS), ns, ntab)); ty = np.zeros_like(tx); ty2 = np.zeros_like(tx)
    for p, prop in enumerate(PROPS):
        for s in range(ns):
            x, y = tabs[(s, prop)]
            assert len(x) == ntab
            tx[p, s] = x
            ty[p, s] = y
            ty2[p, s] = set_spline(x, y, 0.0, 0.0)
    out.update(n_species=np.array(ns), n_reactions=np.array(nr), mmass=mm, diff_vol=np.array(dv),
               form_enthalpy=np.array(hf), tab_x=tx, tab_y=ty, tab_y2=ty2,
               species=np.array(sorted(names, key=names.get)))
    return out
