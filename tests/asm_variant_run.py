"""One implicit residual + BSR assembly of a golden state, written to an .npz (helper of
tests/test_gpu_assembly.py, run as a subprocess so that the assembly variant the library caches from the
environment — RX_ASM_CONV, read once per process by rx_fuse_conv — can differ between runs).

usage: python tests/asm_variant_run.py CASE SPATIAL_ORDER OUT.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests.test_gpu_parity import golden, make_solver  # noqa: E402


def main():
    case, order, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    g = golden(case)
    s, (nDim, nVar, nPV, nG, ns) = make_solver(g, implicit=True, spatial_order=order)
    if "dt" in g:  # the assembly itself does not read it (AddVal2Diag comes with the implicit step)
        s.upload("DT", g["dt"])
    if order:  # the MUSCL branch reads the gradient (and, 2ND_ORDER_LIMITER, the limiter) of the state
        s.SetPrimitive_Gradient_LS()
        if order == 2:
            s.SetPrimitive_Limiter()
    s.Preprocessing_zero()
    s.Upwind_Residual()
    s.Viscous_Residual()
    s.Source_Residual()
    s.sync()
    np.savez(out, res=s.download("RES"), jac=s.download("JAC"))
    s.close()


if __name__ == "__main__":
    main()
