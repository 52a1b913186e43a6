"""Host-side Python mirror of the reactive-RANS hot path on MI355X.

The compute lives in librx.so (hand-written HIP kernels for gfx950 behind the C ABI of
include/rx.h). This module only marshals arrays through that ABI; it never computes physics and
has no CPU fallback: on a machine without a HIP device the context creation fails loudly.

The class and method names mirror the reference's CSolver / CNumerics call surface
(SU2_CFD/include/solver_reactive.hpp): Preprocessing-time fields are uploaded, then
Upwind_Residual / Viscous_Residual / Source_Residual / SetTime_Step / SetPrimitive_Gradient_LS /
SetPrimitive_Limiter / ExplicitEuler_Iteration / ImplicitEuler_Iteration run on the device.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librx.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "rx.h")

# rx_status
(RX_OK, RX_ERR_ARG, RX_ERR_HIP, RX_ERR_NAN, RX_ERR_RANGE, RX_ERR_NONPHYS, RX_ERR_DIVERGED, RX_ERR_STATE, RX_ERR_COMM,
 RX_ERR_UNSUPPORTED) = range(10)
# rx_field
FIELDS = ["U", "V", "DPDU", "DTDU", "MU", "KAPPA", "DIJ", "GRAD", "LIMITER", "TKE", "OMEGA", "MUT", "SIGMAK", "GRADK",
          "EDDY", "RES", "DT", "LAMBDA_INV", "LAMBDA_VISC", "JAC", "ILU", "SOL", "RHS", "STRAIN", "F1", "F2", "CDKW",
          "WALLDIST"]
F = {name: k for k, name in enumerate(FIELDS)}
# rx_kernel
KERNELS = ["CONV", "VISC", "SOURCE", "GRAD", "LIMITER", "DT", "SPMV", "ILU_BUILD", "ILU_APPLY", "LUSGS", "KRYLOV",
           "UPDATE", "SOLVE", "VISC_JAC", "ASSEMBLE", "STRAIN", "PRIMITIVE", "SST_GRAD", "SST_UPW", "SST_VISC", "SST_SOURCE",
           "SST_SYSTEM", "SST_SOLVE", "SST_POST", "BC", "SST_BC"]
K = {name: k for k, name in enumerate(KERNELS)}


class RxError(RuntimeError):
    """A failed rx_* call: status = the rx_status code, index = rx_last_error_index (the first offending point /
    edge a kernel flagged, -1 if none)."""

    def __init__(self, msg, status=None, index=-1):
        super().__init__(msg)
        self.status = status
        self.index = index


class MechDesc(C.Structure):
    _fields_ = [("n_species", C.c_int32), ("n_reactions", C.c_int32), ("n_tab", C.c_int32),
                ("mmass", C.c_void_p), ("diff_vol", C.c_void_p),
                ("stoich_reac", C.c_void_p), ("stoich_prod", C.c_void_p),
                ("exp_reac", C.c_void_p), ("exp_prod", C.c_void_p),
                ("A", C.c_void_p), ("beta", C.c_void_p), ("Ta", C.c_void_p),
                ("A_back", C.c_void_p), ("beta_back", C.c_void_p), ("Ta_back", C.c_void_p),
                ("reversible", C.c_void_p), ("has_backward", C.c_void_p),
                ("tab_x", C.c_void_p), ("tab_y", C.c_void_p), ("tab_y2", C.c_void_p)]


class MeshDesc(C.Structure):
    _fields_ = [("n_dim", C.c_int32), ("n_point", C.c_int64), ("n_edge", C.c_int64), ("n_bvert", C.c_int64),
                ("edges", C.c_void_p), ("edge_normal", C.c_void_p), ("coord", C.c_void_p), ("volume", C.c_void_p),
                ("nbr_ptr", C.c_void_p), ("nbr", C.c_void_p), ("bvert", C.c_void_p), ("bvert_normal", C.c_void_p),
                ("n_part", C.c_int64), ("part_ptr", C.c_void_p),
                ("n_domain", C.c_int64), ("n_neigh", C.c_int32), ("neigh", C.c_void_p), ("send_ptr", C.c_void_p),
                ("send_idx", C.c_void_p), ("recv_ptr", C.c_void_p), ("global_id", C.c_void_p)]


SENDRECV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int64),
                          C.POINTER(C.c_double), C.POINTER(C.c_int64), C.POINTER(C.c_double), C.c_int32)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int32)


class HostComm(C.Structure):
    """rx_host_comm: the host-staged transport (the reference's MPI SendReceive / Allreduce pattern)."""
    _fields_ = [("user", C.c_void_p), ("sendrecv", SENDRECV_FN), ("allreduce", ALLREDUCE_FN)]


class Cfg(C.Structure):
    _fields_ = [("mach_inf", C.c_double), ("T_ref", C.c_double), ("E_ref", C.c_double), ("R_ref", C.c_double),
                ("rho_ref", C.c_double), ("t_ref", C.c_double), ("prandtl_lam", C.c_double),
                ("prandtl_turb", C.c_double), ("lewis_turb", C.c_double), ("c_mu", C.c_double),
                ("pasr_lb", C.c_double), ("cfl", C.c_double), ("max_delta_time", C.c_double),
                ("ref_elem_length", C.c_double), ("limiter_coeff", C.c_double), ("lin_tol", C.c_double),
                ("relaxation", C.c_double), ("implicit", C.c_int32), ("rans", C.c_int32), ("lin_iter", C.c_int32),
                ("lin_prec", C.c_int32), ("spatial_order", C.c_int32), ("clip_temp", C.c_int32),
                ("t_min", C.c_double), ("t_max", C.c_double), ("p_ref", C.c_double), ("visc_ref", C.c_double),
                ("cond_ref", C.c_double), ("vel_ref", C.c_double), ("len_ref", C.c_double),
                ("slope_limiter", C.c_int32), ("ignition", C.c_int32), ("fuel_index", C.c_int32),
                ("oxidizer_index", C.c_int32), ("ignition_iter", C.c_int64), ("ignition_temp", C.c_double),
                ("grad_method", C.c_int32), ("lin_solver", C.c_int32), ("lin_restart", C.c_int32)]

# rx_lin_prec / rx_lin_solver (include/rx.h): LINEAR_SOLVER_PREC and LINEAR_SOLVER
PREC_LU_SGS, PREC_ILU, PREC_JACOBI = 0, 1, 2
LIN_FGMRES, LIN_BCGSTAB, LIN_RESTARTED_FGMRES, LIN_SMOOTHER_LUSGS, LIN_SMOOTHER_JACOBI, LIN_SMOOTHER_ILU = range(6)


class BcDesc(C.Structure):
    """rx_bc_desc: boundary markers of Space_Integration (next-3)."""
    _fields_ = [("n_marker", C.c_int32), ("kind", C.c_void_p), ("data", C.c_void_p), ("normal_neighbor", C.c_void_p),
                ("inlet_kind", C.c_int32), ("tke_inf", C.c_double), ("kine_inf", C.c_double),
                ("omega_inf", C.c_double)]


ERR_PHASE_CALL, ERR_PHASE_UPWIND = 0, 1  # rx_err_phase (rx_last_error_phase)
LIMITER_VENKATAKRISHNAN, LIMITER_BARTH_JESPERSEN = 0, 1  # rx_slope_limiter

BC_NONE, BC_INLET, BC_OUTLET, BC_ISOTHERMAL, BC_HEATFLUX, BC_EULER, BC_SUP_INLET, BC_SUP_OUTLET = range(8)
EULER_WALL_ENUM = 1  # the reference's BC_TYPE value of EULER_WALL (Common/include/option_structure.hpp:750)
INLET_TOTAL_CONDITIONS, INLET_MASS_FLOW, INLET_TEMPERATURE_IMPOSE = 0, 1, 2


def bc_from_reference(bc_marker, bc_params, normal_neighbor):
    """rx_bc_desc inputs from the reference's marker table (oracle/ref_harness bc_marker / bc_params: rows
    [KindBC, a, b, dir[3], Y[Ns]]; bc_params[11:18] = the reference's INLET_FLOW, OUTLET_FLOW, ISOTHERMAL,
    HEAT_FLUX, TOTAL_CONDITIONS, MASS_FLOW, TEMPERATURE_IMPOSE enum values, bc_params[27] EULER_WALL,
    bc_params[28:30] SUPERSONIC_INLET / SUPERSONIC_OUTLET). Other marker kinds (SYMMETRY_PLANE) map to BC_NONE."""
    p = np.asarray(bc_params, dtype=np.float64)
    k_in, k_out, k_iso, k_hf, k_tot, k_mf, k_ti = (int(x) for x in p[11:18])
    k_eu = int(p[27]) if len(p) > 27 else EULER_WALL_ENUM
    kmap = {k_in: BC_INLET, k_out: BC_OUTLET, k_iso: BC_ISOTHERMAL, k_hf: BC_HEATFLUX, k_eu: BC_EULER}
    if len(p) > 29:
        kmap.update({int(p[28]): BC_SUP_INLET, int(p[29]): BC_SUP_OUTLET})
    md = np.ascontiguousarray(bc_marker, dtype=np.float64)
    kinds = np.array([kmap.get(int(k), BC_NONE) for k in md[:, 0]], dtype=np.int32)
    inlet = {k_tot: INLET_TOTAL_CONDITIONS, k_mf: INLET_MASS_FLOW, k_ti: INLET_TEMPERATURE_IMPOSE}[int(p[0])]
    return dict(kind=kinds, data=md, normal_neighbor=np.ascontiguousarray(normal_neighbor, dtype=np.int64),
                inlet_kind=inlet, tke_inf=float(p[1]), kine_inf=float(p[2]), omega_inf=float(p[3]))


_lib = None


def build():
    """Compile librx.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-j4", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        # RX_LIB: an in-tree build variant of librx.so for same-box A/B measurements (tools/gpu_ab.sh)
        path = os.environ.get("RX_LIB", LIB_PATH)
        if not os.path.exists(path):
            raise RxError(f"librx.so not built ({path}); run __graft_entry__.build()")
        _lib = C.CDLL(path)
        _lib.rx_status_string.restype = C.c_char_p
        _lib.rx_last_error_index.restype = C.c_int64
        _lib.rx_ctx_create.argtypes = [C.POINTER(MeshDesc), C.POINTER(MechDesc), C.POINTER(Cfg), C.c_int,
                                       C.POINTER(C.c_void_p)]
        for name in ("rx_ctx_destroy", "rx_sync", "rx_residual_zero", "rx_edge_flux_conv", "rx_edge_flux_visc",
                     "rx_cell_source_pasr", "rx_grad_lsq", "rx_grad_gg", "rx_limiter_venkat", "rx_time_step", "rx_ilu0_build"):
            getattr(_lib, name).argtypes = [C.c_void_p]
        _lib.rx_upload.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int64]
        _lib.rx_download.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int64]
        _lib.rx_field_size.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int64)]
        _lib.rx_bsr_pattern.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        _lib.rx_bsr_spmv.argtypes = [C.c_void_p, C.c_int, C.c_int]
        _lib.rx_ilu0_apply.argtypes = [C.c_void_p, C.c_int, C.c_int]
        _lib.rx_lusgs_apply.argtypes = [C.c_void_p, C.c_int, C.c_int]
        _lib.rx_fgmres.argtypes = [C.c_void_p, C.c_double, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_double)]
        if hasattr(_lib, "rx_linear_solve"):  # an RX_LIB A/B variant built before it may lack it
            _lib.rx_linear_solve.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_double)]
        if hasattr(_lib, "rx_set_system_fold"):  # (an RX_LIB A/B variant built before round 5's cycle v lacks it)
            _lib.rx_set_system_fold.argtypes = [C.c_void_p, C.c_int]
        _lib.rx_explicit_euler.argtypes = [C.c_void_p, C.c_void_p]
        _lib.rx_implicit_euler.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]
        _lib.rx_explicit_rk.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_void_p]
        _lib.rx_set_primitive.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int64)]
        _lib.rx_profile_enable.argtypes = [C.c_void_p, C.c_int]
        _lib.rx_profile_read.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int64)]
        _lib.rx_last_error_index.argtypes = [C.c_void_p]
        if hasattr(_lib, "rx_last_error_phase"):
            _lib.rx_last_error_phase.argtypes = [C.c_void_p]
        _lib.rx_comm_unique_id.argtypes = [C.c_void_p]
        _lib.rx_comm_init.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        _lib.rx_comm_init_host.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(HostComm)]
        _lib.rx_halo_exchange.argtypes = [C.c_void_p, C.c_int]
        _lib.rx_sst_create.argtypes = [C.POINTER(MeshDesc), C.c_void_p, C.POINTER(Cfg), C.POINTER(C.c_void_p)]
        for name in ("rx_strain_mag", "rx_sst_preprocessing", "rx_sst_upwind", "rx_sst_viscous", "rx_sst_source",
                     "rx_sst_postprocessing"):
            getattr(_lib, name).argtypes = [C.c_void_p]
        _lib.rx_sst_implicit_euler.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]
        _lib.rx_bc_set.argtypes = [C.c_void_p, C.POINTER(BcDesc)]
        _lib.rx_bc_flow.argtypes = [C.c_void_p]
        _lib.rx_bc_sst.argtypes = [C.c_void_p]
        # rx_io.h (host-side setup and file formats)
        _lib.rx_mesh_read_su2.argtypes = [C.c_char_p, C.POINTER(C.c_void_p)]
        _lib.rx_mesh_destroy.argtypes = [C.c_void_p]
        _lib.rx_mesh_destroy.restype = None
        _lib.rx_mesh_info.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                      C.POINTER(C.c_int64), C.POINTER(C.c_int32)]
        _lib.rx_mesh_marker_tag.argtypes = [C.c_void_p, C.c_int32]
        _lib.rx_mesh_marker_tag.restype = C.c_char_p
        _lib.rx_mesh_describe.argtypes = [C.c_void_p, C.POINTER(MeshDesc)]
        for name in ("rx_mesh_global_index", "rx_mesh_normal_neighbor"):
            getattr(_lib, name).argtypes = [C.c_void_p]
            getattr(_lib, name).restype = C.POINTER(C.c_int64)
        _lib.rx_mesh_wall_distance.argtypes = [C.c_void_p, C.c_void_p]
        _lib.rx_mesh_wall_distance.restype = C.POINTER(C.c_double)
        _lib.rx_mech_read.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_void_p)]
        _lib.rx_mech_destroy.argtypes = [C.c_void_p]
        _lib.rx_mech_destroy.restype = None
        _lib.rx_mech_describe.argtypes = [C.c_void_p, C.POINTER(MechDesc)]
        _lib.rx_mech_species.argtypes = [C.c_void_p, C.c_int32]
        _lib.rx_mech_species.restype = C.c_char_p
        _lib.rx_mech_formation_enthalpy.argtypes = [C.c_void_p, C.c_int32]
        _lib.rx_mech_formation_enthalpy.restype = C.c_double
        _lib.rx_restart_write.argtypes = [C.c_char_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_int64]
        _lib.rx_restart_read.argtypes = [C.c_char_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
        _lib.rx_cfg_default.argtypes = [C.POINTER(Cfg)]
        _lib.rx_cfg_default.restype = None
        _lib.rx_case_read.argtypes = [C.c_char_p, C.POINTER(C.c_void_p)]
        _lib.rx_case_destroy.argtypes = [C.c_void_p]
        _lib.rx_case_destroy.restype = None
        _lib.rx_case_error.restype = C.c_char_p
        for name in ("rx_case_mesh", "rx_case_mech"):
            getattr(_lib, name).argtypes = [C.c_void_p]
            getattr(_lib, name).restype = C.c_void_p
        _lib.rx_case_cfg.argtypes = [C.c_void_p, C.POINTER(Cfg), C.POINTER(Cfg)]
        _lib.rx_case_bc.argtypes = [C.c_void_p, C.POINTER(BcDesc)]
        _lib.rx_case_rk.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.POINTER(C.c_double))]
        _lib.rx_case_free_stream.argtypes = [C.c_void_p] + [C.POINTER(C.c_double)] * 4
    return _lib


def comm_unique_id() -> bytes:
    """ncclGetUniqueId (128 bytes) for rx_comm_init; create on one rank and broadcast."""
    buf = C.create_string_buffer(128)
    _chk(lib().rx_comm_unique_id(buf), "rx_comm_unique_id")
    return buf.raw


class TorchHostTransport:
    """rx_host_comm over torch.distributed point-to-point and all_gather (gloo on CPU tensors): the
    reference's MPI_Isend/Irecv halo exchange and MPI_Allreduce (as a rank-ordered sum), for ranks that cannot
    share RCCL (several ranks on one GPU, CPU-side validation)."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.error = None

        def sendrecv(user, n_neigh, neigh, send_ptr, send, recv_ptr, recv, stride):
            try:
                reqs = []
                for k in range(n_neigh):
                    s0, s1 = send_ptr[k] * stride, send_ptr[k + 1] * stride
                    r0, r1 = recv_ptr[k] * stride, recv_ptr[k + 1] * stride
                    if s1 > s0:
                        sb = torch.from_numpy(np.ctypeslib.as_array(send, shape=(s1,))[s0:s1])
                        reqs.append(dist.isend(sb, int(neigh[k]), group=self.group))
                    if r1 > r0:
                        rb = torch.from_numpy(np.ctypeslib.as_array(recv, shape=(r1,))[r0:r1])
                        reqs.append(dist.irecv(rb, int(neigh[k]), group=self.group))
                for r in reqs:
                    r.wait()
                return 0
            except Exception as e:  # surfaced as RX_ERR_COMM
                self.error = e
                return 1

        def allreduce(user, inp, out, count):
            # rx_host_comm's contract: the rank-ordered sum (all-gather, then ((in_0 + in_1) + in_2) + ...)
            try:
                t = torch.from_numpy(np.ctypeslib.as_array(inp, shape=(count,)).copy())
                parts = [torch.empty_like(t) for _ in range(dist.get_world_size(group=self.group))]
                dist.all_gather(parts, t, group=self.group)
                acc = parts[0].numpy().copy()
                for p in parts[1:]:
                    acc += p.numpy()
                np.ctypeslib.as_array(out, shape=(count,))[:] = acc
                return 0
            except Exception as e:
                self.error = e
                return 1

        self._cb = (SENDRECV_FN(sendrecv), ALLREDUCE_FN(allreduce))  # keep alive
        self.desc = HostComm(None, self._cb[0], self._cb[1])


def header_symbols():
    """Function names declared in include/rx.h and include/rx_io.h (the ABI contract)."""
    import re
    out = set()
    for h in (HEADER, os.path.join(os.path.dirname(HEADER), "rx_io.h")):
        txt = open(h).read()
        out |= set(re.findall(r"^\s*(?:int|int64_t|void|double|const char \*|const int64_t \*|const double \*)\s*"
                              r"(rx_[a-z0-9_]+)\s*\(", txt, re.M))
    return sorted(out)


def _chk(rc, what, ctx=None):
    if rc != RX_OK:
        msg = lib().rx_status_string(rc).decode()
        idx = lib().rx_last_error_index(ctx) if ctx is not None else -1
        if rc == RX_ERR_NAN and ctx is not None and lib().rx_last_error_phase(ctx) == ERR_PHASE_UPWIND:
            # the implicit AUSM pass runs inside the 2-D node-centric assembly: the reference's upwind loop error
            what, msg = "Upwind_Residual", "NaN found in the upwind residual"
        raise RxError(f"{what}: {msg} (status {rc}, index {idx})", status=rc, index=idx)


class Mechanism:
    """Flat mechanism arrays (same keys as oracle/mech.py / the golden files' mech_* arrays)."""

    def __init__(self, arrays, prefix="mech_"):
        g = {k[len(prefix):]: arrays[k] for k in arrays if k.startswith(prefix)}
        f8 = lambda k: np.ascontiguousarray(g[k], dtype=np.float64)
        i4 = lambda k: np.ascontiguousarray(g[k], dtype=np.int32)
        self.ns = int(g["n_species"])
        self.nr = int(g["n_reactions"])
        self.ntab = int(g["tab_x"].shape[2])
        self._keep = {k: f8(k) for k in ("mmass", "diff_vol", "stoich_reac", "stoich_prod", "exp_reac", "exp_prod",
                                         "A", "beta", "Ta", "A_back", "beta_back", "Ta_back", "tab_x", "tab_y",
                                         "tab_y2")}
        self._keep["reversible"] = i4("reversible")
        self._keep["has_backward"] = i4("has_backward")
        d = MechDesc()
        d.n_species, d.n_reactions, d.n_tab = self.ns, self.nr, self.ntab
        for k, v in self._keep.items():
            setattr(d, k, v.ctypes.data)
        self.desc = d


# The flow CFL of the bench's implicit step (and of default_cfg): the largest CFL at which the reference itself and
# the restatement agree to 1e-10 on the bench state AND FGMRES(5)+ILU(0) actually reduces the residual
# (oracle/calibrate_cfl.py -> profiles/r05_calibration_c2.json, reference compiled here, serial ILU(0), 500 x 200
# jet, 7 species; C3 2000 x 500: profiles/r05_calibration_c3.json): CFL 0.1 (the reference cfg's,
# my_combustion_second_chem_PaSR.cfg:120) 2e-16 with the solve converged in 3 iterations (|b - Ax|/|b| 1.5e-7);
# CFL 1 4e-16, 5 iterations, |b - Ax|/|b| 1.4e-2; CFL 2 6e-12 but 0.94; CFL 5 (rounds 1-4) 6e-4 and 0.99999925 —
# the ILU(0) of that state is numerically singular (profiles/r04_calibration_c2b.json) and the solve is rounding
# noise.
BENCH_CFL = 1.0


def default_cfg(**kw):
    c = dict(mach_inf=0.01819, T_ref=1.0, E_ref=1.0, R_ref=1.0, rho_ref=1.0, t_ref=1.0, prandtl_lam=0.72,
             prandtl_turb=0.9, lewis_turb=1.2, c_mu=0.09, pasr_lb=0.2, cfl=BENCH_CFL, max_delta_time=1e6,
             ref_elem_length=0.1, limiter_coeff=0.5, lin_tol=1e-6, relaxation=1.0, implicit=1, rans=1, lin_iter=5,
             lin_prec=1, spatial_order=0, clip_temp=0, t_min=200.0, t_max=6000.0, p_ref=1.0, visc_ref=1.0,
             cond_ref=1.0, vel_ref=1.0, len_ref=1.0, slope_limiter=0,
             # CConfig defaults (config_structure.cpp:591-603)
             ignition=0, fuel_index=0, oxidizer_index=2, ignition_iter=999999, ignition_temp=1700.0,
             grad_method=0,  # NUM_METHOD_GRAD: 0 WEIGHTED_LEAST_SQUARES, 1 GREEN_GAUSS
             lin_solver=0, lin_restart=10)  # LINEAR_SOLVER (LIN_*), LINEAR_SOLVER_RESTART_FREQUENCY
    c.update(kw)
    cfg = Cfg()
    for k, v in c.items():
        setattr(cfg, k, v)
    return cfg


def mesh_desc(mesh):
    """rx_mesh_desc over contiguous copies of the mesh arrays (kept alive by the returned dict)."""
    nDim = int(mesh.get("n_dim", np.shape(mesh["coord"])[1]))
    keep = {
        "edges": np.ascontiguousarray(mesh["edges"], dtype=np.int64),
        "edge_normal": np.ascontiguousarray(mesh["edge_normal"], dtype=np.float64),
        "coord": np.ascontiguousarray(mesh["coord"], dtype=np.float64),
        "volume": np.ascontiguousarray(mesh["volume"], dtype=np.float64),
        "nbr_ptr": np.ascontiguousarray(mesh["nbr_ptr"], dtype=np.int64),
        "nbr": np.ascontiguousarray(mesh["nbr"], dtype=np.int64),
        "bvert": np.ascontiguousarray(np.asarray(mesh["bvertex"])[:, :2], dtype=np.int64),
        "bvert_normal": np.ascontiguousarray(mesh["bvertex_normal"], dtype=np.float64),
    }
    pp = mesh.get("part_ptr")
    if pp is not None and len(pp) > 2:
        keep["part_ptr"] = np.ascontiguousarray(pp, dtype=np.int64)
    N = len(keep["coord"])
    if "n_domain" in mesh:
        keep["neigh"] = np.ascontiguousarray(mesh["neigh"], dtype=np.int32)
        for k in ("send_ptr", "send_idx", "recv_ptr"):
            keep[k] = np.ascontiguousarray(mesh[k], dtype=np.int64)
        if "l2g" in mesh:  # meshgen.shard: BSR rows in global column order (rx_mesh_desc.global_id)
            keep["global_id"] = np.ascontiguousarray(mesh["l2g"], dtype=np.int64)
    md = MeshDesc()
    md.n_dim, md.n_point, md.n_edge = nDim, N, len(keep["edges"])
    md.n_bvert = len(keep["bvert"])
    md.n_part = len(keep["part_ptr"]) - 1 if "part_ptr" in keep else 0
    if "n_domain" in mesh:
        md.n_domain = int(mesh["n_domain"])
        md.n_neigh = len(keep["neigh"])
    for k, v in keep.items():
        setattr(md, k, v.ctypes.data)
    return keep, md


class ReactiveNSSolver:
    """Device-resident reactive NS + SST flow state with the reference's per-phase entry points."""

    def __init__(self, mesh, mech: Mechanism, cfg: Cfg, device=0):
        self.mech = mech
        self.cfg = cfg
        self.nDim = int(mesh.get("n_dim", np.shape(mesh["coord"])[1]))
        self.N = int(len(mesh["coord"]))
        self.E = int(len(mesh["edges"]))
        self.nVar = mech.ns + self.nDim + 2
        self._mesh_keep, md = mesh_desc(mesh)
        self.n_part = md.n_part if md.n_part > 0 else 1
        self.Nd = int(mesh.get("n_domain", self.N))
        h = C.c_void_p()
        _chk(lib().rx_ctx_create(C.byref(md), C.byref(mech.desc), C.byref(cfg), device, C.byref(h)), "rx_ctx_create")
        self.h = h
        self._mesh_keep = None
        self._children = []

    # ---- distributed (one rank per GPU)
    def comm_init(self, nranks, rank, uid: bytes):
        """Attach an RCCL communicator (uid from comm_unique_id() on one rank)."""
        buf = C.create_string_buffer(uid, 128)
        _chk(lib().rx_comm_init(self.h, nranks, rank, buf), "rx_comm_init", self.h)

    def comm_init_host(self, nranks, rank, transport):
        """Attach a host-staged transport (e.g. TorchHostTransport over gloo)."""
        self._transport = transport
        _chk(lib().rx_comm_init_host(self.h, nranks, rank, C.byref(transport.desc)), "rx_comm_init_host", self.h)

    def halo_exchange(self, field):
        _chk(lib().rx_halo_exchange(self.h, F[field]), f"rx_halo_exchange({field})", self.h)

    def close(self):
        for c in getattr(self, "_children", []):
            c.close()
        if getattr(self, "h", None):
            lib().rx_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- fields
    def size(self, field):
        n = C.c_int64()
        _chk(lib().rx_field_size(self.h, F[field], C.byref(n)), "rx_field_size")
        return n.value

    def upload(self, field, arr):
        a = np.ascontiguousarray(arr, dtype=np.float64).ravel()
        _chk(lib().rx_upload(self.h, F[field], a.ctypes.data, a.size), f"rx_upload({field})", self.h)

    def download(self, field):
        n = self.size(field)
        a = np.empty(n, dtype=np.float64)
        _chk(lib().rx_download(self.h, F[field], a.ctypes.data, n), f"rx_download({field})", self.h)
        return a

    def bsr_pattern(self):
        rp = np.empty(self.N + 1, dtype=np.int64)
        lib().rx_bsr_pattern(self.h, rp.ctypes.data, None)
        col = np.empty(int(rp[-1]), dtype=np.int64)
        lib().rx_bsr_pattern(self.h, None, col.ctypes.data)
        return rp, col

    def set_state(self, st):
        """Upload the node state produced by Preprocessing (primitives, transport, SST fields)."""
        for key, field in (("V", "V"), ("dPdU", "DPDU"), ("dTdU", "DTDU"), ("mu", "MU"), ("kappa", "KAPPA"),
                           ("Dij", "DIJ"), ("grad_prim", "GRAD"), ("turb_k", "TKE"), ("turb_omega", "OMEGA"),
                           ("mu_t", "MUT"), ("sigma_k", "SIGMAK"), ("grad_k", "GRADK"), ("eddy_visc_flow", "EDDY"),
                           ("U", "U")):
            if key in st:
                self.upload(field, st[key])

    # ---- phases (reference CSolver names)
    def _call(self, name, *args):
        _chk(getattr(lib(), name)(self.h, *args), name, self.h)

    def Preprocessing_zero(self):
        self._call("rx_residual_zero")

    def Upwind_Residual(self):
        self._call("rx_edge_flux_conv")

    def Viscous_Residual(self):
        self._call("rx_edge_flux_visc")

    def Source_Residual(self):
        self._call("rx_cell_source_pasr")

    def SetPrimitive_Gradient_LS(self):
        self._call("rx_grad_lsq")

    def SetPrimitive_Gradient_GG(self):
        """CReactiveNSSolver::SetPrimitive_Gradient_GG (solver_direct_reactive.cpp:4784-4880)."""
        self._call("rx_grad_gg")

    def SetPrimitive_Gradient(self):
        """The primitive gradient of NUM_METHOD_GRAD (CReactiveNSSolver::Preprocessing, solver_direct_reactive.cpp:
        4714-4718)."""
        if self.cfg.grad_method == 1:
            self.SetPrimitive_Gradient_GG()
        else:
            self.SetPrimitive_Gradient_LS()

    def SetPrimitive_Limiter(self):
        self._call("rx_limiter_venkat")

    def SetTime_Step(self):
        self._call("rx_time_step")

    def SetStrainMag(self):
        self._call("rx_strain_mag")

    def SetPrimitive_Variables(self, ext_iter=0, count=False):
        """Cons2Prim + transport on the device; returns the non-physical count when count=True (syncs)."""
        n = C.c_int64(0)
        _chk(lib().rx_set_primitive(self.h, int(ext_iter), C.byref(n) if count else None), "rx_set_primitive",
             self.h)
        return n.value if count else None

    def set_bc(self, bc):
        """Boundary markers (dict from bc_from_reference or the same keys)."""
        keep = dict(kind=np.ascontiguousarray(bc["kind"], dtype=np.int32),
                    data=np.ascontiguousarray(bc["data"], dtype=np.float64),
                    nn=np.ascontiguousarray(bc["normal_neighbor"], dtype=np.int64))
        d = BcDesc(len(keep["kind"]), keep["kind"].ctypes.data, keep["data"].ctypes.data, keep["nn"].ctypes.data,
                   int(bc["inlet_kind"]), float(bc.get("tke_inf", 0.0)), float(bc.get("kine_inf", 0.0)),
                   float(bc.get("omega_inf", 0.0)))
        _chk(lib().rx_bc_set(self.h, C.byref(d)), "rx_bc_set", self.h)

    def BC(self):
        """Space_Integration's boundary-condition loops (weak markers, then strong)."""
        self._call("rx_bc_flow")

    def sync(self):
        self._call("rx_sync")

    def spmv(self, x="RHS", y="SOL"):
        self._call("rx_bsr_spmv", F[x], F[y])

    def ilu0_build(self):
        self._call("rx_ilu0_build")

    def ilu0_apply(self, b="RHS", x="SOL"):
        self._call("rx_ilu0_apply", F[b], F[x])

    def lusgs_apply(self, b="RHS", x="SOL"):
        self._call("rx_lusgs_apply", F[b], F[x])

    def fgmres(self, tol=None, m=None):
        it = C.c_int()
        res = C.c_double()
        tol = self.cfg.lin_tol if tol is None else tol
        m = self.cfg.lin_iter if m is None else m
        _chk(lib().rx_fgmres(self.h, tol, m, C.byref(it), C.byref(res)), "rx_fgmres", self.h)
        return it.value, res.value

    def linear_solve(self):
        """CSysSolve::Solve on JAC * SOL = RHS with the cfg's LINEAR_SOLVER / _PREC / _ERROR / _ITER /
        _RESTART_FREQUENCY (rx_linear_solve) -> (iterations, residual norm)."""
        it = C.c_int()
        res = C.c_double()
        _chk(lib().rx_linear_solve(self.h, C.byref(it), C.byref(res)), "rx_linear_solve", self.h)
        return it.value, res.value

    def ExplicitEuler_Iteration(self):
        rms = np.zeros(self.nVar)
        _chk(lib().rx_explicit_euler(self.h, rms.ctypes.data), "rx_explicit_euler", self.h)
        return rms

    def ExplicitRK_Iteration(self, rk_step, alpha):
        rms = np.zeros(self.nVar)
        _chk(lib().rx_explicit_rk(self.h, int(rk_step), float(alpha), rms.ctypes.data), "rx_explicit_rk", self.h)
        return rms

    def ImplicitEuler_Iteration(self):
        rms = np.zeros(self.nVar)
        it = C.c_int()
        _chk(lib().rx_implicit_euler(self.h, rms.ctypes.data, C.byref(it)), "rx_implicit_euler", self.h)
        return rms, it.value

    def profile(self, on=True):
        _chk(lib().rx_profile_enable(self.h, int(on)), "rx_profile_enable")

    def profile_read(self, kernel):
        ms = C.c_double()
        n = C.c_int64()
        lib().rx_profile_read(self.h, K[kernel], C.byref(ms), C.byref(n))
        return ms.value, n.value


def sst_cfg(implicit=1, lin_tol=1e-6, lin_iter=5, lin_prec=1, relaxation_turb=1.0, cfl_red_turb=1.0, grad_method=0,
            spatial_order=0, slope_limiter=0, ref_elem_length=0.1, limiter_coeff=0.5, lin_solver=0, lin_restart=10):
    """rx_cfg for the SST context: RELAXATION_FACTOR_TURB -> relaxation, CFL_REDUCTION_TURB -> cfl, NUM_METHOD_GRAD
    -> grad_method, SPATIAL_ORDER_TURB -> spatial_order (0 1ST_ORDER, 1 2ND_ORDER, 2 2ND_ORDER_LIMITER),
    SLOPE_LIMITER_TURB -> slope_limiter, REF_ELEM_LENGTH / LIMITER_COEFF (the flow's); LINEAR_SOLVER /
    LINEAR_SOLVER_RESTART_FREQUENCY are the flow's (one System.Solve config)."""
    return default_cfg(implicit=implicit, lin_tol=lin_tol, lin_iter=lin_iter, lin_prec=lin_prec,
                       relaxation=relaxation_turb, cfl=cfl_red_turb, grad_method=grad_method,
                       spatial_order=spatial_order, slope_limiter=slope_limiter, ref_elem_length=ref_elem_length,
                       limiter_coeff=limiter_coeff, lin_solver=lin_solver, lin_restart=lin_restart)


class TurbSSTSolver:
    """Device-resident Menter SST solver (CTurbSSTSolver / CTurbSolver surface) bound to a flow solver:
    a second context (k, omega) on the flow context's stream, reading the flow's primitives, laminar and
    eddy viscosity, primitive gradient, StrainMag and time step, and writing back the turbulent fields the
    flow's viscous flux reads (TKE, OMEGA, MUT, GRADK, SIGMAK, EDDY) in Postprocessing."""

    def __init__(self, mesh, flow: ReactiveNSSolver, cfg: Cfg):
        self.flow = flow
        self.cfg = cfg
        self.N, self.nDim, self.nVar = flow.N, flow.nDim, 2
        keep, md = mesh_desc(mesh)
        h = C.c_void_p()
        _chk(lib().rx_sst_create(C.byref(md), flow.h, C.byref(cfg), C.byref(h)), "rx_sst_create")
        self.h = h
        flow._children.append(self)

    def close(self):
        if getattr(self, "h", None):
            lib().rx_ctx_destroy(self.h)
            self.h = None

    size = ReactiveNSSolver.size
    upload = ReactiveNSSolver.upload
    download = ReactiveNSSolver.download
    _call = ReactiveNSSolver._call
    sync = ReactiveNSSolver.sync
    profile = ReactiveNSSolver.profile
    profile_read = ReactiveNSSolver.profile_read
    ilu0_build = ReactiveNSSolver.ilu0_build
    ilu0_apply = ReactiveNSSolver.ilu0_apply

    def set_state(self, T, wall_distance, F1=None, F2=None, CDkw=None):
        self.upload("U", T)
        self.upload("WALLDIST", wall_distance)
        for k, v in (("F1", F1), ("F2", F2), ("CDKW", CDkw)):
            if v is not None:
                self.upload(k, v)

    def Preprocessing(self):
        self._call("rx_sst_preprocessing")

    def Upwind_Residual(self):
        self._call("rx_sst_upwind")

    def Viscous_Residual(self):
        self._call("rx_sst_viscous")

    def Source_Residual(self):
        self._call("rx_sst_source")

    def ImplicitEuler_Iteration(self):
        rms = np.zeros(2)
        it = C.c_int()
        _chk(lib().rx_sst_implicit_euler(self.h, rms.ctypes.data, C.byref(it)), "rx_sst_implicit_euler", self.h)
        return rms, it.value

    def Postprocessing(self):
        self._call("rx_sst_postprocessing")

    def BC(self):
        """The SST boundary-condition loops (after the flow's BC of the same iteration)."""
        self._call("rx_bc_sst")


class SU2Mesh:
    """A mesh read by the reference's SU2 reader and dual-grid preprocessing, restated natively (rx_io.h
    rx_mesh_read_su2: connectivity, RCM ordering, edges, median dual, boundary vertices, normal neighbours).
    mesh() gives the dict ReactiveNSSolver / TurbSSTSolver take; is_wall marks the HEAT_FLUX / ISOTHERMAL markers
    for the wall distance."""

    def __init__(self, path=None, walls=(), handle=None, owner=None):
        """path: read the file; handle: an rx_mesh owned by `owner` (an rx_case), borrowed, never destroyed here."""
        self._owner = owner
        if handle is not None:
            h = C.c_void_p(handle)
            self._borrowed = True
        else:
            h = C.c_void_p()
            _chk(lib().rx_mesh_read_su2(os.fsencode(path), C.byref(h)), f"rx_mesh_read_su2({path})")
            self._borrowed = False
        self.h = h
        nd, n, e, nb, nm = C.c_int32(), C.c_int64(), C.c_int64(), C.c_int64(), C.c_int32()
        lib().rx_mesh_info(h, C.byref(nd), C.byref(n), C.byref(e), C.byref(nb), C.byref(nm))
        self.n_dim, self.N, self.E, self.NB = nd.value, n.value, e.value, nb.value
        self.tags = [lib().rx_mesh_marker_tag(h, k).decode() for k in range(nm.value)]
        md = MeshDesc()
        _chk(lib().rx_mesh_describe(h, C.byref(md)), "rx_mesh_describe")
        self.desc = md
        arr = lambda p, shape, t=np.float64: np.ctypeslib.as_array(C.cast(p, C.POINTER(
            C.c_double if t == np.float64 else C.c_int64)), shape=shape).copy()
        nnb = int(arr(md.nbr_ptr, (self.N + 1,), np.int64)[-1])
        self._mesh = dict(edges=arr(md.edges, (self.E, 2), np.int64), edge_normal=arr(md.edge_normal, (self.E, nd.value)),
                          coord=arr(md.coord, (self.N, nd.value)), volume=arr(md.volume, (self.N,)),
                          nbr_ptr=arr(md.nbr_ptr, (self.N + 1,), np.int64), nbr=arr(md.nbr, (nnb,), np.int64),
                          bvertex=arr(md.bvert, (self.NB, 2), np.int64),
                          bvertex_normal=arr(md.bvert_normal, (self.NB, nd.value)), n_dim=nd.value)
        self.global_index = np.ctypeslib.as_array(lib().rx_mesh_global_index(h), shape=(self.N,)).copy()
        self._mesh["bvertex_pn"] = np.ctypeslib.as_array(lib().rx_mesh_normal_neighbor(h), shape=(self.NB,)).copy()
        if self._borrowed and not walls:
            # a case's mesh (rx_case_read already ran ComputeWall_Distance over its wall markers): take those
            # distances instead of recomputing (and, with no walls given, overwriting) them
            p = lib().rx_mesh_wall_distance(self.h, None)
            self._mesh["wall_distance"] = (np.ctypeslib.as_array(p, shape=(self.N,)).copy() if p
                                           else np.zeros(self.N))
        else:
            self.wall_distance(walls)

    def wall_distance(self, walls):
        flags = np.array([1 if t in walls else 0 for t in self.tags], dtype=np.int32)
        p = lib().rx_mesh_wall_distance(self.h, flags.ctypes.data)
        self._mesh["wall_distance"] = np.ctypeslib.as_array(p, shape=(self.N,)).copy()
        return self._mesh["wall_distance"]

    def mesh(self):
        return dict(self._mesh)

    def write_restart(self, path, U, T, extra=None, ext_iter=0):
        """COutput::SetRestart format (%.15e, global-index order) from U [N][nVar], T [N][2], extra [N][5] (P, T,
        Mach, mu, mu_t) or None."""
        U = np.ascontiguousarray(U, dtype=np.float64)
        T = np.ascontiguousarray(T, dtype=np.float64)
        ex = None if extra is None else np.ascontiguousarray(extra, dtype=np.float64)
        _chk(lib().rx_restart_write(os.fsencode(path), self.h, U.shape[1], U.ctypes.data, T.ctypes.data,
                                    None if ex is None else ex.ctypes.data, int(ext_iter)), "rx_restart_write")

    def read_restart(self, path, n_var):
        U = np.zeros((self.N, n_var))
        T = np.zeros((self.N, 2))
        _chk(lib().rx_restart_read(os.fsencode(path), self.h, n_var, U.ctypes.data, T.ctypes.data), "rx_restart_read")
        return U, T

    def close(self):
        if getattr(self, "h", None):
            if not self._borrowed:
                lib().rx_mesh_destroy(self.h)
            self.h = None
            self._owner = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def read_mechanism(base_dir, list_file):
    """ReactingModelLibrary::Setup restated (rx_io.h rx_mech_read): the mechanism arrays (mech_* keys, as the golden
    files and Mechanism take them) of the library files listed in base_dir/list_file."""
    h = C.c_void_p()
    _chk(lib().rx_mech_read(os.fsencode(base_dir), os.fsencode(list_file), C.byref(h)), f"rx_mech_read({list_file})")
    try:
        return _mech_arrays(h)
    finally:
        lib().rx_mech_destroy(h)


def _mech_arrays(h):
    """mech_* arrays of an rx_mech handle (copies)."""
    if True:
        d = MechDesc()
        _chk(lib().rx_mech_describe(h, C.byref(d)), "rx_mech_describe")
        ns, nr, nt = d.n_species, d.n_reactions, d.n_tab
        f8 = lambda p, shape: (np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_double)), shape=shape).copy()
                               if int(np.prod(shape)) else np.zeros(shape))
        i4 = lambda p, n: (np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_int32)), shape=(n,)).astype(np.int64)
                           if n else np.zeros(0, dtype=np.int64))
        out = dict(n_species=np.array(ns), n_reactions=np.array(nr), mmass=f8(d.mmass, (ns,)),
                   diff_vol=f8(d.diff_vol, (ns,)), stoich_reac=f8(d.stoich_reac, (ns, nr)),
                   stoich_prod=f8(d.stoich_prod, (ns, nr)), exp_reac=f8(d.exp_reac, (nr, ns)),
                   exp_prod=f8(d.exp_prod, (nr, ns)), A=f8(d.A, (nr,)), beta=f8(d.beta, (nr,)), Ta=f8(d.Ta, (nr,)),
                   A_back=f8(d.A_back, (nr,)), beta_back=f8(d.beta_back, (nr,)), Ta_back=f8(d.Ta_back, (nr,)),
                   reversible=i4(d.reversible, nr), has_backward=i4(d.has_backward, nr),
                   tab_x=f8(d.tab_x, (5, ns, nt)), tab_y=f8(d.tab_y, (5, ns, nt)), tab_y2=f8(d.tab_y2, (5, ns, nt)),
                   form_enthalpy=np.array([lib().rx_mech_formation_enthalpy(h, s) for s in range(ns)]),
                   species=np.array([lib().rx_mech_species(h, s).decode() for s in range(ns)]))
        return {"mech_" + k: v for k, v in out.items()}


R_UNGAS = 6.02214129e23 * 1.3806488e-23 * 1.0e3  # J/(kmol K) (physical_chemical_library.hpp:571-579)


def read_cfg(path):
    """The reference's cfg grammar for the keys this path uses (CConfig::SetConfig_Parsing: `KEY= value` lines,
    `%` comments; values kept as strings). Returns {KEY: value}."""
    out = {}
    with open(path) as f:
        for raw in f:
            line = raw.split("%", 1)[0].strip()
            if "=" not in line:
                continue
            k, v = line.split("=", 1)
            out[k.strip().upper()] = v.strip()
    return out


def _cfg_list(v):
    return [t.strip() for t in v.strip().strip("()").replace(";", ",").split(",") if t.strip()]


def _spline(mech, prop, s, T):
    """MathTools::GetSpline (spline.cpp:62-77) on the library tables (host; free-stream values only)."""
    x, y, y2 = (mech["mech_tab_" + k][prop, s] for k in ("x", "y", "y2"))
    if T < x[0] or T > x[-1]:  # GetSpline's std::out_of_range (spline.cpp:63-64)
        raise RxError(f"The required temperature ({T} K) is out of data range")
    h = x[1] - x[0]
    klo = int((T - x[0]) / h + 1)
    a = (x[klo] - T) / h
    b = (T - x[klo - 1]) / h
    return a * y[klo - 1] + b * y[klo] + ((a * a * a - a) * y2[klo - 1] + (b * b * b - b) * y2[klo]) * (h * h) / 6.0


class _Case:
    """Owner of an rx_case handle (the mesh of case_from_cfg borrows from it)."""

    def __init__(self, h):
        self.h = h

    def __del__(self):
        try:
            if self.h:
                lib().rx_case_destroy(self.h)
                self.h = None
        except Exception:
            pass


def _cfg_dict(c: Cfg):
    return {name: getattr(c, name) for name, _ in Cfg._fields_}


def case_from_cfg(cfg_path):
    """The inputs of a reference REACTIVE_RANS case from its cfg, read natively (include/rx_io.h rx_case_read,
    csrc/rx_case.cpp): the mesh (MESH_FILENAME: SU2 reader + dual-grid preprocessing + wall distance to the
    ISOTHERMAL / HEAT_FLUX markers), the library (CONFIG_LIB_FILE), the flow and SST rx_cfg, the boundary markers in
    the mesh's marker order and the free-stream values of SetNondimensionalization. Returns a dict: mesh (SU2Mesh,
    borrowed from the case), mech (mech_* arrays), flow_cfg (keyword dict for default_cfg), sst_cfg (keyword dict for
    default_cfg: the SST context's rx_cfg), bc (rx_bc_desc inputs), rk_alpha (None unless RUNGE-KUTTA_EXPLICIT),
    free_stream."""
    h = C.c_void_p()
    rc = lib().rx_case_read(os.fsencode(cfg_path), C.byref(h))
    if rc != RX_OK:
        raise RxError(f"case_from_cfg({cfg_path}): {lib().rx_case_error().decode()} "
                      f"({lib().rx_status_string(rc).decode()}, status {rc})")
    case = _Case(h)
    mesh = SU2Mesh(handle=lib().rx_case_mesh(h), owner=case)
    mech = _mech_arrays(C.c_void_p(lib().rx_case_mech(h)))
    fc, sc = Cfg(), Cfg()
    _chk(lib().rx_case_cfg(h, C.byref(fc), C.byref(sc)), "rx_case_cfg")
    bd = BcDesc()
    _chk(lib().rx_case_bc(h, C.byref(bd)), "rx_case_bc")
    nm, nb = bd.n_marker, mesh.NB
    kinds = np.ctypeslib.as_array(C.cast(bd.kind, C.POINTER(C.c_int32)), shape=(nm,)).copy()
    ns = int(mech["mech_n_species"])
    data = np.ctypeslib.as_array(C.cast(bd.data, C.POINTER(C.c_double)), shape=(nm, 6 + ns)).copy()
    nn = (np.ctypeslib.as_array(C.cast(bd.normal_neighbor, C.POINTER(C.c_int64)), shape=(nb,)).copy() if nb
          else np.zeros(0, dtype=np.int64))
    bc = dict(kind=kinds, data=data, normal_neighbor=nn, inlet_kind=int(bd.inlet_kind), tke_inf=bd.tke_inf,
              kine_inf=bd.kine_inf, omega_inf=bd.omega_inf)
    n = C.c_int32()
    ap = C.POINTER(C.c_double)()
    _chk(lib().rx_case_rk(h, C.byref(n), C.byref(ap)), "rx_case_rk")
    rk = [ap[k] for k in range(n.value)] if n.value else None
    fs = [C.c_double() for _ in range(4)]
    _chk(lib().rx_case_free_stream(h, *[C.byref(x) for x in fs]), "rx_case_free_stream")
    return dict(mesh=mesh, mech=mech, flow_cfg=_cfg_dict(fc), sst_cfg=_cfg_dict(sc), bc=bc, rk_alpha=rk,
                free_stream=dict(rho=fs[0].value, mu=fs[1].value, T=fs[2].value, P=fs[3].value), case=case)


def Iterate(flow: ReactiveNSSolver, turb, ext_iter=0, limiter=None, rk_alpha=None):
    """One reference outer iteration for REACTIVE_RANS on the device, in the reference's order
    (CMeanFlowIteration::Iterate iteration_structure.cpp:486-560; CMultiGridIntegration::MultiGrid_Iteration
    integration_time.cpp:40-140 with MGLEVEL = 0, whose MultiGrid_Cycle pre-smoothing sweep runs iRKLimit stages
    :144-183; CSingleGridIntegration::SingleGrid_Iteration :770-810). Each flow stage: Preprocessing
    (SetPrimitive_Variables, gradient, StrainMag, the limiter for 2ND_ORDER_LIMITER), Set_OldSolution + SetTime_Step
    at stage 0, Space_Integration (loops + BCs), Time_Integration (integration_structure.cpp:325-335):
    ImplicitEuler_Iteration when the flow cfg is implicit, else ExplicitEuler_Iteration (EULER_EXPLICIT, rk_alpha
    None) or one ExplicitRK_Iteration per RK_ALPHA_COEFF entry (RUNGE-KUTTA_EXPLICIT). Then the flow
    Preprocessing(Output = true) on the updated solution and the SST iteration — or, turb None (a flow context with
    cfg.rans = 0: REACTIVE_NAVIER_STOKES, KIND_TURB_MODEL= NONE), the flow's iteration alone. limiter None: from
    cfg.spatial_order == 2 (SECOND_ORDER_LIMITER, solver_direct_reactive.cpp:4739-4742). Nothing leaves the device
    except the RMS vectors and the linear-solver counts. Returns (rms_flow of the last stage, rms_turb, lin_iters)."""
    if limiter is None:
        limiter = flow.cfg.spatial_order == 2
    implicit = bool(flow.cfg.implicit)
    stages = [None] if implicit or not rk_alpha else list(rk_alpha)
    # nothing reads RES / JAC between the loops and the implicit step here: the assembly may fold the system's V / dt
    # (rx_set_system_fold; the system is bitwise the same)
    fold = implicit and hasattr(lib(), "rx_set_system_fold")
    if fold:
        _chk(lib().rx_set_system_fold(flow.h, 1), "rx_set_system_fold", flow.h)
    try:
        return _iterate_stages(flow, turb, ext_iter, limiter, implicit, stages)
    finally:
        if fold:
            lib().rx_set_system_fold(flow.h, 0)


def _iterate_stages(flow, turb, ext_iter, limiter, implicit, stages):
    """The body of Iterate (below the fold hint)."""

    def preprocess(output):
        flow.SetPrimitive_Variables(ext_iter)
        flow.SetPrimitive_Gradient()
        flow.SetStrainMag()
        if limiter and not output:
            flow.SetPrimitive_Limiter()

    it = 0
    for k, alpha in enumerate(stages):
        preprocess(False)
        if k == 0:
            flow.SetTime_Step()
        flow.Preprocessing_zero()
        flow.Upwind_Residual()
        flow.Viscous_Residual()
        flow.Source_Residual()
        flow.BC()
        if implicit:
            rms, it = flow.ImplicitEuler_Iteration()
        elif alpha is None:
            rms = flow.ExplicitEuler_Iteration()
        else:
            rms = flow.ExplicitRK_Iteration(k, alpha)
    preprocess(True)  # MultiGrid_Iteration's closing Preprocessing(Output = true) (integration_time.cpp:124-126)
    if turb is None:
        # REACTIVE_NAVIER_STOKES without a turbulence model (KIND_TURB_MODEL= NONE, round 6): CMeanFlowIteration::
        # Iterate runs the flow's MultiGrid_Iteration alone (iteration_structure.cpp:531-534), no SST iteration
        return rms, None, (it, 0)
    turb.Preprocessing()
    turb.Upwind_Residual()
    turb.Viscous_Residual()
    turb.Source_Residual()
    turb.BC()
    rms_t, it_t = turb.ImplicitEuler_Iteration()
    turb.Postprocessing()
    return rms, rms_t, (it, it_t)
