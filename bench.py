"""Throughput of the reactive RANS hot path on MI355X: Mcells*iters/s (BASELINE.json metric).

One step = one outer implicit iteration (flow + SST, as CMeanFlowIteration::Iterate runs them) of the
device-resident hot path over the whole mesh (the order CIntegration drives
them):
  flow: SetPrimitive_Gradient_LS -> SetStrainMag -> SetTime_Step -> residual zero -> Upwind_Residual
        (AUSM + Jacobians) -> Viscous_Residual (reactive viscous + SST closure + Jacobians) ->
        Source_Residual (PaSR + Jacobian) -> ImplicitEuler_Iteration (assembly, Vol/dt, ILU(0) build,
        FGMRES(5), clipped update, RMS);
  SST:  Preprocessing (LS gradient) -> Upwind / Viscous / Source residuals with 2x2 Jacobians ->
        ImplicitEuler_Iteration (system, ILU(0), FGMRES(5), conservative clipped update, RMS) ->
        Postprocessing (gradient, F1/F2/CDkw, mu_t, coupling fields the flow reads next step).

Default workload (N=1): BASELINE configs[2], the north-star roofline run — synthetic 2-D reactive jet,
2000x500 = 1M points, 7 species PaSR + SST, implicit FGMRES+ILU0. `--workload c2` runs configs[1]
(500x200, 100k points); `--workload c5` one GPU's share of configs[4], the 3-D extruded jet (1000x50x20 = 1M
points per GPU; with --gpus 8 the slab is the whole 1000x400x20 mesh).
Inputs are resident in HBM before the timed region. Data are synthetic: the mesh replicates the
reference jet geometry (same domain and markers, nx x ny points); the initial field is the reference's
converged PaSR jet (its own 9 000-point mesh, tests/golden/jet9k.npz) linearly interpolated onto it, and
the node records are completed by the reference's start-up preprocessing on the device (see synth.py).

The preconditioner is partitioned like the reference run on `--parts` MPI ranks (RCB partition,
local RCM per part, ILU(0) per rank; default 256 = one rank per CU); `--parts 1` is the serial
reference.

Multi-GPU (`torch.distributed.run --nproc-per-node N`, one rank per GPU): domain decomposition like the reference's
MPI run. `--scaling strong` (the default for c2 / c3: BASELINE configs[3], C4 = the 1M-point C3 jet split over the
GPUs) keeps the global nx x ny mesh and splits it into parts*N partitions (parts per GPU, the N = 1 line's own
partitioning at N = 1); `--scaling weak` (the default for c5, whose per-GPU slab stacks to the whole 1000x400x20 C5
mesh at N = 8) makes the jet N times taller (nx x ny*N points, parts*N partitions). Every rank owns a contiguous
block of `parts` partitions plus one halo layer (meshgen.shard) and exchanges halos over RCCL where the reference
calls SendReceive / Set_MPI_*, with every FGMRES inner product and the RMS all-reduced (rx_comm_init; all-gather +
rank-ordered sum). The first warm-up step runs
eagerly and must give bitwise the RMS of the next (graph-replayed) one, else the graph is disabled.
If the communicator cannot be set up on any rank, the run prints a line with `value: null` and the
reason, and exits with status 3 (no replica fallback: a scaling point is the decomposed mesh or nothing).
Timing = max over ranks; value = all ranks' owned cells.

Prints ONE JSON line (rank 0) with `roofline` for the dominant kernel and `cpu_baseline`: the reference itself
(oracle/_ref, compiled from /root/reference) on configs[1]'s 100k-point sample, one serial process per core of the
host's CPU share at once (`cpu_baseline_reference_1core`: one process alone), beside the CPU restatement (oracle/,
OpenMP on the same share) over one step of the bench mesh (`cpu_baseline_port`); each names its core count and the
host's `nproc`.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WORKLOADS = {
    "c1": dict(nx=100, ny=90, ns=4, desc="configs[0]: 2-D jet 100x90, 4 species"),
    "c2": dict(nx=500, ny=200, ns=7, desc="configs[1]: 2-D reactive jet 500x200 (100k cells), implicit FGMRES+ILU0"),
    "c3": dict(nx=2000, ny=500, ns=7, desc="configs[2]: 2-D reactive jet 2000x500 (1M cells), 7 species PaSR+SST"),
    # configs[4] (3-D extruded jet 1000x400x20 = 8M cells over 8 GPUs): one GPU's share, 1000x50x20 = 1M cells;
    # --gpus N runs the N-times-taller slab (N = 8: the whole C5 mesh)
    "c5": dict(nx=1000, ny=50, nz=20, ns=7,
               desc="configs[4]: 3-D extruded jet, 7 species, implicit; 1000x50x20 per GPU (8 GPUs: 1000x400x20)"),
}
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFS = 78.6       # MI355X FP64 vector spec


def pmc_fp64_flop(kernel, workload_key):
    """FP64 FLOP per launch of `kernel` counted by rocprofv3 (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64,
    tools/pmc_fp64.py -> profiles/r*_fp64*.json; the newest file on this workload wins); else None."""
    import glob
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_fp64*.json")), reverse=True):
        try:
            with open(fn) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload_key and kernel in d.get("kernels", {}):
            return d["kernels"][kernel]["fp64_flop"]
    return None


def ring_groups():
    """Wave groups per ring-sweep workgroup (rx_ilu_ring_groups in rx_sweeps.hip: env RX_ILU_RING_G in 1 / 2 / 4 / 8,
    default 2)."""
    v = os.environ.get("RX_ILU_RING_G", "").strip()
    return int(v) if v in ("1", "4", "8") else 2


def ilu_apply_kernels(N, nnzb, nVar, parts, nDim=2):
    """The ILU(0) apply kernel rx_la_ilu_apply launches for this partitioning (rx_sweeps.hip), in its order: the LDS-ring
    sweeps (round 5; since round 6 also where a partition fits the LDS-resident sweep, unless RX_RING_FIRST=0), the
    LDS-resident sweep when a partition's vector, metadata and columns fit the 160 KiB LDS, else the wide global
    sweeps."""
    rows = -(-N // parts)
    shm = 8 * (rows * nVar + (256 // nVar) * nVar + 1) + 4 * (8 * rows + rows * nnzb // max(N, 1))
    ring = nVar >= 5 and not (os.environ.get("RX_ILU_NO_RING") or os.environ.get("RX_NARROW_APPLY"))
    ring_first = os.environ.get("RX_RING_FIRST", "1") != "0"
    if shm <= 160 * 1024 and not (ring and ring_first):
        return f"k_ilu_apply_lds<{nVar}>"
    if ring:
        # every level has at most 16 * (64 // nVar) rows on the jet partitions (C3 / C5 / a C4 rank: rocprof shows it)
        # template <NV, threads, factor blocks of a row in registers, wave groups>: 3-D rows (up to 7 blocks) take
        # 768 threads with three blocks in registers (rx_ilu_ring_tb; RX_RING_3D=0: the 2-D shape)
        if nDim == 3 and os.environ.get("RX_RING_3D", "1") != "0":
            return f"k_ilu_apply_ring<{nVar}, 768, 3, {min(ring_groups(), 2)}>"
        return f"k_ilu_apply_ring<{nVar}, 1024, 2, {ring_groups()}>"
    if os.environ.get("RX_ILU_SPLIT"):
        return f"k_ilu_fwd_wide<{nVar}, 1024>+k_ilu_bwd_wide<{nVar}, 1024>"
    return f"k_ilu_apply_wide<{nVar}, 1024>"  # both sweeps of a partition in one launch (round 4)


def kernel_models(N, E, nnzb, ns, nDim, lin_iter, parts=256, workload_key=None, max_degree=4,
                  ilu_grouped=os.environ.get("RX_ILU_ROWWAVE") is None):
    """Algorithmic bytes (or flops) per launch of the single-launch kernels timed per phase
    (each unique datum once per sweep)."""
    nVar, nPV, nG = ns + nDim + 2, ns + nDim + 5, ns + nDim + 2
    d = 8
    blk = nVar * nVar * d
    summ = (14 + 5 * nDim + 9 * ns) * d  # visc_summary_size<NS, NDIM>
    hbm = lambda b, name: dict(bound="hbm", work=float(b), unit="GB/s", peak=HBM_PEAK_GBS, kernel=name)
    te, tv = f"<{ns}, {nDim}>", f"<{nVar}>"  # template arguments of the flow kernels (rocprof / PMC names)
    # k_visc_edge's FP64 work: counted by PMC on this workload when a count is committed, else SURVEY §8(d)'s
    # ~9 kflop per edge (the C3 count is 13.9 kflop per edge, profiles/r02_c3_v2_fp64.json)
    visc_flop = pmc_fp64_flop("k_visc_edge" + te, workload_key) or 9000.0 * E
    fused = conv_fused(nDim)
    # the node-centric assembly kernel: k_asm_es (round 6: edge-side teams) unless RX_ASMV_ES=0 or a node has more
    # edges than its workgroup has teams (rx_asmes_teams: 4 * floor(64 / nVar)); else the node-serial k_asm_visc
    asm_kernel = ("k_asm_es" if os.environ.get("RX_ASMV_ES", "1") != "0" and max_degree <= 4 * (64 // nVar)
                  else "k_asm_visc") + te
    models = {
        # k_ausm_edge: V (nPV) and dPdU (nVar) per node once; edge (2 int32 + normal); flux + 2 Jacobians
        "CONV": hbm(N * (nPV + nVar) * d + E * (8 + nDim * d) + E * (nVar * d + 2 * blk), "k_ausm_edge" + te),
        "VISC": dict(bound="fp64", work=float(visc_flop), unit="TFLOP/s", peak=FP64_PEAK_TFS,
                     kernel="k_visc_edge" + te),
        # k_visc_jac (fused assembly): per-edge summary + dT/dU + the edge's two convective blocks in; two viscous
        # blocks (for the diagonals) and the two off-diagonal BSR blocks out
        "VISC_JAC": hbm(E * summ + N * nVar * d + E * 16 + E * 6 * blk, "k_visc_jac" + te),
        # k_assemble: each node's own-side conv + visc blocks (2 per edge each), the edge fluxes, the source
        # Jacobian's species rows and residual in; diagonal blocks + residual out
        "ASSEMBLE": (hbm(4 * E * blk + 2 * E * nVar * d + N * (ns * nVar + nVar) * d + N * (blk + nVar * d),
                         f"k_assemble<{nVar}, {4 if max_degree <= 4 else 8}>")  # register path by max degree
                     if os.environ.get("RX_ASM_VISC", "1") == "0" else
                     # k_asm_visc (round 4: viscous Jacobians made by the node-centric assembly, VISC_JAC not
                     # launched): each edge's two convective blocks, summary record, fluxes and ends' dT/dU in once,
                     # the source rows; the two off-diagonal blocks, the diagonal blocks and the residual out
                     hbm(2 * E * blk + 2 * E * nVar * d + E * summ + N * nVar * d + 24 * E
                         + N * (ns * nVar + nVar) * d + 2 * E * blk + N * (blk + nVar * d), asm_kernel)
                     if not fused else
                     # k_asm_visc with the fused AUSM pass (round 4, k_ausm_edge not launched): V and dP/dU per
                     # node and each edge's normal once, the viscous fluxes, summary records, dT/dU and index
                     # arrays, the source rows; the two off-diagonal blocks, the diagonal blocks and the residual out
                     hbm(N * (nPV + nVar) * d + E * nDim * d + E * nVar * d + E * summ + N * nVar * d + 24 * E
                         + N * (ns * nVar + nVar) * d + 2 * E * blk + N * (blk + nVar * d), asm_kernel)),
        "GRAD": hbm(N * ((nDim + nPV) * d + nG * nDim * d) + (N + 1) * 4 + 2 * E * 4, "k_grad_lsq" + te),
        # k_source: V, dT/dU, volume, omega in; residual + the Jacobian's species rows out
        "SOURCE": hbm(N * (nPV + nVar + 2) * d + N * (nVar + ns * nVar) * d, "k_source" + te),
        # k_ilu_build_grp (the jet meshes: ILU(0) changes only the lower blocks and the diagonal): every
        # block of A in once (the lower blocks and the diagonal of row i, the upper blocks as the A_ji of the rows
        # below), the lower factor blocks W, the factored diagonal and inv(D_i) out. k_ilu_build_part (other meshes,
        # RX_ILU_ROWWAVE=1): A in, the whole factor + inv(D) out
        # (<nVar, false>: one lane group per row, the bench meshes' levels are wider than RX_GRP_PAIR_W)
        "ILU_BUILD": (hbm((nnzb + (nnzb - N) // 2 + 2 * N) * blk, "k_ilu_build_grp" + tv[:-1] + ", false>")
                      if ilu_grouped else
                      hbm((2 * nnzb + N) * blk, "k_ilu_build_part" + tv)),
        # SOLVE phase (inside the FGMRES graph; timed by an eager replay of one step after the timed region):
        # FGMRES's w = A z (k_fg_spmv_stage for the flow blocks, k_fg_spmv_full for the SST's 2x2): every block + its
        # column index once, z gathered, w written
        "SPMV": hbm(nnzb * (blk + 4) + (N + 1) * 4 + 2 * N * nVar * d,
                    ("k_fg_spmv_stage" if nVar > 4 else "k_fg_spmv_full") + tv),
        # ILU(0) apply: L and U blocks + inv(D_i) (= nnzb blocks) + column indices, b in, x out
        "ILU_APPLY": hbm(nnzb * (blk + 4) + 2 * N * nVar * d, ilu_apply_kernels(N, nnzb, nVar, parts, nDim)),
        # round 6: k_set_primitive — U, the previous record's temperature, k and mu_t in; the
        # clamped U, the record (nPV), dP/dU, dT/dU, mu, kappa, D_ij (Ns^2) and the eddy viscosity out
        "PRIMITIVE": hbm(N * (nVar + 3) * d + N * (nVar + nPV + 2 * nVar + 3 + ns * ns) * d, "k_set_primitive" + te),
        # k_sst_upwind (first order): per node its velocity + density, (k, omega), residual and diagonal block in / out,
        # the adjacency pointer; per adjacency entry its index + block position and the off-diagonal 2x2 block in / out;
        # per edge its ends and normal
        "SST_UPW": hbm(N * ((nDim + 1) * d + 2 * d + 4 * d + 64 + 4) + 2 * E * (12 + 64) + E * (8 + nDim * d),
                       f"k_sst_upwind<{nDim}, 0>"),
        # k_sst_visc: per node F1, mu, eddy viscosity, density, coordinates, (k, omega) and their gradient, residual and
        # diagonal block in / out; per adjacency entry and edge as the upwind
        "SST_VISC": hbm(N * ((4 + nDim + 2 + 2 * nDim + 4) * d + 64 + 4) + 2 * E * (12 + 64) + E * (8 + nDim * d),
                        f"k_sst_visc<{nDim}>"),
    }
    if fused:
        del models["CONV"]  # the CONV phase launches no flux kernel (only MUSCL's reconstruction at 2nd order)
    return models


def conv_fused(nDim):
    """Whether the implicit AUSM fluxes and Jacobians are made inside k_asm_visc (rx_fuse_conv, rx_kernels.hip):
    by default in 2-D and 3-D (round 5), never with RX_ASM_CONV=0 or RX_ASM_VISC=0."""
    if os.environ.get("RX_ASM_VISC", "1") == "0":
        return False
    return not os.environ.get("RX_ASM_CONV", "").startswith("0")


def pmc_traffic(kernel, workload_key, field="hbm_bytes"):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes (profiles/r*_pmc*.json, written by
    tools/pmc_summary.py: 2 x FETCH_SIZE + WRITE_SIZE, the guide's gfx950 correction; field "hbm_bytes_calibrated"
    for the SpMV-calibrated figure). The file's workload key must equal bench.py's (`c3 2000x500 ns7 parts256`);
    the newest file on this workload wins; else None."""
    import glob
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc*.json")), reverse=True):
        try:
            with open(fn) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("workload") != workload_key:
            continue
        ks = [d.get("kernels", {}).get(p) for p in kernel.split("+")]  # "a+b": both launches of one phase
        if all(k is not None for k in ks):
            return sum(k.get(field, k["hbm_bytes"]) for k in ks)
    return None


def build_workload(nx, ny, ns, n_part=1, nz=0):
    """Mesh + initial field: the reference's converged PaSR jet interpolated onto the synthetic mesh
    (synth.jet_field_case); the node records are completed on the device by synth.device_preprocess."""
    from tests.rxpkg import synth
    mesh, st, mech, kw = synth.jet_field_case(nx, ny, n_species=ns, n_part=n_part, nz=nz)
    return mesh, st, mech, kw


def cpu_baseline(mesh, st, mech_arrays, kw, ns, cfg, bc=None):
    """One reference outer iteration of the CPU restatement (oracle/, OpenMP over the host cores it is given:
    OMP_NUM_THREADS, 16 on the GPU box) on the same mesh and state: O.outer_iteration (flow Preprocessing, time
    step, loops + boundary conditions, FGMRES(5)+ILU0 update, Preprocessing(Output), SST iteration) — or, with bc
    None (--no-bc), the legacy flow + SST step. The per-edge / per-point / per-rank loops run in parallel with the
    reference's per-item arithmetic (results are thread-count independent); the scatters of the time step and
    the SST system, the inner products and the host orchestration stay serial."""
    from oracle import oracle as O
    om = O.Mechanism(mech_arrays)
    c = dict(cfl=cfg.cfl, max_delta_time=cfg.max_delta_time, prandtl_lam=cfg.prandtl_lam,
             prandtl_turb=cfg.prandtl_turb, lewis_turb=cfg.lewis_turb, mach_inf=cfg.mach_inf, c_mu=cfg.c_mu,
             pasr_lb=cfg.pasr_lb, lin_tol=cfg.lin_tol, lin_iter=cfg.lin_iter, relaxation=cfg.relaxation)
    N = len(st["V"])
    pattern = O.bsr_pattern(N, mesh["edges"])
    nDim = int(np.shape(mesh["coord"])[1])
    if bc is not None:
        from tests.oracle_inputs import outer_iteration_inputs
        mesh_o, state, bco, c = outer_iteration_inputs(mesh, st, cfg, bc)
        t0 = time.perf_counter()
        O.outer_iteration(om, nDim, mesh_o, state, bco, c, 0, pattern, part_ptr=mesh.get("part_ptr"), keep=False)
        what = "1 reference outer iteration (flow + SST, jet boundary conditions)"
    else:
        t0 = time.perf_counter()
        _, info = O.implicit_step(om, nDim, ns, mesh, st, c, pattern=pattern, part_ptr=mesh.get("part_ptr"))
        flow = dict(V=st["V"], grad=info["grad"], mu=st["mu"], eddy=st["eddy_visc_flow"],
                    strain=O.strain_mag(nDim, info["grad"]))
        O.sst_step(nDim, mesh, flow, st["sst_sol"], None, st["sst_F1"], st["sst_F2"], st["sst_CDkw"], info["dt"],
                   dict(lin_tol=cfg.lin_tol, lin_iter=cfg.lin_iter), pattern=pattern, part_ptr=mesh.get("part_ptr"))
        what = "1 outer iteration (flow implicit step + SST step, no boundary conditions)"
    dt = time.perf_counter() - t0
    cores = int(O.lib().orc_num_threads())
    share, nproc = host_cores()
    return dict(value=N / dt / 1e6, unit="Mcells*iters/s", cores=cores, kind="port",
                sample=f"{what} of the same {N}-cell mesh, {cores} host threads ({dt:.2f} s)",
                host_cpu_share=share, host_nproc=nproc)


def host_cores():
    """(CPU share, nproc): the cores this process may run on (the GPU box grants a 16-CPU share of a larger host and
    sets OMP_NUM_THREADS to it) and the host's whole count (os.cpu_count(), what `nproc` reports there)."""
    share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        share = min(share, int(omp))
    return share, os.cpu_count() or share


def cpu_baseline_reference(ns, cfl, nx=500, ny=200, copies=1):
    """The reference itself (SU2's CMeanFlowIteration::Iterate through oracle/ref_harness, compiled from
    /root/reference's sources by oracle/ref_build.mk into oracle/_ref; serial: one MPI rank, one core per process) on
    a bounded sample of the bench workload: the same synthetic jet geometry and interpolated PaSR state
    (synth.field_at) at nx x ny points — by default configs[1]'s 500 x 200 = 100 000-point mesh —, the bench's
    mechanism (`ns` species), EULER_IMPLICIT with ILU0 FGMRES(5) at the bench's CFL and the jet's boundary conditions.
    The time is the harness's own clock around Iterate (it1_wall). On the GPU box one such iteration takes 9-10 s
    (0.010-0.011 Mcells*iters/s; 0.0105 on the 300 x 75 sample of round 4: the per-cell cost does not depend on the
    sample there — the container's slower core gives 0.0033, which is what an earlier note compared with).
    copies > 1: that many independent reference processes at once on as many cores, each on its own copy of the
    sample, the aggregate throughput copies * points / slowest wall — the all-core reference estimate (the MPI build of
    the reference cannot be made here: its run on those cores would split one mesh and add communication, so this
    bounds it from above). None when the harness is not built."""
    harness = os.path.join(ROOT, "oracle", "_ref", "harness")
    if not os.path.exists(harness):
        return None
    import shutil
    import subprocess
    import tempfile
    from tests.casefiles import unpack
    from tests.rxpkg import meshgen, synth
    root = tempfile.mkdtemp(prefix="rx_refbase_")
    try:
        cd = os.path.join(root, "ref", "Test_Cases", "TURBOLENT", "TURBOLENT_COMBUSTION")
        unpack(cd, "jet")
        os.environ["RX_REFERENCE"] = os.path.join(root, "ref")
        from oracle import make_golden as MG
        MG.CASE_DIR = cd
        pts, quads, bnd = meshgen.jet_mesh(nx, ny)
        _, U, k, om, _, _ = synth.field_at(pts, ns)
        state = np.c_[U, k, om]

        def writer(wd):
            meshgen.write_su2(os.path.join(wd, "mesh.su2"), pts, quads, bnd)
            return "mesh.su2"

        wds = []
        for q in range(copies):
            wd = MG.make_workdir(f"refbase{q}", writer, cfl=cfl, order="1ST_ORDER", prec="ILU0", ns=ns, root=root)
            MG.write_state(wd, state)
            wds.append(wd)
        if copies == 1:
            walls = [float(np.ravel(MG.run_harness(wds[0], bsr=False, extra=["--iters", "1"])["it1_wall"])[0])]
        else:
            env = dict(os.environ, OMP_NUM_THREADS="1")
            procs = [subprocess.Popen([harness, "case.cfg", "state.txt", "out", "--iters", "1"], cwd=wd, env=env,
                                      stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL) for wd in wds]
            if any(p.wait() != 0 for p in procs):
                raise RuntimeError("a concurrent reference harness failed")
            walls = []
            for wd in wds:
                man = dict(line.split()[:2] for line in open(os.path.join(wd, "out", "manifest.txt")))
                walls.append(float(np.fromfile(os.path.join(wd, "out", "it1_wall.bin"),
                                               dtype="<" + man["it1_wall"])[0]))
    finally:
        shutil.rmtree(root, ignore_errors=True)
    n = len(pts)
    wall = max(walls)
    share, nproc = host_cores()
    what = (f"1 outer iteration of the reference itself (oracle/_ref harness, serial) on the {nx}x{ny} synthetic jet "
            f"({n} points, {ns} species, EULER_IMPLICIT ILU0 FGMRES(5), jet BCs)")
    if copies == 1:
        return dict(value=round(n / wall / 1e6, 6), unit="Mcells*iters/s", cores=1, kind="reference",
                    sample=f"{what}, one core: {wall:.2f} s", host_cpu_share=share, host_nproc=nproc)
    return dict(value=round(copies * n / wall / 1e6, 6), unit="Mcells*iters/s", cores=copies, kind="reference",
                sample=f"{copies} concurrent copies of {what}, one core each: slowest {wall:.2f} s, fastest "
                       f"{min(walls):.2f} s (aggregate = copies x points / slowest; an upper bound of the reference's "
                       f"MPI run on these cores)", host_cpu_share=share, host_nproc=nproc)


def setup_sharded(rx, args, nx, ny, ns, world, rank, local, dist, nz=0):
    """Build the rank's shard (strong: of the fixed nx x ny jet; weak: of the N-times-taller one) and attach the RCCL
    communicator."""
    from tests.rxpkg import meshgen, synth
    gy = ny if args.scaling == "strong" else ny * world
    mesh, st, mech_arrays, kw = build_workload(nx, gy, ns, args.parts * world, nz)
    sh = meshgen.shard(mesh, world, rank)
    st_l = {k: np.asarray(v)[sh["l2g"]] for k, v in st.items()}
    if args.cfl:
        kw["cfl"] = args.cfl
    cfg = rx.default_cfg(implicit=1, rans=1, lin_prec=1, lin_iter=5, **kw)
    s = rx.ReactiveNSSolver(sh, rx.Mechanism(mech_arrays), cfg, device=local)
    uid = [rx.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    s.comm_init(world, rank, uid[0])
    if not args.no_bc:
        s.set_bc(synth.jet_bc(sh, ns))
    t = rx.TurbSSTSolver(sh, s, rx.sst_cfg())
    st_l = synth.device_preprocess(s, t, sh, st_l)
    return s, t, sh, st_l, mech_arrays, kw, cfg, int(sh["n_domain"])


def set_states(s, t, mesh, st):
    s.set_state(st)
    t.set_state(st["sst_sol"], mesh["wall_distance"], st["sst_F1"], st["sst_F2"], st["sst_CDkw"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--nx", type=int, default=0)
    ap.add_argument("--ny", type=int, default=0)
    ap.add_argument("--nz", type=int, default=0, help="z planes of the 3-D extrusion (c5)")
    ap.add_argument("--species", type=int, default=0)
    ap.add_argument("--parts", type=int, default=256,
                    help="partitions (= the reference's MPI ranks) of the ILU(0)/LU-SGS preconditioner")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-bc", action="store_true",
                    help="legacy step without boundary conditions and without the post-update Preprocessing")
    ap.add_argument("--cfl", type=float, default=0.0, help="CFL_NUMBER (default: the case's)")
    ap.add_argument("--breakdown", action="store_true", help="print per-phase times to stderr")
    ap.add_argument("--scaling", choices=("strong", "weak"), default=None,
                    help="N > 1: strong = split the fixed mesh (default for c2 / c3: C4), weak = N-times-taller mesh "
                         "(default for c5)")
    args = ap.parse_args()
    if args.scaling is None:
        args.scaling = "weak" if args.workload == "c5" else "strong"

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        local = local % max(1, torch.cuda.device_count())  # rehearsal with more ranks than GPUs
        torch.cuda.set_device(local)
        # host-side control only (uid broadcast, barrier, max of the timings): gloo; the data path
        # is the context's own RCCL communicator
        dist.init_process_group("gloo")
    from tests.rxpkg import rx

    wl = dict(WORKLOADS[args.workload])
    nx, ny, ns = args.nx or wl["nx"], args.ny or wl["ny"], args.species or wl["ns"]
    nz = args.nz or wl.get("nz", 0)
    nDim = 3 if nz > 1 else 2
    s = None
    parallelism = "1 GPU"
    n_owned = 0
    if world > 1:
        err = ""
        try:
            s, t, mesh, st, mech_arrays, kw, cfg, n_owned = setup_sharded(rx, args, nx, ny, ns, world, rank, local,
                                                                          dist, nz)
        except Exception as e:  # noqa: BLE001 - reported in the JSON line
            err = repr(e)[:200]
        flags = [None] * world
        dist.all_gather_object(flags, err)
        bad = [f for f in flags if f]
        if bad:
            # no scaling point without the domain decomposition: independent replicas would
            # sum N single-GPU runs into a value a scaling curve must not record, so the line carries no value
            if s is not None:
                s.close()
            if rank == 0:
                print(json.dumps({"metric": "Mcells*iters/s (reactive RANS)", "value": None, "unit": "Mcells*iters/s",
                                  "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": None,
                                  "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
                                  "dtype": "f64", "data": "synthetic",
                                  "config": {"workload": args.workload, "parallelism": "none"},
                                  "error": f"sharded setup failed on a rank: {bad[0]}"}), flush=True)
            dist.destroy_process_group()
            sys.exit(3)
        else:
            parallelism = f"sharded x{world} (RCCL halo exchange + all-reduce)"
    if s is None:
        mesh, st, mech_arrays, kw = build_workload(nx, ny, ns, args.parts, nz)
        if args.cfl:
            kw["cfl"] = args.cfl
        cfg = rx.default_cfg(implicit=1, rans=1, lin_prec=1, lin_iter=5, **kw)
        s = rx.ReactiveNSSolver(mesh, rx.Mechanism(mech_arrays), cfg, device=local)
        if not args.no_bc:
            from tests.rxpkg import synth
            synth_bc = synth.jet_bc(mesh, ns)
            s.set_bc(synth_bc)
        t = rx.TurbSSTSolver(mesh, s, rx.sst_cfg())
        from tests.rxpkg import synth
        st = synth.device_preprocess(s, t, mesh, st)
        set_states(s, t, mesh, st)
        n_owned = s.N
    N, E = s.N, s.E
    rp, col = s.bsr_pattern()
    nnzb = int(rp[-1])

    lin_its = []
    rms_log = []

    ext_iter = [0]

    def step():
        if not args.no_bc:
            # the reference's outer iteration (CMeanFlowIteration::Iterate): flow Preprocessing, time step,
            # loops + boundary conditions, implicit solve, Preprocessing(Output) on the update, SST iteration
            rms, trms, (it, tit) = rx.Iterate(s, t, ext_iter=ext_iter[0])
            ext_iter[0] += 1
        else:
            s.SetPrimitive_Variables()  # Cons2Prim + transport from the U of the previous update (next-1)
            s.SetPrimitive_Gradient()
            s.SetStrainMag()
            s.SetTime_Step()
            s.Preprocessing_zero()
            s.Upwind_Residual()
            s.Viscous_Residual()
            s.Source_Residual()
            rms, it = s.ImplicitEuler_Iteration()
            t.Preprocessing()
            t.Upwind_Residual()
            t.Viscous_Residual()
            t.Source_Residual()
            trms, tit = t.ImplicitEuler_Iteration()
            t.Postprocessing()
        lin_its.append((it, tit))
        rms_log.append(np.r_[rms, trms])

    graph = True
    if parallelism.startswith("sharded"):
        # eager step, then a graph-replayed step from the same state: same systems, same RMS bitwise
        os.environ["RX_NO_GRAPH"] = "1"
        step()
        os.environ.pop("RX_NO_GRAPH")
        set_states(s, t, mesh, st)
        step()
        ok = bool(np.array_equal(rms_log[0], rms_log[1]) and lin_its[0] == lin_its[1])
        oks = [None] * world
        dist.all_gather_object(oks, ok)
        if not all(oks):
            os.environ["RX_NO_GRAPH"] = "1"
            graph = False
    for _ in range(args.warmup):
        step()
    s.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    s.profile(True)
    t.profile(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    s.sync()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    timed_its = list(lin_its[-args.steps:])
    if dist:
        dist.barrier()
        tel = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(tel, op=dist.ReduceOp.MAX)
        el = float(tel.item())
    prof = {k: s.profile_read(k) for k in rx.K}
    tprof = {k: t.profile_read(k) for k in rx.K}
    prof = {k: (prof[k][0] + tprof[k][0], prof[k][1] + tprof[k][1]) for k in rx.K}
    s.profile(False)
    t.profile(False)
    # The SOLVE phase's kernels (inside the FGMRES graph in the timed steps, where no event can bracket them): one
    # more step with the solve launched eagerly (RX_NO_GRAPH=1: the same kernels on the same stream, each in-solve
    # ILU apply and k_fg_spmv_full bracketed by events, rx_krylov.hip), flow context only.
    os.environ["RX_NO_GRAPH"] = "1"
    s.profile(True)
    step()
    s.sync()
    for k in ("SPMV", "ILU_APPLY"):
        prof[k] = s.profile_read(k)
    s.profile(False)
    if graph:
        os.environ.pop("RX_NO_GRAPH", None)

    dims = f"{nx}x{ny}" + (f"x{nz}" if nz > 1 else "")
    wkey = f"{args.workload} {dims} ns{ns} parts{args.parts}"
    max_degree = int(np.bincount(np.asarray(mesh["edges"]).ravel()).max())
    models = kernel_models(N, E, nnzb, ns, nDim, 5, parts=args.parts, workload_key=wkey, max_degree=max_degree)
    phase_ms = {k: v[0] / args.steps for k, v in prof.items() if v[1] > 0 and k not in ("SPMV", "ILU_APPLY")}

    def roof(k):
        ms, n = prof[k]
        avg_s = ms / n / 1e3
        m = models[k]
        scale = 1e9 if m["unit"] == "GB/s" else 1e12
        ach = m["work"] / avg_s / scale
        out = dict(kernel=m["kernel"], phase=k, bound=m["bound"], achieved=round(ach, 2), peak=m["peak"],
                   unit=m["unit"], frac=round(ach / m["peak"], 4), avg_launch_us=round(avg_s * 1e6, 2),
                   launches=int(n))
        if m["unit"] == "GB/s":
            t = pmc_traffic(m["kernel"], wkey)
            tc = pmc_traffic(m["kernel"], wkey, "hbm_bytes_calibrated")
            out["algorithmic_bytes"] = int(m["work"])
            out["traffic"] = None if t is None else int(t)
            out["traffic_spmv_calibrated"] = None if tc is None else int(tc)
            f64 = pmc_fp64_flop(m["kernel"], wkey)
            if f64 is not None:  # the FP64 view beside the HBM one (PMC-counted flops / this run's launch time)
                out["fp64_tflops"] = round(f64 / avg_s / 1e12, 3)
                out["fp64_frac"] = round(f64 / avg_s / 1e12 / FP64_PEAK_TFS, 4)
        else:
            out["algorithmic_flops"] = int(m["work"])
            out["traffic"] = None
        return out

    timed = [k for k in models if prof.get(k, (0, 0))[1] > 0]
    kernels = {k: roof(k) for k in timed}
    # GPU time per step of each single-kernel phase (SPMV / ILU_APPLY: average launch of the eager pass x launches per
    # step, i.e. per linear iteration of the flow solve; ILU_APPLY is one kernel, both sweeps, unless RX_ILU_SPLIT)
    its_mean = float(np.mean([a for a, _ in timed_its]))
    for k in timed:
        per = its_mean if k in ("SPMV", "ILU_APPLY") else prof[k][1] / args.steps
        kernels[k]["ms_per_step"] = round(prof[k][0] / prof[k][1] * per, 4)
    single = [k for k in timed if "+" not in kernels[k]["kernel"]]
    # dominant kernel: the most GPU time per step; the longest single launch beside it
    dom = max(single, key=lambda k: kernels[k]["ms_per_step"])
    longest = max((k for k in single if k != "SPMV"), key=lambda k: prof[k][0] / prof[k][1])

    if world > 1:
        tot = [None] * world
        dist.all_gather_object(tot, n_owned)
        cells = int(sum(tot))
    else:
        cells = N
    out = {
        "metric": "Mcells*iters/s (reactive RANS)",
        "value": round(cells * args.steps / el / 1e6, 4),
        "unit": "Mcells*iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": args.scaling if world == 1 or parallelism.startswith("sharded") else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (reference jet geometry; node records resampled from the reference PaSR jet state)",
        "config": {"workload": f"{args.workload}: {nDim}-D reactive jet {dims}" + (
                       (f" split over {world} GPUs (configs[3], C4)" if args.scaling == "strong" else
                        f" per GPU (global {nx}x{ny * world}" + (f"x{nz})" if nz > 1 else ")"))
                       if parallelism.startswith("sharded") else ""),
                   "cells_per_gpu": n_owned, "halo_points": N - n_owned, "edges": E,
                   "species": ns, "nVar": ns + nDim + 2, "nnz_blocks": nnzb,
                   "time": f"EULER_IMPLICIT flow at CFL {cfg.cfl:g} (rx.BENCH_CFL: reference-pinned, "
                           "profiles/r05_calibration_c2.json) + SST (one reference outer iteration per step" +
                           (", no boundary conditions)" if args.no_bc else ", jet boundary conditions)"),
                   "linear_solver": f"FGMRES(5)+ILU0 (flow {ns + nDim + 2}x{ns + nDim + 2} and SST 2x2 systems)",
                   "partitions": args.parts,
                   "parallelism": parallelism, "solve_graph": graph, "cells_total": cells,
                   "lin_iters_mean": float(np.mean([a for a, _ in timed_its])),
                   "sst_lin_iters_mean": float(np.mean([b for _, b in timed_its]))},
        "roofline": kernels[dom],
        "roofline_longest_launch": kernels[longest],
        # the edge flux: k_ausm_edge, or (fused, the default) the assembly kernel that now evaluates it
        "roofline_edge_flux": kernels.get("CONV") or dict(kernels.get("ASSEMBLE") or {}, fused_into_assembly=True),
        "roofline_kernels": kernels,
        "phase_ms_per_step": {k: round(v, 4) for k, v in phase_ms.items()},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the reference itself on a bounded sample when its harness is built (kind "reference"), beside the
        # restatement on the whole mesh on all host cores (kind "port")
        port = cpu_baseline(mesh, st, mech_arrays, kw, ns, cfg, None if args.no_bc else synth_bc)
        ref = ref1 = None
        if nz <= 1 and not args.no_bc:
            try:
                ref1 = cpu_baseline_reference(ns, cfg.cfl)
                share, _ = host_cores()
                # the reference on every core of the box's CPU share at once, the line's baseline
                ref = cpu_baseline_reference(ns, cfg.cfl, copies=share) if share > 1 else ref1
            except (SystemExit, Exception) as e:  # noqa: BLE001 - the port line stands
                port["reference_error"] = repr(e)[:200]
        out["cpu_baseline"] = ref if ref is not None else (ref1 if ref1 is not None else port)
        out["cpu_baseline_reference_1core"] = ref1
        out["cpu_baseline_port"] = port
    else:
        out["cpu_baseline"] = None
    s.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
