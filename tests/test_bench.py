"""bench.py's kernel bookkeeping (CPU): the ILU(0) apply kernel the bench line names must be the one rx_la_ilu_apply
launches for the workload (rx_sweeps.hip), so that `roofline.kernel` matches the rocprof summary."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_ilu_apply_kernel_names(monkeypatch):
    for v in ("RX_ILU_SPLIT", "RX_ILU_NO_RING", "RX_NARROW_APPLY", "RX_RING_FIRST", "RX_ILU_RING_G"):
        monkeypatch.delenv(v, raising=False)
    # C3: 1M points, 256 partitions of 3 906 rows -> the vector does not fit LDS: the LDS-ring sweeps (round 5)
    assert bench.ilu_apply_kernels(1_000_000, 4_995_000, 11, 256) == "k_ilu_apply_ring<11, 1024, 2, 2>"
    # C5 (3-D, 200x100x100 in 256 partitions): the 3-D ring shape
    assert bench.ilu_apply_kernels(2_000_000, 13_880_000, 12, 256, nDim=3) == "k_ilu_apply_ring<12, 768, 3, 2>"
    # C4's share per GPU at 2048 partitions: 488-row partitions fit LDS, but the ring sweeps come first (round 6)
    assert bench.ilu_apply_kernels(125_000, 624_000, 11, 256) == "k_ilu_apply_ring<11, 1024, 2, 2>"
    monkeypatch.setenv("RX_RING_FIRST", "0")
    assert bench.ilu_apply_kernels(125_000, 624_000, 11, 256) == "k_ilu_apply_lds<11>"
    monkeypatch.setenv("RX_ILU_NO_RING", "1")  # the fused wide sweeps (round 4)
    assert bench.ilu_apply_kernels(1_000_000, 4_995_000, 11, 256) == "k_ilu_apply_wide<11, 1024>"
    assert bench.ilu_apply_kernels(125_000, 624_000, 11, 256) == "k_ilu_apply_lds<11>"
    monkeypatch.setenv("RX_ILU_SPLIT", "1")
    assert bench.ilu_apply_kernels(1_000_000, 4_995_000, 11, 256) == "k_ilu_fwd_wide<11, 1024>+k_ilu_bwd_wide<11, 1024>"


def test_kernel_models_cover_the_timed_phases(monkeypatch):
    monkeypatch.delenv("RX_ASM_CONV", raising=False)
    monkeypatch.delenv("RX_ASM_VISC", raising=False)
    monkeypatch.delenv("RX_ASMV_ES", raising=False)
    m = bench.kernel_models(1_000_000, 1_997_500, 4_995_000, 7, 2, 5)
    for k in ("VISC", "VISC_JAC", "ASSEMBLE", "GRAD", "SOURCE", "ILU_BUILD", "SPMV", "ILU_APPLY"):
        assert k in m and m[k]["kernel"] and m[k]["peak"] > 0, k
    assert m["SPMV"]["unit"] == "GB/s" and m["ILU_APPLY"]["kernel"].startswith("k_ilu_apply_")
    # the node-centric assembly (default) makes the viscous Jacobians and the AUSM fluxes / Jacobians itself:
    # no k_ausm_edge launch in the CONV phase, and no per-edge convective blocks in the assembly's bytes
    # (round 6: with edge-side teams, k_asm_es; the node-serial k_asm_visc with RX_ASMV_ES=0 or a node of more edges
    # than teams)
    assert m["ASSEMBLE"]["kernel"] == "k_asm_es<7, 2>" and "CONV" not in m
    m3 = bench.kernel_models(8_000_000, 23_580_000, 62_000_000, 7, 3, 5, max_degree=6)  # 3-D: fused too (round 5)
    assert m3["ASSEMBLE"]["kernel"] == "k_asm_es<7, 3>" and "CONV" not in m3
    assert bench.kernel_models(1_000, 2_000, 5_000, 7, 3, 5, max_degree=24)["ASSEMBLE"]["kernel"] == "k_asm_visc<7, 3>"
    monkeypatch.setenv("RX_ASMV_ES", "0")
    assert bench.kernel_models(1_000_000, 1_997_500, 4_995_000, 7, 2, 5)["ASSEMBLE"]["kernel"] == "k_asm_visc<7, 2>"
    monkeypatch.delenv("RX_ASMV_ES")
    monkeypatch.setenv("RX_ASM_CONV", "0")
    u = bench.kernel_models(1_000_000, 1_997_500, 4_995_000, 7, 2, 5)
    assert u["CONV"]["kernel"] == "k_ausm_edge<7, 2>" and u["ASSEMBLE"]["kernel"] == "k_asm_es<7, 2>"
    assert u["ASSEMBLE"]["work"] > m["ASSEMBLE"]["work"]
    monkeypatch.setenv("RX_ASM_VISC", "0")
    assert bench.kernel_models(1_000_000, 1_997_500, 4_995_000, 7, 2, 5)["ASSEMBLE"]["kernel"] == "k_assemble<11, 4>"


def test_cpu_baseline_reference_runs_the_compiled_reference():
    """The bench line's cpu_baseline (kind "reference"): the reference's own Iterate on a bounded sample of the
    bench's jet, through the harness compiled from the reference sources (skipped where it is not built)."""
    import pytest
    if not os.path.exists(os.path.join(bench.ROOT, "oracle", "_ref", "harness")):
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    r = bench.cpu_baseline_reference(7, 5.0, nx=40, ny=12)
    assert r["kind"] == "reference" and r["cores"] == 1 and r["value"] > 0 and "480 points" in r["sample"]
