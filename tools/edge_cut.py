"""Edge cut of the solver's partitions of the jet meshes (the reference partitions with METIS
k-way, geometry_structure.cpp:11465-11530; METIS is not installed here, so the comparison is against the
isoperimetric lower bound of the structured nx x ny grid: P parts of A = N/P points, every part a square of
side sqrt(A), cut at least (P * 4 sqrt(A) - 2 (nx + ny)) / 2 edges (part perimeters minus the domain's, each
cut edge shared by two parts), which METIS approaches on such grids). "coord": bisection across the longer
extent in coordinates normalised by the domain's (round 1); "spacing": across the longer extent in mesh
spacings (meshgen.partition_rcb with edges, what build_jet uses).

Round 5: "graph" (meshgen.partition_graph, the multilevel graph partitioner rx_partition_graph) and "metis" (METIS 5's
k-way partitioner compiled from the reference's own vendored sources, oracle/_ref/libmetis.so, on the same graph;
omitted when that library is not built).

usage: python tools/edge_cut.py [c3|c4|c2] > profiles/r05_edge_cut.json
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.rxpkg import meshgen  # noqa: E402

CASES = {"c2": (500, 200), "c3": (2000, 500), "c4": (2000, 4000)}


def cut_stats(edges, part):
    cut = part[edges[:, 0]] != part[edges[:, 1]]
    P = int(part.max()) + 1
    # halo points per part: distinct foreign endpoints of its cut edges
    a, b = edges[cut, 0], edges[cut, 1]
    halo = np.zeros(P, dtype=np.int64)
    for p in range(P):
        m0 = part[a] == p
        m1 = part[b] == p
        halo[p] = len(np.unique(np.r_[b[m0], a[m1]]))
    return int(cut.sum()), int(halo.max()), float(halo.mean())


METIS = os.path.join(ROOT, "oracle", "_ref", "libmetis.so")


def metis_kway(n, edges, P):
    import ctypes as C
    lib = C.CDLL(METIS)
    xadj, adj = meshgen.graph_csr(n, edges)
    x32, a32 = xadj.astype(np.int32), adj.astype(np.int32)
    part = np.zeros(n, dtype=np.int32)
    nv, ncon, np_, obj = C.c_int32(n), C.c_int32(1), C.c_int32(P), C.c_int32()
    lib.METIS_PartGraphKway(C.byref(nv), C.byref(ncon), x32.ctypes.data_as(C.c_void_p), a32.ctypes.data_as(C.c_void_p),
                            None, None, None, C.byref(np_), None, None, None, C.byref(obj),
                            part.ctypes.data_as(C.c_void_p))
    return part.astype(np.int64)


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "c3"
    nx, ny = CASES[case]
    pts, el, bnd = meshgen.jet_mesh(nx, ny)
    # the dual graph's edges are the primal mesh edges (quads: the 4 sides of every element)
    e = np.concatenate([el[:, [0, 1]], el[:, [1, 2]], el[:, [2, 3]], el[:, [3, 0]]])
    e = np.unique(np.sort(e, axis=1), axis=0)
    out = {"bound": "(4 P sqrt(N/P) - 2 (nx + ny)) / 2", "case": case, "grid": [nx, ny], "points": int(len(pts)), "edges": int(len(e)), "partitions": {}}
    for P in ((8, 256, 1024) if case != "c4" else (8, 2048)):
        A = len(pts) / P
        bound = max(P * 2.0 * np.sqrt(A) - (nx + ny), 1.0)
        row = {"lower_bound_cut": round(bound)}
        modes = ["coord", "spacing", "graph"] + (["metis"] if os.path.exists(METIS) else [])
        for mode in modes:
            if mode == "graph":
                part = meshgen.partition_graph(len(pts), e, P)
            elif mode == "metis":
                part = metis_kway(len(pts), e, P)
            else:
                part = meshgen.partition_rcb(pts, P, edges=e if mode == "spacing" else None)
            c, hmax, hmean = cut_stats(e, part)
            row[mode] = {"edge_cut": c, "cut_over_bound": round(c / bound, 3), "halo_max": hmax,
                         "halo_mean": round(hmean, 1)}
        out["partitions"][str(P)] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
