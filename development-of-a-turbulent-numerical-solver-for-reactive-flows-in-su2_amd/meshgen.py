"""Synthetic 2-D jet meshes and their vertex-centred median dual.

Host-side setup, not the hot path. Replicates the layout of the reference's jet combustor mesh
(`Test_Cases/TURBOLENT/TURBOLENT_COMBUSTION/mesh_stretched.su2`: 0.125 x 0.006 m box; markers
Oxidizer_Inlet (left), Outlet (right), upper_wall (top), and a bottom wall split 20:39:40 into
lower_wall_pre / Fuel_Inlet / lower_wall_post) at any nx x ny resolution.

The dual grid follows the reference construction:
  * edges i<j, normal oriented from i to j, accumulated per element face from the edge midpoint to
    the element centroid (`Common/src/dual_grid_structure.cpp:505-530`,
    `Common/src/geometry_structure.cpp` CPhysicalGeometry::SetControlVolume, 2-D branch);
  * dual volume = sum of the triangles (point, edge midpoint, element centroid);
  * boundary vertex normals from the boundary line elements
    (`Common/src/geometry_structure.cpp` CPhysicalGeometry::SetBoundControlVolume, 2-D branch).
Edge order is lexicographic in (i, j) after the point ordering (reference `CGeometry::SetEdges`
discovers edges point by point over sorted neighbour lists, `geometry_structure.cpp:223-252`).
"""
from __future__ import annotations

import numpy as np

MARKERS = ("Oxidizer_Inlet", "Outlet", "upper_wall", "Fuel_Inlet", "lower_wall_pre", "lower_wall_post")
# bottom split of the reference mesh: 20 : 39 : 40 elements out of 99
BOTTOM_SPLIT = (20, 39, 40)


def jet_points(nx: int, ny: int, length=0.125, height=0.006, stretch=1.5):
    """Structured nx x ny points (x fastest), tanh-clustered towards both walls in y."""
    x = np.linspace(0.0, length, nx)
    s = np.linspace(-1.0, 1.0, ny)
    y = 0.5 * height * (1.0 + np.tanh(stretch * s) / np.tanh(stretch))
    y[0], y[-1] = 0.0, height
    X, Y = np.meshgrid(x, y)  # (ny, nx)
    return np.stack([X.ravel(), Y.ravel()], axis=1)


def jet_mesh(nx: int, ny: int, **kw):
    """Points, counter-clockwise quads and boundary line elements per marker."""
    pts = jet_points(nx, ny, **kw)
    pid = np.arange(nx * ny).reshape(ny, nx)
    quads = np.stack([pid[:-1, :-1].ravel(), pid[:-1, 1:].ravel(), pid[1:, 1:].ravel(), pid[1:, :-1].ravel()], axis=1)
    nxe = nx - 1
    a = round(nxe * BOTTOM_SPLIT[0] / 99.0)
    b = round(nxe * (BOTTOM_SPLIT[0] + BOTTOM_SPLIT[1]) / 99.0)
    bottom = np.stack([pid[0, :-1], pid[0, 1:]], axis=1)
    bnd = {
        "Oxidizer_Inlet": np.stack([pid[1:, 0], pid[:-1, 0]], axis=1),
        "Outlet": np.stack([pid[:-1, -1], pid[1:, -1]], axis=1),
        "upper_wall": np.stack([pid[-1, 1:], pid[-1, :-1]], axis=1),
        "Fuel_Inlet": bottom[a:b],
        "lower_wall_pre": bottom[:a],
        "lower_wall_post": bottom[b:],
    }
    return pts, quads, bnd


# 3-D extrusion (config C5): the 2-D markers become side walls / inlets / outlet of the slab, the two z planes are
# symmetry planes (MARKER_SYM; the reactive solvers leave them to CSolver::BC_Sym_Plane, a no-op)
MARKERS3 = MARKERS + ("sym_back", "sym_front")
# CHexahedron::Faces (Common/src/primal_grid_structure.cpp:395), CQuadrilateral::Neighbor_Nodes (:260)
HEX_FACES = np.array([[0, 1, 5, 4], [1, 2, 6, 5], [2, 3, 7, 6], [3, 0, 4, 7], [0, 3, 2, 1], [4, 5, 6, 7]])
QUAD_NEIGHBORS = np.array([[1, 3], [2, 0], [3, 1], [0, 2]])


def jet_mesh3d(nx: int, ny: int, nz: int, depth=0.003, **kw):
    """The 2-D jet extruded over nz planes in z: points (plane-major), VTK-ordered hexahedra and boundary quads per
    marker, ordered counter-clockwise seen from the interior (the orientation CPhysicalGeometry::
    Check_BoundElem_Orientation, geometry_structure.cpp:8825-8960, leaves unflipped)."""
    p2, q2, b2 = jet_mesh(nx, ny, **kw)
    n2 = len(p2)
    z = np.linspace(0.0, depth, nz)
    pts = np.concatenate([np.c_[p2, np.full(n2, zk)] for zk in z])
    hexes = np.concatenate([np.c_[q2 + k * n2, q2 + (k + 1) * n2] for k in range(nz - 1)]).astype(np.int64)
    bnd = {}
    for name in MARKERS:
        l = np.asarray(b2[name], dtype=np.int64)
        bnd[name] = np.concatenate([np.c_[l[:, 0] + k * n2, l[:, 0] + (k + 1) * n2, l[:, 1] + (k + 1) * n2,
                                          l[:, 1] + k * n2] for k in range(nz - 1)])
    bnd["sym_back"] = q2.astype(np.int64)
    bnd["sym_front"] = q2[:, ::-1].astype(np.int64) + (nz - 1) * n2
    return pts, hexes, bnd


def _orient3(c1, c2, c3, c4):
    """The tetrahedral orientation test of Check_IntElem_Orientation (geometry_structure.cpp:8542-8794)."""
    a, b, c = 0.5 * (c2 - c1), 0.5 * (c3 - c1), c4 - c1
    n = np.array([a[1] * b[2] - b[1] * a[2], -(a[0] * b[2] - b[0] * a[2]), a[0] * b[1] - b[0] * a[1]])
    return float(n @ c)


def mixed_mesh3d(nx: int, ny: int, nz: int, **kw):
    """jet_mesh3d with every element kind of the 3-D SU2 reader: the columns of 2-D cells q with q % 3 == 1 are
    split along the bottom-face diagonal (node 0 - node 2) into two prisms (VTK 13) per layer, whose z-plane faces
    become boundary triangles (VTK 5); in the other columns, the cells with (q + k) % 4 == 2 become six pyramids
    (VTK 14) on the hexahedron's faces around an added centroid point, each base ordered so that the reference's
    pyramid test passes (CPyramid::Change_Orientation does nothing); the rest stay hexahedra. Returns pts,
    elems = [(vtk, nodes)], bnd = {marker: [(vtk, nodes)]}."""
    pts, hexes, bnd = jet_mesh3d(nx, ny, nz, **kw)
    nq = len(hexes) // (nz - 1)
    extra, elems = [], []
    n0 = len(pts)
    for c, h in enumerate(hexes):
        k, q = divmod(c, nq)
        if q % 3 == 1:
            elems.append((13, [h[0], h[1], h[2], h[4], h[5], h[6]]))
            elems.append((13, [h[0], h[2], h[3], h[4], h[6], h[7]]))
        elif (q + k) % 4 == 2:
            apex = n0 + len(extra)
            extra.append(pts[h].mean(axis=0))
            X = lambda p: pts[p] if p < n0 else extra[p - n0]  # noqa: E731
            for f in HEX_FACES:
                b = [int(h[v]) for v in f]
                if _orient3(X(b[0]), X(b[1]), X(b[2]), X(apex)) < 0 or _orient3(X(b[2]), X(b[3]), X(b[0]), X(apex)) < 0:
                    b = [b[0], b[3], b[2], b[1]]
                assert _orient3(X(b[0]), X(b[1]), X(b[2]), X(apex)) >= 0 and _orient3(X(b[2]), X(b[3]), X(b[0]), X(apex)) >= 0
                elems.append((14, b + [apex]))
        else:
            elems.append((12, [int(v) for v in h]))
    pts = np.concatenate([pts, np.asarray(extra).reshape(-1, 3)])
    out = {}
    for name, quads in bnd.items():
        lst = []
        for qi, qd in enumerate(quads):
            qd = [int(v) for v in qd]
            if name in ("sym_back", "sym_front") and qi % 3 == 1:
                if name == "sym_back":  # (q0, q1, q2, q3): diagonal q0 - q2
                    lst += [(5, [qd[0], qd[1], qd[2]]), (5, [qd[0], qd[2], qd[3]])]
                else:  # reversed (q3, q2, q1, q0) + offset: the same diagonal
                    lst += [(5, [qd[1], qd[2], qd[3]]), (5, [qd[3], qd[0], qd[1]])]
            else:
                lst.append((9, qd))
        out[name] = lst
    return pts, elems, out


def write_su2_mixed(path: str, pts, elems, bnd):
    """SU2 native mesh file of a mesh with element kinds given per element: elems = [(vtk, nodes)], bnd = {marker:
    [(vtk, nodes)]} in marker order."""
    with open(path, "w") as f:
        f.write(f"NDIME= {pts.shape[1]}\n")
        f.write(f"NELEM= {len(elems)}\n")
        for k, (t, nodes) in enumerate(elems):
            f.write(f"{t} " + " ".join(str(int(v)) for v in nodes) + f" {k}\n")
        f.write(f"NPOIN= {len(pts)}\n")
        for k, p in enumerate(pts):
            f.write(" ".join(f"{c:.17g}" for c in p) + f" {k}\n")
        f.write(f"NMARK= {len(bnd)}\n")
        for name, lst in bnd.items():
            f.write(f"MARKER_TAG= {name}\nMARKER_ELEMS= {len(lst)}\n")
            for t, nodes in lst:
                f.write(f"{t} " + " ".join(str(int(v)) for v in nodes) + "\n")


def median_dual3d(pts, hexes, bnd):
    """3-D median dual of a hexahedral mesh, vectorised restatement of CPhysicalGeometry::SetControlVolume
    (geometry_structure.cpp:10457-10560, 3-D branch): for every face edge (i, j) of every element the triangle
    (edge midpoint, face centroid, element centroid) adds 1/2 (E - e) x (F - e) to the edge normal, negated when
    i > j (CEdge::SetNodes_Coord, dual_grid_structure.cpp:479-505), and the tetrahedra (point, e, F, E) add to
    both dual volumes (CEdge::GetVolume :425-453). Boundary vertex normals: CPhysicalGeometry::SetBoundControlVolume
    (:9595-9660, 3-D branch) with CVertex::SetNodes_Coord (dual_grid_structure.cpp:589-616). Sums are taken in
    numpy order (the reference's element order gives the same values up to rounding)."""
    n = len(pts)
    hexes = np.asarray(hexes, dtype=np.int64)
    edges = element_edges(n, hexes)  # the face edges' set
    ukey = edges[:, 0] * n + edges[:, 1]
    emid = 0.5 * (pts[edges[:, 0]] + pts[edges[:, 1]])
    normal = np.zeros((len(edges), 3))
    vol = np.zeros(n)
    # elements in chunks of `blk` (bounded host memory at C5's 7.6 M hexahedra); np.add.at accumulates in element
    # order either way, and the volume pass keeps its two sweeps (all i ends, then all j ends)
    blk = 1 << 19

    def faces(c0, c1):
        h = hexes[c0:c1]
        ecg = pts[h].mean(axis=1)                                     # (nE, 3)
        fnodes = h[:, HEX_FACES]                                      # (nE, 6, 4)
        fcg = pts[fnodes].mean(axis=2)                                # (nE, 6, 3)
        fi = fnodes.reshape(-1, 4).ravel()
        fj = np.roll(fnodes, -1, axis=2).reshape(-1, 4).ravel()      # (nE*24,)
        F = np.repeat(fcg.reshape(-1, 3), 4, axis=0)
        E = np.repeat(ecg, 24, axis=0)
        inv = np.searchsorted(ukey, np.minimum(fi, fj) * n + np.maximum(fi, fj))
        return fi, fj, F, E, inv

    vj = []  # the j ends' volume terms, added after every i end's
    for c0 in range(0, len(hexes), blk):
        fi, fj, F, E, inv = faces(c0, c0 + blk)
        e = emid[inv]
        contrib = 0.5 * np.cross(E - e, F - e)
        contrib[fi > fj] *= -1.0
        np.add.at(normal, inv, contrib)
        for end, P_ in enumerate((fi, fj)):
            P = pts[P_]
            t = np.abs(np.einsum("ij,ij->i", E - P, np.cross(e - P, F - P))) / 6.0
            if end == 0:
                np.add.at(vol, P_, t)
            else:
                vj.append((P_, t))
    for P_, t in vj:
        np.add.at(vol, P_, t)
    nb_i = np.r_[edges[:, 0], edges[:, 1]]
    nb_j = np.r_[edges[:, 1], edges[:, 0]]
    order = np.lexsort((nb_j, nb_i))
    nb_i, nb_j = nb_i[order], nb_j[order]
    nbr_ptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(nbr_ptr, nb_i + 1, 1)
    nbr_ptr = np.cumsum(nbr_ptr)
    bv, bn = [], []
    for m, name in enumerate(bnd.keys()):
        q = np.asarray(bnd[name], dtype=np.int64)
        C = pts[q].mean(axis=1)
        acc = np.zeros((n, 3))
        for k in range(4):
            V = pts[q[:, k]]
            e0 = 0.5 * (V + pts[q[:, QUAD_NEIGHBORS[k, 0]]])
            e1 = 0.5 * (V + pts[q[:, QUAD_NEIGHBORS[k, 1]]])
            np.add.at(acc, q[:, k], 0.5 * np.cross(V - C, e0 - C) + 0.5 * np.cross(V - e1, C - e1))
        verts = np.unique(q)
        bv.append(np.c_[np.full(len(verts), m), verts])
        bn.append(acc[verts])
    return dict(edges=edges, edge_normal=normal, volume=vol, nbr_ptr=nbr_ptr, nbr=nb_j.astype(np.int64),
                bvertex=np.concatenate(bv).astype(np.int64), bvertex_normal=np.concatenate(bn))


def write_su2(path: str, pts, quads, bnd):
    """SU2 native mesh file: quads (VTK 9) + boundary lines (VTK 3) in 2-D, hexahedra (VTK 12) + boundary quads
    (VTK 9) in 3-D; markers in the order of `bnd`."""
    nd = pts.shape[1]
    elem_t, bnd_t = (9, 3) if nd == 2 else (12, 9)
    with open(path, "w") as f:
        f.write(f"NDIME= {nd}\n")
        f.write(f"NELEM= {len(quads)}\n")
        for k, q in enumerate(quads):
            f.write(f"{elem_t} " + " ".join(str(int(v)) for v in q) + f" {k}\n")
        f.write(f"NPOIN= {len(pts)}\n")
        for k, p in enumerate(pts):
            f.write(" ".join(f"{c:.17g}" for c in p) + f" {k}\n")
        f.write(f"NMARK= {len(bnd)}\n")
        for name in (MARKERS if nd == 2 else bnd.keys()):
            lines = bnd[name]
            f.write(f"MARKER_TAG= {name}\nMARKER_ELEMS= {len(lines)}\n")
            for l in lines:
                f.write(f"{bnd_t} " + " ".join(str(int(v)) for v in l) + "\n")


def element_edges(n, elems):
    """The edge set (i < j, lexicographic) of a quad or hexahedral mesh: the edges median_dual2d / median_dual3d
    produce, without their geometry (the partitioner and the RCM ordering need only the graph)."""
    elems = np.asarray(elems, dtype=np.int64)
    if elems.shape[1] == 4:
        a, b = elems, np.roll(elems, -1, axis=1)
    else:  # hexahedron: the 4 edges of the bottom face, of the top face, and the 4 vertical edges
        a = np.concatenate([elems[:, :4], elems[:, 4:], elems[:, :4]], axis=1)
        b = np.concatenate([np.roll(elems[:, :4], -1, axis=1), np.roll(elems[:, 4:], -1, axis=1), elems[:, 4:]],
                           axis=1)
    lo, hi = np.minimum(a, b).ravel(), np.maximum(a, b).ravel()
    ukey = np.unique(lo * n + hi)
    return np.stack([ukey // n, ukey % n], axis=1).astype(np.int64)


def rcm_order(n, edges):
    """Reverse Cuthill-McKee permutation (new -> old) of the point graph."""
    import scipy.sparse as sp
    from scipy.sparse.csgraph import reverse_cuthill_mckee
    i, j = edges[:, 0], edges[:, 1]
    A = sp.coo_matrix((np.ones(2 * len(i)), (np.r_[i, j], np.r_[j, i])), shape=(n, n)).tocsr()
    return np.asarray(reverse_cuthill_mckee(A, symmetric_mode=True), dtype=np.int64)


def median_dual2d(pts, quads, bnd):
    """Edges (i<j), edge normals, dual volumes, neighbour CSR and boundary vertices.

    Vectorised restatement of the reference 2-D dual construction (see module docstring).
    """
    n = len(pts)
    cg = pts[quads].mean(axis=1)  # element centroids
    faces = np.stack([quads, np.roll(quads, -1, axis=1)], axis=2).reshape(-1, 2)  # (4*nelem, 2)
    fcg = np.repeat(cg, 4, axis=0)
    lo = np.minimum(faces[:, 0], faces[:, 1])
    hi = np.maximum(faces[:, 0], faces[:, 1])
    key = lo * n + hi
    ukey, inv = np.unique(key, return_inverse=True)
    edges = np.stack([ukey // n, ukey % n], axis=1).astype(np.int64)
    emid = 0.5 * (pts[edges[:, 0]] + pts[edges[:, 1]])
    # normal contribution: (Elem_CG - Edge_CG) rotated, oriented from lo to hi
    d = fcg - emid[inv]
    contrib = np.stack([d[:, 1], -d[:, 0]], axis=1)
    flip = faces[:, 0] > faces[:, 1]
    contrib[flip] *= -1.0
    normal = np.zeros((len(edges), 2))
    np.add.at(normal, inv, contrib)
    # dual volumes: triangles (point, edge midpoint, element centroid) on both face ends
    vol = np.zeros(n)
    for end in (0, 1):
        p = pts[faces[:, end]]
        a = emid[inv] - p
        b = fcg - p
        np.add.at(vol, faces[:, end], 0.5 * np.abs(a[:, 0] * b[:, 1] - a[:, 1] * b[:, 0]))
    # neighbour CSR (sorted)
    nb_i = np.r_[edges[:, 0], edges[:, 1]]
    nb_j = np.r_[edges[:, 1], edges[:, 0]]
    order = np.lexsort((nb_j, nb_i))
    nb_i, nb_j = nb_i[order], nb_j[order]
    nbr_ptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(nbr_ptr, nb_i + 1, 1)
    nbr_ptr = np.cumsum(nbr_ptr)
    # boundary vertex normals: each line element gives half its outward normal to each end
    bverts = []
    for m, name in enumerate(MARKERS):
        lines = bnd[name]
        acc = {}
        for l in lines:
            p0, p1 = pts[l[0]], pts[l[1]]
            t = p1 - p0
            half = 0.5 * np.array([-t[1], t[0]])  # CVertex::SetNodes_Coord, both line ends
            for v in (l[0], l[1]):
                acc[v] = acc.get(v, 0.0) + half
        for v in sorted(acc):
            bverts.append((m, v, acc[v][0], acc[v][1]))
    bv = np.array([(b[0], b[1]) for b in bverts], dtype=np.int64)
    bn = np.array([(b[2], b[3]) for b in bverts], dtype=np.float64)
    return dict(edges=edges, edge_normal=normal, volume=vol, nbr_ptr=nbr_ptr, nbr=nb_j.astype(np.int64),
                bvertex=bv, bvertex_normal=bn)


def median_dual(pts, elems, bnd):
    """Median dual of a 2-D quad or 3-D hexahedral mesh."""
    return median_dual3d(pts, elems, bnd) if pts.shape[1] == 3 else median_dual2d(pts, elems, bnd)


def renumber(pts, quads, bnd, perm):
    """Apply a new->old permutation to points and connectivity."""
    old2new = np.empty_like(perm)
    old2new[perm] = np.arange(len(perm))
    return pts[perm], old2new[quads], {k: old2new[v] for k, v in bnd.items()}, old2new


def partition_rcb(coord, n_part: int, edges=None):
    """Recursive coordinate bisection into n_part balanced parts (stand-in for the reference's METIS
    k-way call, geometry_structure.cpp:11465-11530: any partition is valid input, the solver records
    it). Returns the part id of every point.

    edges None: each cut is across the longer extent normalised by the domain's. With the mesh edges, the
    extent is measured in mesh spacings (extent / median length of the part's edges running along that axis),
    i.e. in cells, so parts come out square in the graph and the edge cut approaches the grid's
    isoperimetric bound (tools/edge_cut.py, profiles/r02_edge_cut.json) on stretched meshes too."""
    part = np.zeros(len(coord), dtype=np.int64)
    nd = coord.shape[1]
    if edges is not None:
        edges = np.asarray(edges)
        d = np.abs(coord[edges[:, 1]] - coord[edges[:, 0]])
        along = np.argmax(d, axis=1)
        inside = np.zeros(len(coord), dtype=bool)

    def axis_of(idx, eidx):
        ext = coord[idx].max(axis=0) - coord[idx].min(axis=0)
        if edges is None:
            return int(np.argmax(ext / np.maximum(dom, 1e-300)))
        cells = np.zeros(nd)
        for a in range(nd):
            da = d[eidx[along[eidx] == a], a]
            h = np.median(da) if len(da) else ext[a] / max(1.0, len(idx) ** (1.0 / nd))
            cells[a] = ext[a] / max(h, 1e-300)
        return int(np.argmax(cells))

    def split(idx, eidx, p0, np_):
        if np_ == 1:
            part[idx] = p0
            return
        left = np_ // 2
        ax = axis_of(idx, eidx)
        o = idx[np.argsort(coord[idx, ax], kind="stable")]
        cut = int(round(len(o) * left / np_))
        lo, hi = o[:cut], o[cut:]
        el = eh = None
        if edges is not None:
            inside[lo] = True
            inside[hi] = False
            a, b = inside[edges[eidx, 0]], inside[edges[eidx, 1]]
            el = eidx[a & b]
            eh = eidx[~a & ~b]
        split(lo, el, p0, left)
        split(hi, eh, p0 + left, np_ - left)

    dom = coord.max(axis=0) - coord.min(axis=0)
    split(np.arange(len(coord)), None if edges is None else np.arange(len(edges)), 0, int(n_part))
    return part


def graph_csr(n, edges):
    """CSR adjacency (xadj [n+1], adj) of the undirected edge list, both directions, neighbours in increasing order."""
    e = np.asarray(edges, dtype=np.int64)
    a, b = np.r_[e[:, 0], e[:, 1]], np.r_[e[:, 1], e[:, 0]]
    o = np.lexsort((b, a))
    a, b = a[o], b[o]
    xadj = np.zeros(n + 1, dtype=np.int64)
    np.add.at(xadj, a + 1, 1)
    return np.cumsum(xadj), np.ascontiguousarray(b, dtype=np.int64)


def partition_graph(n, edges, n_part: int, imbalance: float = 0.03):
    """Multilevel graph partition of the points (rx_partition_graph, csrc/rx_part.cpp: recursive bisection with
    heavy-edge coarsening and FM refinement, then a k-way boundary pass) — the graph-based stand-in for the reference's
    METIS call (geometry_structure.cpp:11360-11450), within a few percent of METIS's edge cut on the jet grids
    (tools/edge_cut.py -> profiles/r05_edge_cut.json). Returns the part id of every point."""
    import ctypes as C
    import os
    lib = C.CDLL(os.environ.get("RX_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "librx.so")))
    xadj, adj = graph_csr(n, edges)
    part = np.zeros(n, dtype=np.int32)
    rc = lib.rx_partition_graph(C.c_int64(n), xadj.ctypes.data_as(C.c_void_p), adj.ctypes.data_as(C.c_void_p),
                                C.c_int32(n_part), C.c_double(imbalance), part.ctypes.data_as(C.c_void_p), None)
    if rc != 0:
        raise ValueError(f"rx_partition_graph failed (status {rc})")
    return part.astype(np.int64)


def partition_order(n, edges, part):
    """New->old permutation: partitions in order, each one RCM-ordered on its own subgraph (the
    reference renumbers every rank's domain points with RCM, CPhysicalGeometry::SetRCM_Ordering)."""
    import scipy.sparse as sp
    from scipy.sparse.csgraph import reverse_cuthill_mckee
    i, j = edges[:, 0], edges[:, 1]
    same = part[i] == part[j]
    A = sp.coo_matrix((np.ones(2 * same.sum()), (np.r_[i[same], j[same]], np.r_[j[same], i[same]])),
                      shape=(n, n)).tocsr()
    perm, ptr = [], [0]
    for p in range(int(part.max()) + 1):
        idx = np.nonzero(part == p)[0]
        sub = A[idx][:, idx]
        perm.append(idx[np.asarray(reverse_cuthill_mckee(sub, symmetric_mode=True), dtype=np.int64)])
        ptr.append(ptr[-1] + len(idx))
    return np.concatenate(perm), np.asarray(ptr, dtype=np.int64)


def build_jet(nx: int, ny: int, rcm: bool = True, n_part: int = 1, nz: int = 0, partitioner: str = "coord", **kw):
    """Synthetic jet mesh ready for the solver: RCM-ordered points + median dual (nz > 1: the 3-D extrusion).

    n_part > 1: points are split into n_part RCB parts (the reference's MPI ranks), numbered part by
    part with a local RCM; `part_ptr` gives the row range of every part. partitioner "coord" (default: the
    partitions every golden, size test and bench line was measured on), "spacing" (cuts in mesh spacings:
    within 2 % of the grid's edge-cut bound, profiles/r02_edge_cut.json) or "graph" (partition_graph, the multilevel
    graph partitioner, for meshes whose coordinates say little about their connectivity)."""
    pts, quads, bnd = jet_mesh3d(nx, ny, nz, **kw) if nz > 1 else jet_mesh(nx, ny, **kw)
    median_dual = median_dual3d if nz > 1 else median_dual2d
    part_ptr = np.array([0, len(pts)], dtype=np.int64)
    if n_part > 1:
        e0 = element_edges(len(pts), quads)
        part = (partition_graph(len(pts), e0, n_part) if partitioner == "graph" else
                partition_rcb(pts, n_part, edges=e0 if partitioner == "spacing" else None))
        perm, part_ptr = partition_order(len(pts), e0, part)
        pts, quads, bnd, _ = renumber(pts, quads, bnd, perm)
    elif rcm:
        perm = rcm_order(len(pts), element_edges(len(pts), quads))
        pts, quads, bnd, _ = renumber(pts, quads, bnd, perm)
    dual = median_dual(pts, quads, bnd)
    dual["coord"] = pts
    dual["quads"] = quads
    dual["part_ptr"] = part_ptr
    dual["wall_distance"] = wall_distance(pts, bnd)
    dual["bvertex_pn"] = normal_neighbor(pts, dual["nbr_ptr"], dual["nbr"], dual["bvertex"], dual["bvertex_normal"])
    return dual


def normal_neighbor(coord, nbr_ptr, nbr, bvertex, bvertex_normal):
    """CPhysicalGeometry::FindNormal_Neighbor (Common/src/geometry_structure.cpp:12610-12652): for every boundary
    vertex the neighbour whose edge makes the largest cosine with the vertex normal (the last one on ties, the
    reference's `>=`), with the reference's arithmetic (per-component sums in dimension order, then
    sp / (sqrt(nv) sqrt(nn)); evaluated for all (vertex, neighbour) pairs at once)."""
    coord = np.asarray(coord, dtype=np.float64)
    bv = np.asarray(bvertex)
    nbr_ptr, nbr = np.asarray(nbr_ptr), np.asarray(nbr)
    if len(bv) == 0:
        return np.zeros(0, dtype=np.int64)
    i = bv[:, 1].astype(np.int64)
    cnt = nbr_ptr[i + 1] - nbr_ptr[i]
    seg = np.repeat(np.arange(len(bv)), cnt)
    start = np.cumsum(cnt) - cnt
    j = nbr[np.repeat(nbr_ptr[i], cnt) + (np.arange(cnt.sum()) - np.repeat(start, cnt))]
    n = np.asarray(bvertex_normal, dtype=np.float64)[seg]
    sp = np.zeros(len(j))
    nv = np.zeros(len(j))
    nn = np.zeros(len(j))
    for d in range(coord.shape[1]):
        dc = coord[j, d] - coord[i[seg], d]
        sp += dc * n[:, d]
        nv += dc * dc
        nn += n[:, d] * n[:, d]
    c = sp / (np.sqrt(nv) * np.sqrt(nn))
    cmax = np.maximum.reduceat(c, start)
    # the last neighbour reaching the maximum (the loop's `c >= cmax` keeps moving to later ties)
    pos = np.where(c == cmax[seg], np.arange(len(c)), -1)
    last = np.maximum.reduceat(pos, start)
    return j[last].astype(np.int64)


WALLS = ("upper_wall", "lower_wall_pre", "lower_wall_post")  # the cfg's MARKER_ISOTHERMAL


def wall_distance(pts, bnd):
    """Distance of every point to the nearest wall vertex (CGeometry::ComputeWall_Distance: points of the
    viscous-wall markers; wall points get 0)."""
    from scipy.spatial import cKDTree
    wp = np.unique(np.concatenate([np.asarray(bnd[m]).ravel() for m in WALLS]))
    d, _ = cKDTree(pts[wp]).query(pts, workers=-1)
    return np.ascontiguousarray(d, dtype=np.float64)


def shard(mesh, n_ranks: int, rank: int):
    """The local mesh of one MPI rank / GPU: the rank owns a contiguous block of the global partitions
    (points [g0, g1) of the partition-major numbering) plus one halo layer, like the reference's
    partitioned CGeometry (geometry_structure.cpp:11465-11530: domain points, then halo points).

    Local numbering: own points in global order, then halo points in global order (so the halo is
    contiguous per owning rank). Local edges: every global edge with an own endpoint, in the global edge
    order and orientation (an edge whose halo end has the lower local id keeps its global direction).
    LSQ neighbour lists of own points keep the global order; halo points keep only their local neighbours
    (their gradients are overwritten by the halo exchange). `l2g` (the global point numbers) also orders
    each BSR row by global column (rx_mesh_desc.global_id). So every owned point gathers the same
    contributions in the same order as the undivided mesh: the rank's residual, Jacobian rows, gradient,
    limiter, time step and SpMV rows are bitwise the single-context ones, and only the inner products
    (rank-local partial sums, then the rank-ordered sum) differ.
    The reference's own MPI ranks renumber edges and matrix columns locally (SetEdges / CSysMatrix on the
    rank's CGeometry), which changes rounding but no formula; keeping the global order makes the sharded
    iteration checkable against the undivided oracle. Returns the local mesh dict plus the exchange plan
    (`neigh`, `send_ptr`, `send_idx`, `recv_ptr`, `n_domain`) and `l2g`.
    """
    pp = np.asarray(mesh["part_ptr"], dtype=np.int64)
    P = len(pp) - 1
    assert P % n_ranks == 0 or P >= n_ranks, "need at least one partition per rank"
    pr = np.array_split(np.arange(P), n_ranks)
    rank_ptr = np.array([pp[c[0]] for c in pr] + [pp[-1]], dtype=np.int64)
    g0, g1 = int(rank_ptr[rank]), int(rank_ptr[rank + 1])
    owner = np.searchsorted(rank_ptr, np.arange(pp[-1]), side="right") - 1
    e = np.asarray(mesh["edges"], dtype=np.int64)
    own_e = ((e[:, 0] >= g0) & (e[:, 0] < g1)) | ((e[:, 1] >= g0) & (e[:, 1] < g1))
    ends = np.unique(e[own_e].ravel())
    halo = ends[(ends < g0) | (ends >= g1)]
    n_own = g1 - g0
    l2g = np.concatenate([np.arange(g0, g1, dtype=np.int64), halo])
    g2l = np.full(int(pp[-1]), -1, dtype=np.int64)
    g2l[l2g] = np.arange(len(l2g))
    le = g2l[e[own_e]]
    ln = np.ascontiguousarray(np.asarray(mesh["edge_normal"])[own_e])
    # LSQ neighbours
    nptr_g, nbr_g = np.asarray(mesh["nbr_ptr"]), np.asarray(mesh["nbr"])
    cnt = nptr_g[l2g + 1] - nptr_g[l2g]
    idx = np.repeat(nptr_g[l2g], cnt) + (np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt))
    row = np.repeat(np.arange(len(l2g)), cnt)
    lj = g2l[nbr_g[idx]]
    ok = lj >= 0  # own points have every neighbour locally; halo points keep their local ones
    nbr_l = lj[ok]
    nptr_l = np.zeros(len(l2g) + 1, dtype=np.int64)
    np.add.at(nptr_l, row[ok] + 1, 1)
    nptr_l = np.cumsum(nptr_l)
    # boundary vertices of own points
    bv = np.asarray(mesh["bvertex"])[:, :2]
    keep = (bv[:, 1] >= g0) & (bv[:, 1] < g1)
    lbv = np.stack([bv[keep, 0], bv[keep, 1] - g0], axis=1).astype(np.int64) if keep.any() else np.zeros((0, 2),
                                                                                                         np.int64)
    # exchange plan with every neighbouring rank
    neigh = sorted({int(owner[h]) for h in halo})
    recv_ptr = [0]
    for q in neigh:
        recv_ptr.append(recv_ptr[-1] + int(np.sum(owner[halo] == q)))
    send_ptr, send_idx = [0], []
    for q in neigh:
        # points of mine in rank q's halo, in global order (= q's halo order)
        qa, qb = rank_ptr[q], rank_ptr[q + 1]
        q_e = ((e[:, 0] >= qa) & (e[:, 0] < qb)) | ((e[:, 1] >= qa) & (e[:, 1] < qb))
        qe = np.unique(e[q_e].ravel())
        mine = qe[(qe >= g0) & (qe < g1)]
        send_idx.extend((mine - g0).tolist())
        send_ptr.append(len(send_idx))
    lpp = pp[pr[rank][0]:pr[rank][-1] + 2] - g0
    extra = {"wall_distance": np.asarray(mesh["wall_distance"])[l2g]} if "wall_distance" in mesh else {}
    if "bvertex_pn" in mesh:  # normal neighbours: neighbours of own points, hence local
        extra["bvertex_pn"] = g2l[np.asarray(mesh["bvertex_pn"])[keep]]
    return dict(**extra, edges=le, edge_normal=ln, coord=np.asarray(mesh["coord"])[l2g],
                volume=np.asarray(mesh["volume"])[l2g], nbr_ptr=nptr_l, nbr=nbr_l.astype(np.int64), bvertex=lbv,
                bvertex_normal=np.asarray(mesh["bvertex_normal"])[keep], part_ptr=lpp.astype(np.int64),
                n_domain=n_own, l2g=l2g, neigh=np.asarray(neigh, dtype=np.int32),
                send_ptr=np.asarray(send_ptr, dtype=np.int64), send_idx=np.asarray(send_idx, dtype=np.int64),
                recv_ptr=np.asarray(recv_ptr, dtype=np.int64), rank_ptr=rank_ptr)
