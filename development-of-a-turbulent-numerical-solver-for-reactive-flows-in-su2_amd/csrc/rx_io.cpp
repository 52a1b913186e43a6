// rx_io.cpp — host-side setup and on-disk formats: the SU2 mesh reader with the
// reference's dual-grid preprocessing, the reacting-library file readers and the restart format. See
// include/rx_io.h for the reference functions each entry point restates. Plain C++ (no device code); compiled
// with -ffp-contract=off so the geometry rounds exactly as the x86-64 reference build.
#include "../../include/rx_io.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace {

constexpr double kEPS = 1.0e-16;  // EPS (Common/include/option_structure.hpp)

// ---- primal element tables (Common/src/primal_grid_structure.cpp)
struct ElemType {
  int vtk, nnodes, nfaces;
  int faces[6][4];
  int nnodes_face[6];
  int nneigh[8];
  int neigh[8][4];
};
const ElemType kLine = {3, 2, 1, {{0, 1}}, {2}, {1, 1}, {{1}, {0}}};
const ElemType kTri = {5, 3, 3, {{0, 1}, {1, 2}, {2, 0}}, {2, 2, 2}, {2, 2, 2}, {{1, 2}, {2, 0}, {0, 1}}};
const ElemType kQuad = {9, 4, 4, {{0, 1}, {1, 2}, {2, 3}, {3, 0}}, {2, 2, 2, 2}, {2, 2, 2, 2},
                        {{1, 3}, {2, 0}, {3, 1}, {0, 2}}};
const ElemType kTet = {10, 4, 4, {{0, 2, 1}, {0, 1, 3}, {0, 3, 2}, {1, 2, 3}}, {3, 3, 3, 3}, {3, 3, 3, 3},
                       {{1, 2, 3}, {0, 2, 3}, {0, 1, 3}, {0, 1, 2}}};
const ElemType kHex = {12, 8, 6,
                       {{0, 1, 5, 4}, {1, 2, 6, 5}, {2, 3, 7, 6}, {3, 0, 4, 7}, {0, 3, 2, 1}, {4, 5, 6, 7}},
                       {4, 4, 4, 4, 4, 4}, {3, 3, 3, 3, 3, 3, 3, 3},
                       {{1, 3, 4}, {0, 2, 5}, {1, 3, 6}, {0, 2, 7}, {0, 5, 7}, {4, 6, 1}, {2, 5, 7}, {4, 3, 6}}};
// CPrism / CPyramid (primal_grid_structure.cpp:478-494, 566-582): the triangular faces of a prism and the
// triangular faces of a pyramid carry a repeated fourth entry the face loops never reach (nNodesFace = 3)
const ElemType kPrism = {13, 6, 5, {{3, 4, 1, 0}, {5, 2, 1, 4}, {2, 5, 3, 0}, {0, 1, 2, 2}, {5, 4, 3, 3}},
                         {4, 4, 4, 3, 3}, {3, 3, 3, 3, 3, 3},
                         {{1, 2, 3}, {0, 2, 4}, {1, 0, 5}, {0, 4, 5}, {3, 5, 1}, {4, 3, 2}}};
const ElemType kPyramid = {14, 5, 5, {{0, 3, 2, 1}, {4, 3, 0, 0}, {4, 0, 1, 1}, {2, 4, 1, 1}, {3, 4, 2, 2}},
                           {4, 3, 3, 3, 3}, {3, 3, 3, 3, 4},
                           {{1, 3, 4, 4}, {0, 2, 4, 4}, {1, 3, 4, 4}, {2, 0, 4, 4}, {0, 1, 2, 3}}};
// boundary triangles / quadrilaterals of a 3-D mesh use the 2-D element tables (CTriangle / CQuadrilateral)

const ElemType* elem_type(int vtk) {
  switch (vtk) {
    case 3: return &kLine;
    case 5: return &kTri;
    case 9: return &kQuad;
    case 10: return &kTet;
    case 12: return &kHex;
    case 13: return &kPrism;
    case 14: return &kPyramid;
    default: return nullptr;
  }
}

struct Elem {
  const ElemType* t;
  int64_t n[8];
};

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
  return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}

// "KEY= value" of an SU2 mesh line (the reader matches the keyword at the start of the line)
bool keyword(const std::string& line, const char* key, std::string* val) {
  const size_t n = std::strlen(key);
  if (line.compare(0, n, key) != 0) return false;
  *val = trim(line.substr(n));
  return true;
}

}  // namespace

struct rx_mesh {
  int nDim = 2;
  int64_t N = 0;
  std::vector<double> coord;        // [N][nDim], RCM order
  std::vector<int64_t> gidx;        // [N] global (file) index
  std::vector<Elem> elems;          // interior elements (node ids in RCM order)
  std::vector<std::string> tags;    // MARKER_TAG per marker
  std::vector<std::vector<Elem>> bound;
  std::vector<std::vector<int64_t>> nb, nb_edge;  // neighbour lists (reference order) and their edge ids
  std::vector<int64_t> edges;       // [E][2], i < j, SetEdges discovery order
  std::vector<double> normal, vol;  // [E][nDim], [N]
  std::vector<int64_t> nbr_ptr, nbr;
  std::vector<int64_t> bvert;       // [nB][2] (marker, point)
  std::vector<double> bnormal;      // [nB][nDim]
  std::vector<int64_t> pn;          // [nB] normal neighbour
  std::vector<double> wall;         // [N]
};

namespace {

// CPhysicalGeometry::SetPoint_Connectivity (geometry_structure.cpp:9145-9198): per point, the elements in element
// order, in each the element's neighbour nodes of that point, appended when new (CPoint::SetPoint).
void point_connectivity(rx_mesh& m) {
  std::vector<std::vector<int64_t>> pe(m.N);
  for (size_t e = 0; e < m.elems.size(); ++e)
    for (int a = 0; a < m.elems[e].t->nnodes; ++a) pe[m.elems[e].n[a]].push_back((int64_t)e);
  m.nb.assign(m.N, {});
  for (int64_t i = 0; i < m.N; ++i)
    for (int64_t e : pe[i]) {
      const Elem& el = m.elems[e];
      for (int a = 0; a < el.t->nnodes; ++a)
        if (el.n[a] == i)
          for (int k = 0; k < el.t->nneigh[a]; ++k) {
            const int64_t j = el.n[el.t->neigh[a][k]];
            if (std::find(m.nb[i].begin(), m.nb[i].end(), j) == m.nb[i].end()) m.nb[i].push_back(j);
          }
    }
}

// CPhysicalGeometry::SetRCM_Ordering (:9200-9340): new -> old permutation. Start at the lowest-degree point (the
// first minimum, with node 0's degree as the initial minimum), breadth-first over neighbours in list order, each
// level's new points bubble-sorted by degree (stable), then reversed.
std::vector<int64_t> rcm(const rx_mesh& m) {
  const int64_t n = m.N;
  std::vector<char> inq(n, 0);
  size_t mind = m.nb[0].size();
  int64_t add = 0;
  for (int64_t i = 1; i < n; ++i)
    if (m.nb[i].size() < mind) {
      mind = m.nb[i].size();
      add = i;
    }
  std::vector<int64_t> res{add}, queue;
  size_t head = 0;
  inq[add] = 1;
  do {
    std::vector<int64_t> aux;
    for (int64_t j : m.nb[add])
      if (!inq[j]) aux.push_back(j);
    for (size_t a = 0; a < aux.size(); ++a)
      for (size_t b = 0; b + 1 + a < aux.size(); ++b)
        if (m.nb[aux[b]].size() > m.nb[aux[b + 1]].size()) std::swap(aux[b], aux[b + 1]);
    for (int64_t j : aux) {
      queue.push_back(j);
      inq[j] = 1;
    }
    if (head < queue.size()) {
      add = queue[head++];
      res.push_back(add);
    }
  } while (head < queue.size());
  for (int64_t i = 0; i < n; ++i)
    if (!inq[i]) res.push_back(i);
  std::reverse(res.begin(), res.end());
  return res;
}

// CGeometry::SetEdges (:223-252): edges numbered in discovery order over points and their neighbour lists.
void set_edges(rx_mesh& m) {
  m.nb_edge.assign(m.N, {});
  for (int64_t i = 0; i < m.N; ++i) m.nb_edge[i].assign(m.nb[i].size(), -1);
  m.edges.clear();
  for (int64_t i = 0; i < m.N; ++i)
    for (size_t k = 0; k < m.nb[i].size(); ++k) {
      const int64_t j = m.nb[i][k];
      const auto& nj = m.nb[j];
      const size_t kk = (size_t)(std::find(nj.begin(), nj.end(), i) - nj.begin());
      if (m.nb_edge[j][kk] == -1) {
        const int64_t e = (int64_t)m.edges.size() / 2;
        m.nb_edge[i][k] = e;
        m.nb_edge[j][kk] = e;
        m.edges.push_back(std::min(i, j));
        m.edges.push_back(std::max(i, j));
      } else {
        m.nb_edge[i][k] = m.nb_edge[j][kk];
      }
    }
}

int64_t find_edge(const rx_mesh& m, int64_t i, int64_t j) {
  const auto& ni = m.nb[i];
  const size_t k = (size_t)(std::find(ni.begin(), ni.end(), j) - ni.begin());
  return k < ni.size() ? m.nb_edge[i][k] : -1;
}

// CPrimalGrid::SetCoord_CG (primal_grid_structure.cpp:57-82): element / face centroids, each term divided first.
void elem_cg(const rx_mesh& m, const Elem& el, double* cg, double (*fcg)[3]) {
  const int nd = m.nDim;
  for (int d = 0; d < nd; ++d) {
    cg[d] = 0.0;
    for (int a = 0; a < el.t->nnodes; ++a) cg[d] += m.coord[el.n[a] * nd + d] / double(el.t->nnodes);
  }
  if (!fcg) return;
  for (int f = 0; f < el.t->nfaces; ++f)
    for (int d = 0; d < nd; ++d) {
      fcg[f][d] = 0.0;
      const int nf = el.t->nnodes_face[f];
      for (int a = 0; a < nf; ++a) fcg[f][d] += m.coord[el.n[el.t->faces[f][a]] * nd + d] / double(nf);
    }
}

// CEdge::SetCoord_CG (dual_grid_structure.cpp:412-421)
void edge_cg(const rx_mesh& m, int64_t e, double* cg) {
  for (int d = 0; d < m.nDim; ++d) {
    cg[d] = 0.0;
    for (int k = 0; k < 2; ++k) cg[d] += m.coord[m.edges[2 * e + k] * m.nDim + d] / 2.0;
  }
}

// CPhysicalGeometry::SetControlVolume (geometry_structure.cpp:10457-10560) with CEdge::SetNodes_Coord / GetVolume
// (dual_grid_structure.cpp:423-540), arguments bound as the reference passes them.
void control_volume(rx_mesh& m) {
  const int nd = m.nDim;
  const int64_t E = (int64_t)m.edges.size() / 2;
  m.normal.assign(E * nd, 0.0);
  m.vol.assign(m.N, 0.0);
  for (const Elem& el : m.elems) {
    double cg[3], fcg[6][3];
    elem_cg(m, el, cg, fcg);
    for (int f = 0; f < el.t->nfaces; ++f) {
      const int nef = nd == 2 ? 1 : el.t->nnodes_face[f];
      for (int ef = 0; ef < nef; ++ef) {
        int64_t fi, fj;
        if (nd == 2) {
          fi = el.n[el.t->faces[f][0]];
          fj = el.n[el.t->faces[f][1]];
        } else {
          fi = el.n[el.t->faces[f][ef]];
          fj = el.n[el.t->faces[f][ef + 1 < nef ? ef + 1 : 0]];
        }
        const bool flip = fi > fj;
        const int64_t e = find_edge(m, fi, fj);
        double ecg[3], pi[3] = {0, 0, 0}, pj[3] = {0, 0, 0};
        edge_cg(m, e, ecg);
        for (int d = 0; d < nd; ++d) {
          pi[d] = m.coord[fi * nd + d];
          pj[d] = m.coord[fj * nd + d];
        }
        double* nrm = &m.normal[e * nd];
        if (nd == 2) {
          // SetNodes_Coord(val_coord_Edge_CG, val_coord_Elem_CG): Normal += (Elem[1]-Edge[1], -(Elem[0]-Edge[0]))
          const double* a = flip ? cg : ecg;  // bound to val_coord_Edge_CG
          const double* b = flip ? ecg : cg;  // bound to val_coord_Elem_CG
          nrm[0] += b[1] - a[1];
          nrm[1] += -(b[0] - a[0]);
          // GetVolume(val_coord_Edge_CG = point, val_coord_Elem_CG = edge CG, val_coord_Point = element CG)
          for (int end = 0; end < 2; ++end) {
            const double* p = end ? pj : pi;
            const double va0 = ecg[0] - cg[0], va1 = ecg[1] - cg[1];
            const double vb0 = p[0] - cg[0], vb1 = p[1] - cg[1];
            m.vol[end ? fj : fi] += 0.5 * std::fabs(va0 * vb1 - va1 * vb0);
          }
        } else {
          // SetNodes_Coord(val_coord_Edge_CG, val_coord_FaceElem_CG, val_coord_Elem_CG)
          const double* ve = flip ? fcg[f] : ecg;
          const double* vf = flip ? ecg : fcg[f];
          double va[3], vb[3];
          for (int d = 0; d < 3; ++d) {
            va[d] = cg[d] - ve[d];
            vb[d] = vf[d] - ve[d];
          }
          nrm[0] += 0.5 * (va[1] * vb[2] - va[2] * vb[1]);
          nrm[1] += -0.5 * (va[0] * vb[2] - va[2] * vb[0]);
          nrm[2] += 0.5 * (va[0] * vb[1] - va[1] * vb[0]);
          // GetVolume(Edge_CG = point, FaceElem_CG = edge CG, Elem_CG = face CG, Point = element CG)
          for (int end = 0; end < 2; ++end) {
            const double* p = end ? pj : pi;
            double a3[3], b3[3], c3[3], d3[3];
            for (int d = 0; d < 3; ++d) {
              a3[d] = p[d] - cg[d];
              b3[d] = ecg[d] - cg[d];
              c3[d] = fcg[f][d] - cg[d];
            }
            d3[0] = a3[1] * b3[2] - a3[2] * b3[1];
            d3[1] = -(a3[0] * b3[2] - a3[2] * b3[0]);
            d3[2] = a3[0] * b3[1] - a3[1] * b3[0];
            m.vol[end ? fj : fi] += std::fabs(c3[0] * d3[0] + c3[1] * d3[1] + c3[2] * d3[2]) / 6.0;
          }
        }
      }
    }
  }
  for (int64_t e = 0; e < E; ++e) {
    double a = 0.0;
    for (int d = 0; d < nd; ++d) a += m.normal[e * nd + d] * m.normal[e * nd + d];
    if (std::sqrt(a) == 0.0)
      for (int d = 0; d < nd; ++d) m.normal[e * nd + d] = kEPS * kEPS;
  }
}

// SetVertex (vertices of a marker in order of first appearance) + SetBoundControlVolume (:9595-9660) with
// CVertex::SetNodes_Coord (dual_grid_structure.cpp:589-640).
void bound_control_volume(rx_mesh& m) {
  const int nd = m.nDim;
  m.bvert.clear();
  m.bnormal.clear();
  for (size_t mk = 0; mk < m.bound.size(); ++mk) {
    std::map<int64_t, int64_t> vid;  // point -> vertex index in this marker
    std::vector<int64_t> pts;
    for (const Elem& be : m.bound[mk])
      for (int a = 0; a < be.t->nnodes; ++a)
        if (vid.emplace(be.n[a], (int64_t)pts.size()).second) pts.push_back(be.n[a]);
    std::vector<double> nrm(pts.size() * nd, 0.0);
    for (const Elem& be : m.bound[mk]) {
      double cg[3];
      elem_cg(m, be, cg, nullptr);
      for (int a = 0; a < be.t->nnodes; ++a) {
        const int64_t ip = be.n[a];
        double* vn = &nrm[vid[ip] * nd];
        double vx[3] = {0, 0, 0};
        for (int d = 0; d < nd; ++d) vx[d] = m.coord[ip * nd + d];
        for (int k = 0; k < be.t->nneigh[a]; ++k) {
          const int64_t jp = be.n[be.t->neigh[a][k]];
          double ecg[3];
          edge_cg(m, find_edge(m, ip, jp), ecg);
          if (nd == 2) {
            const double* e = a == 0 ? cg : vx;  // SetNodes_Coord(val_coord_Edge_CG, val_coord_Elem_CG)
            const double* l = a == 0 ? vx : cg;
            if (a <= 1) {
              vn[0] += l[1] - e[1];
              vn[1] += -(l[0] - e[0]);
            }
          } else if (k <= 1) {
            // k = 0: SetNodes_Coord(Elem_CG, Edge_CG, Vertex); k = 1: SetNodes_Coord(Edge_CG, Elem_CG, Vertex)
            const double* ve = k == 0 ? cg : ecg;
            const double* vf = k == 0 ? ecg : cg;
            double va[3], vb[3];
            for (int d = 0; d < 3; ++d) {
              va[d] = vx[d] - ve[d];
              vb[d] = vf[d] - ve[d];
            }
            vn[0] += 0.5 * (va[1] * vb[2] - va[2] * vb[1]);
            vn[1] += -0.5 * (va[0] * vb[2] - va[2] * vb[0]);
            vn[2] += 0.5 * (va[0] * vb[1] - va[1] * vb[0]);
          }
        }
      }
    }
    for (size_t v = 0; v < pts.size(); ++v) {
      double a = 0.0;
      for (int d = 0; d < nd; ++d) a += nrm[v * nd + d] * nrm[v * nd + d];
      if (std::sqrt(a) == 0.0)
        for (int d = 0; d < nd; ++d) nrm[v * nd + d] = kEPS * kEPS;
      m.bvert.push_back((int64_t)mk);
      m.bvert.push_back(pts[v]);
      for (int d = 0; d < nd; ++d) m.bnormal.push_back(nrm[v * nd + d]);
    }
  }
}

// CPhysicalGeometry::FindNormal_Neighbor (:12610-12652): the neighbour whose edge makes the largest cosine with the
// vertex normal (the last one on ties, `>=`).
void normal_neighbors(rx_mesh& m) {
  const int nd = m.nDim;
  const size_t nB = m.bvert.size() / 2;
  m.pn.assign(nB, 0);
  for (size_t b = 0; b < nB; ++b) {
    const int64_t i = m.bvert[2 * b + 1];
    const double* n = &m.bnormal[b * nd];
    int64_t best = 0;
    double cmax = -1.0;
    for (int64_t j : m.nb[i]) {
      double sp = 0.0, nv = 0.0, nn = 0.0;
      for (int d = 0; d < nd; ++d) {
        const double dc = m.coord[j * nd + d] - m.coord[i * nd + d];
        sp += dc * n[d];
        nv += dc * dc;
        nn += n[d] * n[d];
      }
      const double c = sp / (std::sqrt(nv) * std::sqrt(nn));
      if (c >= cmax) {
        best = j;
        cmax = c;
      }
    }
    m.pn[b] = best;
  }
}

// Orientation tests of CPhysicalGeometry::Check_IntElem_Orientation / Check_BoundElem_Orientation: a = (P2 - P1)/2,
// b = (P3 - P1)/2, 2-D test a x b, 3-D test (a x b) . (P4 - P1).
double orient2(const double* c1, const double* c2, const double* c3) {
  double a[2], b[2];
  for (int d = 0; d < 2; ++d) {
    a[d] = 0.5 * (c2[d] - c1[d]);
    b[d] = 0.5 * (c3[d] - c1[d]);
  }
  return a[0] * b[1] - b[0] * a[1];
}
double orient3(const double* c1, const double* c2, const double* c3, const double* c4) {
  double a[3], b[3], c[3], n[3];
  for (int d = 0; d < 3; ++d) {
    a[d] = 0.5 * (c2[d] - c1[d]);
    b[d] = 0.5 * (c3[d] - c1[d]);
    c[d] = c4[d] - c1[d];
  }
  n[0] = a[1] * b[2] - b[1] * a[2];
  n[1] = -(a[0] * b[2] - b[0] * a[2]);
  n[2] = a[0] * b[1] - b[0] * a[1];
  return n[0] * c[0] + n[1] * c[1] + n[2] * c[2];
}

// The prism test of Check_IntElem_Orientation (geometry_structure.cpp:8641-8684): a = (B - A)/2, b = (C - A)/2,
// c = (D0 - E0) + (D1 - E1) + (D2 - E2) (the three edges joining the triangles), test (a x b) . c.
double orient_prism(const double* A, const double* B, const double* Cc, const double* const D[3],
                    const double* const Ee[3]) {
  double a[3], b[3], c[3], n[3];
  for (int d = 0; d < 3; ++d) {
    a[d] = 0.5 * (B[d] - A[d]);
    b[d] = 0.5 * (Cc[d] - A[d]);
    c[d] = (D[0][d] - Ee[0][d]) + (D[1][d] - Ee[1][d]) + (D[2][d] - Ee[2][d]);
  }
  n[0] = a[1] * b[2] - b[1] * a[2];
  n[1] = -(a[0] * b[2] - b[0] * a[2]);
  n[2] = a[0] * b[1] - b[0] * a[1];
  return n[0] * c[0] + n[1] * c[1] + n[2] * c[2];
}

// Change_Orientation of each element kind (primal_grid_structure.cpp)
void change_orientation(Elem& e) {
  switch (e.t->vtk) {
    case 3: std::swap(e.n[0], e.n[1]); break;   // CLine
    case 5: std::swap(e.n[0], e.n[2]); break;   // CTriangle
    case 9: std::swap(e.n[1], e.n[3]); break;   // CQuadrilateral
    case 10: std::swap(e.n[0], e.n[1]); break;  // CTetrahedron
    case 12: {                                   // CHexahedron
      const int64_t o[8] = {e.n[0], e.n[1], e.n[2], e.n[3], e.n[4], e.n[5], e.n[6], e.n[7]};
      const int map[8] = {7, 4, 5, 6, 3, 0, 1, 2};
      for (int k = 0; k < 8; ++k) e.n[k] = o[map[k]];
      break;
    }
    case 13:  // CPrism (primal_grid_structure.cpp:548-560)
      std::swap(e.n[0], e.n[1]);
      std::swap(e.n[3], e.n[4]);
      break;
    case 14: break;  // CPyramid::Change_Orientation only prints "Not defined orientation change" (:622)
  }
}

// Check_IntElem_Orientation (geometry_structure.cpp:8640-8824) and Check_BoundElem_Orientation (:8825-8960, the
// domain point = the first node of the boundary element's volume element, SetBoundVolume, not on the face).
void check_orientation(rx_mesh& m) {
  const int nd = m.nDim;
  auto X = [&](int64_t p) { return &m.coord[p * nd]; };
  for (Elem& e : m.elems) {
    const int64_t* n = e.n;
    bool flip = false;
    if (e.t->vtk == 5) {
      flip = orient2(X(n[0]), X(n[1]), X(n[2])) < 0.0;
    } else if (e.t->vtk == 9) {
      flip = orient2(X(n[0]), X(n[1]), X(n[2])) < 0.0 && orient2(X(n[1]), X(n[2]), X(n[3])) < 0.0 &&
             orient2(X(n[2]), X(n[3]), X(n[0])) < 0.0 && orient2(X(n[3]), X(n[0]), X(n[2])) < 0.0;
    } else if (e.t->vtk == 10) {
      flip = orient3(X(n[0]), X(n[1]), X(n[2]), X(n[3])) < 0.0;
    } else if (e.t->vtk == 12) {
      flip = orient3(X(n[0]), X(n[1]), X(n[2]), X(n[5])) < 0.0 || orient3(X(n[2]), X(n[3]), X(n[0]), X(n[7])) < 0.0 ||
             orient3(X(n[1]), X(n[2]), X(n[3]), X(n[6])) < 0.0 || orient3(X(n[3]), X(n[0]), X(n[1]), X(n[4])) < 0.0;
    } else if (e.t->vtk == 13) {
      const double* lo[3] = {X(n[0]), X(n[1]), X(n[2])};
      const double* up[3] = {X(n[3]), X(n[4]), X(n[5])};
      flip = orient_prism(lo[0], lo[2], lo[1], up, lo) < 0.0 || orient_prism(up[0], up[1], up[2], lo, up) < 0.0;
    } else if (e.t->vtk == 14) {
      flip = orient3(X(n[0]), X(n[1]), X(n[2]), X(n[4])) < 0.0 || orient3(X(n[2]), X(n[3]), X(n[0]), X(n[4])) < 0.0;
    }
    if (flip) change_orientation(e);
  }
  std::vector<std::vector<int64_t>> pe(m.N);
  for (size_t k = 0; k < m.elems.size(); ++k)
    for (int a = 0; a < m.elems[k].t->nnodes; ++a) pe[m.elems[k].n[a]].push_back((int64_t)k);
  for (auto& bm : m.bound)
    for (Elem& be : bm) {
      auto on_face = [&](int64_t p) { return std::find(be.n, be.n + be.t->nnodes, p) != be.n + be.t->nnodes; };
      const Elem* dom = nullptr;  // the volume element holding every node of the face
      for (int64_t k : pe[be.n[0]]) {
        const Elem& e = m.elems[k];
        int hit = 0;
        for (int a = 0; a < be.t->nnodes; ++a) hit += std::find(e.n, e.n + e.t->nnodes, be.n[a]) != e.n + e.t->nnodes;
        if (hit == be.t->nnodes) {
          dom = &e;
          break;
        }
      }
      if (!dom) continue;
      int64_t pd = dom->n[0];
      for (int a = 0; a < dom->t->nnodes; ++a) {
        pd = dom->n[a];
        if (!on_face(pd)) break;
      }
      const int64_t* n = be.n;
      bool flip = false;
      if (be.t->vtk == 3) {
        flip = orient2(X(n[0]), X(n[1]), X(pd)) < 0.0;
      } else if (be.t->vtk == 5) {
        flip = orient3(X(n[0]), X(n[1]), X(n[2]), X(pd)) < 0.0;
      } else if (be.t->vtk == 9) {
        flip = orient3(X(n[0]), X(n[1]), X(n[2]), X(pd)) < 0.0 && orient3(X(n[1]), X(n[2]), X(n[3]), X(pd)) < 0.0 &&
               orient3(X(n[2]), X(n[3]), X(n[0]), X(pd)) < 0.0 && orient3(X(n[3]), X(n[0]), X(n[2]), X(pd)) < 0.0;
      }
      if (flip) change_orientation(be);
    }
}

// file-order mesh -> the reference's preprocessed mesh
void preprocess(rx_mesh& m) {
  point_connectivity(m);
  const std::vector<int64_t> perm = rcm(m);  // new -> old
  std::vector<int64_t> inv(m.N);
  for (int64_t k = 0; k < m.N; ++k) inv[perm[k]] = k;
  std::vector<double> c(m.coord.size());
  m.gidx.assign(m.N, 0);
  for (int64_t k = 0; k < m.N; ++k) {
    m.gidx[k] = perm[k];
    for (int d = 0; d < m.nDim; ++d) c[k * m.nDim + d] = m.coord[perm[k] * m.nDim + d];
  }
  m.coord.swap(c);
  for (Elem& e : m.elems)
    for (int a = 0; a < e.t->nnodes; ++a) e.n[a] = inv[e.n[a]];
  for (auto& bm : m.bound)
    for (Elem& e : bm)
      for (int a = 0; a < e.t->nnodes; ++a) e.n[a] = inv[e.n[a]];
  point_connectivity(m);
  check_orientation(m);  // after the connectivity (neighbour lists keep the file's node order), before the dual
  set_edges(m);
  control_volume(m);
  bound_control_volume(m);
  normal_neighbors(m);
  m.nbr_ptr.assign(1, 0);
  m.nbr.clear();
  for (int64_t i = 0; i < m.N; ++i) {
    m.nbr.insert(m.nbr.end(), m.nb[i].begin(), m.nb[i].end());
    m.nbr_ptr.push_back((int64_t)m.nbr.size());
  }
  m.wall.assign(m.N, 0.0);
}

bool read_elem(std::istringstream& is, Elem* e) {
  int vtk = 0;
  if (!(is >> vtk)) return false;
  e->t = elem_type(vtk);
  if (!e->t) return false;
  for (int a = 0; a < e->t->nnodes; ++a)
    if (!(is >> e->n[a])) return false;
  return true;
}

}  // namespace

extern "C" {

int rx_mesh_read_su2(const char* path, rx_mesh** out) {
  if (!path || !out) return RX_ERR_ARG;
  *out = nullptr;
  std::ifstream f(path);
  if (!f) return RX_ERR_STATE;
  rx_mesh* m = new rx_mesh();
  std::string line, v;
  int64_t nelem = -1, npoin = -1;
  int nmark = -1;
  auto fail = [&](int rc) {
    delete m;
    return rc;
  };
  while (std::getline(f, line)) {
    line = trim(line);
    if (line.empty() || line[0] == '%') continue;
    if (keyword(line, "NDIME=", &v)) {
      m->nDim = std::atoi(v.c_str());
      if (m->nDim != 2 && m->nDim != 3) return fail(RX_ERR_ARG);
    } else if (keyword(line, "NELEM=", &v)) {
      nelem = std::atoll(v.c_str());
      m->elems.resize(nelem);
      for (int64_t e = 0; e < nelem; ++e) {
        if (!std::getline(f, line)) return fail(RX_ERR_STATE);
        std::istringstream is(line);
        if (!read_elem(is, &m->elems[e])) return fail(RX_ERR_ARG);
        const int vtk = m->elems[e].t->vtk;
        if ((m->nDim == 2) != (vtk == 5 || vtk == 9) || vtk == 3) return fail(RX_ERR_ARG);
      }
    } else if (keyword(line, "NPOIN=", &v)) {
      npoin = std::atoll(v.c_str());  // "NPOIN= n [n_domain]": a serial mesh has every point in its domain
      m->N = npoin;
      m->coord.resize(npoin * m->nDim);
      for (int64_t p = 0; p < npoin; ++p) {
        if (!std::getline(f, line)) return fail(RX_ERR_STATE);
        std::istringstream is(line);
        for (int d = 0; d < m->nDim; ++d)
          if (!(is >> m->coord[p * m->nDim + d])) return fail(RX_ERR_STATE);
      }
    } else if (keyword(line, "NMARK=", &v)) {
      nmark = std::atoi(v.c_str());
      for (int k = 0; k < nmark; ++k) {
        std::string tag, cnt;
        while (std::getline(f, line) && !keyword(trim(line), "MARKER_TAG=", &tag)) {
        }
        if (!f) return fail(RX_ERR_STATE);
        while (std::getline(f, line) && !keyword(trim(line), "MARKER_ELEMS=", &cnt)) {
        }
        if (!f) return fail(RX_ERR_STATE);
        const int64_t ne = std::atoll(cnt.c_str());
        m->tags.push_back(tag);
        m->bound.emplace_back(ne);
        for (int64_t e = 0; e < ne; ++e) {
          if (!std::getline(f, line)) return fail(RX_ERR_STATE);
          std::istringstream is(line);
          if (!read_elem(is, &m->bound.back()[e])) return fail(RX_ERR_ARG);
          const int vtk = m->bound.back()[e].t->vtk;
          if (m->nDim == 2 ? vtk != 3 : (vtk != 5 && vtk != 9)) return fail(RX_ERR_ARG);
        }
      }
    }
  }
  if (nelem <= 0 || npoin <= 0 || nmark < 0) return fail(RX_ERR_STATE);
  for (const Elem& e : m->elems)
    for (int a = 0; a < e.t->nnodes; ++a)
      if (e.n[a] < 0 || e.n[a] >= m->N) return fail(RX_ERR_STATE);
  for (const auto& bm : m->bound)
    for (const Elem& e : bm)
      for (int a = 0; a < e.t->nnodes; ++a)
        if (e.n[a] < 0 || e.n[a] >= m->N) return fail(RX_ERR_STATE);
  // CPhysicalGeometry(geometry, config), the partitioned copy the driver solves on (geometry_structure.cpp:2960-3080,
  // 4128-4150), stores the elements grouped by kind — triangles, quadrilaterals, tetrahedra, hexahedra, prisms,
  // pyramids — and each marker's boundary elements as lines, triangles, quadrilaterals, file order within a kind;
  // the point connectivity (and so the RCM order and the edge numbering) follows that order
  auto rank = [](int vtk) {
    const int order[] = {3, 5, 9, 10, 12, 13, 14};
    return (int)(std::find(order, order + 7, vtk) - order);
  };
  auto by_kind = [&](const Elem& a, const Elem& b) { return rank(a.t->vtk) < rank(b.t->vtk); };
  std::stable_sort(m->elems.begin(), m->elems.end(), by_kind);
  for (auto& bm : m->bound) std::stable_sort(bm.begin(), bm.end(), by_kind);
  preprocess(*m);
  *out = m;
  return RX_OK;
}

void rx_mesh_destroy(rx_mesh* mesh) { delete mesh; }

int rx_mesh_info(const rx_mesh* m, int32_t* n_dim, int64_t* n_point, int64_t* n_edge, int64_t* n_bvert,
                 int32_t* n_marker) {
  if (!m) return RX_ERR_ARG;
  if (n_dim) *n_dim = m->nDim;
  if (n_point) *n_point = m->N;
  if (n_edge) *n_edge = (int64_t)m->edges.size() / 2;
  if (n_bvert) *n_bvert = (int64_t)m->bvert.size() / 2;
  if (n_marker) *n_marker = (int32_t)m->tags.size();
  return RX_OK;
}

const char* rx_mesh_marker_tag(const rx_mesh* m, int32_t k) {
  return (m && k >= 0 && k < (int32_t)m->tags.size()) ? m->tags[k].c_str() : nullptr;
}

int rx_mesh_describe(const rx_mesh* m, rx_mesh_desc* d) {
  if (!m || !d) return RX_ERR_ARG;
  std::memset(d, 0, sizeof(*d));
  d->n_dim = m->nDim;
  d->n_point = m->N;
  d->n_edge = (int64_t)m->edges.size() / 2;
  d->n_bvert = (int64_t)m->bvert.size() / 2;
  d->edges = m->edges.data();
  d->edge_normal = m->normal.data();
  d->coord = m->coord.data();
  d->volume = m->vol.data();
  d->nbr_ptr = m->nbr_ptr.data();
  d->nbr = m->nbr.data();
  d->bvert = m->bvert.data();
  d->bvert_normal = m->bnormal.data();
  return RX_OK;
}

const int64_t* rx_mesh_global_index(const rx_mesh* m) { return m ? m->gidx.data() : nullptr; }
const int64_t* rx_mesh_normal_neighbor(const rx_mesh* m) { return m ? m->pn.data() : nullptr; }

const double* rx_mesh_wall_distance(rx_mesh* m, const int32_t* is_wall) {
  if (!m) return nullptr;
  if (!is_wall) return m->wall.empty() ? nullptr : m->wall.data();  // the last computed distances
  const int nd = m->nDim;
  std::vector<int64_t> wp;  // wall vertices in marker / vertex order
  for (size_t b = 0; b < m->bvert.size() / 2; ++b)
    if (is_wall[m->bvert[2 * b]]) wp.push_back(m->bvert[2 * b + 1]);
  m->wall.assign(m->N, 0.0);
  if (wp.empty()) return m->wall.data();
  // exact nearest wall vertex through a uniform bucket grid (the reference's ADT returns the same minimum)
  double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
  for (int d = 0; d < nd; ++d) {
    lo[d] = hi[d] = m->coord[wp[0] * nd + d];
    for (int64_t p : wp) {
      lo[d] = std::min(lo[d], m->coord[p * nd + d]);
      hi[d] = std::max(hi[d], m->coord[p * nd + d]);
    }
  }
  const int64_t nw = (int64_t)wp.size();
  int nc[3] = {1, 1, 1};
  const double per = std::max(1.0, std::pow((double)nw / 4.0, 1.0 / nd));
  double h[3] = {1, 1, 1};
  for (int d = 0; d < nd; ++d) {
    nc[d] = (int)std::max(1.0, std::min(per, 4096.0));
    h[d] = (hi[d] - lo[d]) / nc[d];
    if (!(h[d] > 0.0)) {
      nc[d] = 1;
      h[d] = 1.0;
    }
  }
  auto cell = [&](int d, double x) { return std::min(nc[d] - 1, std::max(0, (int)std::floor((x - lo[d]) / h[d]))); };
  std::vector<std::vector<int64_t>> bucket((size_t)nc[0] * nc[1] * nc[2]);
  for (int64_t p : wp) {
    int c[3] = {0, 0, 0};
    for (int d = 0; d < nd; ++d) c[d] = cell(d, m->coord[p * nd + d]);
    bucket[((size_t)c[2] * nc[1] + c[1]) * nc[0] + c[0]].push_back(p);
  }
  for (int64_t i = 0; i < m->N; ++i) {
    const double* x = &m->coord[i * nd];
    int c[3] = {0, 0, 0};
    for (int d = 0; d < nd; ++d) c[d] = cell(d, x[d]);
    double best2 = INFINITY;
    for (int r = 0;; ++r) {
      // cells at Chebyshev ring r around c; stop once the ring is farther than the best distance
      double ring = INFINITY;
      for (int d = 0; d < nd; ++d) {
        const double lo_d = lo[d] + (c[d] - r) * h[d], hi_d = lo[d] + (c[d] + r + 1) * h[d];
        ring = std::min(ring, std::min(x[d] - lo_d, hi_d - x[d]));
      }
      for (int dz = (nd == 3 ? -r : 0); dz <= (nd == 3 ? r : 0); ++dz)
        for (int dy = -r; dy <= r; ++dy)
          for (int dx = -r; dx <= r; ++dx) {
            if (std::max(std::abs(dx), std::max(std::abs(dy), std::abs(dz))) != r) continue;
            const int cx = c[0] + dx, cy = c[1] + dy, cz = c[2] + dz;
            if (cx < 0 || cy < 0 || cz < 0 || cx >= nc[0] || cy >= nc[1] || cz >= nc[2]) continue;
            for (int64_t p : bucket[((size_t)cz * nc[1] + cy) * nc[0] + cx]) {
              double s = 0.0;
              for (int d = 0; d < nd; ++d) {
                const double t = x[d] - m->coord[p * nd + d];
                s += t * t;
              }
              best2 = std::min(best2, s);
            }
          }
      const bool covered = r >= std::max(nc[0], std::max(nc[1], nc[2]));
      if (covered || (std::isfinite(best2) && ring > 0.0 && ring * ring >= best2)) break;
    }
    m->wall[i] = std::sqrt(best2);
  }
  return m->wall.data();
}

}  // extern "C"

// ================================================================================================
// Reacting-library files (ReactingModelLibrary::Setup, reacting_model_library.cpp:925-1506)
// ================================================================================================
struct rx_mech {
  int ns = 0, nr = 0, ntab = 0;
  std::vector<std::string> names;
  std::vector<double> mm, hf, dv;
  std::vector<double> sr, sp, er, ep;  // [ns][nr], [nr][ns]
  std::vector<double> A, beta, Ta, Ab, betab, Tab;
  std::vector<int32_t> rev, hasb;
  std::vector<double> tx, ty, ty2;  // [5][ns][ntab]: cp, h, s, mu, kappa
};

namespace {

constexpr double kRcal = 1.9858775;  // R_UNGAS_SCAL, cal/(mol K) (physical_chemical_library.hpp:571-579)

// the library's line filter: empty lines and lines starting with a punctuation character are skipped; "STOP" ends
std::vector<std::string> lib_lines(const std::string& path, bool* ok) {
  std::vector<std::string> out;
  std::ifstream f(path);
  *ok = (bool)f;
  std::string line;
  while (std::getline(f, line)) {
    while (!line.empty() && (line.back() == '\r' || line.back() == '\n')) line.pop_back();
    if (line == "STOP") break;
    if (!line.empty() && !std::ispunct((unsigned char)line[0])) out.push_back(line);
  }
  return out;
}

// MathTools::SetSpline's table checks (Common/src/Tools/spline.cpp:12-25): at least 2 points, x sorted and unique,
// and equispaced (GetSpline finds the interval by integer division) — the reference's loop compares the steps
// x[i] - x[i-1] for 2 <= i < n - 1 with the first one exactly (the last step is not compared).
bool spline_table_ok(const double* x, int n) {
  if (n < 2) return false;
  for (int i = 1; i < n; ++i)
    if (!(x[i - 1] < x[i])) return false;  // sorted and unique
  const double step = x[1] - x[0];
  for (int i = 2; i < n - 1; ++i)
    if (x[i] - x[i - 1] != step) return false;
  return true;
}

// MathTools::SetSpline (spline.cpp:10-58), called with zero end slopes
void set_spline(const double* x, const double* y, int n, double* y2, double yp1 = 0.0, double ypn = 0.0) {
  std::vector<double> u(n, 0.0);
  if (yp1 > 0.99e30) {
    y2[0] = 0.0;
  } else {
    y2[0] = -0.5;
    u[0] = (3.0 / (x[1] - x[0])) * ((y[1] - y[0]) / (x[1] - x[0]) - yp1);
  }
  for (int i = 2; i < n; ++i) {
    const double sig = (x[i - 1] - x[i - 2]) / (x[i] - x[i - 2]);
    const double p = sig * y2[i - 2] + 2.0;
    y2[i - 1] = (sig - 1.0) / p;
    u[i - 1] = (y[i] - y[i - 1]) / (x[i] - x[i - 1]) - (y[i - 1] - y[i - 2]) / (x[i - 1] - x[i - 2]);
    u[i - 1] = (6.0 * u[i - 1] / (x[i] - x[i - 2]) - sig * u[i - 2]) / p;
  }
  double qn, un;
  if (ypn > 0.99e30) {
    qn = un = 0.0;
  } else {
    qn = 0.5;
    un = (3.0 / (x[n - 1] - x[n - 2])) * (ypn - (y[n - 1] - y[n - 2]) / (x[n - 1] - x[n - 2]));
  }
  y2[n - 1] = (un - qn * u[n - 2]) / (qn * y2[n - 2] + 1.0);
  for (int k = n - 1; k > 0; --k) y2[k - 1] = y2[k - 1] * y2[k] + u[k - 1];
}

// MathTools::Parse_Terms (utility.cpp:12-86), iterative form of the recursive parser
bool parse_terms(std::string line, int r, bool is_rev, bool is_reac, rx_mech& m, std::vector<double>& stoich) {
  auto punct = [](char c) { return std::ispunct((unsigned char)c) != 0; };
  while (true) {
    const size_t size = line.size();
    size_t idx = 0;
    while (idx < size && !(std::isdigit((unsigned char)line[idx]) || std::isalpha((unsigned char)line[idx]))) ++idx;
    if (idx >= size) return false;
    std::string coeff;
    while (idx < size && (std::isdigit((unsigned char)line[idx]) || punct(line[idx]))) coeff += line[idx++];
    std::string symbol;
    while (true) {
      while (idx < size && (std::isalpha((unsigned char)line[idx]) || std::isdigit((unsigned char)line[idx])))
        symbol += line[idx++];
      if (!(idx < size && !punct(line[idx]) && !std::isspace((unsigned char)line[idx]) && line[idx] != '+')) break;
    }
    const auto it = std::find(m.names.begin(), m.names.end(), symbol);
    if (it == m.names.end()) return false;
    const int s = (int)(it - m.names.begin());
    const double coefficient = coeff.empty() ? 1.0 : std::stod(coeff);
    stoich[(size_t)s * m.nr + r] += coefficient;
    std::string exp_coeff;
    if (idx < size && punct(line[idx])) {
      ++idx;
      while (idx < size && (std::isdigit((unsigned char)line[idx]) || punct(line[idx]))) exp_coeff += line[idx++];
    }
    if (!exp_coeff.empty()) {
      const double e = std::stod(exp_coeff);
      if (is_reac) m.er[(size_t)r * m.ns + s] += e;
      else if (is_rev) m.ep[(size_t)r * m.ns + s] += e;
    } else if (is_reac) {
      m.er[(size_t)r * m.ns + s] += stoich[(size_t)s * m.nr + r];
    }
    if (idx == size) return true;
    line = line.substr(idx + 1);
    if (line.empty()) return true;
  }
}

std::string join(const std::string& dir, const std::string& f) { return dir.empty() ? f : dir + "/" + f; }

}  // namespace

extern "C" {

int rx_mech_read(const char* base_dir, const char* list_file, rx_mech** out) {
  if (!base_dir || !list_file || !out) return RX_ERR_ARG;
  *out = nullptr;
  const std::string dir(base_dir);
  bool ok = false;
  const std::vector<std::string> files = lib_lines(join(dir, list_file), &ok);
  if (!ok || files.empty()) return RX_ERR_STATE;
  rx_mech* m = new rx_mech();
  auto fail = [&](int rc) {
    delete m;
    return rc;
  };
  // mixture: number of species, then name, molar mass, formation enthalpy, diffusion volume
  const std::vector<std::string> mix = lib_lines(join(dir, trim(files[0])), &ok);
  if (!ok || mix.empty()) return fail(RX_ERR_STATE);
  m->ns = std::atoi(mix[0].c_str());
  if (m->ns < 1 || (int)mix.size() < 1 + m->ns) return fail(RX_ERR_STATE);
  for (int s = 0; s < m->ns; ++s) {
    std::istringstream is(mix[1 + s]);
    std::string name;
    double a, b, c;
    if (!(is >> name >> a >> b >> c)) return fail(RX_ERR_STATE);
    m->names.push_back(name);
    m->mm.push_back(a);
    m->hf.push_back(b);
    m->dv.push_back(c);
  }
  const int ns = m->ns;
  const bool has_chem = (int)files.size() == 2 * ns + 2;
  if (has_chem) {
    const std::vector<std::string> chem = lib_lines(join(dir, trim(files[1])), &ok);
    if (!ok || chem.size() < 2) return fail(RX_ERR_STATE);
    const int nr = m->nr = std::atoi(chem[0].c_str());
    std::istringstream us(chem[1]);
    std::string units;
    us >> units;
    const bool cgs = units == "CGS";
    m->sr.assign((size_t)ns * nr, 0.0);
    m->sp.assign((size_t)ns * nr, 0.0);
    m->er.assign((size_t)nr * ns, 0.0);
    m->ep.assign((size_t)nr * ns, 0.0);
    for (auto* v : {&m->A, &m->beta, &m->Ta, &m->Ab, &m->betab, &m->Tab}) v->assign(nr, 0.0);
    m->rev.assign(nr, 0);
    m->hasb.assign(nr, 0);
    int n_line = 2, r = -1;
    for (size_t q = 2; q < chem.size(); ++q, ++n_line) {
      const std::string& line = chem[q];
      if (n_line % 2 == 0 && n_line < 2 * nr + 1) {
        ++r;
        const bool is_rev = line.find('<') != std::string::npos;
        m->rev[r] = is_rev;
        const size_t major = line.find('>');
        if (major == std::string::npos) return fail(RX_ERR_STATE);
        const std::string reac = line.substr(0, line.find(is_rev ? '<' : '='));
        const std::string prod = line.substr(major + 1);
        if (!parse_terms(reac, r, is_rev, true, *m, m->sr) || !parse_terms(prod, r, is_rev, false, *m, m->sp))
          return fail(RX_ERR_STATE);
      } else if (n_line % 2 == 1 && n_line < 2 * nr + 2) {
        std::istringstream is(line);
        double a, b, c;
        if (!(is >> a >> b >> c)) return fail(RX_ERR_STATE);
        m->A[r] = a;
        m->beta[r] = b;
        m->Ta[r] = cgs ? c / kRcal : c;
      } else {
        const std::string key = "Available Backward Rate reaction";
        if (line.find(key) != std::string::npos && line.size() > 32) {
          const std::string rest = line.substr(32);
          const int rr = std::atoi(rest.substr(0, rest.find(':')).c_str()) - 1;
          if (rr < 0 || rr >= nr || rest.size() < 3) return fail(RX_ERR_STATE);
          std::istringstream is(rest.substr(3));
          double a, b, c;
          if (!(is >> a >> b >> c)) return fail(RX_ERR_STATE);
          m->hasb[rr] = 1;
          m->Ab[rr] = a;
          m->betab[rr] = b;
          m->Tab[rr] = cgs ? c / kRcal : c;
        }
        if (line.find("Extra Forward terms reaction") != std::string::npos ||
            line.find("Extra Backward terms reaction") != std::string::npos)
          return fail(RX_ERR_ARG);  // not used by the shipped mechanisms
      }
    }
    for (int rr = 0; rr < nr; ++rr)
      if (m->rev[rr] && !m->hasb[rr])
        for (int s = 0; s < ns; ++s)
          m->ep[(size_t)rr * ns + s] = m->er[(size_t)rr * ns + s] + m->sp[(size_t)s * nr + rr] - m->sr[(size_t)s * nr + rr];
    if (cgs)
      for (int rr = 0; rr < nr; ++rr) {
        double se = 0.0, sb = 0.0;
        for (int s = 0; s < ns; ++s) {
          se += m->er[(size_t)rr * ns + s];
          sb += m->ep[(size_t)rr * ns + s];
        }
        m->A[rr] *= std::pow(10.0, 6.0 * (1.0 - se));
        if (m->hasb[rr]) m->Ab[rr] *= std::pow(10.0, 6.0 * (1.0 - sb));
      }
  }
  // per-species tables: transport (T, mu, kappa) then thermo (T, cp, h, s) file of each species
  const int off = has_chem ? 0 : 1;
  if ((int)files.size() < 2 * ns + 2 - off) return fail(RX_ERR_STATE);
  std::vector<std::vector<double>> tabs((size_t)5 * ns * 2);  // [prop][s] -> (x, y) interleaved
  for (int q = 0; q < ns; ++q)
    for (int kind = 0; kind < 2; ++kind) {
      const std::vector<std::string> ls = lib_lines(join(dir, trim(files[2 * q + 2 + kind - off])), &ok);
      if (!ok || ls.size() < 3) return fail(RX_ERR_STATE);
      const auto it = std::find(m->names.begin(), m->names.end(), trim(ls[0]));
      if (it == m->names.end()) return fail(RX_ERR_STATE);
      const int s = (int)(it - m->names.begin());
      for (size_t l = 1; l < ls.size(); ++l) {
        std::istringstream is(ls[l]);
        double T, a, b, c = 0.0;
        if (!(is >> T >> a >> b)) return fail(RX_ERR_STATE);
        if (kind == 1 && !(is >> c)) return fail(RX_ERR_STATE);
        // props: 0 cp, 1 h, 2 s (thermo); 3 mu, 4 kappa (transport)
        const int p0 = kind == 0 ? 3 : 0;
        const double vals[3] = {a, b, c};
        for (int k = 0; k < (kind == 0 ? 2 : 3); ++k) {
          auto& t = tabs[((size_t)(p0 + k) * ns + s)];
          t.push_back(T);
          t.push_back(vals[k]);
        }
      }
    }
  m->ntab = (int)tabs[0].size() / 2;
  const int nt = m->ntab;
  if (nt < 3) return fail(RX_ERR_STATE);
  m->tx.assign((size_t)5 * ns * nt, 0.0);
  m->ty.assign(m->tx.size(), 0.0);
  m->ty2.assign(m->tx.size(), 0.0);
  for (int p = 0; p < 5; ++p)
    for (int s = 0; s < ns; ++s) {
      const auto& t = tabs[(size_t)p * ns + s];
      if ((int)t.size() != 2 * nt) return fail(RX_ERR_STATE);
      double* x = &m->tx[((size_t)p * ns + s) * nt];
      double* y = &m->ty[((size_t)p * ns + s) * nt];
      for (int k = 0; k < nt; ++k) {
        x[k] = t[2 * k];
        y[k] = t[2 * k + 1];
      }
      if (!spline_table_ok(x, nt)) return fail(RX_ERR_STATE);
      set_spline(x, y, nt, &m->ty2[((size_t)p * ns + s) * nt]);
    }
  *out = m;
  return RX_OK;
}

void rx_mech_destroy(rx_mech* mech) { delete mech; }

int rx_mech_describe(const rx_mech* m, rx_mech_desc* d) {
  if (!m || !d) return RX_ERR_ARG;
  d->n_species = m->ns;
  d->n_reactions = m->nr;
  d->n_tab = m->ntab;
  d->mmass = m->mm.data();
  d->diff_vol = m->dv.data();
  d->stoich_reac = m->sr.data();
  d->stoich_prod = m->sp.data();
  d->exp_reac = m->er.data();
  d->exp_prod = m->ep.data();
  d->A = m->A.data();
  d->beta = m->beta.data();
  d->Ta = m->Ta.data();
  d->A_back = m->Ab.data();
  d->beta_back = m->betab.data();
  d->Ta_back = m->Tab.data();
  d->reversible = m->rev.data();
  d->has_backward = m->hasb.data();
  d->tab_x = m->tx.data();
  d->tab_y = m->ty.data();
  d->tab_y2 = m->ty2.data();
  return RX_OK;
}

const char* rx_mech_species(const rx_mech* m, int32_t s) {
  return (m && s >= 0 && s < m->ns) ? m->names[s].c_str() : nullptr;
}

double rx_mech_formation_enthalpy(const rx_mech* m, int32_t s) {
  return (m && s >= 0 && s < m->ns) ? m->hf[s] : 0.0;
}

// ================================================================================================
// Restart files (COutput::SetRestart output_structure.cpp:3858-4060; Load_Restart solver_direct_reactive.cpp:566-686)
// ================================================================================================
int rx_restart_write(const char* path, const rx_mesh* m, int32_t n_var, const double* U, const double* T,
                     const double* extra, int64_t ext_iter) {
  if (!path || !m || n_var < 1 || !U || !T) return RX_ERR_ARG;
  std::ofstream f(path);
  if (!f) return RX_ERR_STATE;
  f.precision(15);
  const int nd = m->nDim;
  f << "\"PointID\"";
  f << (nd == 2 ? "\t\"x\"\t\"y\"" : "\t\"x\"\t\"y\"\t\"z\"");
  for (int v = 0; v < n_var + 2; ++v) f << "\t\"Conservative_" << v + 1 << "\"";
  if (extra) f << "\t\"Pressure\"\t\"Temperature\"\t\"Mach\"\t\"Laminar_Viscosity\"\t\"<greek>m</greek><sub>t</sub>\"";
  f << "\n";
  std::vector<int64_t> local(m->N);  // global (file) index -> mesh point
  for (int64_t i = 0; i < m->N; ++i) local[m->gidx[i]] = i;
  for (int64_t g = 0; g < m->N; ++g) {
    const int64_t i = local[g];
    f << g << "\t";
    for (int d = 0; d < nd; ++d) f << std::scientific << m->coord[i * nd + d] << "\t";
    for (int v = 0; v < n_var; ++v) f << std::scientific << U[i * n_var + v] << "\t";
    for (int v = 0; v < 2; ++v) f << std::scientific << T[i * 2 + v] << "\t";
    if (extra)
      for (int v = 0; v < 5; ++v) f << std::scientific << extra[i * 5 + v] << "\t";
    f << "\n";
  }
  // trailer (output_structure.cpp:4056-4065): the doubles AoA - offset, AoS - offset, INITIAL_BCTHRUST (CConfig
  // default 4000) and dCD/dCL, still in scientific at precision 15; then the integer EXT_ITER (+ 1)
  f << "AOA= " << 0.0 << "\n";
  f << "SIDESLIP_ANGLE= " << 0.0 << "\n";
  f << "INITIAL_BCTHRUST= " << 4000.0 << "\n";
  f << "DCD_DCL_VALUE= " << 0.0 << "\n";
  f << "EXT_ITER= " << ext_iter + 1 << "\n";
  return f ? RX_OK : RX_ERR_STATE;
}

int rx_restart_read(const char* path, const rx_mesh* m, int32_t n_var, double* U, double* T) {
  if (!path || !m || n_var < 1 || !U) return RX_ERR_ARG;
  std::ifstream f(path);
  if (!f) return RX_ERR_STATE;
  std::string line;
  std::getline(f, line);  // header
  std::vector<int64_t> local(m->N);
  for (int64_t i = 0; i < m->N; ++i) local[m->gidx[i]] = i;
  const int nd = m->nDim;
  for (int64_t g = 0; g < m->N; ++g) {
    if (!std::getline(f, line)) return RX_ERR_STATE;  // "doesn't match with the mesh file"
    std::istringstream is(line);
    int64_t index;
    double dull;
    if (!(is >> index)) return RX_ERR_STATE;
    for (int d = 0; d < nd; ++d) is >> dull;
    const int64_t i = local[g];
    for (int v = 0; v < n_var; ++v)
      if (!(is >> U[i * n_var + v])) return RX_ERR_STATE;
    if (T)
      for (int v = 0; v < 2; ++v)
        if (!(is >> T[i * 2 + v])) return RX_ERR_STATE;
  }
  return RX_OK;
}

}  // extern "C"
