// rx_part.cpp — multilevel graph partitioning (host): splits a mesh's point graph into the partitions that stand for
// the reference's MPI ranks (include/rx.h, rx_mesh_desc.part_ptr) and into the ranks of a distributed run.
//
// The reference partitions with METIS 5 (CPhysicalGeometry::SetColorGrid, Common/src/geometry_structure.cpp:11360-
// 11450: METIS_PartMeshNodal on its triangulated elements). This is an independent multilevel recursive bisection of
// the same family: heavy-edge-matching coarsening, a greedy graph-growing bisection of the coarsest graph (the best of
// several seeds), then Fiduccia-Mattheyses boundary refinement at every level while projecting back, with a balance
// constraint per bisection. Deterministic: a fixed-seed generator, so a graph always gets the same partition.
// tools/edge_cut.py and tests/test_partition.py compare its edge cut with METIS compiled from the reference's own
// sources (oracle/ref_build.mk `metis`).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <queue>
#include <random>
#include <vector>

#include "../../include/rx_io.h"

namespace {

struct Graph {
  int n = 0;
  std::vector<int> xadj, adj, ew, vw;  // CSR adjacency with edge weights, vertex weights
  int64_t total_vw() const {
    int64_t s = 0;
    for (int w : vw) s += w;
    return s;
  }
};

// Heavy-edge matching: vertices in a random order match their unmatched neighbour of largest edge weight (lightest
// vertex on ties); cmap[v] = coarse vertex. Returns the coarse graph.
Graph coarsen(const Graph& g, std::vector<int>& cmap, std::mt19937& rng, const int32_t* label = nullptr) {
  std::vector<int> perm(g.n), match(g.n, -1);
  for (int v = 0; v < g.n; ++v) perm[v] = v;
  std::shuffle(perm.begin(), perm.end(), rng);
  for (int v : perm) {
    if (match[v] >= 0) continue;
    int best = -1, bw = -1;
    for (int k = g.xadj[v]; k < g.xadj[v + 1]; ++k) {
      const int u = g.adj[k];
      if (match[u] >= 0 || u == v || (label && label[u] != label[v])) continue;
      if (g.ew[k] > bw || (g.ew[k] == bw && g.vw[u] < g.vw[best])) {
        best = u;
        bw = g.ew[k];
      }
    }
    if (best < 0) {
      match[v] = v;
    } else {
      match[v] = best;
      match[best] = v;
    }
  }
  cmap.assign(g.n, -1);
  int nc = 0;
  for (int v : perm)
    if (cmap[v] < 0) {
      cmap[v] = nc;
      cmap[match[v]] = nc;
      ++nc;
    }
  Graph c;
  c.n = nc;
  c.vw.assign(nc, 0);
  std::vector<int> first(nc, -1), second(nc, -1);
  for (int v = 0; v < g.n; ++v) {
    const int cv = cmap[v];
    c.vw[cv] += g.vw[v];
    if (first[cv] < 0) first[cv] = v;
    else second[cv] = v;
  }
  c.xadj.assign(nc + 1, 0);
  std::vector<int> slot(nc, -1);  // position of coarse neighbour u in the current row
  for (int cv = 0; cv < nc; ++cv) {
    const int row0 = (int)c.adj.size();
    for (int v : {first[cv], second[cv]}) {
      if (v < 0) continue;
      for (int k = g.xadj[v]; k < g.xadj[v + 1]; ++k) {
        const int cu = cmap[g.adj[k]];
        if (cu == cv) continue;
        if (slot[cu] >= row0) {
          c.ew[slot[cu]] += g.ew[k];
        } else {
          slot[cu] = (int)c.adj.size();
          c.adj.push_back(cu);
          c.ew.push_back(g.ew[k]);
        }
      }
    }
    c.xadj[cv + 1] = (int)c.adj.size();
  }
  return c;
}

int64_t cut_of(const Graph& g, const std::vector<int>& where) {
  int64_t cut = 0;
  for (int v = 0; v < g.n; ++v)
    for (int k = g.xadj[v]; k < g.xadj[v + 1]; ++k)
      if (where[g.adj[k]] != where[v]) cut += g.ew[k];
  return cut / 2;
}

// Fiduccia-Mattheyses passes on a bisection: moves of the best gain (external - internal degree) from a side whose
// move keeps the other side within its bound, vertices locked once moved, each pass rolled back to its best prefix
// (lowest cut among balanced states; an unbalanced start is first driven into balance). maxw: the side bounds.
void fm_refine(const Graph& g, std::vector<int>& where, const int64_t (&maxw)[2], int passes) {
  std::vector<int> gain(g.n);
  std::vector<char> locked(g.n);
  int64_t pw[2] = {0, 0};
  for (int v = 0; v < g.n; ++v) pw[where[v]] += g.vw[v];
  auto compute_gain = [&](int v) {
    int ext = 0, in = 0;
    for (int k = g.xadj[v]; k < g.xadj[v + 1]; ++k) (where[g.adj[k]] == where[v] ? in : ext) += g.ew[k];
    return ext - in;
  };
  auto over = [&](const int64_t (&w)[2]) { return std::max<int64_t>(0, w[0] - maxw[0]) + std::max<int64_t>(0, w[1] - maxw[1]); };
  for (int pass = 0; pass < passes; ++pass) {
    int64_t cut = cut_of(g, where);
    std::priority_queue<std::pair<int, int>> q[2];  // (gain, vertex), lazily updated
    for (int v = 0; v < g.n; ++v) {
      gain[v] = compute_gain(v);
      locked[v] = 0;
      bool boundary = false;
      for (int k = g.xadj[v]; k < g.xadj[v + 1] && !boundary; ++k) boundary = where[g.adj[k]] != where[v];
      if (boundary || over(pw) > 0) q[where[v]].push({gain[v], v});
    }
    std::vector<int> moves;
    int64_t best_cut = cut, best_over = over(pw);
    size_t best_len = 0;
    // moves without improvement before the pass ends
    const size_t limit = std::min<size_t>(5000, std::max<size_t>(200, (size_t)g.n / 20));
    while (moves.size() < (size_t)g.n) {
      // the side to move from: the overweight one, else the one whose best move is better (and allowed)
      int from = -1;
      for (int s = 0; s < 2; ++s)
        while (!q[s].empty() && (locked[q[s].top().second] || where[q[s].top().second] != s ||
                                 q[s].top().first != gain[q[s].top().second]))
          q[s].pop();
      if (pw[0] > maxw[0]) from = 0;
      else if (pw[1] > maxw[1]) from = 1;
      else {
        int bg = INT32_MIN;
        for (int s = 0; s < 2; ++s)
          if (!q[s].empty() && pw[1 - s] + g.vw[q[s].top().second] <= maxw[1 - s] && q[s].top().first > bg) {
            bg = q[s].top().first;
            from = s;
          }
      }
      if (from < 0 || q[from].empty()) break;
      const int v = q[from].top().second;
      q[from].pop();
      locked[v] = 1;
      where[v] = 1 - from;
      pw[from] -= g.vw[v];
      pw[1 - from] += g.vw[v];
      cut -= gain[v];
      moves.push_back(v);
      for (int k = g.xadj[v]; k < g.xadj[v + 1]; ++k) {
        const int u = g.adj[k];
        if (locked[u]) continue;
        gain[u] += (where[u] == where[v]) ? -2 * g.ew[k] : 2 * g.ew[k];
        q[where[u]].push({gain[u], u});
      }
      const int64_t ov = over(pw);
      if (ov < best_over || (ov == best_over && cut < best_cut)) {
        best_over = ov;
        best_cut = cut;
        best_len = moves.size();
      } else if (moves.size() - best_len > limit) {
        break;
      }
    }
    for (size_t m = moves.size(); m > best_len; --m) {  // roll back to the best prefix
      const int v = moves[m - 1];
      pw[where[v]] -= g.vw[v];
      where[v] = 1 - where[v];
      pw[where[v]] += g.vw[v];
    }
    if (best_len == 0) break;  // no improving prefix: converged
  }
}

// Greedy graph growing: a region grown breadth-first from a seed until it holds the target weight; the best cut of
// `trials` seeds after refinement.
std::vector<int> initial_bisection(const Graph& g, int64_t target0, const int64_t (&maxw)[2], std::mt19937& rng) {
  std::vector<int> best;
  int64_t best_cut = -1, best_ov = -1;
  const int trials = g.n < 8 ? 1 : 8;
  std::uniform_int_distribution<int> pick(0, std::max(0, g.n - 1));
  for (int t = 0; t < trials; ++t) {
    std::vector<int> where(g.n, 1);
    std::vector<char> seen(g.n, 0);
    std::vector<int> fifo;
    int64_t w0 = 0;
    int head = 0;
    int seed = pick(rng);
    while (w0 < target0) {
      if (head == (int)fifo.size()) {  // the region's component is exhausted: restart from an unseen vertex
        int s = -1;
        for (int k = 0; k < g.n && s < 0; ++k)
          if (!seen[(seed + k) % g.n]) s = (seed + k) % g.n;
        if (s < 0) break;
        seen[s] = 1;
        fifo.push_back(s);
      }
      const int v = fifo[head++];
      if (w0 + g.vw[v] > maxw[0] && w0 > 0) continue;
      where[v] = 0;
      w0 += g.vw[v];
      for (int k = g.xadj[v]; k < g.xadj[v + 1]; ++k)
        if (!seen[g.adj[k]]) {
          seen[g.adj[k]] = 1;
          fifo.push_back(g.adj[k]);
        }
    }
    fm_refine(g, where, maxw, 4);
    int64_t pw0 = 0;
    for (int v = 0; v < g.n; ++v)
      if (where[v] == 0) pw0 += g.vw[v];
    const int64_t tot = g.total_vw();
    const int64_t ov = std::max<int64_t>(0, pw0 - maxw[0]) + std::max<int64_t>(0, tot - pw0 - maxw[1]);
    const int64_t c = cut_of(g, where);
    if (best_cut < 0 || ov < best_ov || (ov == best_ov && c < best_cut)) {
      best = where;
      best_cut = c;
      best_ov = ov;
    }
  }
  return best;
}

// Multilevel bisection of g with side 0 holding `frac` of the weight (balance tolerance eps per side); each side keeps
// at least min0 / min1 of the weight (its part count: no part comes out empty whatever eps).
std::vector<int> bisect(const Graph& g, double frac, double eps, std::mt19937& rng, int64_t min0 = 0,
                        int64_t min1 = 0) {
  const int64_t tot = g.total_vw();
  const int64_t t0 = (int64_t)(frac * (double)tot + 0.5);
  std::vector<Graph> levels{g};
  std::vector<std::vector<int>> maps;
  while (levels.back().n > 120) {
    std::vector<int> cmap;
    Graph c = coarsen(levels.back(), cmap, rng);
    if (c.n > 0.95 * levels.back().n) break;  // matching stalled (stars, isolated vertices)
    maps.push_back(std::move(cmap));
    levels.push_back(std::move(c));
  }
  auto bounds = [&](const Graph& h, int64_t (&maxw)[2]) {
    int maxv = 0;
    for (int w : h.vw) maxv = std::max(maxv, w);
    // the tolerance, widened on coarse levels by one coarse vertex (so a balanced move exists)
    maxw[0] = (int64_t)((double)t0 * (1.0 + eps)) + (h.n == g.n ? 0 : maxv);
    maxw[1] = (int64_t)((double)(tot - t0) * (1.0 + eps)) + (h.n == g.n ? 0 : maxv);
    maxw[0] = std::min(maxw[0], tot - min1 + (h.n == g.n ? 0 : maxv));
    maxw[1] = std::min(maxw[1], tot - min0 + (h.n == g.n ? 0 : maxv));
  };
  int64_t maxw[2];
  bounds(levels.back(), maxw);
  std::vector<int> where = initial_bisection(levels.back(), t0, maxw, rng);
  for (int l = (int)levels.size() - 2; l >= 0; --l) {
    std::vector<int> fine(levels[l].n);
    for (int v = 0; v < levels[l].n; ++v) fine[v] = where[maps[l][v]];
    where.swap(fine);
    bounds(levels[l], maxw);
    fm_refine(levels[l], where, maxw, l == 0 ? 6 : 3);
  }
  return where;
}

Graph induced(const Graph& g, const std::vector<int>& verts, std::vector<int>& local) {
  Graph s;
  s.n = (int)verts.size();
  for (int i = 0; i < s.n; ++i) local[verts[i]] = i;
  s.xadj.assign(s.n + 1, 0);
  s.vw.resize(s.n);
  for (int i = 0; i < s.n; ++i) {
    const int v = verts[i];
    s.vw[i] = g.vw[v];
    for (int k = g.xadj[v]; k < g.xadj[v + 1]; ++k)
      if (local[g.adj[k]] >= 0) {
        s.adj.push_back(local[g.adj[k]]);
        s.ew.push_back(g.ew[k]);
      }
    s.xadj[i + 1] = (int)s.adj.size();
  }
  for (int v : verts) local[v] = -1;
  return s;
}

// Recursive bisection: nparts parts numbered from p0; the sides get floor(nparts / 2) and the rest.
void recurse(const Graph& g, const std::vector<int>& verts, int nparts, int p0, double eps, std::mt19937& rng,
             std::vector<int>& local, int32_t* part) {
  if (nparts == 1 || verts.empty()) {
    for (int v : verts) part[v] = p0;
    return;
  }
  const int left = nparts / 2;
  const Graph s = induced(g, verts, local);
  const std::vector<int> where = bisect(s, (double)left / nparts, eps, rng, left, nparts - left);
  std::vector<int> a, b;
  for (int i = 0; i < s.n; ++i) (where[i] == 0 ? a : b).push_back(verts[i]);
  recurse(g, a, left, p0, eps, rng, local, part);
  recurse(g, b, nparts - left, p0 + left, eps, rng, local, part);
}

// Greedy k-way boundary refinement of one level (vertex weights) in place; returns the number of moves.
int64_t kway_greedy(const Graph& g, int32_t* part, std::vector<int64_t>& pw, int64_t minw, int64_t maxw,
                    std::vector<int>& conn, std::vector<int>& touched) {
  int64_t moved = 0;
  for (int v = 0; v < g.n; ++v) {
    const int p = part[v];
    touched.clear();
    for (int k = g.xadj[v]; k < g.xadj[v + 1]; ++k) {
      const int q = part[g.adj[k]];
      if (conn[q] == 0) touched.push_back(q);
      conn[q] += g.ew[k];
    }
    int best = p, bg = 0;
    for (int q : touched)
      if (q != p && pw[q] + g.vw[v] <= maxw && pw[p] - g.vw[v] >= minw) {
        const int gq = conn[q] - conn[p];
        // a strictly better cut, or an equal one that moves weight to a lighter part
        if (gq > bg || (gq == bg && gq == 0 && best == p && pw[q] + g.vw[v] < pw[p])) {
          bg = gq;
          best = q;
        }
      }
    for (int q : touched) conn[q] = 0;
    conn[p] = 0;
    if (best != p) {
      pw[p] -= g.vw[v];
      pw[best] += g.vw[v];
      part[v] = best;
      ++moved;
    }
  }
  return moved;
}

// k-way refinement over a hierarchy: the graph coarsened with matches inside a part only (so the partition carries
// to every level), then greedy boundary passes from the coarsest level down — coarse moves shift whole clusters.
void kway_vcycle(const Graph& g, int32_t* part, int nparts, int64_t minw, int64_t maxw, std::mt19937& rng) {
  std::vector<Graph> levels{g};
  std::vector<std::vector<int>> maps;
  std::vector<std::vector<int32_t>> parts{std::vector<int32_t>(part, part + g.n)};
  while (levels.back().n > 40 * nparts) {
    std::vector<int> cmap;
    Graph c = coarsen(levels.back(), cmap, rng, parts.back().data());
    if (c.n > 0.9 * levels.back().n) break;
    std::vector<int32_t> cp(c.n);
    for (int v = 0; v < levels.back().n; ++v) cp[cmap[v]] = parts.back()[v];
    maps.push_back(std::move(cmap));
    levels.push_back(std::move(c));
    parts.push_back(std::move(cp));
  }
  std::vector<int> conn(nparts, 0), touched;
  for (int l = (int)levels.size() - 1; l >= 0; --l) {
    if (l + 1 < (int)levels.size())  // project the coarser level's refined partition
      for (int v = 0; v < levels[l].n; ++v) parts[l][v] = parts[l + 1][maps[l][v]];
    std::vector<int64_t> pw(nparts, 0);
    for (int v = 0; v < levels[l].n; ++v) pw[parts[l][v]] += levels[l].vw[v];
    for (int pass = 0; pass < 6; ++pass)
      if (!kway_greedy(levels[l], parts[l].data(), pw, minw, maxw, conn, touched)) break;
  }
  std::copy(parts[0].begin(), parts[0].end(), part);
}

}  // namespace

extern "C" int rx_partition_graph(int64_t n, const int64_t* xadj, const int64_t* adj, int32_t nparts, double imbalance,
                                  int32_t* part, int64_t* edge_cut) {
  if (n < 0 || n >= (1LL << 31) || nparts < 1 || !part || (n > 0 && (!xadj || !adj)) || imbalance < 0.0)
    return RX_ERR_ARG;
  if (nparts > n && n > 0) return RX_ERR_ARG;
  // a CSR offset array: starts at 0, never decreases, and its total fits the int32 adjacency
  if (n > 0) {
    if (xadj[0] != 0 || xadj[n] >= (1LL << 31)) return RX_ERR_ARG;
    for (int64_t v = 0; v < n; ++v)
      if (xadj[v + 1] < xadj[v]) return RX_ERR_ARG;
  }
  Graph g;
  g.n = (int)n;
  g.xadj.resize(n + 1);
  for (int64_t v = 0; v <= n; ++v) g.xadj[v] = (int)xadj[v];
  g.adj.resize(g.xadj[n]);
  for (int64_t k = 0; k < xadj[n]; ++k) {
    if (adj[k] < 0 || adj[k] >= n) return RX_ERR_ARG;
    g.adj[k] = (int)adj[k];
  }
  g.ew.assign(g.adj.size(), 1);
  g.vw.assign(n, 1);
  std::mt19937 rng(20261018u);
  std::vector<int> verts(n), local(n, -1);
  for (int v = 0; v < (int)n; ++v) verts[v] = v;
  // the per-bisection tolerance compounding to `imbalance` over the log2(nparts) levels
  int levels = 0;
  while ((1 << levels) < nparts) ++levels;
  const double eps = levels ? std::max(0.0, std::pow(1.0 + imbalance, 1.0 / levels) - 1.0) : 0.0;
  recurse(g, verts, nparts, 0, eps, rng, local, part);
  if (nparts > 2) {
    const double mean = (double)n / nparts;
    kway_vcycle(g, part, nparts, std::max<int64_t>(1, (int64_t)std::floor(mean * (1.0 - imbalance))),
                (int64_t)std::ceil(mean * (1.0 + imbalance)), rng);
  }
  {  // every part holds a vertex (the bisection's per-side minimum and the k-way pass's floor of one vertex)
    std::vector<char> used(nparts, 0);
    for (int64_t v = 0; v < n; ++v) used[part[v]] = 1;
    for (int p = 0; p < nparts && n > 0; ++p)
      if (!used[p]) return RX_ERR_RANGE;
  }
  if (edge_cut) {
    std::vector<int> w(part, part + n);
    *edge_cut = cut_of(g, w);
  }
  return RX_OK;
}
