/* rx_io.h — host-side setup and on-disk formats of the reactive-RANS path, C ABI.
 *
 * What the reference's driver does before the first iteration, restated natively (C++ in librx.so, no GPU):
 *   rx_mesh_read_su2   CPhysicalGeometry's SU2 ASCII reader (Common/src/geometry_structure.cpp:4819), then
 *                      CGeometry preprocessing in CDriver::Geometrical_Preprocessing's order
 *                      (SU2_CFD/src/driver_structure.cpp:552-585): SetPoint_Connectivity (:9145-9198),
 *                      SetRCM_Ordering (:9200-9340), SetPoint_Connectivity again, SetEdges (:223-252),
 *                      SetVertex, SetCoord_CG (:9518-9590), SetControlVolume (:10457-10560, median dual, edge
 *                      normals and dual volumes in the reference's element / face accumulation order),
 *                      SetBoundControlVolume (:9595-9660), FindNormal_Neighbor (:12610-12652); and
 *                      ComputeWall_Distance (nearest vertex of the HEAT_FLUX / ISOTHERMAL markers).
 *                      Serial reader (one rank); elements: triangle, quadrilateral (2-D), tetrahedron,
 *                      hexahedron (3-D); boundary: line (2-D), triangle, quadrilateral (3-D). Inverted elements
 *                      are flipped as Check_IntElem_Orientation / Check_BoundElem_Orientation do
 *                      (geometry_structure.cpp:8640-8960), after the connectivity, as the reference orders it.
 *   rx_mech_read       ReactingModelLibrary::Setup (Common/src/Framework/reacting_model_library.cpp:925-1506):
 *                      file list, mixture, chemistry (Parse_Terms Common/src/Tools/utility.cpp:12-86, CGS->SI
 *                      :1122-1132, Ta/R_cal :1209-1210, reversible product exponents :1113-1120, backward-rate
 *                      line :1218-1260), thermo / transport tables with spline second derivatives
 *                      (Common/src/Tools/spline.cpp:10-58, clamped zero-slope ends).
 *   rx_restart_write   COutput::SetRestart (SU2_CFD/src/output_structure.cpp:3858-4060) for REACTIVE_RANS:
 *                      header, one line per point in global-index order (index, coordinates, flow
 *                      conservatives, k, omega[, Pressure, Temperature, Mach, Laminar_Viscosity, mu_t]) at
 *                      precision(15) scientific, tab-separated, then the AOA / SIDESLIP / BCTHRUST / DCD_DCL /
 *                      EXT_ITER trailer.
 *   rx_restart_read    CReactiveEulerSolver::Load_Restart (solver_direct_reactive.cpp:566-686) + the SST
 *                      solver's restart columns (solver_direct_turbulent.cpp:2838-2850).
 *                      Elements: triangles / quadrilaterals (2-D), tetrahedra, hexahedra, prisms (VTK 13) and
 *                      pyramids (VTK 14) with the reference's tables (primal_grid_structure.cpp:478-622) and its
 *                      orientation tests (geometry_structure.cpp:8641-8794; a pyramid is never re-oriented:
 *                      CPyramid::Change_Orientation only prints); boundary lines (2-D), triangles / quads (3-D).
 *                      rx_mech_read rejects (RX_ERR_STATE) a property table that is not sorted, unique and
 *                      equispaced, as SetSpline's assertions do (spline.cpp:12-25): GetSpline locates the interval
 *                      by integer division.
 * Errors: RX_ERR_ARG (bad argument / malformed or unknown element line), RX_ERR_STATE (unreadable or malformed file; the reference exits). Points of an rx_mesh are in the reference's RCM order; global_index maps them to the file.
 */
#ifndef RX_IO_H
#define RX_IO_H

#include <stdint.h>

#include "rx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rx_mesh rx_mesh;
int rx_mesh_read_su2(const char *path, rx_mesh **out);
void rx_mesh_destroy(rx_mesh *mesh);
/* sizes: n_dim, points, edges, boundary vertices, markers */
int rx_mesh_info(const rx_mesh *mesh, int32_t *n_dim, int64_t *n_point, int64_t *n_edge, int64_t *n_bvert,
                 int32_t *n_marker);
/* MARKER_TAG of marker m (file order) or NULL */
const char *rx_mesh_marker_tag(const rx_mesh *mesh, int32_t m);
/* rx_mesh_desc over the mesh's arrays (one partition, single rank); valid until rx_mesh_destroy */
int rx_mesh_describe(const rx_mesh *mesh, rx_mesh_desc *out);
/* global (file) index of every point [N]; normal neighbour of every boundary vertex [n_bvert] */
const int64_t *rx_mesh_global_index(const rx_mesh *mesh);
const int64_t *rx_mesh_normal_neighbor(const rx_mesh *mesh);
/* ComputeWall_Distance: is_wall[n_marker] != 0 for the HEAT_FLUX / ISOTHERMAL markers of the cfg; distance of every
 * point to the nearest vertex of those markers (0 everywhere when there is none). Returns a pointer to [N].
 * is_wall NULL: the distances of the last call (rx_case_read computes them from the cfg's wall markers). */
const double *rx_mesh_wall_distance(rx_mesh *mesh, const int32_t *is_wall);

typedef struct rx_mech rx_mech;
int rx_mech_read(const char *base_dir, const char *list_file, rx_mech **out);
void rx_mech_destroy(rx_mech *mech);
int rx_mech_describe(const rx_mech *mech, rx_mech_desc *out); /* valid until rx_mech_destroy */
const char *rx_mech_species(const rx_mech *mech, int32_t s);  /* SPECIES name of species s */
double rx_mech_formation_enthalpy(const rx_mech *mech, int32_t s);

/* A reference case from its cfg (rx_case.cpp): CConfig::SetConfig_Parsing's grammar for the keys of this path, the
 * mesh (MESH_FILENAME, rx_mesh_read_su2) and library (CONFIG_LIB_FILE, rx_mech_read) relative to the cfg's directory,
 * the flow and SST rx_cfg (CConfig defaults for keys left out; SST: RELAXATION_FACTOR_TURB -> relaxation,
 * CFL_REDUCTION_TURB -> cfl), the markers in the mesh's marker order (MARKER_INLET / INLET_TYPE / INLET_MASS_FRAC,
 * MARKER_OUTLET, MARKER_ISOTHERMAL, MARKER_HEATFLUX, MARKER_EULER, MARKER_SYM), the wall distance to the
 * ISOTHERMAL / HEAT_FLUX markers, Mach_inf (CConfig::SetMach with the frozen sound speed) and the free-stream
 * turbulence of SetNondimensionalization (solver_direct_reactive.cpp:4534-4590). DIMENSIONAL cases only. Keys the
 * path does not implement give RX_ERR_UNSUPPORTED (message: rx_case_error). The mesh / mech / bc arrays belong to
 * the case until rx_case_destroy. */
typedef struct rx_case rx_case;
void rx_cfg_default(rx_cfg *cfg); /* the defaults of every rx_cfg field (jet values; refs 1; no ignition) */
int rx_case_read(const char *cfg_path, rx_case **out);
void rx_case_destroy(rx_case *c);
const char *rx_case_error(void);  /* message of the last failed rx_case_read (this thread) */
rx_mesh *rx_case_mesh(rx_case *c);
rx_mech *rx_case_mech(rx_case *c);
int rx_case_cfg(const rx_case *c, rx_cfg *flow, rx_cfg *sst);
int rx_case_bc(const rx_case *c, rx_bc_desc *bc);
/* RK_ALPHA_COEFF of a RUNGE-KUTTA_EXPLICIT case (n_stage 0 otherwise: EULER_EXPLICIT / EULER_IMPLICIT) */
int rx_case_rk(const rx_case *c, int32_t *n_stage, const double **alpha);
int rx_case_free_stream(const rx_case *c, double *rho, double *mu, double *T, double *P);

/* U [N][n_var] flow conservatives and T [N][2] (k, omega) in the mesh's point order; extra [N][5] (Pressure,
 * Temperature, Mach, Laminar_Viscosity, Eddy_Viscosity) or NULL (the reference's low-memory output). */
int rx_restart_write(const char *path, const rx_mesh *mesh, int32_t n_var, const double *U, const double *T,
                     const double *extra, int64_t ext_iter);
int rx_restart_read(const char *path, const rx_mesh *mesh, int32_t n_var, double *U, double *T);

/* Multilevel recursive-bisection partition of a graph (CSR xadj[n+1] / adj, both directions of every edge, no self
 * loops, unit weights) into nparts parts of n / nparts vertices within a relative `imbalance` (e.g. 0.03): part[n]
 * receives each vertex's part, edge_cut (may be NULL) the number of cut edges. Deterministic. The stand-in for the
 * reference's METIS call (CPhysicalGeometry::SetColorGrid, Common/src/geometry_structure.cpp:11360-11450; csrc/
 * rx_part.cpp); meshgen.partition_graph orders the parts into rx_mesh_desc.part_ptr. */
int rx_partition_graph(int64_t n, const int64_t *xadj, const int64_t *adj, int32_t nparts, double imbalance,
                       int32_t *part, int64_t *edge_cut);

#ifdef __cplusplus
}
#endif
#endif /* RX_IO_H */
