/*
 * oracle.h -- CPU restatement of the reference polygoniser hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity checker for the MI355X path.  It is plain C99, single threaded and
 * follows the reference ynotstartups/implisolid (js_iteration_2/) function by function; every
 * function cites the reference file:line it restates.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product (implisolid_amd/) never links it.
 *
 * Pinning: the reference has no tests, fixtures or golden vectors and cannot be
 * compiled here (Boost/Eigen/emscripten.h absent, F2), so this oracle is "parity unpinned" in the
 * sense of the task statement: it is a faithful restatement checked by construction and by
 * property tests, not by reference-produced vectors.  Library functions the reference calls are
 * pinned where possible: acosf is restated from glibc 2.35 and checked bit-exact over all
 * 2,130,706,434 floats in [-1,1] against this container's libm (tests/test_oracle_libm.py).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math).
 */
#ifndef IMPLI_ORACLE_H
#define IMPLI_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* node types (the MP5 "type" strings the factory accepts, object_factory.hpp:86-653) */
enum {
    OR_UNION = 0,      /* transformed_union         implicit_function/transformed_union.hpp      */
    OR_INTERSECTION,   /* transformed_intersection  implicit_function/transformed_intersection.hpp */
    OR_DIFFERENCE,     /* transformed_subtract      implicit_function/transformed_subtract.hpp   */
    OR_ELLIPSOID,      /* egg                       implicit_function/egg.hpp                    */
    OR_CUBE,           /* cube (rabbit SDF table)   implicit_function/cube.hpp                   */
    OR_CYLINDER,       /* scylinder                 implicit_function/scylinder.hpp              */
    OR_CONE,           /* scone                     implicit_function/scone.hpp                  */
    OR_HEART,          /* heart                     implicit_function/heart.hpp                  */
    OR_TORUS,          /* torus                     implicit_function/torus.hpp                  */
    OR_DMUSHROOM,      /* linearly_transformed(double_mushroom) object_factory.hpp:86-100       */
    OR_SCREW,          /* screw (identity transformation_matrix)  implicit_function/screw.hpp   */
    OR_LID,            /* top_bottom_lid            implicit_function/top_bottom_lid.hpp         */
    OR_HALF_PLANE,     /* half_plane                implicit_function/half_plane.hpp             */
    OR_TETRA,          /* tetrahedron               implicit_function/tetrahedron.hpp            */
    OR_METABALLS,      /* meta_ball_Rydgard         implicit_function/meta_balls_Rydgard.hpp     */
    OR_EXTRUSION,      /* extrusion (convex n-gon)  implicit_function/extrusion.hpp + 2d/GDT/convex_polygon.hpp */
    OR_SCREW_TBB,      /* inf_top_bot_bound(screw)  implicit_function/inf_top_bot_bound.hpp ("screw_gradient_wrong") */
    OR_NTYPES
};

typedef struct {
    int32_t type;
    int32_t child[2];   /* node indices, -1 when unused */
    float m[12];        /* transf_matrix, row-major 3x4, as read from the MP5 JSON */
    float minv[12];     /* inv_transf_matrix, filled by or_tree_prepare */
    float prm[128];     /* primitive parameters: screw {twist_rate, r0, delta};
                           half_plane {unit plane_vector xyz, plane_point xyz};
                           tetrahedron {a, b, c, d} x 4 planes; meta_balls {x, y, z, strength,
                           subtract} x 4 balls; extrusion {n, (nx, ny, n0) x n edges} */
} or_node;

/* basic_functions.hpp:77-128 invert_matrix (ublas LU in float). returns 1 on success. */
int or_invert_matrix(const float in12[12], float out12[12]);

/* fills minv of every node */
void or_tree_prepare(or_node* nodes, int n);

/* implicit_function::eval_implicit / eval_gradient over a batch (implicit_function.hpp:35-36) */
void or_eval(const or_node* nodes, int root, const float* xyz, int64_t n, float* f_out);
void or_grad(const or_node* nodes, int root, const float* xyz, int64_t n, float* g_out);

/* glibc-2.35 sinf (x86_64 FMA variant), atanf, atan2f restatements (or_libm.c) */
float or_sinf(float x);
float or_atanf(float x);
float or_atan2f(float y, float x);
int64_t or_libm_check(int which, uint32_t start, uint32_t stride, uint64_t count);
/* glibc-2.35 double cos (x86_64 FMA variant, s_sin.c __cos) restated (or_libm.c): the screw gradient */
double or_cos(double x);
int64_t or_cos_check(uint64_t start, uint64_t count, double lim);
void or_cos_apply(const double* a, int64_t n, double* out, int glibc);

/* glibc-2.35 acosf restatement (vertex_resampling.hpp:75 calls std::acos(float)) */
float or_acosf(float x);
int64_t or_acosf_check(uint32_t start, uint32_t stride, uint64_t count);

/* ---- marching cubes: MarchingCubes::produce_mesh (marching_cubes.hpp:1728-1738) ---- */
typedef struct {
    float* verts;      /* 3*nv floats (malloc'ed, free with or_mesh_free) */
    int32_t* faces;    /* 3*nf ints */
    int64_t nv, nf;
} or_mesh;

/* box = {xmin,xmax,ymin,ymax,zmin,zmax}; returns 0 on success */
int or_marching_cubes(const or_node* nodes, int root, int resolution, const float box[6], or_mesh* out);
void or_mesh_free(or_mesh* m);

/* the sampled field (res^3, sealed) for inspection: res = resolution + 5 */
int or_mc_field(const or_node* nodes, int root, int resolution, const float box[6], float* field_out);

/* ---- OB02 (polygonizer_algorithm_ob02.hpp steps 1-3) ---- */
/* step 1: apply_vertex_resampling_to_MC_buffers__VMS (apply_v_s_to_mc_buffers.hpp:280-326) */
int or_vertex_resampling(const or_node* nodes, int root, float c,
                         float* verts, int64_t nv, const int32_t* faces, int64_t nf,
                         float* centroids_out /* nullable, 3*nf */);
/* step 2: centroids_projection (centroids_projection.cpp:1219-1311).
   projected centroids are written to centroids_out (3*nf, nullable); verts updated if qem. */
int or_centroids_projection(const or_node* nodes, int root,
                            float* verts, int64_t nv, const int32_t* faces, int64_t nf,
                            int enable_qem, float* centroids_out, float* avg_edge_out);
/* step 3: my_subdiv_ (centroids_projection.cpp:1314-1367): 1-to-4 subdivision of every face, then
   randomize_verts with glibc rand() (process-global state, see or_srand).  *vout / *fout are
   malloc'ed (free with or_free). */
int or_subdivide(const float* verts, int64_t nv, const int32_t* faces, int64_t nf, float amplitude,
                 float** vout, int64_t* nv_out, int32_t** fout);
void or_srand(unsigned seed);
int or_rand(void);
void or_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
