/*
 * implisolid.h -- C ABI of the MI355X-native implicit-surface polygoniser.
 *
 * Drop-in replacement for the extern "C" interface of ImpliSolid's mcc2.cpp.  Every declaration
 * below names the reference declaration it replaces (/root/reference/js_iteration_2/mcc2.cpp,
 * declarations :88-134, definitions as cited).  Signatures, argument meaning, ownership and error
 * behaviour are the reference's; the work runs on the GPU (HIP, gfx950).
 *
 * Thread-safety: like the reference, one global geometry slot and one direct-eval slot; not
 * reentrant.  build_geometry returns after the result is host resident.
 */
#ifndef IMPLISOLID_H
#define IMPLISOLID_H

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- mesh API ------------------------------------------------------------------------------ */
/* mcc2.cpp:89 / :446-464  polygonise the MP5 shape with the given mc_settings JSON.  Refuses (with
   a message) while a previous result is active: call finish_geometry() first (:316-319). */
void build_geometry(const char* shape_parameters_json, const char* mc_parameters_json);
/* mcc2.cpp:90 (declared, body commented out at :296-302): build_geometry + worker call specs
   ({"progressCallback_id", "call_id", "shape_id"}, worker_call_specs.hpp:28-40; each -1 when
   absent).  Progress updates carry those ids (see implisolid_set_progress_callback). */
void build_geometry_u(const char* shape_parameters_json, const char* mc_parameters_json, const char* call_specs);
/* Additive: the progress hook of build_geometry / build_geometry_u -- the reference's
   polygonizer::send_mesh_back_to_client (polygonizer_algorithm_ob02.hpp:180-220), which posts the
   current mesh to wwapi.send_progress_update (js/worker_api.js:399-416) after marching cubes
   (mcc2.cpp:351), after each repeat's vertex resampling (:372) and after each centroid projection
   (:390).  The callback runs synchronously on the calling thread with the intermediate mesh
   (library-owned, valid during the call; get_v_ptr / get_f_ptr / get_v_size / get_f_size read the
   same mesh meanwhile) and the call specs' ids (-1 for plain build_geometry).  NULL unregisters. */
typedef void (*implisolid_progress_callback)(const float* verts, int n_verts, const int32_t* faces, int n_faces,
                                             int progress_callback_id, int shape_id, int call_id, void* user);
void implisolid_set_progress_callback(implisolid_progress_callback cb, void* user);
/* mcc2.cpp:91 / :470-473  vertex count */
int get_v_size(void);
/* mcc2.cpp:92 / :466-469  face count */
int get_f_size(void);
/* mcc2.cpp:93 / :496-511  copy 3*fcount int32 vertex indices */
void get_f(int* f_out, int fcount);
/* mcc2.cpp:94 / :474-492  copy 3*vcount float32 coordinates */
void get_v(float* v_out, int vcount);
/* mcc2.cpp:95 / :540-552  release the slot (buffers stay valid until the next build) */
void finish_geometry(void);
/* mcc2.cpp:96 / :521-525  library-owned int32 triplets */
void* get_f_ptr(void);
/* mcc2.cpp:97 / :515-519  library-owned float32 xyz */
void* get_v_ptr(void);

/* ---- direct evaluation API ------------------------------------------------------------------ */
/* mcc2.cpp:106 / :726-741  returns 1, or 0 if an object is already set */
int set_object(const char* shape_parameters_json, bool ignore_root_matrix);
/* mcc2.cpp:107 / :743-763 */
bool unset_object(int id);
/* mcc2.cpp:109 / :765-799  0 <= n < 50000 points, float32 xyz */
bool set_x(void* verts, int n);
/* mcc2.cpp:110 / :800-812 */
void unset_x(void);
/* mcc2.cpp:112 / :815-822 */
void calculate_implicit_values(void);
/* mcc2.cpp:113 / :827-829 */
void* get_values_ptr(void);
/* mcc2.cpp:114 / :830-832 */
int get_values_size(void);
/* mcc2.cpp:116 / :834-889  with normalize_and_invert: g <- -g/|g| (factor -42 if |g| <= 1e-4) */
void calculate_implicit_gradients(bool normalize_and_invert);
/* mcc2.cpp:117 / :890-903 */
void* get_gradients_ptr(void);
/* mcc2.cpp:118 / :904-911  = 3n */
int get_gradients_size(void);

/* ---- misc ------------------------------------------------------------------------------------ */
/* mcc2.cpp:122 / :203-209  debug point sets (pre/post_resampling_vertices, pre/post_p_centroids,
   pre/post_qem_verts); NULL if absent */
void* get_pointset_ptr(char* id);
/* mcc2.cpp:123 / :210-215 */
int get_pointset_size(char* id);
/* mcc2.cpp:126 / :574-617  build information */
void about(void);

/* ---- additive API (not in the reference) ---------------------------------------------------- */
/* last error message of this thread's calls ("" if none) */
const char* implisolid_last_error(void);
/* 0 (default): abort() where the reference aborts (bad settings, unknown MP5 type);
   1: print the same message, record it in implisolid_last_error() and return */
void implisolid_set_error_mode(int mode);

/* Additive: per-brick interval pruning of the field evaluation (process-wide; environment
 * IMPLISOLID_PRUNE=<level> sets the initial level).  0 off; 1 CSG operands proven irrelevant over a
 * brick are skipped (field bit-identical); 2 (default) additionally fills bricks that are
 * sign-definite together with their face neighbours with +-1 (only their sign is ever read, so
 * the mesh is bit-identical). */
void implisolid_set_pruning(int level);

/* Additive, host only: the library's process-global glibc rand() generator, which the subdivision
 * noise draws from (randomize_verts, basic_functions.hpp:551-557, calls the C library's rand()).
 * It starts in glibc's unseeded state (srand(1)); implisolid_srand/implisolid_rand behave as
 * srand/rand; implisolid_rand_skip(n) discards n draws (jump-ahead, O(log n)). */
void implisolid_srand(unsigned seed);
int implisolid_rand(void);
void implisolid_rand_skip(uint64_t n);

/* Additive, host only: the parsed mc-settings (polygoniser_settings.hpp:147-305 semantics).
 * ints = resolution, ignore_root_matrix, overall_repeats, vresampl.iters, projection, qem, subdiv;
 * floats = vresampl.c, debug.post_subdiv_noise.  0, or -1 with implisolid_last_error() set where
 * the reference would abort() (error mode 0 aborts, as the reference). */
int implisolid_parse_settings(const char* mc_json, float box[6], int32_t ints[7], float floats[2]);

/* Additive, host only: Z-slab decomposition used by the slab API -- rank owns cell layers
 * [out[0], out[1]) and recomputes out[2] (0/1) halo layers below. */
int implisolid_slab_partition(int R, int rank, int nranks, int32_t out[3]);
/* Additive: balanced Z-slab cuts (nranks + 1 cell-layer boundaries, cuts[0] = 1, cuts[nranks] =
 * R + 3; rank r owns layers [cuts[r], cuts[r+1])).  Runs the interval pass of the whole grid once
 * on the current HIP device and splits the estimated work (listed bricks per layer) evenly; every
 * rank computing it gets the same cuts, so no exchange is needed (blocking). */
int implisolid_slab_balance(const char* shape_json, const char* mc_json, int nranks, int32_t* cuts);
/* host only: the same split from per-sample-layer listed-brick counts of the whole grid
 * (n_layers = R + 3) and the bricks per layer */
int implisolid_cuts_from_layer_work(const int64_t* listed, int n_layers, int64_t bricks_per_layer, int R, int nranks,
                                    int32_t* cuts);
/* Additive: the devices build_geometry uses for marching cubes (HIP ordinals; n <= 0 or NULL: the
 * current device only).  With n > 1 the grid is split into n balanced Z-slabs, slab r on device
 * ids[r] (a device may repeat), the slabs' meshes are concatenated in rank order on the host --
 * byte-identical to one device -- and the OB02 steps run on ids[0]. */
int implisolid_set_devices(const int32_t* ids, int n);
/* Additive diagnostics of the OB02 steps (polygonizer_algorithm_ob02.hpp:74-157 keeps per-step
 * timers, timer.hpp:33-75).  With profiling on, build_geometry drains its stream at every stage
 * boundary and sums each stage's wall time, and counts the projection's implicit evaluations (off
 * by default: the stages then overlap and nothing is counted).  last_build_stats (blocking) returns
 * [bisections that hit the 200-round cap (F8e), projection evaluations (profiled builds),
 *  last average edge length, ms of: topology, vertex resampling, edge-length fold, projection, QEM,
 *  subdivision, result fetch (profiled builds), faces, vertices, OB02 passes that ran the JIT point
 *  module] of the last build. */
void implisolid_ob02_profile(int on);
int implisolid_last_build_stats(double out[13]);
/* evaluate n >= 0 points (no 50k limit) of the current set_object(); grad may be NULL */
int implisolid_eval_points(const float* xyz, int64_t n, float* f_out, float* grad_out);
/* Additive, diagnostics: the device restatements of glibc 2.35 sinf (which 0: out = sinf(a)),
   atanf (1) and atan2f (2: out = atan2f(a, b)) that the screw family calls (screw.hpp:20-36,
   std::sin / std::atan2 on floats), on n host operands; 0 or -1 with implisolid_last_error() */
int implisolid_debug_libm(int which, const float* a, const float* b, int64_t n, float* out);
/* Additive, diagnostics: the device restatement of glibc 2.35's double cos (x86_64 FMA variant) that
   the screw gradient calls (screw.hpp:178-180, cos(M_PI * (...))), on n host doubles; 0 or -1 */
int implisolid_debug_cos(const double* a, int64_t n, double* out);
/* Additive, diagnostics: the edge-length fold of the projection (compute_average_edge_length,
   centroids_projection.cpp:70-82: s = 0; s += e[k] in order, float) on n host terms, computed as
   build_geometry computes it -- the chunk table and the device walk; *sum_out = s, *table_chunks
   (may be NULL) = chunks the walk took from the table.  0, or -1 with implisolid_last_error(). */
int implisolid_debug_fold(const float* terms, int64_t n, float* sum_out, int64_t* table_chunks);

/* host-only: compile an MP5 tree to the node program; info = {n_instr, depth, n_mats, 0};
   mats_out receives n_mats inverse matrices (12 floats each, up to 256) */
/* Additive, host only (no GPU): generate and hipRTC-compile the tree kernel for this shape.
 * Returns the code-object size (> 0), or -1 with implisolid_last_error(); optionally copies the
 * generated source (NUL-terminated, truncated to capacity) and the compile time in seconds. */
int64_t implisolid_jit_compile(const char* shape_json, char* source_out, int64_t capacity, double* seconds);
/* the same for the shape's point module (the OB02 passes and direct evaluation over straight-line
 * tree code; used by build_geometry's OB02 steps and implisolid_eval_points once loaded) */
int64_t implisolid_jit_compile_points(const char* shape_json, char* source_out, int64_t capacity, double* seconds);
int implisolid_program_info(const char* shape_json, int ignore_root_matrix, int32_t info[4], float* mats_out);

/* Device-resident slab pipeline (benchmarks / multi-GPU Z-slab runs).  A slab engine owns the
   device buffers of one Z-slab of one object on the current HIP device.  `stream` is a
   hipStream_t (may be NULL).  The launches (eval, count, emit*, copy_*) are stream-ordered and do
   not block; implisolid_slab_counts, _download, _stats* and _kernel_times* block on their stream;
   the setup calls (create*, set_offsets) synchronise the device, since the buffers they reset or
   write may still be read by kernels of an earlier call on another stream. */
typedef struct implisolid_slab implisolid_slab;
implisolid_slab* implisolid_slab_create(const char* shape_json, const char* mc_json, int rank, int nranks);
/* async device-to-device copy of the slab's emitted mesh (nv vertices, nf faces, as counted) into
 * caller-owned device buffers on the slab's device (the multi-process output gather) */
int implisolid_slab_copy_mesh(implisolid_slab* s, float* d_verts, int32_t* d_faces, int64_t nv, int64_t nf, void* stream);
/* the slab of cell layers [z0, z1) (e.g. from implisolid_slab_balance); a halo layer below if z0 > 1 */
implisolid_slab* implisolid_slab_create_range(const char* shape_json, const char* mc_json, int z0, int z1);
void implisolid_slab_destroy(implisolid_slab* s);
int implisolid_slab_eval(implisolid_slab* s, void* stream);            /* field (K1) */
int implisolid_slab_count(implisolid_slab* s, void* stream);           /* counts + scan (K2) */
/* d_offsets: device uint32[2] = this slab's {vertex, face} offset in the global numbering, or NULL
   for the host-set offsets (implisolid_slab_set_offsets, default 0) */
int implisolid_slab_emit(implisolid_slab* s, const uint32_t* d_offsets, void* stream);
/* emit in two halves, so that the count all-gather can overlap the vertex pass: verts needs no
   offsets (slab-local ids); faces takes d_offsets as above, or d_gathered = every rank's
   copy_counts (device uint32[nranks][4], rank order) and this slab's rank, from which it forms
   its vertex offset on the device */
int implisolid_slab_emit_verts(implisolid_slab* s, void* stream);
int implisolid_slab_emit_faces(implisolid_slab* s, const uint32_t* d_offsets, const uint32_t* d_gathered, int rank,
                               void* stream);
/* device uint32[16]: [2] owned verts incl. halo, [3] faces, [4] active cells, [5] halo verts */
const uint32_t* implisolid_slab_counters(implisolid_slab* s);
/* blocking: out[0] = vertices, out[1] = faces of this slab, out[2] = overflow flag; grows the
   output buffers when needed (then emit again) */
int implisolid_slab_counts(implisolid_slab* s, void* stream, uint32_t out[3]);
int implisolid_slab_grid(implisolid_slab* s, int32_t out[8]);
/* async device copy of counters[2..5] (owned verts incl. halo, faces, active cells, halo verts)
   into d_dst (uint32[4]) on `stream` -- for device-side all-gathers */
int implisolid_slab_copy_counts(implisolid_slab* s, uint32_t* d_dst, void* stream);
int implisolid_slab_set_offsets(implisolid_slab* s, uint32_t voff, uint32_t foff);
/* blocking copy of the slab's emitted vertices (3*V floats) and faces (3*F ints, global ids) */
int implisolid_slab_download(implisolid_slab* s, float* verts, int32_t* faces, void* stream);   /* R, res, cz0, cz1, cz_emit, fz0, fz1, depth */
float* implisolid_slab_verts(implisolid_slab* s);     /* device pointers */
int32_t* implisolid_slab_faces(implisolid_slab* s);
float* implisolid_slab_field(implisolid_slab* s);
/* blocking copy of the slab's stored field samples (n*n*layers floats, x fastest, converted from
 * the device's brick-major storage); with out == NULL returns the sample count only.
 * implisolid_slab_field's device pointer is brick-major (8x8x2-sample bricks, x fastest inside). */
int64_t implisolid_slab_read_field(implisolid_slab* s, float* out, int64_t capacity);
/* per-kernel HIP-event timing (stream-ordered, no synchronisation) of the following eval /
 * count / emit calls; kernel_times blocks and returns milliseconds of the last timed calls for
 * [brick pass, field eval, MC count, unit scan, vertex emission, face emission] */
int implisolid_slab_set_timing(implisolid_slab* s, int on);
/* after count: [units, non-empty units, owned vertices (incl. halo), triangles, active cells,
 * halo-owned vertices, cells, mixed coarse boxes of the last eval] (blocking) */
int implisolid_slab_stats(implisolid_slab* s, int64_t out[8]);
/* the same figures, then [halo-owned vertices as the vertex pass reads them (counter word 1, must
 * equal [5]), unit parts]: writes min(n, 10) values and returns how many exist (10), or -1 */
int implisolid_slab_stats_n(implisolid_slab* s, int64_t* out, int n);
/* the tree kernels the slab's last eval ran: 0 the interpreter, 1 the shape's JIT module, 2 the
 * object's baked JIT module */
int implisolid_slab_used_jit(implisolid_slab* s);
/* process-wide tree-kernel JIT mode for objects set from now on (environment IMPLISOLID_JIT):
 *   0 off (interpreter kernels only), 1 sync (hipRTC compiles before the first eval of a new shape),
 *   2 async (default: compilation runs on background threads, evals use the interpreter kernels
 *   until the module is loaded -- a never-seen shape pays no compile latency).  Compiled code
 *   objects are kept in a disk cache (IMPLISOLID_JIT_CACHE).  Results are bit-identical in every mode. */
void implisolid_set_jit(int mode);
/* tree modules with the object's matrices baked in as literals (IMPLISOLID_JIT_BAKE): 0 never (one
 * module per tree shape, matrices read from memory), 1 every object (one module per object), 2
 * (default) hot objects: an engine that evaluates the same object 4 times requests its baked module
 * (in the background in async mode) and switches to it once loaded.  Bit-identical in every mode. */
void implisolid_set_jit_bake(int mode);
/* block until all scheduled tree-kernel compilations have finished */
void implisolid_jit_wait(void);
/* [mode, bake, modules compiled, modules read from the disk cache], total compile seconds */
void implisolid_jit_stats(int32_t out[4], double* compile_seconds);
/* bound on the loaded tree modules (IMPLISOLID_JIT_MAX_MODULES, default 1024, at least 8): past it
 * the least recently requested modules no engine holds are unloaded (a later request recompiles or
 * reads the disk cache).  Unloads happen at trim points -- set_object and implisolid_jit_wait, where
 * the device is synchronised anyway -- so between them the loaded modules may exceed the bound; a
 * request evicts on its own only once the cache is 4x over it (4 n modules is the hard bound).
 * Replaces nothing in mcc2.cpp: the reference interprets its trees. */
void implisolid_set_jit_max_modules(int n);
/* [modules resident, bound, modules unloaded so far] */
void implisolid_jit_modules(int32_t out[3]);
int implisolid_slab_kernel_times(implisolid_slab* s, float ms[6]);
/* the same timing per kernel: [coarse interval pass, brick refine, brick fill, field eval, MC count,
 * unit scan, vertex emission (k_mc_cells), face emission (k_mc_faces)] */
int implisolid_slab_kernel_times_each(implisolid_slab* s, float ms[8]);
/* blocking copy of the slab's sample signs (1: value < 0), n*n*layers bytes, x fastest; with
 * out == NULL returns the count.  At pruning level 2 sign-filled bricks keep no field values, so
 * this (not the field) is the complete sign information marching cubes uses. */
int64_t implisolid_slab_read_signs(implisolid_slab* s, uint8_t* out, int64_t capacity);
/* bricks of the last slab eval: out = [bricks, mixed-sign bricks, sign-filled bricks] (blocking);
 * sign-filled = no value computed (claimed neighbour candidates, which were evaluated, excluded) */
int implisolid_slab_brick_stats(implisolid_slab* s, int64_t out[3]);

/* Object stream (BASELINE config 5): n objects polygonised with the same mc settings, each with
 * its own buffers.  create runs each object once to size its outputs, then:
 *   n_streams <= 0 (merged): run() launches every stage of eval + MC once for all objects (block row
 *     y = object y; the interpreter kernels, no per-object compilation);
 *   n_streams >= 1: compiles every tree kernel (parallel hipRTC), captures each object's eval +
 *     count + emit in a hipGraph (direct launches when capture is unavailable, or with
 *     IMPLISOLID_NO_GRAPH=1), and run() replays them round-robin over n_streams streams joined back
 *     into `stream`.
 * run is async on `stream`; counts and download block.  info = {objects, streams, graphs (1/0),
 * merged (1/0)} and the JIT compile seconds. */
typedef struct implisolid_batch implisolid_batch;
implisolid_batch* implisolid_batch_create(const char* const* shapes, int n, const char* mc_json, int n_streams);
int implisolid_batch_run(implisolid_batch* b, void* stream);
int implisolid_batch_info(implisolid_batch* b, int32_t out[4], double* jit_seconds);
int implisolid_batch_counts(implisolid_batch* b, int i, uint32_t out[3]);
int implisolid_batch_download(implisolid_batch* b, int i, float* verts, int32_t* faces);
void implisolid_batch_destroy(implisolid_batch* b);

/* The OB02 loop (polygonizer steps 1-3, polygonizer_algorithm_ob02.hpp:74-157) on one Z-slab shard of
 * a multi-GPU build: every rank loads the whole MC mesh (device pointers on the current device) and
 * owns the vertices [v0, v1) of its slab.  resample / project (+ QEM per the mc settings) update only
 * the owned vertices, evaluating the faces that touch them (and their edge neighbours for the
 * resampling weights); the edge-length fold runs over every face on every rank.  After each step
 * that moves vertices, the caller exchanges the owned ranges: get_verts copies the current
 * vertices (3 nv floats) into a device buffer, set_verts takes them back.  Every call blocks;
 * ranges = [v0, v1, work faces f0, f1, centroid faces f0, f1].  Results are byte-identical to the
 * single-device loop.  0, or -1 with implisolid_last_error(). */
typedef struct implisolid_ob02 implisolid_ob02;
implisolid_ob02* implisolid_ob02_create(const char* shape_json, const char* mc_json);
void implisolid_ob02_destroy(implisolid_ob02* h);
int implisolid_ob02_load(implisolid_ob02* h, const float* d_verts, int64_t nv, const int32_t* d_faces, int64_t nf, int64_t v0,
                         int64_t v1);
int implisolid_ob02_resample(implisolid_ob02* h);
int implisolid_ob02_project(implisolid_ob02* h);
int implisolid_ob02_subdivide(implisolid_ob02* h, float amplitude);
int implisolid_ob02_counts(implisolid_ob02* h, int64_t out[2]);
int implisolid_ob02_ranges(implisolid_ob02* h, int64_t out[6]);
int implisolid_ob02_get_verts(implisolid_ob02* h, float* d_dst);
int implisolid_ob02_set_verts(implisolid_ob02* h, const float* d_src);
int implisolid_ob02_download(implisolid_ob02* h, float* verts, int32_t* faces);
/* Stream-ordered form of the same loop (distributed.ob02_sharded): no host synchronisation per step.
 *   attach: like load, ordered after `after_stream` by an event (no device synchronisation), and
 *     d_verts (3 nv floats, the caller's, kept alive until destroy or the next attach/load) becomes
 *     the working vertex array itself: the steps update it in place and the caller's exchange
 *     writes the other ranks' ranges into it.  Two small read-backs size the shard's ranges.
 *   stream: the handle's HIP stream; the caller enqueues its collectives on it (and orders its
 *     own streams after it).
 *   resample_async / project_async: the steps, enqueued on that stream.
 *   unpack: after an all-gather of every rank's owned range into equal rows (row r = rank r's
 *     3 (voff[r+1] - voff[r]) floats at d_rows + r row_len; voff: host int64[world + 1]), one kernel
 *     on the stream copies every row but `self` into the vertex array.
 *   halo: [h0, h1), the vertices the next resampling reads (those of the faces whose centroids its
 *     weights use): between a QEM and a resampling only they must be exchanged; the edge-length
 *     fold of a projection reads every vertex. */
int implisolid_ob02_attach(implisolid_ob02* h, float* d_verts, int64_t nv, const int32_t* d_faces, int64_t nf, int64_t v0,
                           int64_t v1, void* after_stream);
void* implisolid_ob02_stream(implisolid_ob02* h);
int implisolid_ob02_resample_async(implisolid_ob02* h);
int implisolid_ob02_project_async(implisolid_ob02* h);
int implisolid_ob02_unpack(implisolid_ob02* h, const float* d_rows, int64_t row_len, const int64_t* voff, int world, int self);
int implisolid_ob02_halo(implisolid_ob02* h, int64_t out[2]);

#ifdef __cplusplus
}
#endif
#endif
