// ob02.hpp -- the Ohtake-Belyaev refinement loop on the GPU (polygonizer steps 1-3).
#pragma once
#include <chrono>
#include <future>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "engine.hpp"

namespace impli {

struct EdgeTab;   // ob02.hip: open-addressed (vmin, vmax) table of the current faces
struct PertDev;   // ob02.hip: a face count's perturbation table on one device (process-wide cache)

// Ob02's range block (int64 fields of rng_): [kRngWork, +2) work faces, [kRngCen, +2) centroid
// faces, [kRngHalo, +2) halo vertices, [kRngOwn, +2) owned vertices (half-open), then four
// (min, max) scratch pairs of the range passes (work faces, centroid faces, halo vertices, and the
// vertices whose umbrellas a shard's topology holds)
constexpr int kRngWork = 0, kRngCen = 2, kRngHalo = 4, kRngOwn = 6, kRngScratch = 8, kRngFields = 16;

class Ob02 {
public:
    Ob02(Engine& e, hipStream_t s);
    ~Ob02();
    Ob02(const Ob02&) = delete;
    Ob02& operator=(const Ob02&) = delete;
    // takes a copy of the MC mesh (device pointers) and builds the face/vertex topology; resets
    // the point sets and counters, so one Ob02 serves many builds (its buffers are grow-only)
    // d_work (optional): the caller's vertex array (3 nv floats, kept alive by the caller until the
    // next load) becomes the working one in place -- the steps update it and a sharded caller's
    // exchange writes into it directly; d_verts is then ignored
    // normals_ahead: the caller's next step is vertex_resampling (build_geometry's loop), whose
    // centroid normals then run beside the topology passes
    void load_mesh(const float* d_verts, int64_t nv, const int32_t* d_faces, int64_t nf, float* d_work = nullptr,
                   bool normals_ahead = false);
    // Z-slab sharding of the loop (one Ob02 per rank, each holding the whole mesh): this rank owns
    // vertices [v0, v1) (its slab's).  Resampling and QEM then update only those; the per-face
    // passes run over the faces touching them (the work faces, a contiguous range: faces are in
    // z-major cell order and an owned vertex's faces lie in the slab's layers and the first layer
    // above) and, for the resampling weights, their edge neighbours as well.  The edge-length fold
    // runs over every face on every rank (the same serial chain, no exchange).  After each step
    // that moves vertices the caller exchanges the owned ranges (set_verts) before the next step.
    // Call after load_mesh; v0 = 0, v1 = nv restores the whole mesh.
    void set_owned_vertices(int64_t v0, int64_t v1);
    // load_mesh + set_owned_vertices for a shard in one pass: the ranges are found while the mesh is
    // copied, and the topology (umbrellas, faces of faces) is built only where the shard's passes
    // read it -- the umbrellas of the owned vertices and of the work faces' vertices, the faces of
    // faces of the work faces -- instead of over the whole mesh on every rank.  v0 = 0, v1 = nv is
    // load_mesh + set_owned_vertices(0, nv).
    void load_shard(const float* d_verts, int64_t nv, const int32_t* d_faces, int64_t nf, float* d_work, int64_t v0,
                    int64_t v1);
    // [v0, v1, work faces f0, f1, centroid faces f0, f1, halo vertices h0, h1]: [h0, h1) are the
    // vertices the next resampling reads (those of the centroid faces), so after a step only they
    // must be current before another resampling (the edge-length fold reads every vertex).  The
    // ranges are found on the device in stream order; this reads them back (blocking) once per
    // set_owned_vertices.
    void ranges(int64_t out[8]);
    // the exchange after a vertex-moving step: rows holds every rank's owned range (row r: rank r's
    // 3 (voff[r+1] - voff[r]) floats at r row_len), copied into the vertex array except row `self`,
    // on the stream (no host synchronisation)
    void unpack_ranges(const float* d_rows, int64_t row_len, const std::vector<int64_t>& voff, int self);
    hipStream_t stream() const { return s; }
    // device pointer of the current vertices (3 nv floats; valid until the next step)
    float* d_verts() { return verts_.as<float>(); }
    // step 1: apply_vertex_resampling_to_MC_buffers__VMS (apply_v_s_to_mc_buffers.hpp:280-326)
    void vertex_resampling(float c);
    // step 2: centroids_projection (centroids_projection.cpp:1219-1311)
    void centroids_projection(bool enable_qem);
    // step 3: my_subdiv_ (centroids_projection.cpp:1314-1367): 1-to-4 split of every face, then
    // randomize_verts noise from the process-global glibc rand() (host.hpp GlibcRand)
    void subdivide(float amplitude);
    int64_t n_verts() const { return nv; }
    int64_t n_faces() const { return nf; }
    // blocking copy of the current mesh to host
    void fetch(float* verts, int32_t* faces);
    // host copies of the point sets stored since load_mesh (blocking)
    const std::map<std::string, std::vector<float>>& pointsets();
    // the last projection's average edge length (blocking: read back from the device once)
    float last_average_edge();
    // after read_counters(): bisections that hit the cap, implicit evaluations of the projection
    // (counted only while profiling)
    void read_counters();
    uint32_t bisection_cap_hits() const { return cap_hits_; }
    uint64_t projection_evals() const { return evals_; }
    int64_t jit_launches() const { return jit_launches_; }
    // profiling: the stream is drained at every stage boundary and the wall time of each stage is
    // summed since load_mesh (topology, resampling, edge-length fold, projection, QEM, subdivision,
    // fetch); evaluations are counted.  Off by default (the stages then overlap freely).
    enum { kStageTopology, kStageResample, kStageEdgeFold, kStageProject, kStageQem, kStageSubdiv, kStageFetch, kStages };
    void set_profile(bool on) { profile_ = on; }
    const double* stage_ms() const { return stage_ms_; }
    bool capture_pointsets = true;
    bool capture_replace = true;   // false: skip the replacing point sets (a later store overwrites them)

private:
    void store_pointset(const char* key, const float* d, int64_t n, bool keep_first);
    void build_topology(bool deg_zeroed = false);   // deg_zeroed: deg_[0..nv] already 0 (load_mesh)
    void begin_load(const float*& d_verts, int64_t nv, int64_t nf, float* d_work);   // host state of a load
    void reserve_topology();
    void launch_centroid_normals(hipStream_t q);
    void scan(uint32_t* in, uint32_t* out, int64_t n, bool zero_in = false);   // exclusive, out[n] = total; zero_in: in[] left 0
    EdgeTab edge_table();
    void rand_tables(int64_t lanes);
    void add_rand_noise(float amplitude);
    hipStream_t start_edge_fold();
    void finish_edge_fold();
    void start_perturbations();
    void whole_ranges();
    const float* perturbations();
    struct Stage {   // profiling scope: stage k from construction to next() / destruction
        Ob02* ob;
        int stage;
        std::chrono::steady_clock::time_point t0;
        Stage(Ob02* o, int k);
        void next(int k);
        ~Stage();
    };

    Engine& E;
    hipStream_t s;
    int64_t nv = 0, nf = 0;
    DevBuf verts_, faces_, vnew_, cen_, nrm_, w_, fof_, uoff_, ulst_, etab_, deg_, proj_, grad_, fn_, norms_,
        pend_, misc_, fnew_, rtab_, scan_tmp_;
    bool topo_valid_ = false;
    bool topo_partial_ = false;   // the topology covers only a shard's ranges (load_shard)
    bool etab_valid_ = false;   // the edge table (subdivision only) matches the current faces
    int64_t own_v0_ = 0, own_v1_ = 0;   // owned vertices
    // the range block in device memory (int64, kRng* below): work faces (touching an owned vertex),
    // centroid faces (whose centroid / normal the work faces' weights read), halo vertices (those
    // faces' vertices: the next resampling's input), owned vertices, and the range passes' scratch
    DevBuf rng_;
    int64_t hrng_[8] = {};              // host copy (ranges()), valid if hrng_valid_
    bool hrng_valid_ = false;
    int64_t est_work_ = 0, est_cen_ = 0;   // grid sizes of the per-face passes (the kernels grid-stride)
    bool sharded_ = false;
    int64_t rand_hi_rows_ = 0;
    float avg_edge_ = 0.f;
    bool avg_valid_ = true;      // avg_edge_ holds the last fold's average (else read fold_out_)
    uint32_t cap_hits_ = 0;
    uint64_t evals_ = 0;
    int64_t jit_launches_ = 0;   // OB02 passes that ran the JIT point module (since load_mesh)
    bool profile_ = false;
    double stage_ms_[kStages] = {};
    DevBuf fold_sum_;                        // the fold's chunk table (fold.hpp), built on the device
    DevBuf fold_out_;                        // FoldOut (ob02_device.hpp): sum, average, alpha list
    hipStream_t side_s_ = nullptr;           // the projection's prep pass, beside the fold's walk on s
    hipEvent_t cnormals_done_ = nullptr;     // a new mesh's centroid normals, beside its topology passes
    bool normals_ahead_ = false;             // cen_ / nrm_ of the loaded mesh are on their way (load_mesh)
    hipEvent_t mesh_ready_ = nullptr, prep_done_ = nullptr;
    hipEvent_t early_done_ = nullptr, normals_done_ = nullptr;   // the QEM normals beside the late pass
    DevBuf dir_, evals_buf_;
    std::future<std::shared_ptr<const std::vector<float>>> pert_job_;
    std::shared_ptr<PertDev> pert_dev_;   // the device table in use (process-wide cache, ob02.hip)
    int64_t pert_nf_ = -1;
    struct Snapshot {
        DevBuf buf;
        int64_t n = 0;
        bool valid = false;   // stored since the last load_mesh (the buffer is kept across builds)
    };
    std::map<std::string, Snapshot> snaps_;
    std::map<std::string, std::vector<float>> pointsets_;
};

// the edge-length fold alone on n host terms (diagnostics, tests): the device's serial-chain sum
float debug_fold(const float* h_terms, int64_t n, int* table_chunks, long long* stats = nullptr, int* trace = nullptr);

}  // namespace impli
