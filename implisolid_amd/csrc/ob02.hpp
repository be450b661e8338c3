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

class Ob02 {
public:
    Ob02(Engine& e, hipStream_t s);
    ~Ob02();
    Ob02(const Ob02&) = delete;
    Ob02& operator=(const Ob02&) = delete;
    // takes a copy of the MC mesh (device pointers) and builds the face/vertex topology; resets
    // the point sets and counters, so one Ob02 serves many builds (its buffers are grow-only)
    void load_mesh(const float* d_verts, int64_t nv, const int32_t* d_faces, int64_t nf);
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
    float last_average_edge() const { return avg_edge_; }
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

private:
    void store_pointset(const char* key, const float* d, int64_t n, bool keep_first);
    void build_topology();
    void scan(const uint32_t* in, uint32_t* out, int64_t n);   // exclusive, out[n] = total
    EdgeTab edge_table();
    void rand_tables(int64_t lanes);
    void add_rand_noise(float amplitude);
    void start_edge_fold();
    float finish_edge_fold();
    void start_perturbations();
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
        alphas_, pert_, pend_, misc_, fnew_, rtab_, scan_tmp_;
    bool topo_valid_ = false;
    int64_t rand_hi_rows_ = 0;
    float avg_edge_ = 0.f;
    uint32_t cap_hits_ = 0;
    uint64_t evals_ = 0;
    int64_t jit_launches_ = 0;   // OB02 passes that ran the JIT point module (since load_mesh)
    bool profile_ = false;
    double stage_ms_[kStages] = {};
    HostBuf host_norms_;                     // pinned: the edge-length terms and the fold's table (D2H)
    DevBuf fold_sum_;                        // the fold's chunk table (fold.hpp), built on the device
    hipEvent_t norms_ready_ = nullptr;
    hipStream_t copy_s_ = nullptr;           // the fold's D2H copies, beside the projection's prep pass
    hipEvent_t table_done_ = nullptr;
    DevBuf dir_, evals_buf_;
    std::vector<float> alphas_host_;         // kept until the next projection (async H2D source)
    std::future<std::shared_ptr<const std::vector<float>>> pert_job_;
    std::shared_ptr<const std::vector<float>> pert_host_;
    int64_t pert_nf_ = -1;
    bool pert_uploaded_ = false;
    struct Snapshot {
        DevBuf buf;
        int64_t n = 0;
    };
    std::map<std::string, Snapshot> snaps_;
    std::map<std::string, std::vector<float>> pointsets_;
};

}  // namespace impli
