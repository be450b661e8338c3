// ob02.hpp -- the Ohtake-Belyaev refinement loop on the GPU (polygonizer steps 1-3).
#pragma once
#include <map>
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
    uint32_t bisection_cap_hits() const { return cap_hits_; }
    bool capture_pointsets = true;

private:
    void store_pointset(const char* key, const float* d, int64_t n, bool keep_first);
    void build_topology();
    void scan(const uint32_t* in, uint32_t* out, int64_t n);   // exclusive, out[n] = total
    EdgeTab edge_table();
    void rand_tables(int64_t lanes);
    void add_rand_noise(float amplitude);
    float average_edge_length();

    Engine& E;
    hipStream_t s;
    int64_t nv = 0, nf = 0;
    DevBuf verts_, faces_, vnew_, cen_, nrm_, w_, fof_, uoff_, ulst_, etab_, deg_, proj_, grad_, fn_, norms_,
        alphas_, pert_, pend_, misc_, fnew_, rtab_, scan_tmp_;
    bool topo_valid_ = false;
    int64_t rand_hi_rows_ = 0;
    float avg_edge_ = 0.f;
    uint32_t cap_hits_ = 0;
    struct Snapshot {
        DevBuf buf;
        int64_t n = 0;
    };
    std::map<std::string, Snapshot> snaps_;
    std::map<std::string, std::vector<float>> pointsets_;
};

}  // namespace impli
