// abi.hip -- the extern "C" drop-in boundary (mcc2.cpp:88-134) over the MI355X engine.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <map>
#include <memory>
#include <string>
#include <vector>
#include <thread>
#include <mutex>
#include <algorithm>

#include "../../include/implisolid.h"
#include "engine.hpp"
#include "batch_device.hpp"
#include "brick_modes.hpp"
#include "jit.hpp"

#include <chrono>
#include <rocprofiler-sdk-roctx/roctx.h>
#include "host.hpp"
#include "ob02.hpp"

using namespace impli;

namespace {

int g_error_mode = 0;           // 0: abort like the reference, 1: report and return
thread_local std::string g_last_error;

void report(const std::string& msg, bool reference_aborts) {
    g_last_error = msg;
    std::fprintf(stderr, "%s\n", msg.c_str());
    if (reference_aborts && g_error_mode == 0) std::abort();
}

// The host mesh of the last build, in pinned memory (D2H at full PCIe rate, where pageable memory
// goes through the driver's staging copies) that resize() does not zero (a vector zero-filled 13 MB
// per 512^3 build before the copy overwrote it).  Grow-only; kept until exit.
template <class T>
struct PinnedVec {
    T* p = nullptr;
    size_t n = 0, cap = 0;
    size_t size() const { return n; }
    T* data() { return p; }
    const T* data() const { return p; }
    void resize(size_t m) {
        if (m > cap) {
            const size_t nc = std::max(m, cap + cap / 2);
            T* q = nullptr;
            if (hipHostMalloc((void**)&q, nc * sizeof(T), hipHostMallocDefault) != hipSuccess || !q)
                throw HipError("host mesh: pinned allocation failed");
            if (n) std::memcpy(q, p, n * sizeof(T));
            if (p) (void)hipHostFree(p);
            p = q;
            cap = nc;
        }
        n = m;
    }
};
struct GeometryState {               // state_t, mcc2.cpp:165-193
    bool active = false;
    PinnedVec<float> verts;
    PinnedVec<int32_t> faces;
};
GeometryState g_state;

// worker_call_sepcs_t (worker_call_specs.hpp:7-47): the ids a progress update carries back to the
// caller; build_geometry uses the default (all -1), build_geometry_u the parsed call specs
struct CallSpecs {
    int progress_callback_id = -1, call_id = -1, shape_id = -1;
};
implisolid_progress_callback g_progress = nullptr;
void* g_progress_user = nullptr;

// polygonizer::send_mesh_back_to_client (polygonizer_algorithm_ob02.hpp:180-220): the reference
// hands the current mesh to wwapi.send_progress_update through EM_ASM after marching cubes, after
// each repeat's resampling and after each projection.  Here the registered callback gets it; as in
// the reference, get_v_ptr / get_f_ptr / get_v_size / get_f_size read that intermediate mesh while
// the callback runs.  Nothing is copied when no callback is registered.
void send_mesh_back_to_client(Ob02* ob, const CallSpecs& cs) {
    if (!g_progress) return;
    if (ob) {
        g_state.verts.resize((size_t)ob->n_verts() * 3);
        g_state.faces.resize((size_t)ob->n_faces() * 3);
        ob->fetch(g_state.verts.data(), g_state.faces.data());
    }
    g_progress(g_state.verts.data(), (int)(g_state.verts.size() / 3), g_state.faces.data(),
               (int)(g_state.faces.size() / 3), cs.progress_callback_id, cs.shape_id, cs.call_id, g_progress_user);
}

std::map<std::string, std::vector<float>> g_pointsets;   // pointset_set.hpp:8
std::unique_ptr<Ob02> g_ob02;   // the refinement state of the last build
// At exit the refinement state is left to the process (released, not destroyed): its destructor
// waits for its perturbation thread and frees HIP streams, events and memory, which a namespace-scope
// static would do after the runtime's own teardown.  Registered at the first Ob02, so it runs before
// g_ob02's destructor.
static Ob02* new_ob02(Engine& E, hipStream_t s) {
    static std::once_flag once;
    std::call_once(once, [] { std::atexit([] { (void)g_ob02.release(); }); });
    return new Ob02(E, s);
}
// The point sets (get_pointset_*) live on the device in g_ob02's snapshots; they are copied to
// g_pointsets only when asked for after a build (a D2H copy of every set per build cost ~0.25 ms)
bool g_pointsets_dirty = false;
void materialize_pointsets() {
    if (!g_pointsets_dirty || !g_ob02) return;
    // STORE_POINTSET (pointset_set.hpp:11-25) replaces; vertex_resampling.hpp:176-211 uses
    // map::emplace on a never-cleared global, so the first resampling point sets persist
    for (auto& kv : g_ob02->pointsets()) {
        const bool first_wins = kv.first == "pre_resampling_vertices" || kv.first == "post_resampling_vertices";
        if (first_wins && g_pointsets.count(kv.first)) continue;
        g_pointsets[kv.first] = kv.second;
    }
    g_pointsets_dirty = false;
}
bool g_ob02_profile = false;
bool g_last_refined = false;   // the last build ran the refinement loop (implisolid_last_build_stats)

struct EvalService {                 // ifunction_service, mcc2.cpp:699-705
    bool has_object = false;
    bool has_x = false;
    std::vector<float> x, f, grad;
};
EvalService g_eval;

Engine& engine() {
    static std::unique_ptr<Engine> e;
    if (!e) e.reset(new Engine());
    return *e;
}

hipStream_t abi_stream() {
    static hipStream_t s = nullptr;
    if (!s) IMPLI_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return s;
}

hipStream_t abi_copy_stream() {   // the vertices' device-to-host copy beside the face pass
    static hipStream_t s = nullptr;
    if (!s) IMPLI_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return s;
}

// ---- build_geometry over several devices (implisolid_set_devices) -------------------------------
std::vector<int> g_devices;   // empty: the current device only

struct DeviceGuard {          // restores the caller's current device
    int prev = 0;
    DeviceGuard() { (void)hipGetDevice(&prev); }
    ~DeviceGuard() { (void)hipSetDevice(prev); }
};

struct SlabEngine {           // one slab's engine and stream on its device, kept across builds
    int device = 0;
    hipStream_t stream = nullptr;
    std::unique_ptr<Engine> engine;
    ~SlabEngine() {
        if (stream) {
            (void)hipSetDevice(device);
            engine.reset();
            (void)hipStreamDestroy(stream);
        }
    }
};
std::vector<std::unique_ptr<SlabEngine>> g_slab_engines;

// polygonize_step_0 on g_devices: balanced cuts (cached per object and grid), every slab evaluated
// and counted on its device concurrently, vertex / face offsets from the counts (host), emission,
// and the slabs' meshes copied into the host result at their offsets -- byte-identical to one GPU.
void multi_device_mc(const Program& prog, const MCSettings& st, PinnedVec<float>& verts, PinnedVec<int32_t>& faces) {
    DeviceGuard guard;
    const int n = (int)g_devices.size();
    while ((int)g_slab_engines.size() < n) {
        const int d = g_devices[g_slab_engines.size()];
        IMPLI_HIP(hipSetDevice(d));
        std::unique_ptr<SlabEngine> se(new SlabEngine());
        se->device = d;
        IMPLI_HIP(hipStreamCreateWithFlags(&se->stream, hipStreamNonBlocking));
        se->engine.reset(new Engine());
        g_slab_engines.push_back(std::move(se));
    }
    static std::string cut_key;
    static std::vector<int> cuts;
    std::string key((const char*)&prog, sizeof(Program));
    key.append((const char*)&st.resolution, sizeof st.resolution).append((const char*)st.box, sizeof st.box);
    key.append((const char*)&n, sizeof n);
    if (key != cut_key) {
        IMPLI_HIP(hipSetDevice(g_devices[0]));
        cuts = balance_cuts(prog, st.resolution, st.box, n, g_slab_engines[0]->stream);
        cut_key = key;
    }
    for (int r = 0; r < n; ++r) {   // eval + count, all devices in flight
        SlabEngine& se = *g_slab_engines[(size_t)r];
        IMPLI_HIP(hipSetDevice(se.device));
        se.engine->set_object(prog);
        se.engine->set_slab(st.resolution, st.box, SlabRange{cuts[(size_t)r], cuts[(size_t)r + 1], 0});
        se.engine->eval_field(se.stream);
        se.engine->count(se.stream);
    }
    std::vector<SlabCounts> c((size_t)n);
    std::vector<int64_t> voff((size_t)n + 1, 0), foff((size_t)n + 1, 0);
    for (int r = 0; r < n; ++r) {
        SlabEngine& se = *g_slab_engines[(size_t)r];
        IMPLI_HIP(hipSetDevice(se.device));
        c[(size_t)r] = se.engine->read_counts(se.stream, nullptr);
        se.engine->ensure_capacity(c[(size_t)r]);
        voff[(size_t)r + 1] = voff[(size_t)r] + c[(size_t)r].n_verts();
        foff[(size_t)r + 1] = foff[(size_t)r] + c[(size_t)r].n_faces();
    }
    if (voff[(size_t)n] >= ((int64_t)1 << 31) || foff[(size_t)n] >= ((int64_t)1 << 31))
        throw InputError("build_geometry: the mesh exceeds 2^31 vertices or faces");
    for (int r = 0; r < n; ++r) {
        SlabEngine& se = *g_slab_engines[(size_t)r];
        IMPLI_HIP(hipSetDevice(se.device));
        se.engine->set_offsets((uint32_t)voff[(size_t)r], (uint32_t)foff[(size_t)r]);
        se.engine->emit(nullptr, se.stream);
    }
    verts.resize((size_t)voff[(size_t)n] * 3);
    faces.resize((size_t)foff[(size_t)n] * 3);
    for (int r = 0; r < n; ++r) {
        SlabEngine& se = *g_slab_engines[(size_t)r];
        IMPLI_HIP(hipSetDevice(se.device));
        bool of = false;
        const SlabCounts cr = se.engine->read_counts(se.stream, &of);
        if (of) throw HipError("build_geometry: slab output overflow after sizing");
        se.engine->download(verts.data() + 3 * voff[(size_t)r], faces.data() + 3 * foff[(size_t)r], cr, se.stream);
    }
}

void grand_algorithm(const char* shape_json, const MCSettings& st, const CallSpecs& cs) {   // mcc2.cpp:309-444
    if (g_state.active) {
        report("build_geometry() called in a bad state.", false);
        return;
    }
    Program prog = compile_mp5(shape_json, st.ignore_root_matrix);
    Engine& E = engine();
    hipStream_t s = abi_stream();
    E.set_object(prog);
    int64_t nv = 0, nf = 0;
    std::unique_ptr<Ob02>& ob_ptr = g_ob02;   // one refinement state, its buffers reused by every build
    // the MC faces' early copy to the host (below); a build that ended in an error left it to finish
    static hipEvent_t faces_copied = nullptr;
    bool faces_early = false;
    if (faces_copied) (void)hipEventSynchronize(faces_copied);
    if (!g_devices.empty()) {
        // polygonize_step_0 over several devices: balanced Z-slabs, concatenated on the host
        multi_device_mc(prog, st, g_state.verts, g_state.faces);
        nv = (int64_t)g_state.verts.size() / 3;
        nf = (int64_t)g_state.faces.size() / 3;
        const bool refine = st.overall_repeats > 0 && (st.vresampl_iters > 0 || st.projection || st.subdiv);
        if (!refine) {
            g_last_refined = false;
            send_mesh_back_to_client(nullptr, cs);   // mcc2.cpp:351
            // the repeats of an empty loop still report after their (empty) resampling (:372)
            for (int rep = 0; rep < st.overall_repeats; ++rep) send_mesh_back_to_client(nullptr, cs);
            g_state.active = true;
            return;
        }
        DevBuf& dv = E.scratch(8);
        DevBuf& df = E.scratch(9);
        dv.reserve((size_t)nv * 12 + 16);
        df.reserve((size_t)nf * 12 + 16);
        IMPLI_HIP(hipMemcpyAsync(dv.p, g_state.verts.data(), (size_t)nv * 12, hipMemcpyHostToDevice, s));
        IMPLI_HIP(hipMemcpyAsync(df.p, g_state.faces.data(), (size_t)nf * 12, hipMemcpyHostToDevice, s));
        if (!ob_ptr) ob_ptr.reset(new_ob02(E, s));
        ob_ptr->set_profile(g_ob02_profile);
        ob_ptr->load_mesh(dv.as<float>(), nv, df.as<int32_t>(), nf);
    } else {
        E.set_grid(st.resolution, st.box, 0, 1);
        const bool refine = st.overall_repeats > 0 && (st.vresampl_iters > 0 || st.projection || st.subdiv);
        if (!refine) {   // the MC mesh is the result: straight into the library's pinned result buffers
            roctxRangePush("marching cubes");
            E.marching_cubes_to_host(s, abi_copy_stream(), [](int64_t v, int64_t f, float** hv, int32_t** hf) {
                g_state.verts.resize((size_t)v * 3);
                g_state.faces.resize((size_t)f * 3);
                *hv = g_state.verts.data();
                *hf = g_state.faces.data();
            });
            roctxRangePop();
            g_last_refined = false;
            send_mesh_back_to_client(nullptr, cs);   // mcc2.cpp:351
            // the repeats of an empty loop still report after their (empty) resampling (:372)
            for (int rep = 0; rep < st.overall_repeats; ++rep) send_mesh_back_to_client(nullptr, cs);
            g_state.active = true;
            return;
        }
        roctxRangePush("marching cubes");
        SlabCounts c = E.marching_cubes(s);   // polygonize_step_0
        roctxRangePop();
        nv = c.n_verts();
        nf = c.n_faces();
        // without subdivision the loop never changes the faces: the MC faces go to the host on the
        // copy stream while the loop runs (8.6 MB at 512^3, ~0.17 ms of PCIe), only the vertices at
        // the end.  (A progress callback reads intermediate meshes through the same buffers: then
        // everything is fetched as before.)
        faces_early = !st.subdiv && !g_progress && nf > 0 && !g_ob02_profile;
        if (faces_early) {
            static hipEvent_t mc_done = nullptr;
            if (!mc_done) IMPLI_HIP(hipEventCreateWithFlags(&mc_done, hipEventDisableTiming));
            if (!faces_copied) IMPLI_HIP(hipEventCreateWithFlags(&faces_copied, hipEventDisableTiming));
            g_state.faces.resize((size_t)nf * 3);   // before the copy: the buffer does not move under it
            IMPLI_HIP(hipEventRecord(mc_done, s));
            IMPLI_HIP(hipStreamWaitEvent(abi_copy_stream(), mc_done, 0));
            IMPLI_HIP(hipMemcpyAsync(g_state.faces.data(), E.d_faces(), (size_t)nf * 12, hipMemcpyDeviceToHost,
                                     abi_copy_stream()));
            IMPLI_HIP(hipEventRecord(faces_copied, abi_copy_stream()));
        }
        if (!ob_ptr) ob_ptr.reset(new_ob02(E, s));
        ob_ptr->set_profile(g_ob02_profile);
        // the loop starts with a resampling: its centroid normals go beside the topology passes
        ob_ptr->load_mesh(E.d_verts(), nv, E.d_faces(), nf, nullptr, st.overall_repeats > 0 && st.vresampl_iters > 0);
    }
    Ob02& ob = *ob_ptr;
    g_last_refined = true;
    send_mesh_back_to_client(&ob, cs);   // after polygonize_step_0 (mcc2.cpp:351)
    for (int rep = 0; rep < st.overall_repeats; ++rep) {
        // a replacing point set keeps its last store: only the last repeat's need a snapshot
        ob.capture_replace = rep == st.overall_repeats - 1;
        for (int i = 0; i < st.vresampl_iters; ++i) ob.vertex_resampling(st.vresampl_c);   // step 1
        send_mesh_back_to_client(&ob, cs);                                             // mcc2.cpp:372
        if (st.projection) {
            ob.centroids_projection(st.qem);                                            // step 2
            send_mesh_back_to_client(&ob, cs);                                         // mcc2.cpp:390
        }
        if (st.subdiv && (st.overall_repeats <= 1 || rep == st.overall_repeats - 1)) {
            // polygonize_step_3 (polygonizer_algorithm_ob02.hpp:119-157): the noise is applied only
            // on the last repeat, scaled by the constant 10
            const bool is_last = rep == st.overall_repeats - 1;
            const float scale_noise = (float)(1.0 * 10.0);
            ob.subdivide(is_last ? st.post_subdiv_noise * scale_noise : 0.0f);
        }
    }
    nv = ob.n_verts();
    nf = ob.n_faces();
    g_state.verts.resize((size_t)nv * 3);
    if (faces_early && (int64_t)g_state.faces.size() == 3 * nf) {
        ob.fetch(g_state.verts.data(), nullptr);
        IMPLI_HIP(hipEventSynchronize(faces_copied));
    } else {
        if (faces_early) IMPLI_HIP(hipEventSynchronize(faces_copied));   // (never: the faces did not change)
        g_state.faces.resize((size_t)nf * 3);
        ob.fetch(g_state.verts.data(), g_state.faces.data());
    }
    ob.capture_replace = true;
    g_pointsets_dirty = true;              // copied to the host when asked for
    g_state.active = true;                 // polygonize_terminate, ob02:163-176
}

}  // namespace

extern "C" {

const char* implisolid_last_error(void) { return g_last_error.c_str(); }
void implisolid_set_error_mode(int mode) { g_error_mode = mode; }

void implisolid_srand(unsigned seed) { impli::process_rand().seed_(seed); }
int implisolid_rand(void) { return impli::process_rand().next(); }
void implisolid_rand_skip(uint64_t n) { impli::process_rand().skip(n); }

void implisolid_set_pruning(int level) { impli::Engine::set_pruning(level); }

int implisolid_parse_settings(const char* mc_json, float box[6], int32_t ints[7], float floats[2]) {
    g_last_error.clear();
    try {
        const MCSettings s = parse_mc_settings(mc_json);
        for (int k = 0; k < 6; ++k) box[k] = s.box[k];
        ints[0] = s.resolution;
        ints[1] = s.ignore_root_matrix;
        ints[2] = s.overall_repeats;
        ints[3] = s.vresampl_iters;
        ints[4] = s.projection;
        ints[5] = s.qem;
        ints[6] = s.subdiv;
        floats[0] = s.vresampl_c;
        floats[1] = s.post_subdiv_noise;
    } catch (const std::exception& e) {
        report(e.what(), true);   // polygoniser_settings.hpp:297-301 aborts
        return -1;
    }
    return 0;
}

int implisolid_slab_partition(int R, int rank, int nranks, int32_t out[3]) {
    g_last_error.clear();
    try {
        const SlabRange r = slab_partition(R, rank, nranks);
        out[0] = r.z0;
        out[1] = r.z1;
        out[2] = r.halo;
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}

void implisolid_set_progress_callback(implisolid_progress_callback cb, void* user) {
    g_progress = cb;
    g_progress_user = user;
}

static void build_geometry_specs(const char* shape_json, const char* mc_json, const CallSpecs& cs) {
    g_last_error.clear();
    MCSettings st;
    try {
        st = parse_mc_settings(mc_json);
    } catch (const InputError& e) {
        report(e.what(), true);
        return;
    }
    try {
        roctxRangePush("build_geometry");
        struct Pop { ~Pop() { roctxRangePop(); } } pop;
        grand_algorithm(shape_json, st, cs);
    } catch (const InputError& e) {
        report(e.what(), true);
    } catch (const std::exception& e) {
        report(std::string("build_geometry failed: ") + e.what(), false);
    }
}

void build_geometry(const char* shape_json, const char* mc_json) {   // worker_call_sepcs_t() defaults
    build_geometry_specs(shape_json, mc_json, CallSpecs{});
}

void build_geometry_u(const char* shape_json, const char* mc_json, const char* call_specs) {
    CallSpecs cs;
    try {   // worker_call_sepcs_t(json), worker_call_specs.hpp:28-40: get<int>(key, -1)
        const Json j = Json::parse(call_specs ? call_specs : "{}");
        cs.progress_callback_id = j.get_int("progressCallback_id", -1);
        cs.call_id = j.get_int("call_id", -1);
        cs.shape_id = j.get_int("shape_id", -1);
    } catch (const JsonError& e) {
        report(std::string("call_specs: ") + e.what(), true);
        return;
    }
    build_geometry_specs(shape_json, mc_json, cs);
}

void implisolid_ob02_profile(int on) { g_ob02_profile = on != 0; }

int implisolid_last_build_stats(double out[13]) {
    g_last_error.clear();
    for (int k = 0; k < 13; ++k) out[k] = 0.0;
    if (!g_ob02 || !g_last_refined) return 0;
    try {
        g_ob02->read_counters();
        out[0] = g_ob02->bisection_cap_hits();
        out[1] = (double)g_ob02->projection_evals();
        out[2] = g_ob02->last_average_edge();
        for (int k = 0; k < Ob02::kStages; ++k) out[3 + k] = g_ob02->stage_ms()[k];
        out[3 + Ob02::kStages] = (double)g_ob02->n_faces();
        out[4 + Ob02::kStages] = (double)g_ob02->n_verts();
        out[5 + Ob02::kStages] = (double)g_ob02->jit_launches();
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}

int get_v_size(void) { return (int)(g_state.verts.size() / 3); }
int get_f_size(void) { return (int)(g_state.faces.size() / 3); }

void get_v(float* v_out, int vcount) {
    const size_t n = g_state.verts.size();
    std::memcpy(v_out, g_state.verts.data(), n * sizeof(float));
    if ((size_t)vcount * 3 != n) std::fprintf(stderr, "sizes dont match: %g %d\n", (double)n / 3., vcount);
}

void get_f(int* f_out, int fcount) {
    const size_t n = g_state.faces.size();
    std::memcpy(f_out, g_state.faces.data(), n * sizeof(int));
    if ((size_t)fcount * 3 != n) std::fprintf(stderr, "sizes dont match: %g %d\n", (double)n / 3., fcount);
}

void* get_v_ptr(void) { return g_state.verts.data(); }
void* get_f_ptr(void) { return g_state.faces.data(); }

void finish_geometry(void) { g_state.active = false; }

// ---- direct evaluation ------------------------------------------------------------------------
int set_object(const char* shape_json, bool ignore_root_matrix) {
    if (g_eval.has_object) {
        report("Error: You cannot unset() the object before a set_object(json).", false);
        return 0;
    }
    try {
        Program p = compile_mp5(shape_json, ignore_root_matrix);
        engine().set_object(p);
    } catch (const InputError& e) {
        report(e.what(), true);
        return 0;
    } catch (const std::exception& e) {
        report(e.what(), false);
        return 0;
    }
    g_eval.has_object = true;
    return 1;
}

bool unset_object(int id) {
    if (!g_eval.has_object) {
        report("Error: You cannot unset() the object before a set_object(json).", false);
        return false;
    }
    if (id <= 0) {
        report("Incorrect ID: use the same id returned by set_object(json).", false);
        return false;
    }
    if (id != 1) {
        report("Incorrect ID. For now, The only id is 1", false);
        return false;
    }
    g_eval.has_object = false;
    return true;
}

bool set_x(void* verts, int n) {
    if (g_eval.has_x) {
        report("Error: You set() before unset()ing the previous set().", false);
        return false;
    }
    if (n < 0 || n >= 10000 * 5) {
        report("Error: n is outside [0, 50000].", false);
        return false;
    }
    const float* p = static_cast<const float*>(verts);
    g_eval.x.assign(p, p + 3 * (size_t)n);
    g_eval.f.assign((size_t)n, 0.f);
    g_eval.grad.assign(3 * (size_t)n, 0.f);
    g_eval.has_x = true;
    return true;
}

void unset_x(void) {
    if (!g_eval.has_x) {
        report("Error: You cannot unset() before a set().", false);
        return;
    }
    g_eval.has_x = false;
    g_eval.x.clear();
    g_eval.f.clear();
    g_eval.grad.clear();
}

int implisolid_eval_points(const float* xyz, int64_t n, float* f_out, float* grad_out) {
    if (!g_eval.has_object) {
        report("Error: You need to set_x() and set_object() first.", false);
        return -1;
    }
    if (n <= 0) return 0;
    try {
        Engine& E = engine();
        hipStream_t s = abi_stream();
        DevBuf& dx = E.scratch(0);
        DevBuf& df = E.scratch(1);
        DevBuf& dg = E.scratch(2);
        dx.reserve((size_t)n * 12);
        df.reserve((size_t)n * 4);
        if (grad_out) dg.reserve((size_t)n * 12);
        IMPLI_HIP(hipMemcpyAsync(dx.p, xyz, (size_t)n * 12, hipMemcpyHostToDevice, s));
        E.eval_points(dx.as<float>(), n, df.as<float>(), grad_out ? dg.as<float>() : nullptr, s);
        if (f_out) IMPLI_HIP(hipMemcpyAsync(f_out, df.p, (size_t)n * 4, hipMemcpyDeviceToHost, s));
        if (grad_out) IMPLI_HIP(hipMemcpyAsync(grad_out, dg.p, (size_t)n * 12, hipMemcpyDeviceToHost, s));
        IMPLI_HIP(hipStreamSynchronize(s));
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}

int implisolid_debug_fold(const float* terms, int64_t n, float* sum_out, int64_t* table_chunks) {
    if (n < 0 || (n && !terms) || !sum_out) {
        report("implisolid_debug_fold: bad arguments", false);
        return -1;
    }
    try {
        (void)engine();   // the device context
        int tc = 0;
        static long long st[14];
        static int tr[256];
        *sum_out = debug_fold(terms, n, &tc, st, tr);
        if (std::getenv("IMPLISOLID_FOLD_TRACE")) {
            for (int i = 0; i < 256 && i < st[0] + st[1] + st[2]; ++i)
                std::fprintf(stderr, "%s k=%d E=%d\n", (tr[i] >> 28) == 1 ? "table" : (tr[i] >> 28) == 3 ? "jump " : (tr[i] >> 28) == 4 ? "fast+" : (tr[i] >> 28) == 5 ? "fast-" : (tr[i] >> 28) == 6 ? "fastX" : "term ",
                             tr[i] & 0xfffff, ((tr[i] >> 20) & 0xff) - 64);
        }
        if (std::getenv("IMPLISOLID_FOLD_STATS"))
            std::fprintf(stderr, "fold n=%lld steps: zero/single %lld run-lookups %lld scans %lld term-chunks %lld (serial %lld, "
                         "global term loads %lld); cycles: stage %lld walk %lld (lookups %lld scans %lld serial %lld "
                         "segments %lld; waiting for staged terms %lld)\n",
                         (long long)n, st[0], st[1], st[2], st[3], st[10], st[11], st[4], st[5], st[6], st[7], st[8], st[9], st[12]);
        if (table_chunks) *table_chunks = tc;
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}

int implisolid_debug_libm(int which, const float* a, const float* b, int64_t n, float* out) {
    if (which < 0 || which > 2 || n < 0 || (n && (!a || !out || (which == 2 && !b)))) {
        report("implisolid_debug_libm: bad arguments", false);
        return -1;
    }
    if (n == 0) return 0;
    try {
        Engine& E = engine();
        hipStream_t s = abi_stream();
        DevBuf& da = E.scratch(0);
        DevBuf& db = E.scratch(1);
        DevBuf& dout = E.scratch(2);
        da.reserve((size_t)n * 4);
        if (which == 2) db.reserve((size_t)n * 4);
        dout.reserve((size_t)n * 4);
        IMPLI_HIP(hipMemcpyAsync(da.p, a, (size_t)n * 4, hipMemcpyHostToDevice, s));
        if (which == 2) IMPLI_HIP(hipMemcpyAsync(db.p, b, (size_t)n * 4, hipMemcpyHostToDevice, s));
        launch_libm_probe(which, da.as<float>(), which == 2 ? db.as<float>() : nullptr, n, dout.as<float>(), s);
        IMPLI_HIP(hipGetLastError());
        IMPLI_HIP(hipMemcpyAsync(out, dout.p, (size_t)n * 4, hipMemcpyDeviceToHost, s));
        IMPLI_HIP(hipStreamSynchronize(s));
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}

int implisolid_debug_cos(const double* a, int64_t n, double* out) {
    if (n < 0 || (n && (!a || !out))) {
        report("implisolid_debug_cos: bad arguments", false);
        return -1;
    }
    if (n == 0) return 0;
    try {
        Engine& E = engine();
        hipStream_t s = abi_stream();
        DevBuf& da = E.scratch(0);
        DevBuf& dout = E.scratch(2);
        da.reserve((size_t)n * 8);
        dout.reserve((size_t)n * 8);
        IMPLI_HIP(hipMemcpyAsync(da.p, a, (size_t)n * 8, hipMemcpyHostToDevice, s));
        launch_cos_probe(da.as<double>(), n, dout.as<double>(), s);
        IMPLI_HIP(hipGetLastError());
        IMPLI_HIP(hipMemcpyAsync(out, dout.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
        IMPLI_HIP(hipStreamSynchronize(s));
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}

void calculate_implicit_values(void) {
    if (!g_eval.has_x || !g_eval.has_object) {
        report("Error: You need to set_x() and set_object() first.", false);
        return;
    }
    implisolid_eval_points(g_eval.x.data(), (int64_t)g_eval.f.size(), g_eval.f.data(), nullptr);
}

void* get_values_ptr(void) { return g_eval.has_x ? g_eval.f.data() : nullptr; }
int get_values_size(void) { return (int)g_eval.f.size(); }

void calculate_implicit_gradients(bool normalize_and_invert) {
    if (!g_eval.has_x || !g_eval.has_object) {
        report("Error: You need to set_x() and set_object() first.", false);
        return;
    }
    const int64_t n = (int64_t)g_eval.f.size();
    std::vector<float> fv((size_t)n);
    implisolid_eval_points(g_eval.x.data(), n, fv.data(), g_eval.grad.data());
    if (normalize_and_invert) {   // mcc2.cpp:852-871
        int problems = 0;
        for (int64_t i = 0; i < n; ++i) {
            float* g = &g_eval.grad[3 * i];
            const float x = g[0], y = g[1], z = g[2];
            const float norm = std::sqrt(x * x + y * y + z * z);
            float factor;
            if (norm > 0.0001) factor = (float)(-1.0 / (double)norm);
            else { factor = -42.0f; problems++; }
            g[0] = x * factor; g[1] = y * factor; g[2] = z * factor;
        }
        if (problems > 0) std::fprintf(stderr, " problems %d\n", problems);
    }
}

void* get_gradients_ptr(void) {
    if (!g_eval.has_x || !g_eval.has_object) {
        report("Error: You need to set_x() and set_object() first.", false);
        return nullptr;
    }
    return g_eval.grad.data();
}

int get_gradients_size(void) {
    if (!g_eval.has_x || !g_eval.has_object) {
        report("Error: You need to set_x() and set_object() first.", false);
        return 0;
    }
    return (int)g_eval.grad.size();
}

void* get_pointset_ptr(char* id) {
    materialize_pointsets();
    auto it = g_pointsets.find(std::string(id));
    return it == g_pointsets.end() ? nullptr : it->second.data();
}
int get_pointset_size(char* id) {
    materialize_pointsets();
    auto it = g_pointsets.find(std::string(id));
    return it == g_pointsets.end() ? 0 : (int)(it->second.size() / 3);
}

void about(void) {
    // mcc2.cpp:574-576 prints __DATE__ __TIME__ on its second line.  The library is built
    // reproducibly (the round's profiles name its hash): the Makefile passes SOURCE_DATE_EPOCH (the
    // reproducible-builds convention) when it is set, formatted as __DATE__ __TIME__ are (UTC)
#ifdef IMPLI_SOURCE_DATE_EPOCH
    {
        const time_t t = (time_t)IMPLI_SOURCE_DATE_EPOCH;
        struct tm u;
        gmtime_r(&t, &u);
        char buf[64];
        std::strftime(buf, sizeof buf, "%b %e %Y %H:%M:%S", &u);
        std::fprintf(stderr, "Build Info: \n%s\n", buf);
    }
#else
    std::fprintf(stderr, "Build Info: \nreproducible build\n");
#endif
    std::fprintf(stderr, "implisolid-mi355x: HIP gfx950 polygoniser (eval + marching cubes + OB02)\n");
    std::fprintf(stderr, "CONFIG: ROOT_TOLERANCE=%g \n", (double)(float)(0.001 / 10.0));
}

static int64_t jit_compile_kind(const char* shape_json, int kind, char* source_out, int64_t capacity, double* seconds) {
    g_last_error.clear();
    try {
        const Program p = compile_mp5(shape_json, false);
        // (bake mode 1, "always": the value-baked source of this object)
        const std::string src = kind == TreeJit::kPoints ? TreeJit::point_source(p)
                                                         : TreeJit::kernel_source(p, TreeJit::instance().bake() == TreeJit::kBakeAlways);
        if (source_out && capacity > 0) {
            const size_t n = std::min<size_t>(src.size(), (size_t)capacity - 1);
            std::memcpy(source_out, src.data(), n);
            source_out[n] = 0;
        }
        const auto t0 = std::chrono::steady_clock::now();
        const std::vector<char> code = TreeJit::compile(src);
        if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return (int64_t)code.size();
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
}

int64_t implisolid_jit_compile(const char* shape_json, char* source_out, int64_t capacity, double* seconds) {
    return jit_compile_kind(shape_json, TreeJit::kBricks, source_out, capacity, seconds);
}

int64_t implisolid_jit_compile_points(const char* shape_json, char* source_out, int64_t capacity, double* seconds) {
    return jit_compile_kind(shape_json, TreeJit::kPoints, source_out, capacity, seconds);
}

int implisolid_program_info(const char* shape_json, int ignore_root_matrix, int32_t info[4], float* mats_out) {
    g_last_error.clear();
    try {
        const Program p = compile_mp5(shape_json, ignore_root_matrix != 0);
        info[0] = p.n_instr;
        info[1] = p.max_depth;
        info[2] = p.n_mats;
        info[3] = 0;
        if (mats_out) std::memcpy(mats_out, p.mats, sizeof(float) * 12 * (size_t)p.n_mats);
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}

// ---- device slab pipeline ----------------------------------------------------------------------
struct implisolid_slab {
    Engine engine;
};

implisolid_slab* implisolid_slab_create_range(const char* shape_json, const char* mc_json, int z0, int z1) {
    g_last_error.clear();
    try {
        MCSettings st = parse_mc_settings(mc_json);
        Program p = compile_mp5(shape_json, st.ignore_root_matrix);
        auto* s = new implisolid_slab();
        s->engine.set_object(p);
        s->engine.set_slab(st.resolution, st.box, SlabRange{z0, z1, 0});
        return s;
    } catch (const std::exception& e) {
        report(e.what(), false);
        return nullptr;
    }
}

int implisolid_slab_balance(const char* shape_json, const char* mc_json, int nranks, int32_t* cuts) {
    g_last_error.clear();
    try {
        const MCSettings st = parse_mc_settings(mc_json);
        const Program p = compile_mp5(shape_json, st.ignore_root_matrix);
        const std::vector<int> c = balance_cuts(p, st.resolution, st.box, nranks, nullptr);
        for (size_t k = 0; k < c.size(); ++k) cuts[k] = c[k];
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}

int implisolid_cuts_from_layer_work(const int64_t* listed, int n_layers, int64_t bricks_per_layer, int R, int nranks,
                                    int32_t* cuts) {
    g_last_error.clear();
    try {
        const std::vector<int> c =
            cuts_from_layer_work(std::vector<int64_t>(listed, listed + n_layers), bricks_per_layer, R, nranks);
        for (size_t k = 0; k < c.size(); ++k) cuts[k] = c[k];
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}

int implisolid_set_devices(const int32_t* ids, int n) {
    g_last_error.clear();
    try {
        std::vector<int> d;
        int count = 0;
        if (ids && n > 0) IMPLI_HIP(hipGetDeviceCount(&count));
        for (int k = 0; ids && k < n; ++k) {
            if (ids[k] < 0 || ids[k] >= count) throw InputError("implisolid_set_devices: no HIP device " + std::to_string(ids[k]));
            d.push_back(ids[k]);
        }
        g_devices = d.size() > 1 ? d : std::vector<int>{};
        g_slab_engines.clear();
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}

implisolid_slab* implisolid_slab_create(const char* shape_json, const char* mc_json, int rank, int nranks) {
    g_last_error.clear();
    try {
        MCSettings st = parse_mc_settings(mc_json);
        Program p = compile_mp5(shape_json, st.ignore_root_matrix);
        auto* s = new implisolid_slab();
        s->engine.set_object(p);
        s->engine.set_grid(st.resolution, st.box, rank, nranks);
        return s;
    } catch (const std::exception& e) {
        report(e.what(), false);
        return nullptr;
    }
}
void implisolid_slab_destroy(implisolid_slab* s) { delete s; }

#define SLAB_TRY(expr)                                 \
    try {                                              \
        expr;                                          \
    } catch (const std::exception& e) {                \
        report(e.what(), false);                       \
        return -1;                                     \
    }                                                  \
    return 0;

int implisolid_slab_eval(implisolid_slab* s, void* stream) { SLAB_TRY(s->engine.eval_field((hipStream_t)stream)) }
int implisolid_slab_count(implisolid_slab* s, void* stream) { SLAB_TRY(s->engine.count((hipStream_t)stream)) }
int implisolid_slab_emit(implisolid_slab* s, const uint32_t* d_offsets, void* stream) {
    SLAB_TRY(s->engine.emit(d_offsets, (hipStream_t)stream))
}
int implisolid_slab_emit_verts(implisolid_slab* s, void* stream) {
    SLAB_TRY(s->engine.emit_verts((hipStream_t)stream))
}
int implisolid_slab_emit_faces(implisolid_slab* s, const uint32_t* d_offsets, const uint32_t* d_gathered, int rank,
                               void* stream) {
    SLAB_TRY(s->engine.emit_faces(d_offsets, d_gathered, rank, (hipStream_t)stream))
}
const uint32_t* implisolid_slab_counters(implisolid_slab* s) { return s->engine.d_counters(); }
int implisolid_slab_counts(implisolid_slab* s, void* stream, uint32_t out[3]) {
    try {
        bool of = false;
        SlabCounts c = s->engine.read_counts((hipStream_t)stream, &of);
        const bool grew = s->engine.ensure_capacity(c);
        out[0] = c.n_verts();
        out[1] = c.n_faces();
        out[2] = (of || grew) ? 1u : 0u;
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}
int implisolid_slab_grid(implisolid_slab* s, int32_t out[8]) {
    const GridDesc& g = s->engine.grid();
    const int32_t v[8] = {g.R, g.res, g.cz0, g.cz1, g.cz_emit, g.fz0, g.fz1, s->engine.depth()};
    std::memcpy(out, v, sizeof v);
    return 0;
}
int implisolid_slab_copy_counts(implisolid_slab* s, uint32_t* d_dst, void* stream) {
    SLAB_TRY(IMPLI_HIP(hipMemcpyAsync(d_dst, s->engine.d_counters() + 2, 4 * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                                      (hipStream_t)stream)))
}
int implisolid_slab_copy_mesh(implisolid_slab* s, float* d_verts, int32_t* d_faces, int64_t nv, int64_t nf, void* stream) {
    SLAB_TRY(
        if (nv > 0) IMPLI_HIP(hipMemcpyAsync(d_verts, s->engine.d_verts(), (size_t)nv * 12, hipMemcpyDeviceToDevice, (hipStream_t)stream));
        if (nf > 0) IMPLI_HIP(hipMemcpyAsync(d_faces, s->engine.d_faces(), (size_t)nf * 12, hipMemcpyDeviceToDevice, (hipStream_t)stream)))
}
int implisolid_slab_set_offsets(implisolid_slab* s, uint32_t voff, uint32_t foff) {
    SLAB_TRY(s->engine.set_offsets(voff, foff))
}
int implisolid_slab_download(implisolid_slab* s, float* verts, int32_t* faces, void* stream) {
    try {
        bool of = false;
        const SlabCounts c = s->engine.read_counts((hipStream_t)stream, &of);
        if (of) throw HipError("slab output overflowed; call implisolid_slab_counts and emit again");
        s->engine.download(verts, faces, c, (hipStream_t)stream);
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}
float* implisolid_slab_verts(implisolid_slab* s) { return s->engine.d_verts(); }
int32_t* implisolid_slab_faces(implisolid_slab* s) { return s->engine.d_faces(); }
float* implisolid_slab_field(implisolid_slab* s) { return s->engine.d_field(); }

int implisolid_slab_stats_n(implisolid_slab* s, int64_t* out, int n) {
    constexpr int kStats = 10;
    try {
        if (!out || n < 0) throw InputError("slab_stats: null output or negative length");
        uint32_t c[16];
        s->engine.raw_counters(c, 0);
        const GridDesc& g = s->engine.grid();
        const int64_t v[kStats] = {
            n_units(g),
            c[6],        // non-empty units (c[0] counts their parts)
            c[2], c[3], c[4], c[5],
            g.n_cells,
            c[14],       // mixed coarse boxes of the last eval (the fill kernel's copy of [13])
            c[1],        // the vertex pass's copy of the halo count (mc_types.hpp counters)
            c[0]};       // unit parts
        for (int k = 0; k < n && k < kStats; ++k) out[k] = v[k];
        return kStats;
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
}

int implisolid_slab_stats(implisolid_slab* s, int64_t out[8]) {   // the original 8 figures
    return implisolid_slab_stats_n(s, out, 8) < 0 ? -1 : 0;
}

int implisolid_slab_used_jit(implisolid_slab* s) { return s->engine.used_baked() ? 2 : s->engine.used_jit() ? 1 : 0; }
void implisolid_set_jit(int mode) { TreeJit::instance().set_mode(mode); }
void implisolid_set_jit_bake(int mode) { TreeJit::instance().set_bake(mode); }
void implisolid_jit_wait(void) { TreeJit::instance().wait_idle(); }
void implisolid_jit_stats(int32_t out[4], double* compile_seconds) {
    TreeJit& j = TreeJit::instance();
    out[0] = j.mode();
    out[1] = j.bake();
    out[2] = j.compiled();
    out[3] = j.disk_hits();
    if (compile_seconds) *compile_seconds = j.compile_seconds();
}
void implisolid_set_jit_max_modules(int n) { TreeJit::instance().set_max_modules(n); }
void implisolid_jit_modules(int32_t out[3]) {
    TreeJit& j = TreeJit::instance();
    out[0] = j.modules();
    out[1] = j.max_modules();
    out[2] = j.evicted();
}

int implisolid_slab_set_timing(implisolid_slab* s, int on) { SLAB_TRY(s->engine.set_timing(on != 0)) }
int implisolid_slab_kernel_times(implisolid_slab* s, float ms[6]) { SLAB_TRY(s->engine.kernel_times(ms)) }
int implisolid_slab_kernel_times_each(implisolid_slab* s, float ms[8]) { SLAB_TRY(s->engine.kernel_times_each(ms)) }

int64_t implisolid_slab_read_signs(implisolid_slab* s, uint8_t* out, int64_t capacity) {
    try {
        const GridDesc& g = s->engine.grid();
        const int64_t rows = (int64_t)g.n * (g.fz1 - g.fz0), rw = sign_row_words(g);
        const int64_t n = rows * g.n;
        if (out) {
            if (capacity < n) throw InputError("implisolid_slab_read_signs: buffer too small");
            std::vector<uint64_t> w((size_t)(rows * rw));
            IMPLI_HIP(hipDeviceSynchronize());
            IMPLI_HIP(hipMemcpy(w.data(), s->engine.d_signs(), w.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
            for (int64_t r = 0; r < rows; ++r)
                for (int x = 0; x < g.n; ++x) out[r * g.n + x] = (uint8_t)((w[(size_t)(r * rw + x / 64)] >> (x % 64)) & 1u);
        }
        return n;
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
}

int implisolid_slab_brick_stats(implisolid_slab* s, int64_t out[3]) {
    try {
        s->engine.brick_stats(out, 0);
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}

int64_t implisolid_slab_read_field(implisolid_slab* s, float* out, int64_t capacity) {
    try {
        const GridDesc& g = s->engine.grid();
        const int64_t n = (int64_t)g.n * g.n * (int64_t)(g.fz1 - g.fz0);
        if (out) {
            if (capacity < n) throw InputError("implisolid_slab_read_field: buffer too small");
            IMPLI_HIP(hipDeviceSynchronize());
            // the field is stored brick-major (grid.hpp field_index): copy it whole, then lay the
            // stored samples out x fastest, then y, then layer
            std::vector<float> raw((size_t)field_samples(g));
            if (!raw.empty())
                IMPLI_HIP(hipMemcpy(raw.data(), s->engine.d_field(), raw.size() * sizeof(float), hipMemcpyDeviceToHost));
            const int layers = g.fz1 - g.fz0;
            for (int l = 0; l < layers; ++l)
                for (int y = 0; y < g.n; ++y)
                    for (int x = 0; x < g.n; ++x)
                        out[((int64_t)l * g.n + y) * g.n + x] = raw[(size_t)field_index(g, x, y, l)];
        }
        return n;
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
}

// ---- object stream (config 5): one engine per object, each object's eval + count + emit captured
//      once in a hipGraph and replayed; objects spread over a few streams ----------------------------
// merged object streams: pipelines the shallow class is split into (IMPLISOLID_BATCH_GROUPS, 1-8)
static int batch_groups() {
    static const int k = [] {
        const char* e = std::getenv("IMPLISOLID_BATCH_GROUPS");
        const int v = e ? std::atoi(e) : kBatchGroups;
        return v < 1 ? 1 : v > 8 ? 8 : v;
    }();
    return k;
}

struct implisolid_batch {
    DevBuf progs;                        // merged: every object's Program, one upload (the engines read them)
    DevBuf counts;                       // merged: every row's counter block, gathered for one read-back
    DevBuf resets;                       // merged: the fresh engines' buffer resets (ZeroPiece list)
    std::vector<std::unique_ptr<Engine>> engines;
    bool merged = false;                 // one launch per stage for all objects (ObjArgs rows)
    DevBuf objs;                         // merged: ObjArgs[n] on the device, shallow objects first
    int depth = 0;
    // merged: objects of tree depth <= kBatchShallowDepth (rows [0, n_shallow)) run the interval and
    // eval passes with 9-slot node stacks (four waves per SIMD), the rest with 12 or 16
    int n_shallow = 0, depth_shallow = 0, depth_deep = 0, vdepth_shallow = 0, vdepth_deep = 0;
    // merged: the groups run as independent pipelines (eval passes + marching cubes), group 0 on the
    // caller's stream, group k on streams[k - 1]: {first row, rows, stack depth}
    struct Group { int row0, n, depth, vdepth; };
    std::vector<Group> groups;
    std::vector<hipGraphExec_t> execs;   // empty when capture is unavailable (direct launches)
    std::vector<hipStream_t> streams;
    std::vector<hipEvent_t> events;      // fork (0) and one join event per stream
    double jit_seconds = 0;
};

static void batch_merged_enqueue(implisolid_batch* b, hipStream_t s);

// object streams' HIP streams and events, cached per device for the process's later batches
static std::mutex g_batch_cache_mu;
static std::map<int, std::vector<hipStream_t>> g_batch_streams;
static std::map<int, std::vector<hipEvent_t>> g_batch_events;
static int current_device() {
    int d = 0;
    IMPLI_HIP(hipGetDevice(&d));
    return d;
}
static hipStream_t batch_take_stream() {
    const int d = current_device();
    {
        std::lock_guard<std::mutex> lk(g_batch_cache_mu);
        auto& v = g_batch_streams[d];
        if (!v.empty()) {
            hipStream_t q = v.back();
            v.pop_back();
            return q;
        }
    }
    hipStream_t q;
    IMPLI_HIP(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
    return q;
}
static hipEvent_t batch_take_event() {
    const int d = current_device();
    {
        std::lock_guard<std::mutex> lk(g_batch_cache_mu);
        auto& v = g_batch_events[d];
        if (!v.empty()) {
            hipEvent_t e = v.back();
            v.pop_back();
            return e;
        }
    }
    hipEvent_t e;
    IMPLI_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
}

implisolid_batch* implisolid_batch_create(const char* const* shapes, int n, const char* mc_json, int n_streams) {
    g_last_error.clear();
    auto* b = new implisolid_batch();
    try {
        if (n <= 0) throw InputError("implisolid_batch_create: no objects");
        const MCSettings st = parse_mc_settings(mc_json);
        static const bool timing = std::getenv("IMPLISOLID_BATCH_TIMING") != nullptr;   // diagnostics
        auto t_start = std::chrono::steady_clock::now();
        size_t pool0[4] = {0, 0, 0, 0};
        if (timing) DevBuf::pool_stats(pool0);
        // the MP5 programs, parsed and compiled on host threads (a few tens of us each)
        std::vector<Program> progs((size_t)n);
        {
            const int nt = std::max(1, std::min({n / 8, 8, (int)std::thread::hardware_concurrency()}));
            std::vector<std::string> errs((size_t)nt);
            std::vector<std::thread> ths;
            for (int t = 0; t < nt; ++t)
                ths.emplace_back([&, t] {
                    try {
                        for (int i = t; i < n; i += nt) progs[(size_t)i] = compile_mp5(shapes[i], st.ignore_root_matrix);
                    } catch (const std::exception& e) {
                        errs[(size_t)t] = e.what();
                    }
                });
            for (auto& th : ths) th.join();
            for (auto& e : errs)
                if (!e.empty()) throw InputError(e);
        }
        // n_streams <= 0: merged launches (the interpreter kernels, every stage once for all
        // objects); otherwise one hipGraph per object (JIT tree kernels when enabled) over streams
        b->merged = n_streams <= 0 && Engine::pruning() > 0;
        if (b->merged) {
            // the merged kernels keep the objects' list prefix in LDS (kMaxBatchObjects entries) and
            // index every object's refine items with one 32-bit flat index
            if (n > kMaxBatchObjects)
                throw InputError("implisolid_batch_create: merged launches hold at most " + std::to_string(kMaxBatchObjects) +
                                 " objects; use n_streams >= 1 (per-object graphs) for larger batches");
            const float* bx = st.box;
            const GridDesc g = make_grid(st.resolution, bx, 1, st.resolution + 3, 1);
            const uint64_t items = (uint64_t)n * (uint64_t)coarse_grid(g).n_bricks * kCZ * kRefineSplit;
            if (items >= (1ull << 32))
                throw InputError("implisolid_batch_create: " + std::to_string(n) + " objects at this resolution exceed the "
                                 "merged refine pass's 32-bit item index; use fewer objects or n_streams >= 1");
        }
        const auto t0 = std::chrono::steady_clock::now();
        struct Held {   // precompile()'s references, dropped once the engines hold their own
            std::vector<TreeJit::Slot*> s;
            ~Held() { for (auto* x : s) TreeJit::instance().release(x); }
        } held;
        if (Engine::pruning() > 0 && !b->merged) held.s = TreeJit::instance().precompile(progs, 16);
        b->jit_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        // merged: the shallow class in batch_groups() pipelines, the deep class (if any) in one more
        const int ns = b->merged ? batch_groups() : std::max(1, std::min(n_streams, 8));
        // (the deep class's stream at the lowest priority measured 0.5 % faster alone, but with the
        // bench's earlier legs' streams alive the two pipelines then shared a hardware queue: 0.85 ms
        // per pass, profiles/r05zr_*; default priority).  Streams and events come from a process-wide
        // cache (batch_take_stream): an object stream creates batch after batch.
        for (int k = 0; k < ns; ++k) b->streams.push_back(batch_take_stream());
        for (int k = 0; k <= ns; ++k) b->events.push_back(batch_take_event());
        hipStream_t s0 = b->streams[0];
        // IMPLISOLID_BATCH_TIMING=1 (diagnostics): the setup's phases summed over the objects, on stderr
        double ph[4] = {0, 0, 0, 0};
        const double t_compile = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
        auto tick = [](std::chrono::steady_clock::time_point& t) {
            const auto now = std::chrono::steady_clock::now();
            const double d = std::chrono::duration<double>(now - t).count();
            t = now;
            return d;
        };
        auto tp = std::chrono::steady_clock::now();
        std::vector<ZeroPiece> pieces;   // merged: uploaded below, read until the first pass's sync
        if (b->merged) {
            // merged launches: the programs in one upload, every engine's buffers set up on s0 without
            // device synchronisations (fresh engines; the pool serves them without hipMalloc from the
            // second batch of a process on), no warm run per object -- the merged fill writes the unit
            // marks from the first pass -- and one merged pass below sizes the outputs of all
            b->progs.reserve((size_t)n * sizeof(Program));
            IMPLI_HIP(hipMemcpyAsync(b->progs.p, progs.data(), (size_t)n * sizeof(Program), hipMemcpyHostToDevice, s0));
            const SlabRange whole = slab_partition(st.resolution, 0, 1);
            std::vector<ZeroRange> resets;   // every engine's buffer resets, cleared by one launch below
            for (int i = 0; i < n; ++i) {
                b->engines.emplace_back(new Engine(s0, &resets));
                Engine& E = *b->engines.back();
                if (timing) ph[0] += tick(tp);
                E.set_hot_bake(false);
                E.set_object(progs[(size_t)i], b->progs.as<Program>() + i);
                if (timing) ph[1] += tick(tp);
                E.set_slab(st.resolution, st.box, whole, false, s0);
                E.arm_merged();
                E.detach_resets();
                if (timing) ph[2] += tick(tp);
            }
            for (const ZeroRange& r : resets) {
                if ((uintptr_t)r.p % 16 != 0) {   // (pool blocks are hipMalloc'd: never taken)
                    IMPLI_HIP(hipMemsetAsync(r.p, 0, r.n, s0));
                    continue;
                }
                for (size_t o = 0; o < r.n; o += kZeroPieceBytes)
                    pieces.push_back({(uint64_t)(uintptr_t)r.p + o, (uint32_t)std::min<size_t>(kZeroPieceBytes, r.n - o), 0});
            }
            b->resets.reserve(std::max<size_t>(pieces.size(), 1) * sizeof(ZeroPiece));
            IMPLI_HIP(hipMemcpyAsync(b->resets.p, pieces.data(), pieces.size() * sizeof(ZeroPiece), hipMemcpyHostToDevice, s0));
            launch_zero_pieces(b->resets.as<ZeroPiece>(), (int)pieces.size(), s0);
            if (timing) ph[2] += tick(tp);
        } else {
            for (int i = 0; i < n; ++i) {   // warm run: JIT lookup, output capacities from the real counts
                b->engines.emplace_back(new Engine());
                Engine& E = *b->engines.back();
                if (timing) ph[0] += tick(tp);
                E.set_hot_bake(false);   // graphs capture the modules found now
                E.set_object(progs[(size_t)i]);
                if (timing) ph[1] += tick(tp);
                E.set_grid(st.resolution, st.box, 0, 1);
                if (timing) ph[2] += tick(tp);
                E.marching_cubes(s0);
                if (timing) ph[3] += tick(tp);
            }
        }
        if (timing)
            std::fprintf(stderr, "implisolid_batch_create: %d objects: engines %.2f ms, set_object %.2f ms, set_grid %.2f ms, "
                                 "warm runs %.2f ms\n", n, ph[0] * 1e3, ph[1] * 1e3, ph[2] * 1e3, ph[3] * 1e3);
        if (b->merged) {   // the objects' device state, one row each; every object has the same grid
            std::vector<ObjArgs> rows;
            std::vector<Engine*> order;   // the engine of each row
            for (int pass = 0; pass < 2; ++pass)   // shallow objects first (launch_batch_eval's classes)
                for (auto& e : b->engines) {
                    const bool shallow = e->depth() <= kBatchShallowDepth;
                    if (shallow != (pass == 0)) continue;
                    rows.push_back(e->obj_args());
                    order.push_back(e.get());
                    b->depth = std::max(b->depth, e->depth());
                    int& d = shallow ? b->depth_shallow : b->depth_deep;
                    d = std::max(d, e->depth());
                    int& vd = shallow ? b->vdepth_shallow : b->vdepth_deep;
                    vd = std::max(vd, e->vdepth());
                    b->n_shallow += shallow ? 1 : 0;
                }
            // groups: the shallow rows split into batch_groups() consecutive runs, then the deep rows
            const int K = std::max(1, std::min(batch_groups(), b->n_shallow));
            for (int k = 0; k < K && b->n_shallow > 0; ++k) {
                const int r0 = b->n_shallow * k / K, r1 = b->n_shallow * (k + 1) / K;
                if (r1 > r0) b->groups.push_back({r0, r1 - r0, b->depth_shallow, b->vdepth_shallow});
            }
            if (n > b->n_shallow) b->groups.push_back({b->n_shallow, n - b->n_shallow, b->depth_deep, b->vdepth_deep});
            b->objs.reserve(rows.size() * sizeof(ObjArgs));
            IMPLI_HIP(hipMemcpyAsync(b->objs.p, rows.data(), rows.size() * sizeof(ObjArgs), hipMemcpyHostToDevice, s0));
            // the first merged pass: every object's counts in one read-back; an object whose mesh
            // outgrew the set_slab capacities grows its buffers and the pass runs again
            static std::mutex hc_mu;
            static HostBuf hc;   // pinned, process-wide (a hipHostMalloc per batch cost more than the pass)
            std::lock_guard<std::mutex> hc_lock(hc_mu);
            hc.reserve((size_t)n * kCounterWords * sizeof(uint32_t));
            DevBuf& dc = b->counts;
            dc.reserve((size_t)n * kCounterWords * sizeof(uint32_t));
            for (int pass = 0;; ++pass) {
                batch_merged_enqueue(b, s0);
                launch_gather_counters(b->objs.as<ObjArgs>(), n, dc.as<uint32_t>(), s0);   // every row's block
                IMPLI_HIP(hipMemcpyAsync(hc.p, dc.p, (size_t)n * kCounterWords * sizeof(uint32_t), hipMemcpyDeviceToHost, s0));
                IMPLI_HIP(hipStreamSynchronize(s0));
                bool grew = false;
                for (int r = 0; r < n; ++r) {
                    const uint32_t* h = hc.as<uint32_t>() + (size_t)r * kCounterWords;
                    const SlabCounts c{h[2], h[3], h[4], h[5]};
                    if (h[kOverflowWord] || !order[(size_t)r]->fits(c)) {
                        if (pass) throw HipError("object stream: output capacity overflow after resize");
                        order[(size_t)r]->ensure_capacity(c);
                        rows[(size_t)r] = order[(size_t)r]->obj_args();
                        IMPLI_HIP(hipMemsetAsync(const_cast<uint32_t*>(order[(size_t)r]->d_counters()) + kOverflowWord, 0,
                                                 4 * sizeof(uint32_t), s0));
                        grew = true;
                    }
                }
                if (!grew) break;
                IMPLI_HIP(hipMemcpyAsync(b->objs.p, rows.data(), rows.size() * sizeof(ObjArgs), hipMemcpyHostToDevice, s0));
            }
            if (timing) {
                ph[3] += tick(tp);
                size_t pool1[4];
                DevBuf::pool_stats(pool1);
                std::fprintf(stderr, "implisolid_batch_create (merged): compile + streams %.2f ms, first pass + counts %.2f ms; "
                                     "pool: %zu hipMalloc, %zu hipFree during the setup, %.1f MB cached before (%.1f MB "
                                     "awaiting a sync)\n",
                             t_compile * 1e3, ph[3] * 1e3, pool1[2] - pool0[2], pool1[3] - pool0[3],
                             (pool0[0] + pool0[1]) / 1e6, pool0[1] / 1e6);
            }
            // (the whole pass captured as one graph and replayed: 0.548-0.557 ms against 0.499-0.501
            // with direct launches, profiles/r05zq_config5_merged_graph_ab.txt)
            return b;
        }
        bool graphs = !std::getenv("IMPLISOLID_NO_GRAPH");
        for (int i = 0; i < n && graphs; ++i) {
            hipGraph_t g = nullptr;
            hipGraphExec_t x = nullptr;
            if (hipStreamBeginCapture(s0, hipStreamCaptureModeRelaxed) != hipSuccess) { graphs = false; break; }
            bool ok = true;
            try {
                b->engines[(size_t)i]->eval_field(s0);
                b->engines[(size_t)i]->count(s0);
                b->engines[(size_t)i]->emit(nullptr, s0);
            } catch (const std::exception&) {
                ok = false;
            }
            const hipError_t ec = hipStreamEndCapture(s0, &g);
            if (!ok || ec != hipSuccess || !g || hipGraphInstantiate(&x, g, nullptr, nullptr, 0) != hipSuccess) {
                if (g) (void)hipGraphDestroy(g);
                (void)hipGetLastError();
                graphs = false;
                break;
            }
            (void)hipGraphDestroy(g);
            b->execs.push_back(x);
        }
        if (!graphs) {
            for (auto x : b->execs) (void)hipGraphExecDestroy(x);
            b->execs.clear();
            std::fprintf(stderr, "implisolid: stream capture unavailable, the batch launches directly\n");
        }
        IMPLI_HIP(hipStreamSynchronize(s0));
    } catch (const std::exception& e) {
        report(e.what(), false);
        implisolid_batch_destroy(b);
        return nullptr;
    }
    return b;
}

// one merged pass enqueued on s: the groups' pipelines forked from s and joined back to it
static void batch_merged_enqueue(implisolid_batch* b, hipStream_t s) {
    Engine& E0 = *b->engines[0];
    const int fill = Engine::pruning() >= 2 ? 1 : 0;
    // each group's pipeline -- interval and eval passes, then marching cubes -- on its own
    // stream: one group's latency-bound launches (the coarse pass, the list fills, the count
    // and scan of few objects) run beside another's throughput-bound eval; the deep class
    // (few objects, 12- or 16-slot stacks) is the last group.  Forked from and joined to the
    // caller's stream.
    const int ng = (int)b->groups.size();
    if (ng > 1) {
        IMPLI_HIP(hipEventRecord(b->events[0], s));
        for (int k = 1; k < ng; ++k) IMPLI_HIP(hipStreamWaitEvent(b->streams[(size_t)k - 1], b->events[0], 0));
    }
    for (int k = ng - 1; k >= 0; --k) {   // the deep class first: its passes are the longest chain
        const implisolid_batch::Group& gr = b->groups[(size_t)k];
        hipStream_t q = k == 0 ? s : b->streams[(size_t)k - 1];
        const ObjArgs* rows = b->objs.as<ObjArgs>() + gr.row0;
        launch_batch_eval(rows, gr.n, gr.depth, gr.vdepth, E0.d_rabbit(), E0.tab_range(), E0.grid(), fill, q);
        launch_batch_mc(rows, gr.n, E0.d_cases(), E0.grid(), q);
    }
    for (int k = 1; k < ng; ++k) {
        IMPLI_HIP(hipEventRecord(b->events[(size_t)k], b->streams[(size_t)k - 1]));
        IMPLI_HIP(hipStreamWaitEvent(s, b->events[(size_t)k], 0));
    }
    IMPLI_HIP(hipGetLastError());
}

int implisolid_batch_run(implisolid_batch* b, void* stream) {
    try {
        hipStream_t s = (hipStream_t)stream;
        if (b->merged) {
            batch_merged_enqueue(b, s);
            return 0;
        }
        const int ns = (int)b->streams.size();
        IMPLI_HIP(hipEventRecord(b->events[0], s));
        for (int k = 0; k < ns; ++k) IMPLI_HIP(hipStreamWaitEvent(b->streams[(size_t)k], b->events[0], 0));
        for (size_t i = 0; i < b->engines.size(); ++i) {
            hipStream_t q = b->streams[i % (size_t)ns];
            if (!b->execs.empty()) {
                IMPLI_HIP(hipGraphLaunch(b->execs[i], q));
            } else {
                b->engines[i]->eval_field(q);
                b->engines[i]->count(q);
                b->engines[i]->emit(nullptr, q);
            }
        }
        for (int k = 0; k < ns; ++k) {
            IMPLI_HIP(hipEventRecord(b->events[(size_t)k + 1], b->streams[(size_t)k]));
            IMPLI_HIP(hipStreamWaitEvent(s, b->events[(size_t)k + 1], 0));
        }
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}

int implisolid_batch_info(implisolid_batch* b, int32_t out[4], double* jit_seconds) {
    out[0] = (int32_t)b->engines.size();
    out[1] = (int32_t)b->streams.size();
    out[2] = b->execs.empty() ? 0 : 1;
    out[3] = b->merged ? 1 : 0;
    if (jit_seconds) *jit_seconds = b->jit_seconds;
    return 0;
}

int implisolid_batch_counts(implisolid_batch* b, int i, uint32_t out[3]) {
    try {
        if (i < 0 || i >= (int)b->engines.size()) throw InputError("implisolid_batch_counts: bad index");
        for (auto q : b->streams) IMPLI_HIP(hipStreamSynchronize(q));
        if (b->merged) IMPLI_HIP(hipDeviceSynchronize());   // run() went to the caller's stream
        bool of = false;
        const SlabCounts c = b->engines[(size_t)i]->read_counts(b->streams[0], &of);
        out[0] = c.n_verts();
        out[1] = c.n_faces();
        out[2] = of ? 1u : 0u;
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}

int implisolid_batch_download(implisolid_batch* b, int i, float* verts, int32_t* faces) {
    try {
        if (i < 0 || i >= (int)b->engines.size()) throw InputError("implisolid_batch_download: bad index");
        for (auto q : b->streams) IMPLI_HIP(hipStreamSynchronize(q));
        if (b->merged) IMPLI_HIP(hipDeviceSynchronize());
        bool of = false;
        Engine& E = *b->engines[(size_t)i];
        const SlabCounts c = E.read_counts(b->streams[0], &of);
        if (of) throw HipError("batch object overflowed its output capacity");
        E.download(verts, faces, c, b->streams[0]);
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}

// ---- the OB02 loop on a Z-slab shard (one object per rank; Ob02::set_owned_vertices) -------------
struct implisolid_ob02 {
    std::unique_ptr<Engine> engine;
    std::unique_ptr<Ob02> ob;
    MCSettings st;
    hipStream_t stream = nullptr;
    hipEvent_t ev = nullptr;   // implisolid_ob02_attach: orders the stream after the caller's
    ~implisolid_ob02() {
        ob.reset();
        engine.reset();
        if (ev) (void)hipEventDestroy(ev);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

implisolid_ob02* implisolid_ob02_create(const char* shape_json, const char* mc_json) {
    g_last_error.clear();
    auto* h = new implisolid_ob02();
    try {
        h->st = parse_mc_settings(mc_json);
        const Program p = compile_mp5(shape_json, h->st.ignore_root_matrix);
        IMPLI_HIP(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
        h->engine.reset(new Engine());
        h->engine->set_object(p);
        h->ob.reset(new Ob02(*h->engine, h->stream));
        h->ob->capture_pointsets = false;
    } catch (const std::exception& e) {
        report(e.what(), false);
        delete h;
        return nullptr;
    }
    return h;
}

void implisolid_ob02_destroy(implisolid_ob02* h) {
    if (!h) return;
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    delete h;
}

#define OB02_TRY(expr)                                 \
    try {                                              \
        expr;                                          \
    } catch (const std::exception& e) {                \
        report(e.what(), false);                       \
        return -1;                                     \
    }                                                  \
    return 0;

int implisolid_ob02_load(implisolid_ob02* h, const float* d_verts, int64_t nv, const int32_t* d_faces, int64_t nf, int64_t v0,
                         int64_t v1) {
    OB02_TRY({
        if (nv < 0 || nf < 0 || (nv && !d_verts) || (nf && !d_faces)) throw InputError("implisolid_ob02_load: bad mesh");
        IMPLI_HIP(hipDeviceSynchronize());   // the caller's copies of the mesh are complete
        h->ob->load_shard(d_verts, nv, d_faces, nf, nullptr, v0, v1);
        IMPLI_HIP(hipStreamSynchronize(h->stream));
    })
}

int implisolid_ob02_attach(implisolid_ob02* h, float* d_verts, int64_t nv, const int32_t* d_faces, int64_t nf, int64_t v0,
                           int64_t v1, void* after_stream) {
    OB02_TRY({
        if (nv < 0 || nf < 0 || (nv && !d_verts) || (nf && !d_faces)) throw InputError("implisolid_ob02_attach: bad mesh");
        // stream-ordered after the caller's stream (its copies of the mesh), no device synchronisation
        if (!h->ev) IMPLI_HIP(hipEventCreateWithFlags(&h->ev, hipEventDisableTiming));
        IMPLI_HIP(hipEventRecord(h->ev, (hipStream_t)after_stream));
        IMPLI_HIP(hipStreamWaitEvent(h->stream, h->ev, 0));
        h->ob->load_shard(d_verts, nv, d_faces, nf, d_verts, v0, v1);
    })
}

void* implisolid_ob02_stream(implisolid_ob02* h) { return h ? (void*)h->stream : nullptr; }

int implisolid_ob02_resample_async(implisolid_ob02* h) { OB02_TRY(h->ob->vertex_resampling(h->st.vresampl_c)) }

int implisolid_ob02_project_async(implisolid_ob02* h) { OB02_TRY(h->ob->centroids_projection(h->st.qem != 0)) }

int implisolid_ob02_unpack(implisolid_ob02* h, const float* d_rows, int64_t row_len, const int64_t* voff, int world, int self) {
    OB02_TRY({
        if (world < 1 || !voff || (!d_rows && world > 1)) throw InputError("implisolid_ob02_unpack: bad arguments");
        h->ob->unpack_ranges(d_rows, row_len, std::vector<int64_t>(voff, voff + world + 1), self);
    })
}

int implisolid_ob02_resample(implisolid_ob02* h) {
    OB02_TRY({
        h->ob->vertex_resampling(h->st.vresampl_c);
        IMPLI_HIP(hipStreamSynchronize(h->stream));
    })
}

int implisolid_ob02_project(implisolid_ob02* h) {
    OB02_TRY({
        h->ob->centroids_projection(h->st.qem != 0);
        IMPLI_HIP(hipStreamSynchronize(h->stream));
    })
}

int implisolid_ob02_subdivide(implisolid_ob02* h, float amplitude) {
    OB02_TRY({
        h->ob->subdivide(amplitude);
        IMPLI_HIP(hipStreamSynchronize(h->stream));
    })
}

int implisolid_ob02_counts(implisolid_ob02* h, int64_t out[2]) {
    out[0] = h->ob->n_verts();
    out[1] = h->ob->n_faces();
    return 0;
}

int implisolid_ob02_ranges(implisolid_ob02* h, int64_t out[6]) {
    int64_t r[8];
    h->ob->ranges(r);
    for (int k = 0; k < 6; ++k) out[k] = r[k];
    return 0;
}

int implisolid_ob02_halo(implisolid_ob02* h, int64_t out[2]) {
    int64_t r[8];
    h->ob->ranges(r);
    out[0] = r[6];
    out[1] = r[7];
    return 0;
}

int implisolid_ob02_get_verts(implisolid_ob02* h, float* d_dst) {
    OB02_TRY({
        const int64_t nv = h->ob->n_verts();
        if (nv) IMPLI_HIP(hipMemcpyAsync(d_dst, h->ob->d_verts(), (size_t)nv * 12, hipMemcpyDeviceToDevice, h->stream));
        IMPLI_HIP(hipStreamSynchronize(h->stream));
    })
}

int implisolid_ob02_set_verts(implisolid_ob02* h, const float* d_src) {
    OB02_TRY({
        const int64_t nv = h->ob->n_verts();
        IMPLI_HIP(hipDeviceSynchronize());   // the caller's exchange into d_src is complete
        if (nv) IMPLI_HIP(hipMemcpyAsync(h->ob->d_verts(), d_src, (size_t)nv * 12, hipMemcpyDeviceToDevice, h->stream));
        IMPLI_HIP(hipStreamSynchronize(h->stream));
    })
}

int implisolid_ob02_download(implisolid_ob02* h, float* verts, int32_t* faces) {
    OB02_TRY(h->ob->fetch(verts, faces))
}

void implisolid_batch_destroy(implisolid_batch* b) {
    if (!b) return;
    for (auto q : b->streams) (void)hipStreamSynchronize(q);
    for (auto x : b->execs) (void)hipGraphExecDestroy(x);
    {   // the streams and events go back to the cache (the streams are idle: synchronised above)
        int d = 0;
        (void)hipGetDevice(&d);
        std::lock_guard<std::mutex> lk(g_batch_cache_mu);
        for (auto e : b->events) g_batch_events[d].push_back(e);
        for (auto q : b->streams) g_batch_streams[d].push_back(q);
    }
    b->objs.release();
    delete b;
}

}  // extern "C"
