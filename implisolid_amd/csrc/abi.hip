// abi.hip -- the extern "C" drop-in boundary (mcc2.cpp:88-134) over the MI355X engine.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/implisolid.h"
#include "engine.hpp"
#include "jit.hpp"

#include <chrono>
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

struct GeometryState {               // state_t, mcc2.cpp:165-193
    bool active = false;
    std::vector<float> verts;
    std::vector<int32_t> faces;
};
GeometryState g_state;

std::map<std::string, std::vector<float>> g_pointsets;   // pointset_set.hpp:8

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

void grand_algorithm(const char* shape_json, const MCSettings& st) {   // mcc2.cpp:309-444
    if (g_state.active) {
        report("build_geometry() called in a bad state.", false);
        return;
    }
    Program prog = compile_mp5(shape_json, st.ignore_root_matrix);
    Engine& E = engine();
    hipStream_t s = abi_stream();
    E.set_object(prog);
    E.set_grid(st.resolution, st.box, 0, 1);
    SlabCounts c = E.marching_cubes(s);   // polygonize_step_0
    int64_t nv = c.n_verts(), nf = c.n_faces();
    static std::unique_ptr<Ob02> ob_ptr;   // one refinement state, its buffers reused by every build
    if (!ob_ptr) ob_ptr.reset(new Ob02(E, s));
    Ob02& ob = *ob_ptr;
    ob.load_mesh(E.d_verts(), nv, E.d_faces(), nf);
    for (int rep = 0; rep < st.overall_repeats; ++rep) {
        for (int i = 0; i < st.vresampl_iters; ++i) ob.vertex_resampling(st.vresampl_c);   // step 1
        if (st.projection) ob.centroids_projection(st.qem);                             // step 2
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
    g_state.faces.resize((size_t)nf * 3);
    ob.fetch(g_state.verts.data(), g_state.faces.data());
    // STORE_POINTSET (pointset_set.hpp:11-25) replaces; vertex_resampling.hpp:176-211 uses
    // map::emplace on a never-cleared global, so the first resampling point sets persist
    for (auto& kv : ob.pointsets()) {
        const bool first_wins = kv.first == "pre_resampling_vertices" || kv.first == "post_resampling_vertices";
        if (first_wins && g_pointsets.count(kv.first)) continue;
        g_pointsets[kv.first] = kv.second;
    }
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

void build_geometry(const char* shape_json, const char* mc_json) {
    g_last_error.clear();
    MCSettings st;
    try {
        st = parse_mc_settings(mc_json);
    } catch (const InputError& e) {
        report(e.what(), true);
        return;
    }
    try {
        grand_algorithm(shape_json, st);
    } catch (const InputError& e) {
        report(e.what(), true);
    } catch (const std::exception& e) {
        report(std::string("build_geometry failed: ") + e.what(), false);
    }
}

void build_geometry_u(const char* shape_json, const char* mc_json, const char* call_specs) {
    try {
        (void)Json::parse(call_specs ? call_specs : "{}");   // worker_call_specs.hpp:28-40
    } catch (const JsonError& e) {
        report(std::string("call_specs: ") + e.what(), true);
        return;
    }
    build_geometry(shape_json, mc_json);
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
    auto it = g_pointsets.find(std::string(id));
    return it == g_pointsets.end() ? nullptr : it->second.data();
}
int get_pointset_size(char* id) {
    auto it = g_pointsets.find(std::string(id));
    return it == g_pointsets.end() ? 0 : (int)(it->second.size() / 3);
}

void about(void) {
    std::fprintf(stderr, "Build Info: \n%s %s\n", __DATE__, __TIME__);
    std::fprintf(stderr, "implisolid-mi355x: HIP gfx950 polygoniser (eval + marching cubes + OB02)\n");
    std::fprintf(stderr, "CONFIG: ROOT_TOLERANCE=%g \n", (double)(float)(0.001 / 10.0));
}

int64_t implisolid_jit_compile(const char* shape_json, char* source_out, int64_t capacity, double* seconds) {
    g_last_error.clear();
    try {
        const Program p = compile_mp5(shape_json, false);
        const std::string src = TreeJit::kernel_source(p);
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

int implisolid_slab_stats(implisolid_slab* s, int64_t out[10]) {
    try {
        uint32_t c[16];
        s->engine.raw_counters(c, 0);
        const GridDesc& g = s->engine.grid();
        out[0] = n_units(g);
        out[1] = c[6];   // non-empty units (c[0] counts their parts)
        out[2] = c[2];
        out[3] = c[3];
        out[4] = c[4];
        out[5] = c[5];
        out[6] = g.n_cells;
        out[7] = c[14];   // mixed coarse boxes of the last eval (the fill kernel's copy of [13])
        out[8] = c[1];    // the vertex pass's copy of the halo count (mc_types.hpp counters)
        out[9] = c[0];    // unit parts
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
    return 0;
}

int implisolid_slab_used_jit(implisolid_slab* s) { return s->engine.used_jit() ? 1 : 0; }
void implisolid_set_jit(int on) { TreeJit::instance().set_enabled(on != 0); }

int implisolid_slab_set_timing(implisolid_slab* s, int on) { SLAB_TRY(s->engine.set_timing(on != 0)) }
int implisolid_slab_kernel_times(implisolid_slab* s, float ms[6]) { SLAB_TRY(s->engine.kernel_times(ms)) }

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
            IMPLI_HIP(hipMemcpy(out, s->engine.d_field(), (size_t)n * sizeof(float), hipMemcpyDeviceToHost));
        }
        return n;
    } catch (const std::exception& e) {
        report(e.what(), false);
        return -1;
    }
}

// ---- object stream (config 5): one engine per object, each object's eval + count + emit captured
//      once in a hipGraph and replayed; objects spread over a few streams ----------------------------
struct implisolid_batch {
    std::vector<std::unique_ptr<Engine>> engines;
    std::vector<hipGraphExec_t> execs;   // empty when capture is unavailable (direct launches)
    std::vector<hipStream_t> streams;
    std::vector<hipEvent_t> events;      // fork (0) and one join event per stream
    double jit_seconds = 0;
};

implisolid_batch* implisolid_batch_create(const char* const* shapes, int n, const char* mc_json, int n_streams) {
    g_last_error.clear();
    auto* b = new implisolid_batch();
    try {
        if (n <= 0) throw InputError("implisolid_batch_create: no objects");
        const MCSettings st = parse_mc_settings(mc_json);
        std::vector<Program> progs;
        for (int i = 0; i < n; ++i) progs.push_back(compile_mp5(shapes[i], st.ignore_root_matrix));
        const auto t0 = std::chrono::steady_clock::now();
        if (Engine::pruning() > 0) TreeJit::instance().precompile(progs, 16);
        b->jit_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        const int ns = std::max(1, std::min(n_streams, 8));
        for (int k = 0; k < ns; ++k) {
            hipStream_t q;
            IMPLI_HIP(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
            b->streams.push_back(q);
        }
        for (int k = 0; k <= ns; ++k) {
            hipEvent_t e;
            IMPLI_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            b->events.push_back(e);
        }
        hipStream_t s0 = b->streams[0];
        for (int i = 0; i < n; ++i) {   // warm run: JIT lookup, output capacities from the real counts
            b->engines.emplace_back(new Engine());
            Engine& E = *b->engines.back();
            E.set_object(progs[(size_t)i]);
            E.set_grid(st.resolution, st.box, 0, 1);
            E.marching_cubes(s0);
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

int implisolid_batch_run(implisolid_batch* b, void* stream) {
    try {
        hipStream_t s = (hipStream_t)stream;
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
    out[3] = 0;
    if (jit_seconds) *jit_seconds = b->jit_seconds;
    return 0;
}

int implisolid_batch_counts(implisolid_batch* b, int i, uint32_t out[3]) {
    try {
        if (i < 0 || i >= (int)b->engines.size()) throw InputError("implisolid_batch_counts: bad index");
        for (auto q : b->streams) IMPLI_HIP(hipStreamSynchronize(q));
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

void implisolid_batch_destroy(implisolid_batch* b) {
    if (!b) return;
    for (auto q : b->streams) (void)hipStreamSynchronize(q);
    for (auto x : b->execs) (void)hipGraphExecDestroy(x);
    for (auto e : b->events) (void)hipEventDestroy(e);
    for (auto q : b->streams) (void)hipStreamDestroy(q);
    delete b;
}

}  // extern "C"
