// engine.hip -- buffer management and stage sequencing for the MI355X polygoniser.
#include "engine.hpp"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>

#include <cstddef>

#include "ifunc_device.hpp"
#include "jit.hpp"

namespace impli {

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw HipError(std::string(what) + ": " + hipGetErrorString(e));
}

// ---- the device-memory pool behind DevBuf ----------------------------------------------------------
// Size classes of four steps per octave (at most 25 % over the request), 256 B and up; blocks above
// kPoolMaxBlock (the field of a large grid) and any block past the cached-bytes cap go back
// to hipFree as before.  A released block waits in `pending` until the next allocation that would
// reuse it synchronises the device once (hipFree used to synchronise on every call): a kernel still
// reading it on some stream is done by then.
namespace {
constexpr size_t kPoolMaxBlock = size_t(256) << 20, kPoolMinCached = size_t(4) << 30;
struct DevicePool {
    std::map<size_t, std::vector<void*>> ready, pending;
    size_t ready_bytes = 0, pending_bytes = 0;
    size_t cap = 0;   // cached bytes at most: 1/16 of the device's memory, at least kPoolMinCached
};
size_t pool_cap(DevicePool& P, int d) {
    if (!P.cap) {
        size_t total = 0;
        if (hipDeviceTotalMem(&total, d) != hipSuccess) total = 0;
        P.cap = std::max(kPoolMinCached, total / 16);   // 18 GB of an MI355X's 288
    }
    return P.cap;
}
std::mutex g_pool_mu;
std::map<int, DevicePool> g_pools;
std::atomic<size_t> g_pool_mallocs{0}, g_pool_frees{0};
size_t pool_class(size_t n) {
    size_t c = 256;
    while (c < n) c <<= 1;                      // the octave's top
    const size_t q = c >> 3;                    // c / 2 + k c / 8, k = 1..4
    for (size_t k = 5; k <= 8; ++k)
        if (n <= q * k && q * k >= 256) return q * k;
    return c;
}
}  // namespace

void DevBuf::reserve(size_t n) {
    if (n <= bytes && p) return;
    release();
    int d = 0;
    IMPLI_HIP(hipGetDevice(&d));
    const size_t want = pool_class(n < 256 ? 256 : n);
    if (want <= kPoolMaxBlock) {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        DevicePool& P = g_pools[d];
        auto take = [&](std::map<size_t, std::vector<void*>>& m, size_t& counted) -> void* {
            auto it = m.find(want);
            if (it == m.end() || it->second.empty()) return nullptr;
            void* q = it->second.back();
            it->second.pop_back();
            counted -= want;
            return q;
        };
        void* q = take(P.ready, P.ready_bytes);
        if (!q && P.pending.count(want) && !P.pending[want].empty()) {
            IMPLI_HIP(hipDeviceSynchronize());   // every pending block's last user is done
            for (auto& kv : P.pending)
                for (void* b : kv.second) P.ready[kv.first].push_back(b);
            P.ready_bytes += P.pending_bytes;
            P.pending.clear();
            P.pending_bytes = 0;
            q = take(P.ready, P.ready_bytes);
        }
        if (q) {
            p = q;
            bytes = want;
            dev = d;
            return;
        }
    }
    IMPLI_HIP(hipMalloc(&p, want));
    g_pool_mallocs.fetch_add(1, std::memory_order_relaxed);
    bytes = want;
    dev = d;
}
void DevBuf::release() {
    if (p && !ext) {
        bool cached = false;
        if (bytes <= kPoolMaxBlock && dev >= 0 && pool_class(bytes) == bytes) {
            std::lock_guard<std::mutex> lk(g_pool_mu);
            DevicePool& P = g_pools[dev];
            if (P.ready_bytes + P.pending_bytes + bytes <= pool_cap(P, dev)) {
                P.pending[bytes].push_back(p);
                P.pending_bytes += bytes;
                cached = true;
            }
        }
        if (!cached) {
            (void)hipFree(p);
            g_pool_frees.fetch_add(1, std::memory_order_relaxed);
        }
    }
    p = nullptr;
    bytes = 0;
    ext = false;
    dev = -1;
}
void DevBuf::pool_stats(size_t out[4]) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    out[0] = out[1] = 0;
    out[2] = g_pool_mallocs.load(std::memory_order_relaxed);
    out[3] = g_pool_frees.load(std::memory_order_relaxed);
    for (auto& kv : g_pools) {
        out[0] += kv.second.ready_bytes;
        out[1] += kv.second.pending_bytes;
    }
}
void DevBuf::pool_trim() {
    int d = 0;
    IMPLI_HIP(hipGetDevice(&d));
    std::lock_guard<std::mutex> lk(g_pool_mu);
    auto it = g_pools.find(d);
    if (it == g_pools.end()) return;
    IMPLI_HIP(hipDeviceSynchronize());
    for (auto* m : {&it->second.ready, &it->second.pending})
        for (auto& kv : *m)
            for (void* b : kv.second) (void)hipFree(b);
    g_pools.erase(it);
}

void HostBuf::reserve(size_t n) {
    if (n <= bytes && p) return;
    release();
    size_t want = n < 256 ? 256 : n;
    IMPLI_HIP(hipHostMalloc(&p, want, hipHostMallocDefault));
    bytes = want;
}
void HostBuf::release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
}

static std::atomic<int> g_pruning{-1};

void Engine::set_pruning(int level) { g_pruning.store(level < 0 ? 0 : level > 2 ? 2 : level); }
int Engine::pruning() {
    int v = g_pruning.load();
    if (v < 0) {
        const char* e = std::getenv("IMPLISOLID_PRUNE");
        v = e ? std::atoi(e) : 2;
        v = v < 0 ? 0 : v > 2 ? 2 : v;
        g_pruning.store(v);
    }
    return v;
}

void Engine::brick_stats(int64_t out[3], hipStream_t s) {
    const BrickGrid bg = brick_grid(grid_);
    std::vector<uint8_t> f((size_t)bg.n_bricks);   // fill[b] = class | fill class << 4 (k_brick_fill)
    IMPLI_HIP(hipStreamSynchronize(s));
    if (bg.n_bricks) IMPLI_HIP(hipMemcpy(f.data(), fill_.p, f.size(), hipMemcpyDeviceToHost));
    int64_t mixed = 0, filled = 0;
    for (int b = 0; b < bg.n_bricks; ++b) {
        mixed += (f[b] & 3) == kBrickMixed;
        filled += ((f[b] >> 4) & 3) != 0 && !(f[b] & kBrickClaimed);   // claimed candidates were evaluated
    }
    out[0] = bg.n_bricks;
    out[1] = pruning() > 0 ? mixed : bg.n_bricks;
    out[2] = filled;
}

// The rabbit table (+ block min / max) and the marching-cubes case table are the same for every
// engine: built once per device and shared (an object stream creates one engine per object: each used
// to rebuild both on the host and upload them with blocking copies).  They live as long as the process.
namespace {
struct SharedTables {
    void* rabbit = nullptr;
    size_t rabbit_bytes = 0;
    void* cases = nullptr;
};
std::mutex g_tables_mu;
std::map<int, SharedTables> g_tables;   // per device
float2 g_tab_range{0.f, 0.f};

const std::vector<float>& rabbit_host_table() {
    static const std::vector<float> all = [] {
        // rabbit table + the object's trailing members (F8d: out-of-table reads) + zero padding
        std::vector<float> tab(dev::kRabbitPadded, 0.f);
        for (int i = 0; i < dev::kRabbitN; ++i) std::memcpy(&tab[i], &IMPLI_RABBIT_BITS[i], 4);
        const uint32_t tail[4] = {IMPLI_RABBIT_GRID_SIZE_BITS, IMPLI_RABBIT_ORIGIN_X_BITS, IMPLI_RABBIT_ORIGIN_Y_BITS,
                                  IMPLI_RABBIT_ORIGIN_Z_BITS};
        std::memcpy(&tab[dev::kRabbitN], tail, sizeof tail);
        g_tab_range = float2{tab[0], tab[0]};
        for (float v : tab) {
            g_tab_range.x = v < g_tab_range.x ? v : g_tab_range.x;
            g_tab_range.y = v > g_tab_range.y ? v : g_tab_range.y;
        }
        // block min / max of the eight reads at every flat index (ifunc_device.hpp kRabbitBlockMinMax)
        const int sx = IMPLI_RABBIT_NX, sxy = IMPLI_RABBIT_NX * IMPLI_RABBIT_NY;
        std::vector<float> a(tab);
        a.resize((size_t)dev::kRabbitPadded * 3, 0.f);
        for (int b = 0; b < dev::kRabbitPadded; ++b) {
            float lo = INFINITY, hi = -INFINITY;
            for (int d : {0, 1, sx, sx + 1, sxy, sxy + 1, sxy + sx, sxy + sx + 1}) {
                const float v = b + d < dev::kRabbitPadded ? tab[b + d] : 0.f;
                lo = v < lo ? v : lo;
                hi = v > hi ? v : hi;
            }
            a[dev::kRabbitPadded + 2 * b] = lo;
            a[dev::kRabbitPadded + 2 * b + 1] = hi;
        }
        return a;
    }();
    return all;
}
}  // namespace

Engine::Engine(hipStream_t setup, std::vector<ZeroRange>* resets) : resets_(resets) {
    int dev = 0;
    IMPLI_HIP(hipGetDevice(&dev));
    {
        std::lock_guard<std::mutex> lk(g_tables_mu);
        SharedTables& t = g_tables[dev];
        if (!t.rabbit) {
            const std::vector<float>& all = rabbit_host_table();
            CaseInfo cases[256];
            build_case_table(cases);
            void* r = nullptr;
            void* c = nullptr;
            IMPLI_HIP(hipMalloc(&r, all.size() * sizeof(float)));
            IMPLI_HIP(hipMalloc(&c, sizeof cases));
            IMPLI_HIP(hipMemcpy(r, all.data(), all.size() * sizeof(float), hipMemcpyHostToDevice));
            IMPLI_HIP(hipMemcpy(c, cases, sizeof cases, hipMemcpyHostToDevice));
            t.rabbit = r;
            t.rabbit_bytes = all.size() * sizeof(float);
            t.cases = c;
        }
        rabbit_.attach(t.rabbit, t.rabbit_bytes);
        cases_.attach(t.cases, sizeof(CaseInfo) * 256);
        tab_range_ = g_tab_range;
    }
    prog_.reserve(sizeof(Program));
    counters_.reserve(kCounterWords * sizeof(uint32_t));
    offsets_.reserve(16);
    if (resets_) {
        resets_->push_back({counters_.p, kCounterWords * sizeof(uint32_t)});
        resets_->push_back({offsets_.p, 16});
    } else if (setup) {
        IMPLI_HIP(hipMemsetAsync(counters_.p, 0, kCounterWords * sizeof(uint32_t), setup));   // [13] starts at 0 (grid.hpp)
        IMPLI_HIP(hipMemsetAsync(offsets_.p, 0, 16, setup));
    } else {
        IMPLI_HIP(hipMemset(counters_.p, 0, kCounterWords * sizeof(uint32_t)));
        IMPLI_HIP(hipMemset(offsets_.p, 0, 16));
    }
}

void Engine::set_offsets(uint32_t voff, uint32_t foff) {
    const uint32_t h[2] = {voff, foff};
    IMPLI_HIP(hipDeviceSynchronize());   // no kernel of an earlier emit may still read them
    IMPLI_HIP(hipMemcpy(offsets_.p, h, sizeof h, hipMemcpyHostToDevice));
}

void Engine::download(float* verts, int32_t* faces, const SlabCounts& c, hipStream_t s) {
    if (c.n_verts()) IMPLI_HIP(hipMemcpyAsync(verts, verts_.p, (size_t)c.n_verts() * 12, hipMemcpyDeviceToHost, s));
    if (c.n_faces()) IMPLI_HIP(hipMemcpyAsync(faces, faces_.p, (size_t)c.n_faces() * 12, hipMemcpyDeviceToHost, s));
    IMPLI_HIP(hipStreamSynchronize(s));
}

void Engine::set_timing(bool on) {
    if (on && !ev_[0])
        for (auto& e : ev_) IMPLI_HIP(hipEventCreate(&e));
    timing_ = on;
}

void Engine::kernel_times_each(float out[kTimedEachKernel]) {
    if (!ev_[0]) throw InputError("kernel timing was never enabled");
    IMPLI_HIP(hipEventSynchronize(ev_[8]));
    const int pairs[kTimedEachKernel][2] = {{0, 9}, {9, 10}, {10, 1}, {1, 2}, {3, 4}, {4, 5}, {6, 7}, {7, 8}};
    for (int k = 0; k < kTimedEachKernel; ++k) {
        float ms = 0.f;
        IMPLI_HIP(hipEventElapsedTime(&ms, ev_[pairs[k][0]], ev_[pairs[k][1]]));
        out[k] = ms;
    }
}

void Engine::kernel_times(float out[kTimedKernels]) {
    if (!ev_[0]) throw InputError("kernel timing was never enabled");
    IMPLI_HIP(hipEventSynchronize(ev_[8]));
    const int pairs[kTimedKernels][2] = {{0, 1}, {1, 2}, {3, 4}, {4, 5}, {6, 7}, {7, 8}};
    for (int k = 0; k < kTimedKernels; ++k) {
        float ms = 0.f;
        IMPLI_HIP(hipEventElapsedTime(&ms, ev_[pairs[k][0]], ev_[pairs[k][1]]));
        out[k] = ms;
    }
}

Engine::~Engine() {
    for (auto& e : ev_)
        if (e) (void)hipEventDestroy(e);
    if (ev_counts_) (void)hipEventDestroy(ev_counts_);
    if (ev_verts_) (void)hipEventDestroy(ev_verts_);
    DevBuf* all[] = {&offsets_, &cmodes_, &ccls_, &clist_, &modes_, &cls_, &fill_, &blist_, &prog_, &rabbit_, &cases_, &field_, &signs_, &scan_blk_, &unit_cnt_, &unit_part_, &unit_cmask_, &ulist_, &upart_, &umark_, &counters_, &lmodes_, &claimed_, &vid_,
                     &records_, &verts_, &faces_};
    for (auto* b : all) b->release();
    for (auto& b : scratch_) b.release();
    // the buffers went to the pool (no hipFree and its implicit synchronisation): the modules'
    // last launches must be done before release_jit may unload them
    if (jit_slot_ || bake_slot_ || pt_slot_ || pt_bake_slot_) (void)hipDeviceSynchronize();
    release_jit();
}

void Engine::release_jit() {
    TreeJit& J = TreeJit::instance();
    J.release(jit_slot_);
    J.release(bake_slot_);
    J.release(pt_slot_);
    J.release(pt_bake_slot_);
    jit_slot_ = bake_slot_ = pt_slot_ = pt_bake_slot_ = nullptr;
    jit_requested_ = bake_requested_ = pt_requested_ = pt_bake_requested_ = false;
    pt_uses_ = 0;
    jit_fn_ = nullptr;
    jit_iv_ = JitIntervalKernels{};
}

// the value stack's high-water mark of a program run without pruning (a pruned run skips a whole
// operand subtree and its CSG node's pop together, so it never holds more)
int program_vdepth(const Program& p) {
    int vp = 0, best = 1;
    for (int pc = 0; pc < p.n_instr; ++pc) {
        const Instr& I = p.instr[pc];
        if (I.op == OP_PRIM) best = std::max(best, ++vp);
        else if (I.op != OP_XFORM) vp = std::max(0, vp - 1);
    }
    return best;
}

void Engine::set_object(const Program& prog, const Program* d_prog) {
    // the same object again (repeated builds): keep its modules and its eval count
    if (have_object_ && !d_prog && std::memcmp(&prog, &prog_host_, sizeof(Program)) == 0) return;
    // the engine's kernels run on caller streams (often non-blocking): nothing in flight may still
    // read the program being replaced (a fresh engine has launched nothing)
    if (have_object_ || have_grid_) IMPLI_HIP(hipDeviceSynchronize());
    if (d_prog) {
        prog_.attach(const_cast<Program*>(d_prog), sizeof(Program));
    } else {
        if (prog_.ext) prog_.release();
        prog_.reserve(sizeof(Program));
        IMPLI_HIP(hipMemcpy(prog_.p, &prog, sizeof(Program), hipMemcpyHostToDevice));
    }
    depth_ = prog.max_depth;
    vdepth_ = program_vdepth(prog);
    n_csg_ = prog.n_csg;
    prog_host_ = prog;
    release_jit();
    TreeJit::instance().trim();   // the device is synchronised here: a safe point to unload modules
    evals_ = 0;
    jit_fn_ = nullptr;
    have_object_ = true;
    ++obj_gen_;   // the grid's buffers hold the previous object's field and signs: set_slab resets them
}

void Engine::set_grid(int R, const float box[6], int rank, int nranks) {
    set_slab(R, box, slab_partition(R, rank, nranks));   // one halo layer below (owner rule)
}

void Engine::arm_merged() {
    if (!have_grid_ || !have_object_ || probe_only_) throw InputError("engine: arm_merged needs an object and a grid");
    if (mark_id_ == 0) mark_id_ = 1;   // the unit marks were reset to 0 with the grid
    marks_valid_ = true;
}

void Engine::set_slab(int R, const float box[6], const SlabRange& sr_in, bool probe_only, hipStream_t setup) {
    const SlabRange sr = slab_range(R, sr_in.z0, sr_in.z1);   // validated, 32-bit limits checked
    // the same grid and object again (repeated builds of build_geometry): every buffer keeps its size
    // and its invariants (umark ids only grow, the sign pieces past a row's last brick stay 0,
    // counters are cleared in-kernel), so there is nothing to reset and nothing to wait for.  A new
    // object on the same grid resets the field (unlisted bricks read as 0) and the sign bitmap
    // (bricks the new object leaves unlisted must not keep the old object's signs).
    if (have_grid_ && !probe_only && !probe_only_ && key_R_ == R && key_z0_ == sr.z0 && key_z1_ == sr.z1 &&
        key_obj_gen_ == obj_gen_ && std::memcmp(key_box_, box, sizeof key_box_) == 0)
        return;
    key_R_ = -1;   // set again once the buffers below are valid
    // the buffers below are reset on the null stream, which a non-blocking caller stream does not
    // order against: no earlier kernel may still run (a fresh engine has launched none), and the
    // resets finish before the next launch
    const bool fresh_async = setup && !have_grid_;   // an object stream's fresh engine (see engine.hpp)
    if (have_grid_) IMPLI_HIP(hipDeviceSynchronize());
    auto zero = [&](void* p, size_t n) {
        if (fresh_async && resets_) resets_->push_back({p, n});
        else if (fresh_async) IMPLI_HIP(hipMemsetAsync(p, 0, n, setup));
        else IMPLI_HIP(hipMemset(p, 0, n));
    };
    grid_ = make_grid(R, box, sr.z0 - sr.halo, sr.z1, sr.z0);
    probe_only_ = probe_only;
    modes_.reserve((size_t)(brick_grid(grid_).n_bricks + 1) * sizeof(uint64_t));
    cls_.reserve((size_t)brick_grid(grid_).n_bricks + 64);
    cmodes_.reserve((size_t)(coarse_grid(grid_).n_bricks + 1) * sizeof(uint64_t));
    ccls_.reserve((size_t)coarse_grid(grid_).n_bricks + 64);
    clist_.reserve(((size_t)coarse_grid(grid_).n_bricks + 16) * sizeof(uint32_t));
    fill_.reserve((size_t)brick_grid(grid_).n_bricks + 64);
    blist_.reserve(((size_t)brick_grid(grid_).n_bricks + 16) * sizeof(uint32_t));
    lmodes_.reserve(((size_t)brick_grid(grid_).n_bricks + 16) * sizeof(uint64_t));
    claimed_.reserve(((size_t)brick_grid(grid_).n_bricks + 16) * sizeof(uint32_t));   // merged eval's second pass
    if (n_chunks(grid_) > kMaxChunks) throw InputError("grid: more than 8189 cells per row");
    const size_t mark_bytes = (size_t)(n_units(grid_) * n_chunks(grid_) + 1) * sizeof(uint32_t);
    umark_.reserve(mark_bytes);
    zero(umark_.p, mark_bytes);   // ids start at 1
    marks_valid_ = false;
    mark_id_ = 0;
    const size_t sign_bytes = (size_t)grid_.n * (grid_.fz1 - grid_.fz0) * sign_row_words(grid_) * sizeof(uint64_t);
    signs_.reserve(sign_bytes + 64);
    // the pieces past the last brick of a row are never written by the pruned path: keep them 0
    zero(signs_.p, sign_bytes + 64);
    if (probe_only) {   // interval_pass / listed_per_layer only
        IMPLI_HIP(hipDeviceSynchronize());
        have_grid_ = true;
        return;
    }
    const size_t field_bytes = (size_t)field_samples(grid_) * sizeof(float);   // brick-major (grid.hpp)
    field_.reserve(field_bytes);
    // the pruned eval writes only the listed bricks: the rest of the field reads as 0, not as
    // whatever the allocation held (deterministic read_field; nothing on the path reads it, so an
    // object stream's engines skip it)
    if (!fresh_async) IMPLI_HIP(hipMemset(field_.p, 0, field_bytes));
    unit_cnt_.reserve((size_t)(n_groups(grid_) * kGroupUnits + 1) * sizeof(uint4));
    unit_part_.reserve((size_t)(n_groups(grid_) * kGroupUnits + 1) * sizeof(uint32_t));
    unit_cmask_.reserve((size_t)(n_groups(grid_) * kGroupUnits + 1) * sizeof(uint32_t));
    scan_blk_.reserve((size_t)(n_groups(grid_) + 1) * (kScanParts + 1) * sizeof(uint32_t));
    ulist_.reserve((size_t)(n_units(grid_) * kMaxParts + 1) * sizeof(uint4));
    upart_.reserve((size_t)(n_units(grid_) * kMaxParts + 1) * sizeof(uint32_t));
    const int64_t m2 = (int64_t)grid_.m * grid_.m;
    // owned-id triples by cell id (mc_types.hpp vid): 12 B per cell of the slab (1.6 GB at 512^3),
    // written only for the ~0.3 % of cells owning a crossing edge
    vid_.reserve((size_t)(grid_.n_cells + 1) * 3 * sizeof(uint32_t));
    ensure_capacity(SlabCounts{(uint32_t)std::min<int64_t>(6 * m2, 1u << 31), (uint32_t)std::min<int64_t>(12 * m2, 1u << 31),
                               (uint32_t)std::min<int64_t>(6 * m2, 1u << 31), 0});
    if (!fresh_async) IMPLI_HIP(hipDeviceSynchronize());
    have_grid_ = true;
    key_R_ = R;
    key_z0_ = sr.z0;
    key_z1_ = sr.z1;
    key_obj_gen_ = obj_gen_;
    std::memcpy(key_box_, box, sizeof key_box_);
}

bool Engine::ensure_capacity(const SlabCounts& c) {
    bool grew = false;
    auto grow = [&](DevBuf& b, int64_t& cap, int64_t need, size_t elem) {
        if (need <= cap) return;
        int64_t nc = cap ? cap : 1024;
        while (nc < need) nc *= 2;
        b.reserve((size_t)nc * elem);
        cap = nc;
        grew = true;
    };
    grow(verts_, cap_v_, (int64_t)c.n_verts() + 1, 3 * sizeof(float));
    grow(faces_, cap_f_, (int64_t)c.n_faces() + 1, 3 * sizeof(int32_t));
    grow(records_, cap_rec_, (int64_t)c.act_total + 1, sizeof(uint4));
    return grew;
}

MCBuffers Engine::buffers() const {
    MCBuffers b{};
    b.field = field_.as<float>();
    b.signs = signs_.as<uint64_t>();

    b.unit_cnt = unit_cnt_.as<uint4>();
    b.unit_part = unit_part_.as<uint32_t>();
    b.unit_cmask = unit_cmask_.as<uint32_t>();
    b.scan_blk = scan_blk_.as<uint32_t>();
    b.ulist = ulist_.as<uint4>();
    b.upart = upart_.as<uint32_t>();
    b.cap_parts = (uint32_t)(n_units(grid_) * kMaxParts + 1);   // ulist_ / upart_ entries
    b.umark = marks_valid_ ? umark_.as<uint32_t>() : nullptr;
    b.mark_id = mark_id_;
    b.counters = counters_.as<uint32_t>();
    b.vid = vid_.as<uint32_t>();
    b.records = records_.as<uint4>();
    b.verts = verts_.as<float>();
    b.faces = faces_.as<int32_t>();
    b.cap_v = cap_v_;
    b.cap_f = cap_f_;
    b.cap_rec = cap_rec_;
    b.offsets = nullptr;
    b.overflow = counters_.as<uint32_t>() + kOverflowWord;

    return b;
}

void Engine::eval_field(hipStream_t s) {
    if (!have_grid_ || !have_object_) throw InputError("engine: object and grid must be set before eval");
    if (probe_only_) throw InputError("engine: a probe slab has no field (interval_pass only)");
    const int level = pruning();
    // the counter block (list lengths, MC counters, overflow flags) is cleared by the pruned path's
    // first kernel (grid.hpp); the dense path clears it with a memset
    if (level == 0 || brick_grid(grid_).n_bricks <= 0)
        IMPLI_HIP(hipMemsetAsync(counters_.p, 0, kCounterWords * sizeof(uint32_t), s));
    counters_fresh_ = true;
    mark(0, s);
    if (level > 0) {
        ensure_jit(s);
        launch_brick_modes(prog_.as<Program>(), depth_, rabbit_.as<float>(), tab_range_, grid_, cmodes_.as<uint64_t>(),
                           ccls_.as<uint8_t>(), clist_.as<uint32_t>(), counters_.as<uint32_t>(),
                           modes_.as<uint64_t>(), cls_.as<uint8_t>(), s, &jit_iv_, timing_ ? ev_[9] : nullptr);
        mark(10, s);
        uint32_t* d_count = counters_.as<uint32_t>() + kBrickListWord;
        launch_brick_fill(grid_, ccls_.as<uint8_t>(), cmodes_.as<uint64_t>(), cls_.as<uint8_t>(), modes_.as<uint64_t>(),
                          level >= 2, fill_.as<uint8_t>(), blist_.as<uint32_t>(), lmodes_.as<uint64_t>(), d_count,
                          signs_.p, umark_.as<uint32_t>(), ++mark_id_, s);
        marks_valid_ = true;
        mark(1, s);
        const BrickGrid bg = brick_grid(grid_);
        const ClaimCtx cc{level >= 2 ? fill_.as<uint8_t>() : nullptr, ccls_.as<uint8_t>(), modes_.as<uint64_t>(),
                          cmodes_.as<uint64_t>(), bg.nbx, bg.nbx * bg.nby};
        if (jit_fn_) {
            const float* d_mats = reinterpret_cast<const float*>(prog_.as<char>() + offsetof(Program, mats));
            TreeJit::launch_bricks(jit_fn_, d_mats, rabbit_.as<float>(), grid_, bg, lmodes_.as<uint64_t>(),
                                   blist_.as<uint32_t>(), d_count, field_.as<float>(), signs_.p, cc, eval_bricks_grid(grid_),
                                   s);
        } else {
            launch_eval_bricks_interp(prog_.as<Program>(), depth_, rabbit_.as<float>(), grid_, lmodes_.as<uint64_t>(),
                                      blist_.as<uint32_t>(), d_count, field_.as<float>(), signs_.p, cc, s);
        }
    } else {
        marks_valid_ = false;   // dense field: MC counts every unit
        IMPLI_HIP(hipMemsetAsync(fill_.p, 0, (size_t)brick_grid(grid_).n_bricks, s));   // nothing filled
        mark(9, s);
        mark(10, s);
        mark(1, s);
        launch_eval_field(prog_.as<Program>(), depth_, rabbit_.as<float>(), grid_, field_.as<float>(), s);
        launch_signs_from_field(grid_, field_.as<float>(), signs_.as<uint64_t>(), s);
    }
    mark(2, s);
    IMPLI_HIP(hipGetLastError());
}

void Engine::interval_pass(hipStream_t s) {
    if (!have_grid_ || !have_object_) throw InputError("engine: object and grid must be set before the interval pass");
    if (brick_grid(grid_).n_bricks <= 0) return;
    ensure_jit(s);
    launch_brick_modes(prog_.as<Program>(), depth_, rabbit_.as<float>(), tab_range_, grid_, cmodes_.as<uint64_t>(),
                       ccls_.as<uint8_t>(), clist_.as<uint32_t>(), counters_.as<uint32_t>(), modes_.as<uint64_t>(),
                       cls_.as<uint8_t>(), s, &jit_iv_);
    launch_brick_fill(grid_, ccls_.as<uint8_t>(), cmodes_.as<uint64_t>(), cls_.as<uint8_t>(), modes_.as<uint64_t>(),
                      1, fill_.as<uint8_t>(), blist_.as<uint32_t>(), lmodes_.as<uint64_t>(),
                      counters_.as<uint32_t>() + kBrickListWord, signs_.p, umark_.as<uint32_t>(), ++mark_id_, s);
    marks_valid_ = false;   // no field behind these marks
    counters_fresh_ = true;
    IMPLI_HIP(hipGetLastError());
}

std::vector<int64_t> Engine::listed_per_layer(hipStream_t s) {
    const BrickGrid bg = brick_grid(grid_);
    const int layers = grid_.fz1 - grid_.fz0;
    std::vector<int64_t> out((size_t)layers, 0);
    if (bg.n_bricks <= 0) return out;
    std::vector<uint8_t> f((size_t)bg.n_bricks);   // fill[b] = class | fill class << 4 (k_brick_fill)
    IMPLI_HIP(hipStreamSynchronize(s));
    IMPLI_HIP(hipMemcpy(f.data(), fill_.p, f.size(), hipMemcpyDeviceToHost));
    const int plane = bg.nbx * bg.nby;
    for (int bz = 0; bz < bg.nbz; ++bz) {
        int64_t listed = 0;
        for (int k = 0; k < plane; ++k) listed += ((f[(size_t)bz * plane + k] >> 4) & 3) == 0;
        for (int l = bz * kBZ; l < std::min(layers, bz * kBZ + kBZ); ++l) out[(size_t)l] = listed;
    }
    return out;
}

std::vector<int> cuts_from_layer_work(const std::vector<int64_t>& listed, int64_t bricks_per_layer, int R, int nranks) {
    const int L = R + 2;   // cell layers 1 .. L; cell layer c evaluates its lower sample layer c - 1
    if (nranks < 1 || nranks > L) throw InputError("balance: more slabs than cell layers");
    if ((int)listed.size() < L + 1) throw InputError("balance: per-layer counts do not cover the grid");
    // a listed brick costs ~1.3 ns of eval + MC, a brick of the interval / fill passes ~27 ps
    // (DESIGN.md section 6): the per-brick term weighs 0.02 of a listed brick
    constexpr double kAllBrickWeight = 0.02;
    std::vector<double> cum((size_t)L + 1, 0.0);
    for (int c = 1; c <= L; ++c)
        cum[(size_t)c] = cum[(size_t)c - 1] + (double)listed[(size_t)c - 1] / kBZ + kAllBrickWeight * bricks_per_layer / kBZ;
    std::vector<int> cuts((size_t)nranks + 1);
    cuts[0] = 1;
    for (int r = 1; r < nranks; ++r) {
        const double target = cum[(size_t)L] * r / nranks;
        int c = cuts[(size_t)r - 1] + 1;   // at least one layer per slab
        while (c < L && cum[(size_t)c - 1] + 0.5 * (cum[(size_t)c] - cum[(size_t)c - 1]) < target) ++c;
        c = std::min(c, L + 1 - (nranks - r));   // leave one layer for every later slab
        cuts[(size_t)r] = std::max(c, cuts[(size_t)r - 1] + 1);
    }
    cuts[(size_t)nranks] = L + 1;
    return cuts;
}

std::vector<int> balance_cuts(const Program& prog, int R, const float box[6], int nranks, hipStream_t s) {
    if (nranks == 1) return {1, R + 3};
    Engine probe;
    probe.set_object(prog);
    probe.set_slab(R, box, SlabRange{1, R + 3, 0}, true);
    probe.interval_pass(s);
    const BrickGrid bg = brick_grid(probe.grid());
    return cuts_from_layer_work(probe.listed_per_layer(s), (int64_t)bg.nbx * bg.nby, R, nranks);
}

const float* Engine::d_mats() const {
    return reinterpret_cast<const float*>(prog_.as<char>() + offsetof(Program, mats));
}

const TreeJit::PointKernels* Engine::point_jit(hipStream_t s) {
    TreeJit& J = TreeJit::instance();
    if (!pt_requested_) {
        pt_slot_ = J.request(prog_host_, TreeJit::kPoints, J.bake() == TreeJit::kBakeAlways, s);
        pt_requested_ = true;
    }
    // a hot object gets a point module with its matrices baked in, as its brick module does
    // (ensure_jit): here after kBakeAfter builds' worth of OB02 steps (a build of 3 repeats asks
    // twice per repeat: the resampling's normals, the projection)
    if (++pt_uses_ >= 6 * TreeJit::kBakeAfter && !pt_bake_requested_ && allow_hot_bake_ && J.bake() == TreeJit::kBakeHot &&
        pt_slot_) {
        pt_bake_slot_ = J.request(prog_host_, TreeJit::kPoints, true, s);
        pt_bake_requested_ = true;
    }
    if (pt_bake_slot_ && pt_bake_slot_->ready.load(std::memory_order_acquire)) return &pt_bake_slot_->pk;
    return (pt_slot_ && pt_slot_->ready.load(std::memory_order_acquire)) ? &pt_slot_->pk : nullptr;
}

void Engine::ensure_jit(hipStream_t s) {
    // the object's tree module is requested once (TreeJit: compiled now, or on a background thread
    // while the interpreter kernels run); every eval uses it as soon as it is loaded
    TreeJit& J = TreeJit::instance();
    if (!jit_requested_) {
        jit_slot_ = J.request(prog_host_, TreeJit::kBricks, J.bake() == TreeJit::kBakeAlways, s);
        jit_requested_ = true;
    }
    // a hot object (evaluated kBakeAfter times since set_object) gets its baked module
    if (++evals_ >= TreeJit::kBakeAfter && !bake_requested_ && allow_hot_bake_ && J.bake() == TreeJit::kBakeHot &&
        jit_slot_) {
        bake_slot_ = J.request(prog_host_, TreeJit::kBricks, true, s);
        bake_requested_ = true;
    }
    const TreeJit::Slot* use = bake_slot_ && bake_slot_->ready.load(std::memory_order_acquire) ? bake_slot_
                               : jit_slot_ && jit_slot_->ready.load(std::memory_order_acquire) ? jit_slot_
                                                                                                : nullptr;
    if (use) {
        jit_fn_ = use->k.bricks;
        jit_iv_.coarse = use->k.coarse;
        jit_iv_.refine = use->k.refine;
    } else {
        jit_fn_ = nullptr;
        jit_iv_ = JitIntervalKernels{};
    }
}

void Engine::count(hipStream_t s) {
    if (!counters_fresh_) {   // a repeated count: reset the MC counters and overflow flags (eval_field did)
        IMPLI_HIP(hipMemsetAsync(counters_.p, 0, kBrickListWord * sizeof(uint32_t), s));
        IMPLI_HIP(hipMemsetAsync(counters_.as<uint32_t>() + kOverflowWord, 0, 4 * sizeof(uint32_t), s));
    }
    counters_fresh_ = false;
    MCBuffers b = buffers();
    mark(3, s);
    launch_mc_count(cases_.as<CaseInfo>(), grid_, b, s);
    mark(4, s);
    launch_mc_scan(grid_, b, s);
    mark(5, s);
    IMPLI_HIP(hipGetLastError());
}

void Engine::emit(const uint32_t* d_offsets, hipStream_t s) {
    emit_verts(s);
    emit_faces(d_offsets, nullptr, 0, s);
}

void Engine::emit_verts(hipStream_t s) {   // vertex positions and ids are slab-local: no offsets
    MCBuffers b = buffers();
    mark(6, s);
    launch_mc_verts(cases_.as<CaseInfo>(), grid_, b, s);
    mark(7, s);
    IMPLI_HIP(hipGetLastError());
}

void Engine::emit_faces(const uint32_t* d_offsets, const uint32_t* d_gathered, int rank, hipStream_t s) {
    MCBuffers b = buffers();
    if (d_gathered) {
        b.offsets = nullptr;
        b.gathered = d_gathered;
        b.rank = rank;
    } else {
        b.offsets = d_offsets ? d_offsets : offsets_.as<uint32_t>();
    }
    launch_mc_faces(cases_.as<CaseInfo>(), grid_, b, s);
    mark(8, s);
    IMPLI_HIP(hipGetLastError());
}

// the counter block's first kOverflowWord + 1 words in one copy into pinned memory (two copies into
// pageable stack memory took ~60 us of staging per build)
static_assert(kOverflowWord + 1 <= kCounterWords, "counter block layout");
void Engine::raw_counters(uint32_t out[16], hipStream_t s) {
    hcounters_.reserve(kCounterWords * sizeof(uint32_t));
    IMPLI_HIP(hipMemcpyAsync(hcounters_.p, counters_.p, 16 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    IMPLI_HIP(hipStreamSynchronize(s));
    std::memcpy(out, hcounters_.p, 16 * sizeof(uint32_t));
}

SlabCounts Engine::read_counts(hipStream_t s, bool* overflow) {
    hcounters_.reserve(kCounterWords * sizeof(uint32_t));
    IMPLI_HIP(hipMemcpyAsync(hcounters_.p, counters_.p, (kOverflowWord + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    IMPLI_HIP(hipStreamSynchronize(s));
    const uint32_t* h = hcounters_.as<uint32_t>();
    if (overflow) *overflow = h[kOverflowWord] != 0;
    return SlabCounts{h[2], h[3], h[4], h[5]};
}

SlabCounts Engine::marching_cubes(hipStream_t s) {
    eval_field(s);
    count(s);
    emit(nullptr, s);
    bool of = false;
    SlabCounts c = read_counts(s, &of);
    if (of || ensure_capacity(c)) {
        ensure_capacity(c);
        IMPLI_HIP(hipMemsetAsync(counters_.as<uint32_t>() + kOverflowWord, 0, 4 * sizeof(uint32_t), s));
        emit(nullptr, s);
        c = read_counts(s, &of);
        if (of) throw HipError("marching cubes: output capacity overflow after resize");
    }
    return c;
}

SlabCounts Engine::marching_cubes_to_host(hipStream_t s, hipStream_t cs,
                                          const std::function<void(int64_t, int64_t, float**, int32_t**)>& host) {
    if (!ev_counts_) IMPLI_HIP(hipEventCreateWithFlags(&ev_counts_, hipEventDisableTiming));
    if (!ev_verts_) IMPLI_HIP(hipEventCreateWithFlags(&ev_verts_, hipEventDisableTiming));
    hcounters_.reserve(kCounterWords * sizeof(uint32_t));
    uint32_t* h = hcounters_.as<uint32_t>();
    eval_field(s);
    count(s);
    // the totals land in pinned memory while the emission kernels run behind them
    IMPLI_HIP(hipMemcpyAsync(h, counters_.p, (kOverflowWord + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    IMPLI_HIP(hipEventRecord(ev_counts_, s));
    emit_verts(s);
    IMPLI_HIP(hipEventRecord(ev_verts_, s));
    emit_faces(nullptr, nullptr, 0, s);
    IMPLI_HIP(hipEventSynchronize(ev_counts_));
    SlabCounts c{h[2], h[3], h[4], h[5]};
    if (!fits(c)) {   // the emission wrote past nothing (it checks its capacity): grow, emit again
        IMPLI_HIP(hipStreamSynchronize(s));
        ensure_capacity(c);
        IMPLI_HIP(hipMemsetAsync(counters_.as<uint32_t>() + kOverflowWord, 0, 4 * sizeof(uint32_t), s));
        emit(nullptr, s);
        bool of = false;
        c = read_counts(s, &of);
        if (of) throw HipError("marching cubes: output capacity overflow after resize");
        float* hv = nullptr;
        int32_t* hf = nullptr;
        host(c.n_verts(), c.n_faces(), &hv, &hf);
        download(hv, hf, c, s);
        return c;
    }
    float* hv = nullptr;
    int32_t* hf = nullptr;
    host(c.n_verts(), c.n_faces(), &hv, &hf);
    if (c.n_verts()) {
        IMPLI_HIP(hipStreamWaitEvent(cs, ev_verts_, 0));
        IMPLI_HIP(hipMemcpyAsync(hv, verts_.p, (size_t)c.n_verts() * 12, hipMemcpyDeviceToHost, cs));
    }
    if (c.n_faces()) IMPLI_HIP(hipMemcpyAsync(hf, faces_.p, (size_t)c.n_faces() * 12, hipMemcpyDeviceToHost, s));
    IMPLI_HIP(hipMemcpyAsync(h + kOverflowWord, counters_.as<uint32_t>() + kOverflowWord, sizeof(uint32_t),
                             hipMemcpyDeviceToHost, s));
    IMPLI_HIP(hipStreamSynchronize(cs));
    IMPLI_HIP(hipStreamSynchronize(s));
    if (h[kOverflowWord] != 0) throw HipError("marching cubes: output overflow within capacity");
    return c;
}

ObjArgs Engine::obj_args() const {
    if (!marks_valid_) throw InputError("engine: obj_args needs one pruned eval_field first");
    ObjArgs o{};
    o.prog = prog_.as<Program>();
    o.cmodes = cmodes_.as<uint64_t>();
    o.ccls = ccls_.as<uint8_t>();
    o.clist = clist_.as<uint32_t>();
    o.modes = modes_.as<uint64_t>();
    o.cls = cls_.as<uint8_t>();
    o.fill = fill_.as<uint8_t>();
    o.blist = blist_.as<uint32_t>();
    o.lmodes = lmodes_.as<uint64_t>();
    o.umark = umark_.as<uint32_t>();
    o.mark_id = mark_id_;
    o.field = field_.as<float>();
    o.signs = signs_.p;
    o.counters = counters_.as<uint32_t>();
    o.claimed = claimed_.as<uint32_t>();
    o.mc = buffers();
    o.mc.offsets = offsets_.as<uint32_t>();
    return o;
}

void Engine::eval_points(const float* d_xyz, int64_t n, float* d_f, float* d_grad, hipStream_t s) {
    if (!have_object_) throw InputError("engine: no object set");
    if (const TreeJit::PointKernels* pk = point_jit(s)) {
        if (n <= 0) return;
        const float* m = d_mats();
        const float* tab = rabbit_.as<float>();
        void* args[] = {&m, &tab, &d_xyz, &n, &d_f, &d_grad};
        TreeJit::launch(pk->points, (unsigned)((n + 255) / 256), args, s, "impli_pt_points");
        IMPLI_HIP(hipGetLastError());
        return;
    }
    launch_eval_points(prog_.as<Program>(), depth_, rabbit_.as<float>(), d_xyz, n, d_f, d_grad, s);
    IMPLI_HIP(hipGetLastError());
}

}  // namespace impli
