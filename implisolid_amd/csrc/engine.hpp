// engine.hpp -- device-resident polygoniser state for one GPU (one Z-slab of one object).
#pragma once
#include <functional>
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "host.hpp"
#include "jit.hpp"
#include "kernels.hpp"

namespace impli {

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
void hip_check(hipError_t e, const char* what);
#define IMPLI_HIP(x) ::impli::hip_check((x), #x)

// grow-only device buffer.  Its memory comes from a per-device caching pool (engine.hip): a released
// block is reused for a later reserve of its size class only after a device synchronisation (the
// guarantee hipFree's implicit synchronisation gave), so an object stream's engines, created and
// destroyed batch after batch, allocate nothing after the first batch.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    bool ext = false;   // caller-owned memory (attach): never freed; a reserve past it allocates anew
    int dev = -1;       // the device the block was allocated on (its pool)
    void reserve(size_t n);
    void release();
    void attach(void* q, size_t n) {
        release();
        p = q;
        bytes = n;
        ext = true;
    }
    // the pool's cached bytes on every device: [0] reusable, [1] awaiting a device synchronisation,
    // [2] hipMalloc calls so far (reserves the pool could not serve), [3] hipFree calls
    static void pool_stats(size_t out[4]);
    // free every cached block of the current device (synchronises it)
    static void pool_trim();
    template <class T> T* as() const { return static_cast<T*>(p); }
};

// pinned host memory (grow-only), for device-to-host copies at full PCIe rate
struct HostBuf {
    void* p = nullptr;
    size_t bytes = 0;
    void reserve(size_t n);
    void release();
    template <class T> T* as() const { return static_cast<T*>(p); }
};

struct SlabCounts {
    uint32_t own_total, tri_total, act_total, halo_own;
    uint32_t n_verts() const { return own_total - halo_own; }
    uint32_t n_faces() const { return tri_total; }
};


// Balanced Z-slab cuts: nranks + 1 cell-layer boundaries (cuts[0] = 1, cuts[nranks] = R + 3) that
// split the grid's estimated work evenly.  The work of a cell layer is its lower sample layer's
// share of the bricks the pruned eval lists (field values + marching cubes scale with them) plus a
// small per-brick term for the interval / fill passes over every brick.  Runs the interval pass of
// the whole grid once on the current device (deterministic: every rank computes the same cuts).
std::vector<int> balance_cuts(const Program& prog, int R, const float box[6], int nranks, hipStream_t stream);
// the same from per-stored-layer listed-brick counts of the whole grid (host-only, tested on CPU)
std::vector<int> cuts_from_layer_work(const std::vector<int64_t>& listed_per_layer, int64_t bricks_per_layer, int R,
                                      int nranks);

struct ZeroRange { void* p; size_t n; };

class Engine {
public:
    // setup: the counter block's reset goes on this stream (an object stream's fresh engines, set up
    // back to back on it without device synchronisations), else on the null stream.  resets: the
    // fresh engine's buffer resets (here and in set_slab) are appended to it instead, for the caller
    // to clear on `setup` before any launch of the engine (launch_zero_pieces); detach_resets()
    // once the engine is set up
    explicit Engine(hipStream_t setup = nullptr, std::vector<ZeroRange>* resets = nullptr);
    ~Engine();

    // object + grid.  rank/nranks select a Z-slab of cell layers (rank 0 of 1 = whole grid), or
    // set_slab takes the slab's layer range itself (balanced cuts, balance_cuts below).
    // probe_only: allocate only what the interval pass needs (interval_pass, listed_per_layer).
    // d_prog: the program already on the device (an object stream uploads all its programs at once;
    // the engine reads it there, it must outlive the engine's use)
    void set_object(const Program& prog, const Program* d_prog = nullptr);
    void set_grid(int R, const float box[6], int rank, int nranks);
    // setup: a fresh engine's buffer resets go on this stream, without device synchronisations
    // (an object stream sets up its engines back to back; every later launch of theirs is on it)
    void set_slab(int R, const float box[6], const SlabRange& sr, bool probe_only = false, hipStream_t setup = nullptr);
    // an object stream's merged launches without a warm eval of this engine: the merged fill writes
    // its unit marks (id 1) from the first pass on
    void arm_merged();
    void detach_resets() { resets_ = nullptr; }
    // the pruned eval's interval and fill passes alone (no field values), then per stored sample
    // layer of the slab: the number of bricks listed for evaluation (blocking)
    void interval_pass(hipStream_t stream);
    std::vector<int64_t> listed_per_layer(hipStream_t stream);

    // the MC pipeline, all asynchronous on `stream`
    void eval_field(hipStream_t stream);
    void count(hipStream_t stream);                           // K2 + scan
    void emit(const uint32_t* d_offsets, hipStream_t stream); // K3 + K4 (offsets: [Voff, Foff] or null)
    void emit_verts(hipStream_t stream);                       // K3 alone (needs no offsets)
    // K4 alone; d_gathered (all ranks' copy_counts, uint32[world][4]) gives Voff on the device
    void emit_faces(const uint32_t* d_offsets, const uint32_t* d_gathered, int rank, hipStream_t stream);
    // host-side offsets used when emit() gets no device offsets
    void set_offsets(uint32_t voff, uint32_t foff);
    // blocking copy of this slab's emitted mesh
    void download(float* verts, int32_t* faces, const SlabCounts& c, hipStream_t stream);
    // blocking: totals of this slab and the overflow flag
    SlabCounts read_counts(hipStream_t stream, bool* overflow);
    // make sure the output buffers can hold the counted mesh (re-run emit() after growing)
    bool ensure_capacity(const SlabCounts& c);
    bool fits(const SlabCounts& c) const {   // the output buffers hold the counted mesh as they are
        return (int64_t)c.n_verts() + 1 <= cap_v_ && (int64_t)c.n_faces() + 1 <= cap_f_ &&
               (int64_t)c.act_total + 1 <= cap_rec_;
    }

    // whole single-GPU marching cubes: eval + count + emit (+ retry on overflow); returns counts
    SlabCounts marching_cubes(hipStream_t stream);
    // the same straight to host memory, with the copies overlapped: the counts are read back while
    // the emission kernels run, `host(nv, nf, &verts, &faces)` then sizes the host result, the
    // vertices' copy runs on copy_stream beside the face pass and the faces' copy follows it on
    // stream (blocking until both have landed)
    SlabCounts marching_cubes_to_host(hipStream_t stream, hipStream_t copy_stream,
                                      const std::function<void(int64_t, int64_t, float**, int32_t**)>& host);

    // this object's state for the merged launches of an object stream (kernels.hpp ObjArgs); the
    // pruned path after one eval_field (its unit marks), valid until the buffers grow
    ObjArgs obj_args() const;
    float2 tab_range() const { return tab_range_; }
    const CaseInfo* d_cases() const { return cases_.as<CaseInfo>(); }

    // direct evaluation at device points
    void eval_points(const float* d_xyz, int64_t n, float* d_f, float* d_grad, hipStream_t stream);

    const GridDesc& grid() const { return grid_; }
    float* d_verts() const { return verts_.as<float>(); }
    int32_t* d_faces() const { return faces_.as<int32_t>(); }
    float* d_field() const { return field_.as<float>(); }
    const uint64_t* d_signs() const { return signs_.as<uint64_t>(); }
    const uint32_t* d_counters() const { return counters_.as<uint32_t>(); }
    int depth() const { return depth_; }
    // the most values the object's postfix program holds at once (the value stacks' depth)
    int vdepth() const { return vdepth_; }
    const Program* d_program() const { return prog_.as<Program>(); }
    // true if the last eval_field ran the JIT-compiled tree kernel
    bool used_jit() const { return jit_fn_ != nullptr; }
    // ... and whether that was the object's baked module (TreeJit bake modes)
    bool used_baked() const { return jit_fn_ != nullptr && bake_slot_ && jit_fn_ == bake_slot_->k.bricks; }
    const float* d_rabbit() const { return rabbit_.as<float>(); }
    // the object's matrices as the JIT kernels read them (the Program's mats array)
    const float* d_mats() const;
    // the object's point module (OB02 passes, direct evaluation): requested on first use (compiled
    // in the background in async mode); null until loaded -- the interpreter kernels run meanwhile
    const TreeJit::PointKernels* point_jit(hipStream_t s = nullptr);

    DevBuf& scratch(int k) { return scratch_[k]; }
    // engines whose kernels are captured once (object streams): no switch to a baked module later
    void set_hot_bake(bool on) { allow_hot_bake_ = on; }

    // per-brick interval pruning of the field evaluation (process-wide level, default 2;
    // IMPLISOLID_PRUNE=<level> or implisolid_set_pruning(level)):
    //   0 off, 1 CSG operand pruning (field bit-identical), 2 + sign-only bricks (mesh bit-identical)
    static void set_pruning(int level);
    static int pruning();
    // per-kernel HIP-event timing of the next eval/count/emit calls (stream-ordered, no sync);
    // kernel_times() blocks and returns ms for: brick pass, field eval, MC count, unit scan,
    // vertex emission, face emission
    static constexpr int kTimedKernels = 6;
    void set_timing(bool on);
    void kernel_times(float out[kTimedKernels]);
    // the same, one figure per kernel: coarse interval pass, brick refine, fill, field eval, MC
    // count, unit scan, vertex emission (k_mc_cells), face emission (k_mc_faces)
    static constexpr int kTimedEachKernel = 8;
    void kernel_times_each(float out[kTimedEachKernel]);
    // raw device counters after count(): [active units, halo own, own, tri, act, halo] (blocking)
    void raw_counters(uint32_t out[16], hipStream_t stream);
    // brick statistics of the last pruned eval: [bricks, mixed, sign-filled]; blocking
    void brick_stats(int64_t out[3], hipStream_t stream);

private:
    MCBuffers buffers() const;

    GridDesc grid_{};
    int depth_ = 1;
    int vdepth_ = 1;
    int n_csg_ = 0;
    Program prog_host_{};
    TreeJit::Slot* jit_slot_ = nullptr;   // the object's module (null: JIT off); may still compile
    bool jit_requested_ = false;
    TreeJit::Slot* bake_slot_ = nullptr;  // its baked module (TreeJit bake modes), preferred once loaded
    bool bake_requested_ = false;
    int evals_ = 0;                        // evals of this object (hot objects get a baked module)
    bool allow_hot_bake_ = true;
    TreeJit::Slot* pt_slot_ = nullptr;     // the point module
    bool pt_requested_ = false;
    TreeJit::Slot* pt_bake_slot_ = nullptr;   // a hot object's point module with its matrices baked in
    bool pt_bake_requested_ = false;
    int pt_uses_ = 0;                         // point_jit calls since set_object (the hot-object count)
    hipFunction_t jit_fn_ = nullptr;       // what the last eval used (null: interpreter)
    bool counters_fresh_ = false;   // eval_field zeroed the counters; the next count() need not
    uint32_t mark_id_ = 0;          // id of the last pruned eval's unit marks (umark_)
    bool marks_valid_ = false;      // the last eval was pruned: count only marked units
    JitIntervalKernels jit_iv_;
    void ensure_jit(hipStream_t s = nullptr);
    void release_jit();   // drop the module references (after the device has synchronised)
    float2 tab_range_{0.f, 0.f};
    bool have_grid_ = false, have_object_ = false, probe_only_ = false;
    std::vector<ZeroRange>* resets_ = nullptr;   // a fresh engine's deferred resets (constructor)
    // the grid set_slab last built its buffers for: setting the same one again keeps them
    int key_R_ = -1, key_z0_ = 0, key_z1_ = 0;
    uint64_t obj_gen_ = 0, key_obj_gen_ = ~0ull;   // set_object's generation / the one the grid's buffers hold
    float key_box_[6] = {};
    HostBuf hcounters_;   // pinned landing zone of read_counts / raw_counters (one small copy)
    hipEvent_t ev_counts_ = nullptr, ev_verts_ = nullptr;   // marching_cubes_to_host
    DevBuf prog_, rabbit_, cases_;
    DevBuf offsets_, cmodes_, ccls_, clist_, modes_, cls_, fill_, blist_, field_, signs_, scan_blk_, unit_cnt_, unit_part_, unit_cmask_, ulist_, upart_, umark_, counters_, lmodes_, claimed_, vid_, records_, verts_, faces_;
    int64_t cap_v_ = 0, cap_f_ = 0, cap_rec_ = 0;
    bool timing_ = false;
    hipEvent_t ev_[11] = {};   // 0-8 phase boundaries, 9 after the coarse pass, 10 after refine
    void mark(int i, hipStream_t s) {
        if (timing_) IMPLI_HIP(hipEventRecord(ev_[i], s));
    }
    DevBuf scratch_[16];
};

}  // namespace impli
