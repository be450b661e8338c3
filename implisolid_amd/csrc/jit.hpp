// jit.hpp -- node programs compiled to straight-line device code (hipRTC), per tree shape.
//
// The interpreter (ifunc_device.hpp) pays for every node with scalar instruction fetches,
// dispatch branches and indexed stack moves.  For the hot brick kernel the tree is instead
// turned into one C++ function: each node a block of straight-line code calling the same
// primitive functions in the same order (bit-identical results), each CSG node a pair of
// wave-uniform branches driven by the brick's pruning modes.  Matrices stay data (read from the
// device Program), so the compiled module depends only on the tree's shape and is cached by it.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <string>
#include <unordered_map>
#include <vector>

#include "grid.hpp"
#include "program.hpp"

namespace impli {

class TreeJit {
public:
    // process-wide instance; IMPLISOLID_JIT=0 disables compilation (interpreter only)
    static TreeJit& instance();

    // C++ source of the tree kernels for this program's shape (no matrices in it), or with the
    // object's transformation matrices baked in as exact literals (bake: one module per object,
    // no matrix loads on the kernels' dependency chains)
    static std::string kernel_source(const Program& p, bool bake = false);
    // C++ source of the point kernels for this shape (OB02 passes and direct evaluation,
    // ob02_device.hpp over straight-line f / (f, grad) code; NaN-exact: no transform specialisation)
    static std::string point_source(const Program& p, bool bake = false);

    // hipRTC-compile the source to a gfx950 code object (no GPU needed); throws with the log
    static std::vector<char> compile(const std::string& src);

    struct Kernels {
        hipFunction_t bricks = nullptr;   // brick-pruned field (eval_bricks_body)
        hipFunction_t coarse = nullptr;   // interval pass, coarse boxes (coarse_modes_body)
        hipFunction_t refine = nullptr;   // interval pass, bricks of mixed boxes (brick_refine_body)
    };
    struct PointKernels {                 // the point module (ob02_device.hpp bodies)
        hipFunction_t cnormals = nullptr, prep = nullptr, early = nullptr, early2 = nullptr, late = nullptr,
                      normals = nullptr, points = nullptr;   // early2: the early search with 2 lanes per face
    };
    enum Kind { kBricks = 0, kPoints = 1 };
    // One compiled module (one source on one device).  `ready` is set (release) once `k` holds the
    // loaded kernels, `failed` if compilation or loading failed.  request() takes a reference and
    // release() drops it; the cache holds at most max_modules() slots and, past that, unloads the
    // least recently requested finished slots nobody references (IMPLISOLID_JIT_MAX_MODULES,
    // default 1024; a long-lived service polygonising ever-new objects keeps bounded device memory).
    // Unloads run at trim() (set_object, wait_idle: device already synchronised); request() itself
    // evicts only when the cache is 4x over the bound, which is therefore the hard bound in between.
    struct Slot {
        std::atomic<bool> ready{false}, failed{false};
        Kernels k;
        PointKernels pk;
        int kind = kBricks;
        hipModule_t mod = nullptr;
        std::string src;
        std::string key;
        int device = 0;
        int refs = 0;             // guarded by mu_
        uint64_t last_use = 0;    // request tick, guarded by mu_
    };
    // Modes (IMPLISOLID_JIT=0|1|2, implisolid_set_jit):
    //   0 off: the interpreter kernels only;
    //   1 sync: request() compiles before it returns (the first call of a new shape waits for hipRTC);
    //   2 async (default): request() returns at once; compilation runs on background threads and the
    //     engine uses the interpreter kernels until the module is ready -- a never-seen shape costs
    //     no compile latency.  Code objects persist in a disk cache (IMPLISOLID_JIT_CACHE=<dir>,
    //     default $XDG_CACHE_HOME or ~/.cache /implisolid_amd; "off" disables it), trimmed to the
    //     IMPLISOLID_JIT_CACHE_MAX (2048) most recently used entries once per process.
    // Variants: shape modules keep the matrices as data (one module per tree shape); baked modules
    // hold the object's matrices as literals (one per object: no matrix loads on the dependency
    // chains, 5 % faster at 512^3).  Bake modes (IMPLISOLID_JIT_BAKE, implisolid_set_jit_bake):
    //   0 never; 1 every object; 2 (default) hot objects -- an engine evaluating the same object
    //   kBakeAfter times requests its baked module (in the background in async mode) and switches
    //   to it once loaded, so objects that change every call never compile one.
    enum Mode { kOff = 0, kSync = 1, kAsync = 2 };
    enum BakeMode { kBakeNever = 0, kBakeAlways = 1, kBakeHot = 2 };
    static constexpr int kBakeAfter = 4;
    // `stream`: the caller's launch stream; while it is being captured into a graph no module is
    // unloaded (an unload synchronises the device), the cache is trimmed by a later request
    Slot* request(const Program& p, int kind = kBricks, bool bake = false, hipStream_t stream = nullptr);
    // drop a reference taken by request() (null is ignored); the caller launches nothing from the
    // slot afterwards and has synchronised whatever it launched
    void release(Slot* slot);
    int modules() const;
    int max_modules() const { return max_modules_.load(); }
    void set_max_modules(int n) { max_modules_.store(n < 8 ? 8 : n); }
    int deferred_evictions() const { return n_deferred_.load(); }
    // block until every scheduled compilation has finished (bench / batch setup)
    void wait_idle();   // ... then trim()
    // unload the least recently used modules nobody holds while the cache is over its bound (a
    // device synchronisation): called where the device is synchronised anyway (Engine::set_object)
    void trim();
    // compile the modules of many programs (sync, up to `threads` host threads); request() then
    // finds them ready.  Returns one reference per program (null where JIT is off or the source
    // failed), which the caller releases once its engines hold their own: until then the module
    // bound cannot evict them.
    std::vector<Slot*> precompile(const std::vector<Program>& progs, int threads);

    // launch the compiled brick kernel (same contract as launch_eval_field_pruned's 2nd kernel)
    static void launch_bricks(hipFunction_t fn, const float* d_mats, const float* d_rabbit, const GridDesc& g,
                              const BrickGrid& bg, const uint64_t* d_modes, const uint32_t* d_list,
                              const uint32_t* d_count, float* d_field, void* d_signs, const ClaimCtx& cc,
                              unsigned blocks, hipStream_t s);

    // launch a compiled kernel with 256-thread blocks; args as for hipModuleLaunchKernel
    static void launch(hipFunction_t fn, unsigned blocks, void** args, hipStream_t s, const char* what);

    int mode() const { return mode_.load(); }
    void set_mode(int m) { mode_.store(m < 0 ? 0 : m > 2 ? 2 : m); }
    int bake() const { return bake_.load(); }
    void set_bake(int b) { bake_.store(b < 0 ? 0 : b > 2 ? 2 : b); }
    bool enabled() const { return mode() != kOff; }
    void set_enabled(bool on) { set_mode(on ? kAsync : kOff); }
    int compiled() const { return n_compiled_.load(); }
    int disk_hits() const { return n_disk_.load(); }
    int evicted() const { return n_evicted_.load(); }
    double compile_seconds() const;

private:
    TreeJit();
    void build(Slot* slot);            // compile (or read from disk) + load; sets ready / failed
    void worker();
    void shutdown();
    void evict_locked(std::vector<Slot*>& out, bool defer);   // pick slots to unload (mu_ held)
    static bool defer_eviction(hipStream_t stream);           // is the caller's stream capturing?
    void unload(std::vector<Slot*>& slots);       // unload and free them (mu_ not held)
    mutable std::mutex mu_;
    uint64_t tick_ = 0;
    std::atomic<int> max_modules_{1024};
    std::atomic<int> n_evicted_{0}, n_deferred_{0};
    std::condition_variable cv_, idle_cv_;
    std::unordered_map<std::string, Slot*> cache_;   // key: device + source
    std::deque<Slot*> queue_;
    std::vector<std::thread> workers_;
    int busy_ = 0;
    bool stop_ = false;
    std::atomic<int> mode_{kAsync};
    std::atomic<int> bake_{kBakeHot};
    std::atomic<int> n_compiled_{0}, n_disk_{0};
    std::atomic<int64_t> compile_us_{0};
    std::string disk_dir_;
};

// the point modules' early projection pass: the two-loop form by default; IMPLISOLID_EARLY_SM=1
// selects the single-loop form (ob02_device.hpp project_early_sm_body, an experiment: slower) and
// IMPLISOLID_EARLY_CHUNK its faces per wave chunk (default 64)
bool early_single_loop();
int early_chunk();

}  // namespace impli
