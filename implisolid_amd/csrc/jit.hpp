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

#include <mutex>
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

    // C++ source of the brick kernel for this program's shape (no matrices in it)
    static std::string kernel_source(const Program& p);

    // hipRTC-compile the source to a gfx950 code object (no GPU needed); throws with the log
    static std::vector<char> compile(const std::string& src);

    // compiled kernels for this shape, compiling on first use; nullptr if disabled or if
    // compilation failed (the failure is logged once and the interpreter kernels are used)
    struct Kernels {
        hipFunction_t bricks = nullptr;   // brick-pruned field (eval_bricks_body)
        hipFunction_t coarse = nullptr;   // interval pass, coarse boxes (coarse_modes_body)
        hipFunction_t refine = nullptr;   // interval pass, bricks of mixed boxes (brick_refine_body)
    };
    Kernels kernels(const Program& p);

    // compile the kernels of many shapes on up to `threads` host threads (hipRTC runs outside the
    // cache lock); shapes already cached are skipped.  kernels() then finds them cached.
    void precompile(const std::vector<Program>& progs, int threads);

    // launch the compiled brick kernel (same contract as launch_eval_field_pruned's 2nd kernel)
    static void launch_bricks(hipFunction_t fn, const float* d_mats, const float* d_rabbit, const GridDesc& g,
                              const BrickGrid& bg, const uint64_t* d_modes, const uint32_t* d_list,
                              const uint32_t* d_count, float* d_field, void* d_signs, unsigned blocks, hipStream_t s);

    // launch a compiled kernel with 256-thread blocks; args as for hipModuleLaunchKernel
    static void launch(hipFunction_t fn, unsigned blocks, void** args, hipStream_t s, const char* what);

    bool enabled() const { return enabled_; }
    void set_enabled(bool on) { enabled_ = on; }
    int compiled() const { return n_compiled_; }
    double compile_seconds() const { return compile_s_; }

private:
    TreeJit();
    struct Entry {
        hipModule_t mod = nullptr;
        Kernels k;
    };
    std::mutex mu_;
    std::unordered_map<std::string, Entry> cache_;
    bool enabled_ = true;
    int n_compiled_ = 0;
    double compile_s_ = 0;
};

}  // namespace impli
