// host.hpp -- host side of the drop-in boundary: mc-settings parser, MP5 factory, matrix inverse.
#pragma once
#include <string>
#include <vector>

#include "json.hpp"
#include "program.hpp"

namespace impli {

// polygoniser_settings.hpp:8-85 mc_settings
struct MCSettings {
    float box[6] = {-1, 1, -1, 1, -1, 1};   // xmin, xmax, ymin, ymax, zmin, zmax
    int resolution = 28;
    bool ignore_root_matrix = false;
    int overall_repeats = 1;
    int vresampl_iters = 0;
    float vresampl_c = 1.0f;
    bool qem = false;
    bool projection = false;
    bool subdiv = true;
    float post_subdiv_noise = 0.01f;
};

// Errors the reference reports with abort() / clog.  The C ABI decides what to do with them
// (abort-compatible by default, see abi.cpp).
struct InputError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// parse_mc_properties_json (polygoniser_settings.hpp:147-305).  Throws InputError where the
// reference sets needs_abort.
MCSettings parse_mc_settings(const char* json_text);

// object_factory (object_factory.hpp:56-758) -> node program.  Throws InputError for unknown or
// unsupported node types (the reference abort()s on unknown ones, :731-734).
Program compile_mp5(const char* shape_json, bool ignore_root_matrix);
Program compile_mp5(const Json& shape, bool ignore_root_matrix);

// Z-slab decomposition of the cell layers 1 .. res-3 (res = R + 5) over nranks: rank r owns
// layers [z0, z1) and recomputes `halo` (0 or 1) layer below z0 (owner rule).
struct SlabRange { int z0, z1, halo; };
SlabRange slab_partition(int R, int rank, int nranks);
// the slab of cell layers [z0, z1); throws if its cells overflow the kernels' 32-bit cell ids
SlabRange slab_range(int R, int z0, int z1);

// glibc rand() / srand() restated (stdlib/random_r.c, TYPE_3: additive feedback
// x_n = x_{n-3} + x_{n-31} mod 2^32, output x_n >> 1; state seeded by the 16807 LCG, 310 outputs
// discarded).  randomize_verts (basic_functions.hpp:551-557) draws from the process-global rand() of
// the native reference build; the library keeps one process-global generator in that state (never
// seeded = srand(1), implisolid_srand to reseed), advanced only by subdivision.
//
// The state is kept as the window of the last 31 terms, so that n draws can be skipped (or handed
// to GPU lanes) with the polynomial z^n mod P(z), P = z^31 - z^28 - 1 over Z/2^32:
//   x_{m+n+j} = sum_i c_i x_{m+i+j}  where  z^n = sum_i c_i z^i  (mod P).
class GlibcRand {
public:
    explicit GlibcRand(unsigned seed = 1) { seed_(seed); }
    void seed_(unsigned seed);
    int32_t next();
    void fill(uint32_t* out, int64_t n) { for (int64_t i = 0; i < n; ++i) out[i] = (uint32_t)next(); }
    // x_m .. x_{m+60}: the window (oldest first) extended by 30 terms; draw k of the future is
    // produced from x_{m+k} and x_{m+k+28}
    void extended_window(uint32_t out[61]) const;
    void skip(uint64_t n);
private:
    uint32_t r_[31];
    int head_ = 0;   // r_[head_] is the oldest term x_{n-31}
};
GlibcRand& process_rand();

// z^n mod (z^31 - z^28 - 1), coefficients mod 2^32
void rand_jump_poly(uint64_t n, uint32_t c[31]);
void rand_poly_mulmod(const uint32_t a[31], const uint32_t b[31], uint32_t out[31]);

// basic_functions.hpp:77-128 invert_matrix (ublas LU on a float 4x4 with last row 0,0,0,1)
bool invert_matrix12(const float in[12], float out[12]);

}  // namespace impli
