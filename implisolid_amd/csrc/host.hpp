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

// basic_functions.hpp:77-128 invert_matrix (ublas LU on a float 4x4 with last row 0,0,0,1)
bool invert_matrix12(const float in[12], float out[12]);

}  // namespace impli
