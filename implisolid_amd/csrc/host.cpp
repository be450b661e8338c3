// host.cpp -- mc-settings parser, MP5-JSON -> node-program compiler, float LU inverse.
#include "host.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>

namespace impli {

// ---------------------------------------------------------------------------------------------
// basic_functions.hpp:77-128.  ublas lu_factorize: per column the first row with the largest |a|
// is the pivot (index_norm_inf), the sub-column is scaled by value_type(1)/pivot, the trailing
// block gets m(r,c) -= l(r)*u(c); lu_substitute: row swaps, unit-lower forward solve, upper back
// solve with "t = e(n,l) /= u(n,n); if (t != 0) e(m,l) -= u(m,n)*t" (triangular.hpp).
bool invert_matrix12(const float in[12], float out[12]) {
    float a[4][4];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c) a[r][c] = in[r * 4 + c];
    a[3][0] = a[3][1] = a[3][2] = 0.f;
    a[3][3] = 1.f;
    int perm[4] = {0, 1, 2, 3};
    for (int i = 0; i < 4; ++i) {
        int piv = i;
        float best = 0.f;
        for (int r = i; r < 4; ++r) {
            float u = std::fabs(a[r][i]);
            if (u > best) { best = u; piv = r; }
        }
        if (a[piv][i] == 0.f) return false;   // singular: the reference returns false, matrix untouched
        if (piv != i) {
            perm[i] = piv;
            for (int c = 0; c < 4; ++c) std::swap(a[piv][c], a[i][c]);
        }
        const float inv = 1.f / a[i][i];
        for (int r = i + 1; r < 4; ++r) a[r][i] *= inv;
        for (int r = i + 1; r < 4; ++r)
            for (int c = i + 1; c < 4; ++c) {
                const float p = a[r][i] * a[i][c];
                a[r][c] -= p;
            }
    }
    float e[4][4];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) e[r][c] = (r == c) ? 1.f : 0.f;
    for (int i = 0; i < 4; ++i)
        if (perm[i] != i)
            for (int c = 0; c < 4; ++c) std::swap(e[i][c], e[perm[i]][c]);
    for (int n = 0; n < 4; ++n)
        for (int l = 0; l < 4; ++l) {
            const float t = e[n][l];
            if (t != 0.f)
                for (int m = n + 1; m < 4; ++m) {
                    const float p = a[m][n] * t;
                    e[m][l] -= p;
                }
        }
    for (int n = 3; n >= 0; --n)
        for (int l = 3; l >= 0; --l) {
            const float t = (e[n][l] /= a[n][n]);
            if (t != 0.f)
                for (int m = n - 1; m >= 0; --m) {
                    const float p = a[m][n] * t;
                    e[m][l] -= p;
                }
        }
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c) out[r * 4 + c] = e[r][c];
    return true;
}

// ---------------------------------------------------------------------------------------------
MCSettings parse_mc_settings(const char* text) {
    Json d;
    try {
        d = Json::parse(text);
    } catch (const JsonError& e) {
        throw InputError(e.what());
    }
    MCSettings s;
    std::string why;
    float box[6];
    const char* keys[6] = {"box.xmin", "box.xmax", "box.ymin", "box.ymax", "box.zmin", "box.zmax"};
    bool ok = true;
    for (int i = 0; i < 6; ++i) {
        float v;
        if (!d.get_float(keys[i], &v) || std::isnan(v)) ok = false;
        box[i] = v;
    }
    if (!ok) {   // :176-191
        for (int i = 0; i < 6; ++i) box[i] = (i % 2) ? 1.f : -1.f;
        why += "  err2 (missing or incorrect box)";
    }
    std::memcpy(s.box, box, sizeof box);
    {   // :193-206 resolution must be an integer-valued number
        const float r = d.get_float("resolution", -1.f);
        // a value no int holds (or NaN) is not an integer resolution: converting it would be
        // undefined behaviour (the reference's cast is; found by the host sanitizer run)
        const bool fits = r > -2147483648.f && r < 2147483648.f;
        int ri = fits ? (int)r : 0;
        if (ri == -1) ri = 28;
        if (!fits || (float)ri != r) why += "  err3 (resolution must be integer)";
        s.resolution = ri;
        if (s.resolution <= 2) why += "  err4 (resolution must be > 2)";
    }
    s.vresampl_c = d.get_float("vresampl.c", 1.0f);
    s.vresampl_iters = d.get_int("vresampl.iters", 0);
    auto read_bool = [&](const char* name, bool dflt, const char* forbidden) {   // :107-141
        int v = d.get_int(name, -1);
        bool r = (v == -1) ? dflt : (v != 0);
        if (d.get_int(forbidden, 9123456) != 9123456) why += std::string("  use ") + name;
        return r;
    };
    s.projection = read_bool("projection.enabled", false, "projection.enable");
    s.qem = read_bool("qem.enabled", false, "qem.enable");
    s.subdiv = read_bool("subdiv.enabled", true, "subdiv.enable");
    s.post_subdiv_noise = d.get_float("debug.post_subdiv_noise", 0.01f);
    s.overall_repeats = d.get_int("overall_repeats", 1);
    s.ignore_root_matrix = d.get_bool("ignore_root_matrix", false);
    if (s.qem && !s.projection) why += "  err7 (qem needs projection)";
    if (s.resolution > 65535) why += "  resolution exceeds the reference's dim_t";
    if (!why.empty()) throw InputError("Aborting because of a problem in mc_settings_from_json. Abort reasons: " + why);
    return s;
}

// ---------------------------------------------------------------------------------------------
namespace {

struct Builder {
    Program p{};
    int depth = 0, max_depth = 0;

    int add_matrix(const float m[12]) {
        if (p.n_mats >= kMaxProgram) throw InputError("MP5 tree too large");
        float inv[12];
        if (!invert_matrix12(m, inv)) throw InputError("singular MP5 matrix");
        std::memcpy(p.mats[p.n_mats], inv, sizeof inv);
        return p.n_mats++;
    }
    int emit(OpCode op, int32_t type, int32_t mat, int32_t csg = -1) {
        if (p.n_instr >= kMaxProgram) throw InputError("MP5 tree too large");
        p.instr[p.n_instr] = Instr{(int16_t)op, (int16_t)type, (int16_t)mat, (int16_t)csg, -1, -1, -1, 0};
        return p.n_instr++;
    }

    static void matrix12(const Json& d, float m[12]) {   // getMatrix12 object_factory.hpp:21-30
        const Json* mj = d.find("matrix");
        if (!mj || mj->kind != Json::Array || mj->items.size() < 12)
            throw InputError("MP5 node needs a 12- or 16-entry \"matrix\"");
        for (int i = 0; i < 12; ++i) {
            float v;
            if (!mj->items[i].second.as_float(&v)) throw InputError("bad matrix entry");
            m[i] = v;
        }
    }

    // raw parameters (not inverted) for primitives that carry them (Instr::prm): ceil(n / 12)
    // consecutive rows of mats[], read as one float array
    int add_params(const float* v, int n) {
        const int rows = (n + 11) / 12;
        if (p.n_mats + rows > kMaxProgram) throw InputError("MP5 tree too large");
        const int first = p.n_mats;
        for (int r = 0; r < rows; ++r) {
            float row[12] = {};
            const int k = std::min(12, n - 12 * r);
            std::memcpy(row, v + 12 * r, sizeof(float) * (size_t)k);
            std::memcpy(p.mats[p.n_mats++], row, sizeof row);
        }
        return first;
    }

    // A "subtree" pushes exactly one value; it sees the parent's local point on top of the stack.
    void leaf(NodeType t, const float m[12], const float* prm = nullptr, int nprm = 0) {
        const int k = add_matrix(m);
        const int pr = prm ? add_params(prm, nprm) : 0;
        emit(OP_XFORM, t, k);
        push_point();
        const int pc = emit(OP_PRIM, t, k);
        p.instr[pc].prm = (int16_t)pr;
        pop_point();
    }

    // screw::getScrewParameters (screw.hpp:380-470) + constructor (:222-330), in float: outer =
    // |v| = 1 for v = (0,1,0), inner = outer / delta_ratio, r0 = inner / 2, delta = outer / 2 -
    // inner / 2, twist_rate = pitch.  ptree get_child/get throw on the missing keys (values unused).
    static void screw_params(const Json& d, float prm[3]) {
        for (const char* k : {"matrix", "v", "pitch", "profile", "end_type", "delta_ratio"})
            if (!d.find(k)) throw InputError(std::string("screw: missing \"") + k + "\"");
        float pitch, ratio;
        if (!d.get_float("pitch", &pitch) || !d.get_float("delta_ratio", &ratio))
            throw InputError("screw: pitch and delta_ratio must be numbers");
        const float outer = 1.0f, inner = outer / ratio;
        prm[0] = pitch;
        prm[1] = inner / 2;
        prm[2] = outer / 2 - inner / 2;
    }
    // half_plane constructor (half_plane.hpp:96-125): plane_vector / |plane_vector| in float, the
    // norm reduced a0 + (a1 + a2); prm = {unit vector, plane_point}
    static void half_plane_params(const float pv[3], const float pp[3], float prm[6]) {
        const float n = std::sqrt(pv[0] * pv[0] + (pv[1] * pv[1] + pv[2] * pv[2]));
        for (int k = 0; k < 3; ++k) {
            prm[k] = pv[k] / n;
            prm[3 + k] = pp[k];
        }
    }
    // tetrahedron (tetrahedron.hpp:20-128; getCorners object_factory.hpp:32-45, a missing corner
    // stays 0): corners moved by the forward node matrix (matrix_vector_product,
    // basic_functions.hpp:140-177), the four calculatePlaneCoefficients planes, each multiplied by
    // the sign (ROOT_TOLERANCE, configs.hpp:33) of its value at the opposite corner
    static void tetra_params(const Json& d, const float m[12], float out[16]) {
        float c[4][3] = {};
        if (const Json* cs = d.find("corners")) {
            if (cs->kind != Json::Array) throw InputError("tetrahedron: \"corners\" must be an array");
            for (size_t i = 0; i < cs->items.size() && i < 4; ++i) {
                const Json& cj = cs->items[i].second;
                for (size_t j = 0; j < cj.items.size() && j < 3; ++j)
                    if (!cj.items[j].second.as_float(&c[i][j])) throw InputError("tetrahedron: bad corner");
            }
        } else {
            throw InputError("tetrahedron: missing \"corners\"");
        }
        float p[4][3];
        for (int i = 0; i < 4; ++i)
            for (int r = 0; r < 3; ++r)
                p[i][r] = m[4 * r] * c[i][0] + m[4 * r + 1] * c[i][1] + m[4 * r + 2] * c[i][2] + m[4 * r + 3];
        auto coef = [](const float* P1, const float* P2, const float* P3, float* o) {
            const float x1 = P1[0], y1 = P1[1], z1 = P1[2], x2 = P2[0], y2 = P2[1], z2 = P2[2], x3 = P3[0], y3 = P3[1],
                        z3 = P3[2];
            o[0] = y1 * z2 - y1 * z3 - y2 * z1 + y2 * z3 + y3 * z1 - y3 * z2;
            o[1] = x1 * z3 - x1 * z2 + x2 * z1 - x2 * z3 - x3 * z1 + x3 * z2;
            o[2] = x1 * y2 - x1 * y3 - x2 * y1 + x2 * y3 + x3 * y1 - x3 * y2;
            o[3] = x1 * y3 * z2 - x1 * y2 * z3 + x2 * y1 * z3 - x2 * y3 * z1 - x3 * y1 * z2 + x3 * y2 * z1;
        };
        coef(p[1], p[2], p[3], out);
        coef(p[0], p[2], p[3], out + 4);
        coef(p[0], p[1], p[3], out + 8);
        coef(p[0], p[1], p[2], out + 12);
        const float tol = (float)(0.001 / 10.0);
        for (int k = 0; k < 4; ++k) {
            float* P = out + 4 * k;
            const float v = P[0] * p[k][0] + P[1] * p[k][1] + P[2] * p[k][2] + P[3];
            const float sg = (v > +tol) ? 1.0f : (v < -tol) ? -1.0f : 0.0f;   // sign(), basic_functions.hpp:22-31
            for (int j = 0; j < 4; ++j) P[j] *= sg;
        }
    }
    // meta_ball_Rydgard (meta_balls_Rydgard.hpp:27-60): 4 blobs, scale 1; ball centres in double
    // (libm sin / cos) stored to float; strength 1.2 / ((sqrt(4) - 1) / 4 + 1), subtract 12
    static void metaball_params(const Json& d, float out[20]) {
        float time = 0.1f;   // get<REAL>("time", 0.1)
        if (d.find("time") && !d.get_float("time", &time)) throw InputError("meta_balls: bad \"time\"");
        const int numblobs = 4;
        for (int i = 0; i < numblobs; ++i) {
            const float x0 = 0.5f, y0 = 0.5f, z0 = 0.5f, D = 1;
            const float ballx = (float)(std::sin(i + 1.26 * time * (1.03 + 0.5 * std::cos(0.21 * i))) * 0.27 * D + 0.5 - x0);
            const float bally = (float)(std::abs(std::cos(i + 1.12 * time * std::cos(1.22 + 0.1424 * i))) * 0.77 * D - y0);
            const float ballz = (float)(std::cos(i + 1.32 * time * 0.1 * std::sin((0.92 + 0.53 * i))) * 0.27 * D + 0.5 - z0);
            const float subtract = 12;
            const float strength = (float)(1.2 / ((std::sqrt((double)numblobs) - 1) / 4 + 1));
            const float v[5] = {ballx, bally, ballz, strength, subtract};
            std::memcpy(out + 5 * i, v, sizeof v);
        }
    }
    // extrusion(eye, size) (extrusion.hpp:61-94) with convex_polygon::update_inner_data
    // (2d/GDT/convex_polygon.hpp:77-93): regular size-gon of radius 0.5 from (0, 0.5),
    // polarToCartesian (basic_functions.hpp:33-36) through std::cos/sin(float); 1/d in double
    static int extrusion_params(const Json& d, float* out) {
        float fs;
        if (!d.get_float("size", &fs)) throw InputError("extrusion: missing \"size\"");
        if (!(fs > -2147483648.f && fs < 2147483648.f)) throw InputError("extrusion: Invalid size");   // no int holds it
        const int size = (int)fs;
        if (size < 3) throw InputError("extrusion: Invalid size");
        if (size > 40) throw InputError("extrusion: size above 40 is not supported");
        const float PI = (float)3.141592653589793238463;   // basic_functions.hpp:8
        const float rot = 2 * PI / size;
        std::vector<float> cx{0.f}, cy{0.5f};
        const float radius = 0.5f;
        for (int i = 1; i < size; ++i) {
            const float theta = (float)(PI / 2.0 + i * rot);
            cx.push_back(radius * std::cos(theta));
            cy.push_back(radius * std::sin(theta));
        }
        out[0] = (float)size;
        for (int i = 0; i < size; ++i) {
            const int j = (i < size - 1) ? i + 1 : 0;
            const float dx = cx[j] - cx[i], dy = cy[j] - cy[i];
            const float dd = std::sqrt(dx * dx + dy * dy);
            const float dinv = (float)((dd > 0.00000001) ? 1.0 / dd : 0.0);
            const float nx = +dy * dinv, ny = -dx * dinv;
            out[1 + 3 * i] = nx;
            out[2 + 3 * i] = ny;
            out[3 + 3 * i] = cx[i] * nx + cy[i] * ny;
        }
        return 1 + 3 * size;
    }

    static void vec3(const Json& d, const char* key, float out[3]) {
        const Json* a = d.find(key);
        if (!a || a->kind != Json::Array || a->items.size() < 3) throw InputError(std::string("half_plane: bad \"") + key + "\"");
        for (int k = 0; k < 3; ++k)
            if (!a->items[k].second.as_float(&out[k])) throw InputError(std::string("half_plane: bad \"") + key + "\"");
    }
    void push_point() { if (++depth > max_depth) max_depth = depth; if (depth >= kMaxDepth) throw InputError("MP5 tree too deep"); }
    void pop_point() { --depth; }

    // node = XFORM(m); child a; child b; CSG(t).  Each operand subtree starts with its own XFORM,
    // which records where the subtree ends so a pruned operand can be skipped in one jump.
    template <class A, class B>
    void csg(NodeType t, const float m[12], A&& a, B&& b) {
        const int k = add_matrix(m);
        const int id = p.n_csg++;
        emit(OP_XFORM, t, k);
        push_point();
        const int a0 = p.n_instr;
        a();
        mark_operand(a0, id, 0);
        const int b0 = p.n_instr;
        b();
        mark_operand(b0, id, 1);
        emit(OP_CSG, t, k, id);
        pop_point();
    }
    void mark_operand(int start, int csg_id, int child) {
        p.instr[start].skip_csg = (int16_t)csg_id;
        p.instr[start].skip_child = (int16_t)child;
        p.instr[start].skip_to = (int16_t)p.n_instr;
    }

    void node(const Json& d, bool ignore) {
        static const float eye[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        std::string t = d.get_string("type", "");
        float m[12];
        struct { const char* name; NodeType t; } prims[] = {
            {"implicit_double_mushroom", NT_DMUSHROOM},        // object_factory.hpp:86-100
            {"icube", NT_CUBE}, {"cube", NT_CUBE},             // :110-119 (rabbit SDF, F3)
            {"icylinder", NT_CYLINDER}, {"cylinder", NT_CYLINDER},  // :121-132
            {"iellipsoid", NT_ELLIPSOID}, {"ellipsoid", NT_ELLIPSOID},  // :134-143
            {"icone", NT_CONE}, {"cone", NT_CONE},             // :144-152
            {"iheart", NT_HEART},                              // :153-162
            {"itorus", NT_TORUS},                              // :163-173
        };
        for (auto& pr : prims)
            if (t == pr.name) {
                matrix12(d, m);
                if (ignore) std::memcpy(m, eye, sizeof m);
                leaf(pr.t, m);
                return;
            }
        if (t == "Union") {   // :537-580: left-deep chain, identity on the intermediate unions
            matrix12(d, m);
            if (ignore) std::memcpy(m, eye, sizeof m);
            const Json* ch = d.find("children");
            if (!ch || ch->kind != Json::Array || ch->items.size() < 2)
                throw InputError("Union needs at least two children");
            union_chain(*ch, (int)ch->items.size() - 1, m);
            return;
        }
        if (t == "Intersection" || t == "Difference") {   // :581-653, binary
            matrix12(d, m);
            if (ignore) std::memcpy(m, eye, sizeof m);
            const Json* ch = d.find("children");
            if (!ch || ch->kind != Json::Array || ch->items.size() < 2)
                throw InputError(t + " needs two children");
            csg(t == "Intersection" ? NT_INTERSECTION : NT_DIFFERENCE, m,
                [&] { node(ch->items[0].second, false); }, [&] { node(ch->items[1].second, false); });
            return;
        }
        if (t == "screw" || t == "inf_screw" || t == "screw_diff_two_plane") {
            float prm[3];
            screw_params(d, prm);
            matrix12(d, m);
            if (ignore) std::memcpy(m, eye, sizeof m);
            if (t == "inf_screw") {   // object_factory.hpp:189-215: the screw under its own matrix
                leaf(NT_SCREW, m, prm, 3);
                return;
            }
            if (t == "screw") {       // :304-351: subtract(screw(identity), top_bottom_lid)
                csg(NT_DIFFERENCE, m, [&] { leaf(NT_SCREW, eye, prm, 3); }, [&] { leaf(NT_LID, eye); });
                return;
            }
            // :216-302: subtract(subtract(screw, half_plane z >= 0.25), half_plane z <= -0.25)
            const float up[3] = {0, 0, 1}, upp[3] = {0, 0, 0.25f}, dn[3] = {0, 0, -1}, dnp[3] = {0, 0, -0.25f};
            float top[6], bot[6];
            half_plane_params(up, upp, top);
            half_plane_params(dn, dnp, bot);
            csg(NT_DIFFERENCE, m,
                [&] { csg(NT_DIFFERENCE, eye, [&] { leaf(NT_SCREW, eye, prm, 3); }, [&] { leaf(NT_HALF_PLANE, eye, top, 6); }); },
                [&] { leaf(NT_HALF_PLANE, eye, bot, 6); });
            return;
        }
        if (t == "screw_gradient_wrong") {
            // :435-479: inf_top_bot_bound(T, screw(T)) -- the screw under the JSON matrix T (no
            // ignore_root_matrix here) bounded by the lid at the same x' = T^-1 x.  The node's
            // gradient applies T^-T twice (inf_top_bot_bound.hpp:142-166 over screw.hpp:476-486),
            // so the primitive carries a copy of the inverse
            float prm[24] = {};
            screw_params(d, prm);
            matrix12(d, m);
            if (!invert_matrix12(m, prm + 12)) throw InputError("singular MP5 matrix");
            leaf(NT_SCREW_TBB, m, prm, 24);
            return;
        }
        if (t == "top_bottom_lid") {   // :480-506: the matrix is read (get_child) and never applied
            matrix12(d, m);
            leaf(NT_LID, eye);
            return;
        }
        if (t == "half_plane") {       // :396-434
            float pv[3], pp[3], prm[6];
            vec3(d, "plane_vector", pv);
            vec3(d, "plane_point", pp);
            matrix12(d, m);
            if (ignore) std::memcpy(m, eye, sizeof m);
            half_plane_params(pv, pp, prm);
            leaf(NT_HALF_PLANE, m, prm, 6);
            return;
        }
        if (t == "tetrahedron") {      // :175-188: the corners are moved, the object itself is not
            float prm[16];
            matrix12(d, m);
            if (ignore) std::memcpy(m, eye, sizeof m);
            tetra_params(d, m, prm);
            leaf(NT_TETRA, eye, prm, 16);
            return;
        }
        if (t == "meta_balls") {       // :654-673
            float prm[20];
            matrix12(d, m);
            if (ignore) std::memcpy(m, eye, sizeof m);
            metaball_params(d, prm);
            leaf(NT_METABALLS, m, prm, 20);
            return;
        }
        if (t == "extrusion") {        // :674-731: subtract(extrusion(eye, size), top_bottom_lid)
            float prm[1 + 3 * 40];
            matrix12(d, m);
            if (ignore) std::memcpy(m, eye, sizeof m);
            const int n = extrusion_params(d, prm);
            csg(NT_DIFFERENCE, m, [&] { leaf(NT_EXTRUSION, eye, prm, n); }, [&] { leaf(NT_LID, eye); });
            return;
        }
        static const char* unsupported[] = {"sdf_3d", "rawjscode"};
        for (auto* u : unsupported)
            if (t == u) throw InputError("MP5 type \"" + t + "\" is outside the implemented node families");
        throw InputError("Invalid object you asked for: \"" + t + "\"");
    }

    // union of children[0..k] = U(union of children[0..k-1], children[k]) with matrix m at the top
    void union_chain(const Json& ch, int k, const float m[12]) {
        static const float eye[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        if (k == 0) {
            node(ch.items[0].second, false);
            return;
        }
        csg(NT_UNION, m, [&] { union_chain(ch, k - 1, eye); }, [&] { node(ch.items[k].second, false); });
    }
};

}  // namespace

Program compile_mp5(const Json& shape, bool ignore_root_matrix) {
    Builder b;
    b.node(shape, ignore_root_matrix);
    b.p.max_depth = b.max_depth + 1;
    for (int i = 0; i < b.p.n_instr; ++i) {   // XFORM patterns (program.hpp XformPattern)
        Instr& I = b.p.instr[i];
        if (I.op != OP_XFORM) continue;
        const float* m = b.p.mats[I.mat];
        bool diag = true;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) {
                const float v = m[4 * r + c];
                uint32_t bits;
                std::memcpy(&bits, &v, 4);
                if (!std::isfinite(v)) diag = false;
                else if (c == 3 && bits == 0x80000000u) diag = false;   // a -0 translation
                else if (c != 3 && c != r && v != 0.f) diag = false;
            }
        I.type = diag ? XF_DIAG : XF_GENERIC;
    }
    return b.p;
}

Program compile_mp5(const char* shape_json, bool ignore_root_matrix) {
    Json d;
    try {
        d = Json::parse(shape_json);
    } catch (const JsonError& e) {
        throw InputError(e.what());
    }
    return compile_mp5(d, ignore_root_matrix);
}

// the largest resolution the settings parser accepts (the reference's dim_t, polygoniser_settings.hpp)
constexpr int kMaxResolution = 65535;

SlabRange slab_range(int R, int z0, int z1) {
    if (R < 1 || R > kMaxResolution) throw InputError("slab_range: resolution out of range");
    const int layers = (R + 5) - 3;   // cell layers 1 .. res-3
    if (z0 < 1 || z1 <= z0 || z1 > layers + 1) throw InputError("slab_range: bad layer range");
    SlabRange r{z0, z1, z0 > 1 ? 1 : 0};
    // 32-bit indexing of one slab (mc_types.hpp / mc_device.hpp): the cell id L of a slab's cells
    // (halo layer included) is a uint32, and so are vertex ids, face rows and the MC counters.
    const int64_t m = (int64_t)R + 2, cells = m * m * (int64_t)(z1 - z0 + r.halo);
    if (cells >= (int64_t)1 << 32)
        throw InputError("slab of " + std::to_string(cells) + " cells exceeds the 2^32-cell limit of one slab (R = " +
                         std::to_string(R) + "): split the grid over more Z-slabs");
    return r;
}

SlabRange slab_partition(int R, int rank, int nranks) {
    if (R < 1 || R > kMaxResolution || nranks < 1 || rank < 0 || rank >= nranks) throw InputError("slab_partition: bad arguments");
    const int layers = (R + 5) - 3;   // cell layers 1 .. res-3
    if (nranks > layers) throw InputError("slab_partition: more slabs than cell layers");
    const int base = layers / nranks, extra = layers % nranks;
    const int z0 = 1 + rank * base + (rank < extra ? rank : extra);
    return slab_range(R, z0, z0 + base + (rank < extra ? 1 : 0));
}

void GlibcRand::seed_(unsigned seed) {   // srandom_r (random_r.c:161-196)
    int32_t word = seed == 0 ? 1 : (int32_t)seed;
    r_[0] = (uint32_t)word;
    for (int i = 1; i < 31; ++i) {        // 16807 * word mod (2^31 - 1), Schrage's method
        const int32_t hi = word / 127773, lo = word % 127773;
        word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        r_[i] = (uint32_t)word;
    }
    head_ = 3;                            // fptr = &state[SEP_3] holds the oldest term
    for (int i = 0; i < 310; ++i) next();
}

int32_t GlibcRand::next() {               // random_r (random_r.c:353-394): *fptr += *rptr
    int b = head_ + 28;
    if (b >= 31) b -= 31;
    const uint32_t v = r_[head_] + r_[b];
    r_[head_] = v;
    if (++head_ == 31) head_ = 0;
    return (int32_t)(v >> 1);
}

void GlibcRand::extended_window(uint32_t out[61]) const {
    for (int j = 0; j < 31; ++j) out[j] = r_[(head_ + j) % 31];
    for (int j = 31; j < 61; ++j) out[j] = out[j - 31] + out[j - 3];
}

void GlibcRand::skip(uint64_t n) {
    uint32_t c[31], x[61];
    rand_jump_poly(n, c);
    extended_window(x);
    for (int j = 0; j < 31; ++j) {
        uint32_t acc = 0;
        for (int i = 0; i < 31; ++i) acc += c[i] * x[i + j];
        r_[j] = acc;
    }
    head_ = 0;
}

void rand_poly_mulmod(const uint32_t a[31], const uint32_t b[31], uint32_t out[31]) {
    uint32_t p[61] = {};
    for (int i = 0; i < 31; ++i)
        for (int j = 0; j < 31; ++j) p[i + j] += a[i] * b[j];
    for (int k = 60; k >= 31; --k) {      // z^k = z^(k-3) + z^(k-31)
        p[k - 3] += p[k];
        p[k - 31] += p[k];
    }
    for (int i = 0; i < 31; ++i) out[i] = p[i];
}

void rand_jump_poly(uint64_t n, uint32_t c[31]) {
    uint32_t base[31] = {}, r[31] = {};
    base[1] = 1;   // z
    r[0] = 1;
    for (; n; n >>= 1) {
        if (n & 1) rand_poly_mulmod(r, base, r);
        rand_poly_mulmod(base, base, base);
    }
    for (int i = 0; i < 31; ++i) c[i] = r[i];
}

GlibcRand& process_rand() {
    static GlibcRand g(1);
    return g;
}

}  // namespace impli
