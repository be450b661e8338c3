/*
 * implisolid_napi.c -- Node-API binding of the C ABI (include/implisolid.h).
 *
 * Lets the reference's JavaScript front-end (js_iteration_2/implisolid_main.js, whose `impli1`
 * service wraps the Emscripten exports with Module.cwrap at :36-70) call the MI355X library from
 * Node instead of the WASM module.  One JS function per mcc2.cpp export, same names and argument
 * meaning; buffers come back as typed-array copies instead of HEAPF32/HEAPU32 views (the JS shim
 * impli1.js keeps the reference call sites unchanged).
 *
 * Build (no node-gyp needed): see Makefile in this directory.
 */
#include <node_api.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/implisolid.h"

#define NAPI_CALL(env, call)                                                  \
    do {                                                                      \
        if ((call) != napi_ok) {                                              \
            napi_throw_error((env), NULL, "implisolid N-API call failed");    \
            return NULL;                                                      \
        }                                                                     \
    } while (0)

static char* arg_string(napi_env env, napi_value v) {
    size_t len = 0;
    if (napi_get_value_string_utf8(env, v, NULL, 0, &len) != napi_ok) return NULL;
    char* s = (char*)malloc(len + 1);
    if (!s) return NULL;
    napi_get_value_string_utf8(env, v, s, len + 1, &len);
    return s;
}

static napi_value undefined(napi_env env) {
    napi_value u;
    napi_get_undefined(env, &u);
    return u;
}

static napi_value number(napi_env env, double x) {
    napi_value v;
    napi_create_double(env, x, &v);
    return v;
}

static napi_value boolean(napi_env env, int b) {
    napi_value v;
    napi_get_boolean(env, b != 0, &v);
    return v;
}

/* typed-array copy of `bytes` at `src` (Float32Array or Uint32Array) */
static napi_value typed_copy(napi_env env, const void* src, size_t count, napi_typedarray_type type) {
    void* data = NULL;
    napi_value buf, arr;
    if (napi_create_arraybuffer(env, count * 4, &data, &buf) != napi_ok) return NULL;
    if (count && src) memcpy(data, src, count * 4);
    if (napi_create_typedarray(env, type, count, buf, 0, &arr) != napi_ok) return NULL;
    return arr;
}

static napi_value js_build_geometry(napi_env env, napi_callback_info info) {   /* mcc2.cpp:89 */
    size_t argc = 2;
    napi_value argv[2];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    char* shape = arg_string(env, argv[0]);
    char* mc = arg_string(env, argv[1]);
    if (shape && mc) build_geometry(shape, mc);
    free(shape);
    free(mc);
    return undefined(env);
}

/* build_geometry_u(shape, mc, call_specs[, progress]) (mcc2.cpp:90): `progress` is called
   synchronously with (verts Float32Array, faces Uint32Array, progressCallback_id, shape_id,
   call_id) at every send_mesh_back_to_client point -- the arguments the reference's worker gives
   wwapi.send_progress_update (js/worker_api.js:399-416). */
static napi_env g_progress_env = NULL;
static napi_value g_progress_fn = NULL;

static void progress_hook(const float* verts, int nv, const int32_t* faces, int nf, int pid, int sid, int cid, void* user) {
    (void)user;
    napi_env env = g_progress_env;
    napi_value argv[5], global, result;
    if (!env || !g_progress_fn) return;
    argv[0] = typed_copy(env, verts, (size_t)nv * 3, napi_float32_array);
    argv[1] = typed_copy(env, faces, (size_t)nf * 3, napi_uint32_array);
    argv[2] = number(env, pid);
    argv[3] = number(env, sid);
    argv[4] = number(env, cid);
    if (!argv[0] || !argv[1]) return;
    napi_get_global(env, &global);
    napi_call_function(env, global, g_progress_fn, 5, argv, &result);
}

static napi_value js_build_geometry_u(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    napi_valuetype t = napi_undefined;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    char* shape = argc > 0 ? arg_string(env, argv[0]) : NULL;
    char* mc = argc > 1 ? arg_string(env, argv[1]) : NULL;
    char* specs = argc > 2 ? arg_string(env, argv[2]) : NULL;
    if (argc > 3) napi_typeof(env, argv[3], &t);
    if (t == napi_function) {
        g_progress_env = env;
        g_progress_fn = argv[3];
        implisolid_set_progress_callback(progress_hook, NULL);
    }
    if (shape && mc) build_geometry_u(shape, mc, specs ? specs : "{}");
    if (t == napi_function) {
        implisolid_set_progress_callback(NULL, NULL);
        g_progress_env = NULL;
        g_progress_fn = NULL;
    }
    free(shape);
    free(mc);
    free(specs);
    return undefined(env);
}

static napi_value js_get_v_size(napi_env env, napi_callback_info info) { (void)info; return number(env, get_v_size()); }
static napi_value js_get_f_size(napi_env env, napi_callback_info info) { (void)info; return number(env, get_f_size()); }

static napi_value js_get_v(napi_env env, napi_callback_info info) {   /* get_v_ptr + HEAPF32 view */
    (void)info;
    return typed_copy(env, get_v_ptr(), (size_t)get_v_size() * 3, napi_float32_array);
}
static napi_value js_get_f(napi_env env, napi_callback_info info) {   /* get_f_ptr + HEAPU32 view */
    (void)info;
    return typed_copy(env, get_f_ptr(), (size_t)get_f_size() * 3, napi_uint32_array);
}
static napi_value js_finish_geometry(napi_env env, napi_callback_info info) {
    (void)info;
    finish_geometry();
    return undefined(env);
}

static napi_value js_set_object(napi_env env, napi_callback_info info) {   /* mcc2.cpp:106 */
    size_t argc = 2;
    napi_value argv[2];
    bool ign = false;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    char* shape = arg_string(env, argv[0]);
    if (argc > 1) napi_get_value_bool(env, argv[1], &ign);
    const int id = shape ? set_object(shape, ign) : 0;
    free(shape);
    return number(env, id);
}
static napi_value js_unset_object(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    int32_t id = 0;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    napi_get_value_int32(env, argv[0], &id);
    return boolean(env, unset_object(id));
}
static napi_value js_set_x(napi_env env, napi_callback_info info) {   /* Float32Array of xyz */
    size_t argc = 1;
    napi_value argv[1];
    napi_typedarray_type type;
    size_t length = 0, offset = 0;
    void* data = NULL;
    napi_value ab;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    NAPI_CALL(env, napi_get_typedarray_info(env, argv[0], &type, &length, &data, &ab, &offset));
    if (type != napi_float32_array) {
        napi_throw_type_error(env, NULL, "set_x expects a Float32Array of xyz triples");
        return NULL;
    }
    return boolean(env, set_x(data, (int)(length / 3)));
}
static napi_value js_unset_x(napi_env env, napi_callback_info info) {
    (void)info;
    unset_x();
    return undefined(env);
}
static napi_value js_calculate_implicit_values(napi_env env, napi_callback_info info) {
    (void)info;
    calculate_implicit_values();
    return undefined(env);
}
static napi_value js_get_values(napi_env env, napi_callback_info info) {
    (void)info;
    return typed_copy(env, get_values_ptr(), (size_t)get_values_size(), napi_float32_array);
}
static napi_value js_calculate_implicit_gradients(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    bool norm = false;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc > 0) napi_get_value_bool(env, argv[0], &norm);
    calculate_implicit_gradients(norm);
    return undefined(env);
}
static napi_value js_get_gradients(napi_env env, napi_callback_info info) {
    (void)info;
    return typed_copy(env, get_gradients_ptr(), (size_t)get_gradients_size(), napi_float32_array);
}
static napi_value js_get_pointset(napi_env env, napi_callback_info info) {   /* mcc2.cpp:122-123 */
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    char* id = arg_string(env, argv[0]);
    napi_value out = NULL;
    if (id) {
        const int n = get_pointset_size(id);
        void* p = get_pointset_ptr(id);
        if (p && n > 0) out = typed_copy(env, p, (size_t)n * 3, napi_float32_array);
    }
    free(id);
    if (!out) napi_get_null(env, &out);
    return out;
}
static napi_value js_about(napi_env env, napi_callback_info info) {
    (void)info;
    about();
    return undefined(env);
}
static napi_value js_last_error(napi_env env, napi_callback_info info) {
    (void)info;
    napi_value s;
    napi_create_string_utf8(env, implisolid_last_error(), NAPI_AUTO_LENGTH, &s);
    return s;
}
static napi_value js_set_error_mode(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    int32_t m = 0;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    napi_get_value_int32(env, argv[0], &m);
    implisolid_set_error_mode(m);
    return undefined(env);
}
static napi_value js_program_info(napi_env env, napi_callback_info info) {   /* host only: compile check */
    size_t argc = 1;
    napi_value argv[1];
    int32_t inf[4] = {0, 0, 0, 0};
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    char* shape = arg_string(env, argv[0]);
    const int rc = shape ? implisolid_program_info(shape, 0, inf, NULL) : -1;
    free(shape);
    return number(env, rc == 0 ? inf[0] : -1);
}

#define EXPORT(name, fn)                                                                  \
    do {                                                                                  \
        napi_value f;                                                                     \
        if (napi_create_function(env, name, NAPI_AUTO_LENGTH, fn, NULL, &f) == napi_ok)   \
            napi_set_named_property(env, exports, name, f);                               \
    } while (0)

static napi_value init(napi_env env, napi_value exports) {
    EXPORT("build_geometry", js_build_geometry);
    EXPORT("build_geometry_u", js_build_geometry_u);
    EXPORT("get_v_size", js_get_v_size);
    EXPORT("get_f_size", js_get_f_size);
    EXPORT("get_v", js_get_v);
    EXPORT("get_f", js_get_f);
    EXPORT("finish_geometry", js_finish_geometry);
    EXPORT("set_object", js_set_object);
    EXPORT("unset_object", js_unset_object);
    EXPORT("set_x", js_set_x);
    EXPORT("unset_x", js_unset_x);
    EXPORT("calculate_implicit_values", js_calculate_implicit_values);
    EXPORT("get_values", js_get_values);
    EXPORT("calculate_implicit_gradients", js_calculate_implicit_gradients);
    EXPORT("get_gradients", js_get_gradients);
    EXPORT("get_pointset", js_get_pointset);
    EXPORT("about", js_about);
    EXPORT("last_error", js_last_error);
    EXPORT("set_error_mode", js_set_error_mode);
    EXPORT("program_info", js_program_info);
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
