// impli1.js -- drop-in for the `impli1` service of the reference's implisolid_main.js (:36-70),
// backed by the MI355X library through the N-API addon instead of Module.cwrap over WASM.
//
// The reference reads results through HEAPF32/HEAPU32 views at get_v_ptr()/get_f_ptr()
// (implisolid_main.js:233-237); here get_v()/get_f() return the same data as typed arrays.
'use strict';
const path = require('path');
const native = require(path.join(__dirname, 'build', 'implisolid.node'));

const impli1 = {
  build_geometry: (mp5_str, params_str) => native.build_geometry(mp5_str, params_str),
  // worker path (worker_api.js:315-345): call_specs = JSON of {progressCallback_id, call_id,
  // shape_id}; progress(verts, faces, progressCallback_id, shape_id, call_id) is called at each
  // send_mesh_back_to_client point, as wwapi.send_progress_update is (worker_api.js:399-416)
  build_geometry_u: (mp5_str, params_str, call_specs, progress) =>
    native.build_geometry_u(mp5_str, params_str, call_specs || '{}', progress),
  get_v_size: () => native.get_v_size(),
  get_f_size: () => native.get_f_size(),
  get_v: () => native.get_v(),              // Float32Array, 3 per vertex
  get_f: () => native.get_f(),              // Uint32Array, 3 per face
  finish_geometry: () => native.finish_geometry(),
  set_object: (mp5_str, ignore_root_matrix) => native.set_object(mp5_str, !!ignore_root_matrix),
  unset_object: (id) => native.unset_object(id),
  set_x: (xyz) => native.set_x(xyz),        // Float32Array of xyz triples (< 50000 points)
  unset_x: () => native.unset_x(),
  calculate_implicit_values: () => native.calculate_implicit_values(),
  get_values: () => native.get_values(),
  calculate_implicit_gradients: (normalize) => native.calculate_implicit_gradients(!!normalize),
  get_gradients: () => native.get_gradients(),
  get_pointset: (id) => native.get_pointset(id),
  about: () => native.about(),
  last_error: () => native.last_error(),
  set_error_mode: (m) => native.set_error_mode(m),
  needs_deallocation: false,
};

// implisolid_main.js:201-249 make_geometry, minus the Emscripten heap views
function make_geometry(mp5_str, params_str, geometry_callback, allocate_buffer) {
  if (typeof params_str !== 'string') params_str = JSON.stringify(params_str);
  if (impli1.needs_deallocation) {
    impli1.finish_geometry();
    impli1.needs_deallocation = false;
  }
  impli1.build_geometry(mp5_str, params_str);
  impli1.needs_deallocation = true;
  return geometry_callback(impli1.get_v(), impli1.get_f(), allocate_buffer);
}

module.exports = { impli1, make_geometry, native };
