// wpt_obj.h — OBJ mesh ingestion: parseObj (src_ts/client/obj_parser.ts:3-51)
// restated over JavaScript's number semantics, so a host that hands the
// library an .obj file gets the vertex soup the reference's client would
// have put into mesh_vertices (wasm_interface.rs:259-293).
//   * lines split on '\n', fields on single spaces (empty fields kept);
//   * "v x y z": parseFloat of fields 1-3 (a missing or malformed field is NaN);
//   * "f a b c": exactly 4 fields or the parse fails ("Non-triangular face in
//     OBJ file"); each corner's vertex index is parseInt of the text before
//     its first '/', minus 1;
//   * everything else ("vn", "#", ...) is ignored;
//   * output: 9 floats per face, the f64 coordinates rounded to f32; a corner
//     whose index is NaN or out of range reads `undefined`, stored as NaN.
#pragma once
#include <stddef.h>

#include <string>
#include <vector>

namespace wpt {

bool parse_obj(const char* text, size_t len, std::vector<float>& out, std::string& err);
// index.ts:216-220's per-axis scale ((8, 8, -8) for the bunny): each f32
// coordinate times the factor in f64, rounded back to f32.
void scale_vertices(std::vector<float>& v, const float scale[3]);

}  // namespace wpt
