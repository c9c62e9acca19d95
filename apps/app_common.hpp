// Shared pieces of the stencil apps: dump files in the reference format and
// result records.
#pragma once

#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "mxs/grid/print.hpp"
#include "mxs/topo/cart.hpp"

namespace mxs {
namespace app {

// Logical (total_width x total_height) window of a tile stored with `g`.
template <typename T>
void dump_tile(std::ostream& os, const T* tile, const TileGeom& g) {
  print_region(os, tile, g.full());
}

inline void append_json(const std::string& path, const std::string& line) {
  if (path.empty()) return;
  std::ofstream f(path, std::ios::app);
  f << line << '\n';
}

#ifndef MXS_GIT_SHA
#define MXS_GIT_SHA "unknown"
#endif

// `, "git": "<sha>", "device": "<desc>"` for the JSON records.
// HIP apps pass mxs::device_description(dev); the host-only app passes "cpu".
inline std::string meta_json(const std::string& device_desc) {
  return std::string(", \"git\": \"") + MXS_GIT_SHA + "\", \"device\": \"" + device_desc + "\"";
}

inline std::string fmt(double v) {
  char b[64];
  std::snprintf(b, sizeof(b), "%.6g", v);
  return b;
}

}  // namespace app
}  // namespace mxs
