// wpt_partition.h — multi-GPU pixel partition.
//
// The reference splits the screen into independent halves per worker
// (wasm_interface.rs:78,90-94) and intends random pixel partitions
// (README.md:87). Here: square tiles in raster order, tile t -> rank
// t % nranks, pixels listed tile by tile in raster order inside the tile.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace wpt {

inline void tile_partition(uint32_t w, uint32_t h, uint32_t rank, uint32_t nranks, uint32_t tile,
                           std::vector<uint32_t>& out) {
  out.clear();
  const uint32_t tx = (w + tile - 1) / tile, ty = (h + tile - 1) / tile;
  for (uint32_t t = rank; t < tx * ty; t += nranks) {
    const uint32_t x0 = (t % tx) * tile, y0 = (t / tx) * tile;
    for (uint32_t y = y0; y < std::min(y0 + tile, h); y++)
      for (uint32_t x = x0; x < std::min(x0 + tile, w); x++) out.push_back(y * w + x);
  }
}

}  // namespace wpt
