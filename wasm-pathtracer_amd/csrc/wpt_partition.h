// wpt_partition.h — multi-GPU pixel partition.
//
// The reference splits the screen into independent halves per worker
// (wasm_interface.rs:78,90-94) and intends random pixel partitions
// (README.md:87). Here: square tiles in raster order, tile t -> rank
// t % nranks, pixels listed tile by tile; inside a tile, 8x8 sub-tiles in
// raster order, raster order inside a sub-tile (a wave's 64 consecutive paths
// are one compact 8x8 pixel block).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace wpt {

constexpr uint32_t kSubTile = 8;

inline void tile_partition(uint32_t w, uint32_t h, uint32_t rank, uint32_t nranks, uint32_t tile,
                           std::vector<uint32_t>& out) {
  out.clear();
  const uint32_t tx = (w + tile - 1) / tile, ty = (h + tile - 1) / tile;
  for (uint32_t t = rank; t < tx * ty; t += nranks) {
    const uint32_t x0 = (t % tx) * tile, y0 = (t / tx) * tile;
    const uint32_t x1 = std::min(x0 + tile, w), y1 = std::min(y0 + tile, h);
    for (uint32_t sy = y0; sy < y1; sy += kSubTile)
      for (uint32_t sx = x0; sx < x1; sx += kSubTile)
        for (uint32_t y = sy; y < std::min(sy + kSubTile, y1); y++)
          for (uint32_t x = sx; x < std::min(sx + kSubTile, x1); x++) out.push_back(y * w + x);
  }
}

// The pixels of columns [x0, x1) of a w-wide, h-high frame, tile by tile
// (tiles of tile x tile in raster order, raster order inside a tile; tile 0:
// plain raster order). A batch of whole sample rounds covers the same
// (pixel, sample) pairs in any pixel order; tile order makes a wave's 64
// consecutive paths a compact pixel block instead of a 64-pixel row.
inline void tile_order(uint32_t w, uint32_t h, uint32_t x0, uint32_t x1, uint32_t tile, std::vector<uint32_t>& out) {
  out.clear();
  out.reserve((size_t)(x1 - x0) * h);
  if (tile == 0) {
    for (uint32_t y = 0; y < h; y++)
      for (uint32_t x = x0; x < x1; x++) out.push_back(y * w + x);
    return;
  }
  for (uint32_t ty = 0; ty < h; ty += tile)
    for (uint32_t tx = x0; tx < x1; tx += tile)
      for (uint32_t y = ty; y < std::min(ty + tile, h); y++)
        for (uint32_t x = tx; x < std::min(tx + tile, x1); x++) out.push_back(y * w + x);
}

}  // namespace wpt
