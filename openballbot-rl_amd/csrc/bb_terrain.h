// bb_terrain.h -- terrain bank generation (bb_terrain.hip), shared with the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bb {

constexpr int HF_N_ = 293;                 // ballbot.xml:23 nrow = ncol = 293
constexpr int HF_VERTS = HF_N_ * HF_N_;
// init-offset window of the reference (ballbot_env.py:546-563 with cell = 5/293):
// centre 146 -/+ 6 cells -> rows/cols [140, 152)
constexpr int HF_WIN0 = 140, HF_WIN1 = 152;

// perlin generator arguments (terrain/perlin.py:8-16 defaults 25, 4, .2, 2, 1)
struct PerlinCfg {
  double scale;       // Python float: x = i / scale in double
  int octaves;
  float persistence;  // parsed as C float by snoise2
  float lacunarity;
  double amplitude;   // (noise + 1) / 2 * amplitude in double
};

// fill bank[t] for t < count with perlin(seeds_dev[t]) and compute the
// per-terrain init offset and max height; enqueued on s
int launch_perlin_bank(float* bank, const int32_t* seeds_dev, int count, const PerlinCfg& cfg, float size_z,
                       float* offset, float* hmax, hipStream_t s);

}  // namespace bb
