// bb_render.h -- depth cameras (bb_render.hip), shared with the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bb_model.h"

namespace bb {

// camera frames in the base body: origin and camera->base rotation (row-major),
// cam_k_body pos/euler (ballbot.xml:44,50) composed with the camera's euler 180 0 0
struct CamRig {
  float p[2][3];
  float R[2][9];
};

struct RenderDev {
  int n;
  const void* qpos;       // T[17][n] (SoA)
  const int* steps;       // steps since reset
  const int* terrain;     // bank slot per env
  const float* bank;
  const float* size_z;
  const float* hmax;      // per terrain: max(hfield)
};

// scratch the launch needs: per (env, camera) scene
size_t scene_bytes(int n);
int launch_depth(bool fp64, const ModelT<float>& m, const CamRig& rig, const RenderDev& d, int H, int W, int every,
                 int force, float dt, void* scenes, float* depth, float* rel_ts, hipStream_t s);

}  // namespace bb
