// rrt_scene_file.h -- host-side owner of a flattened static scene (include/rrt.h
// rrt_scene_file_*).  Filled either from a .rrts file (rrt_host.cpp) or by the native COLLADA
// ingest (rrt_ingest.cpp); `desc` points into the vectors below.
#pragma once
#include <cstdint>
#include <vector>

#include "../../include/rrt.h"

struct rrt_scene_file {
  std::vector<rrt_object_desc> objects;
  std::vector<rrt_bsdf_desc> bsdfs;
  std::vector<rrt_light_desc> lights;
  std::vector<std::vector<double>> dbl;     // per mesh: positions, normals
  std::vector<std::vector<uint32_t>> idx;   // per mesh: triangle indices
  rrt_scene_desc desc{};

  // Point desc (and each mesh object) at the owned arrays.  Meshes take dbl[2k], dbl[2k+1]
  // and idx[k] in object order.
  void finalize() {
    size_t m = 0;
    for (auto& o : objects) {
      if (o.kind != RRT_OBJ_MESH) continue;
      o.positions = dbl[2 * m].data();
      o.normals = dbl[2 * m + 1].data();
      o.indices = idx[m].data();
      ++m;
    }
    desc.n_objects = (uint32_t)objects.size();
    desc.n_bsdfs = (uint32_t)bsdfs.size();
    desc.n_lights = (uint32_t)lights.size();
    desc.objects = objects.data();
    desc.bsdfs = bsdfs.data();
    desc.lights = lights.data();
  }
};
