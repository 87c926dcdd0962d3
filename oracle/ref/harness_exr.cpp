// oracle/ref/harness_exr.cpp -- TEST INFRASTRUCTURE ONLY.  The reference's load_exr
// (main.cpp:42-79, which cannot be compiled here because main.cpp needs GLFW), re-enacted over the
// reference's own vendored tinyexr (CGL/include/CGL/tinyexr.h, compiled from the reference tree).
#define TINYEXR_IMPLEMENTATION
#include "tinyexr.h"

#include <cstdio>
#include <cstdlib>
#include <new>

#include "image.h"

// EnvironmentLight::init accumulates into `new double[h]` without zeroing it
// (environment_light.cpp:25-35): the reference's sampling tables are then built from whatever
// the heap held (observed: values ~1e193 from row 6 on, and a light that always returns the same
// texel).  SURVEY 8(f) fixes the intended semantics as a zeroed marginal_y.  Replacing the global
// array new with a zeroing allocator gives exactly that and changes nothing for code that
// initialises its arrays (a replaceable allocation function, [new.delete]).
void* operator new[](std::size_t n) {
  void* p = std::calloc(1, n ? n : 1);
  if (!p) throw std::bad_alloc();
  return p;
}
void operator delete[](void* p) noexcept { std::free(p); }
void operator delete[](void* p, std::size_t) noexcept { std::free(p); }

using namespace CGL;

HDRImageBuffer* harness_load_exr(const char* file_path) {
  const char* err = nullptr;
  EXRImage exr;
  InitEXRImage(&exr);
  if (ParseMultiChannelEXRHeaderFromFile(&exr, file_path, &err) != 0) {
    std::fprintf(stderr, "Error parsing OpenEXR file: %s\n", err ? err : "?");
    return nullptr;
  }
  for (int i = 0; i < exr.num_channels; i++)
    if (exr.pixel_types[i] == TINYEXR_PIXELTYPE_HALF) exr.requested_pixel_types[i] = TINYEXR_PIXELTYPE_FLOAT;
  if (LoadMultiChannelEXRFromFile(&exr, file_path, &err) != 0) {
    std::fprintf(stderr, "Error loading OpenEXR file: %s\n", err ? err : "?");
    return nullptr;
  }
  HDRImageBuffer* envmap = new HDRImageBuffer();
  envmap->resize(exr.width, exr.height);
  float* channel_r = (float*)exr.images[2];
  float* channel_g = (float*)exr.images[1];
  float* channel_b = (float*)exr.images[0];
  for (size_t i = 0; i < (size_t)exr.width * exr.height; i++)
    envmap->data[i] = Spectrum(channel_r[i], channel_g[i], channel_b[i]);
  return envmap;
}
