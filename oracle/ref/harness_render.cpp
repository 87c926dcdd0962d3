// oracle/ref/harness_render.cpp -- TEST INFRASTRUCTURE ONLY (builds oracle/_ref/ref_render).
//
// Headless driver around the reference renderer's OWN objects (compiled from /root/reference by
// Makefile).  It re-enacts what main() + Application do on the `-f` path
// (main.cpp:81-187, application.cpp:48-97 init, :219-295 load, :180-192 resize,
// :622-628 set_up_pathtracer, application.h:107-110 render_to_file) because application.cpp
// itself needs GL/glu.h, which this image does not have.  Every numeric step is a call into the
// reference (Collada parser, Camera::configure/place/set_screen_size, DynamicScene ->
// get_static_scene, PathTracer ctor/set_* /render_to_file).
//
// Instrumentation (link-time --wrap, no reference source edited):
//   rand()                        -> keyed per-pixel generator (harness_common.h)
//   PathTracer::raytrace_pixel    -> sets the pixel key, calls the real function, records
//                                    (RGB f32, sample count, draw count, work counters)
//   BBox::intersect, BlackHole::next_micro_ray, Sphere::intersect(const Ray&)
//                                 -> per-pixel work counters (AABB tests, micro steps)
//
// Outputs (prefix given by -O):
//   <prefix>.rrts        flattened static scene (format: include/rrt_scene_format.h)
//   <prefix>.rrtc        camera record            (same header)
//   <prefix>_bvh_*.npy   reference BVH in left-first pre-order (node bbox, leaf prim ids)
//   <prefix>_px_*.npy    per-pixel results for the rendered region
//
// Extra flags beyond the reference's getopt string: -S <seed>, -O <prefix>, -Q (dump only).
// -e <file.exr> loads the environment map the way main.cpp:42-79 does (the reference's vendored
// tinyexr, compiled in harness_exr.cpp) and hands it to the PathTracer constructor.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <fstream>
#include <functional>
#include <iostream>
#include <map>
#include <mutex>
#include <sstream>
#include <stack>
#include <thread>
#include <unordered_map>
#include <vector>
#include <unistd.h>

#include "harness_common.h"

#define private public
#define protected public
#include "application.h"  // AppConfig defaults (application.h:41-85); header only
#include "pathtracer.h"
#include "bvh.h"
#include "bsdf.h"
#include "camera.h"
#include "collada/collada.h"
#include "dynamic_scene/ambient_light.h"
#include "dynamic_scene/area_light.h"
#include "dynamic_scene/directional_light.h"
#include "dynamic_scene/mesh.h"
#include "dynamic_scene/point_light.h"
#include "dynamic_scene/sphere.h"
#include "dynamic_scene/spot_light.h"
#include "static_scene/blackhole.h"
#include "static_scene/light.h"
#include "static_scene/object.h"
#include "static_scene/sphere.h"
#include "static_scene/triangle.h"
#include "static_scene/environment_light.h"
#undef private
#undef protected

using namespace CGL;
using CGL::StaticScene::global_black_hole;

namespace harness { thread_local ThreadRng g_rng; }
HDRImageBuffer* harness_load_exr(const char* path);  // harness_exr.cpp (main.cpp:42-79 re-enacted)
using harness::g_rng;

// ------------------------------------------------------------------------------------------
// link-time wraps
// ------------------------------------------------------------------------------------------
extern "C" int __real_rand(void);
extern "C" int __wrap_rand(void) {
  if (g_rng.mode == harness::RAND_KEYED) return harness::keyed_rand(g_rng.key, g_rng.ctr++);
  if (g_rng.mode == harness::RAND_SCRIPTED) {
    if (g_rng.ctr >= g_rng.script_len) { std::fprintf(stderr, "script exhausted\n"); std::abort(); }
    return g_rng.script[g_rng.ctr++];
  }
  std::fprintf(stderr, "[harness] rand() called outside a pixel context\n");
  std::abort();
}

extern "C" bool __real__ZNK3CGL4BBox9intersectERKNS_3RayERdS4_(const BBox*, const Ray&, double&, double&);
extern "C" bool __wrap__ZNK3CGL4BBox9intersectERKNS_3RayERdS4_(const BBox* b, const Ray& r, double& t0, double& t1) {
  ++g_rng.bbox_tests;
  return __real__ZNK3CGL4BBox9intersectERKNS_3RayERdS4_(b, r, t0, t1);
}
extern "C" Ray __real__ZN3CGL11StaticScene9BlackHole14next_micro_rayERKNS_3RayE(StaticScene::BlackHole*, const Ray&);
extern "C" Ray __wrap__ZN3CGL11StaticScene9BlackHole14next_micro_rayERKNS_3RayE(StaticScene::BlackHole* bh, const Ray& r) {
  ++g_rng.micro_steps;
  return __real__ZN3CGL11StaticScene9BlackHole14next_micro_rayERKNS_3RayE(bh, r);
}

struct PixelRecord {
  float rgb[3];
  int32_t count;
  uint32_t draws;
  uint32_t bbox_tests;
  uint32_t micro_steps;
  uint32_t done;
};
static std::vector<PixelRecord> g_pixels;
static size_t g_frame_w = 0, g_frame_h = 0;
static uint64_t g_seed = 0;

extern "C" Spectrum __real__ZN3CGL10PathTracer14raytrace_pixelEmmb(PathTracer*, size_t, size_t, bool);
extern "C" Spectrum __wrap__ZN3CGL10PathTracer14raytrace_pixelEmmb(PathTracer* self, size_t x, size_t y, bool thin) {
  g_rng.mode = harness::RAND_KEYED;
  g_rng.key = harness::pixel_key(g_seed, (uint32_t)x, (uint32_t)y);
  g_rng.ctr = 0;
  g_rng.bbox_tests = 0;
  g_rng.micro_steps = 0;
  Spectrum s = __real__ZN3CGL10PathTracer14raytrace_pixelEmmb(self, x, y, thin);
  g_rng.mode = harness::RAND_UNKEYED;
  PixelRecord& rec = g_pixels[y * g_frame_w + x];
  rec.rgb[0] = s.r; rec.rgb[1] = s.g; rec.rgb[2] = s.b;
  rec.count = self->sampleCountBuffer[x + y * self->frameBuffer.w];
  rec.draws = g_rng.ctr;
  rec.bbox_tests = (uint32_t)g_rng.bbox_tests;
  rec.micro_steps = (uint32_t)g_rng.micro_steps;
  rec.done = 1;
  return s;
}

// ------------------------------------------------------------------------------------------
// dumps
// ------------------------------------------------------------------------------------------
template <class T> static void put(std::vector<unsigned char>& b, const T& v) {
  const unsigned char* p = (const unsigned char*)&v;
  b.insert(b.end(), p, p + sizeof(T));
}
static void put3(std::vector<unsigned char>& b, const Vector3D& v) { put(b, v.x); put(b, v.y); put(b, v.z); }
static void write_file(const std::string& path, const std::vector<unsigned char>& b) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) { std::perror(path.c_str()); std::exit(2); }
  std::fwrite(b.data(), 1, b.size(), f);
  std::fclose(f);
}

// BSDF record: u32 type, u32 pad, f32 p[14]  (64 bytes)
static int bsdf_index(std::vector<BSDF*>& table, BSDF* b) {
  for (size_t i = 0; i < table.size(); ++i) if (table[i] == b) return (int)i;
  table.push_back(b);
  return (int)table.size() - 1;
}
static void put_bsdf(std::vector<unsigned char>& buf, BSDF* b) {
  uint32_t type = 0xffffffffu;
  float p[14] = {0};
  if (auto* d = dynamic_cast<DiffuseBSDF*>(b)) { type = 0; p[0] = d->reflectance.r; p[1] = d->reflectance.g; p[2] = d->reflectance.b; }
  else if (auto* e = dynamic_cast<EmissionBSDF*>(b)) { type = 1; p[0] = e->radiance.r; p[1] = e->radiance.g; p[2] = e->radiance.b; }
  else if (auto* m = dynamic_cast<MirrorBSDF*>(b)) { type = 2; p[0] = m->reflectance.r; p[1] = m->reflectance.g; p[2] = m->reflectance.b; }
  else if (auto* g = dynamic_cast<GlassBSDF*>(b)) {
    type = 3; p[0] = g->transmittance.r; p[1] = g->transmittance.g; p[2] = g->transmittance.b;
    p[3] = g->reflectance.r; p[4] = g->reflectance.g; p[5] = g->reflectance.b; p[6] = g->roughness; p[7] = g->ior;
  } else if (auto* mf = dynamic_cast<MicrofacetBSDF*>(b)) {
    type = 4; p[0] = mf->eta.r; p[1] = mf->eta.g; p[2] = mf->eta.b; p[3] = mf->k.r; p[4] = mf->k.g; p[5] = mf->k.b; p[6] = mf->alpha;
  } else if (auto* rf = dynamic_cast<RefractionBSDF*>(b)) {
    type = 5; p[0] = rf->transmittance.r; p[1] = rf->transmittance.g; p[2] = rf->transmittance.b; p[6] = rf->roughness; p[7] = rf->ior;
  } else { std::fprintf(stderr, "[harness] unknown BSDF type\n"); std::exit(3); }
  put(buf, type); put(buf, (uint32_t)0);
  for (float v : p) put(buf, v);
}

static void dump_scene(const std::string& path, StaticScene::Scene* scene) {
  std::vector<BSDF*> bsdfs;
  std::vector<unsigned char> objs, lights;
  for (StaticScene::SceneObject* o : scene->objects) {
    if (auto* m = dynamic_cast<StaticScene::Mesh*>(o)) {
      size_t nv = 0;
      for (size_t id : m->indices) nv = std::max(nv, id + 1);
      uint32_t ntri = (uint32_t)(m->indices.size() / 3);
      put(objs, (uint32_t)0); put(objs, (uint32_t)bsdf_index(bsdfs, m->bsdf));
      put(objs, (uint32_t)nv); put(objs, ntri);
      for (size_t i = 0; i < nv; ++i) put3(objs, m->positions[i]);
      for (size_t i = 0; i < nv; ++i) put3(objs, m->normals[i]);
      for (size_t id : m->indices) put(objs, (uint32_t)id);
    } else if (auto* s = dynamic_cast<StaticScene::SphereObject*>(o)) {
      put(objs, (uint32_t)1); put(objs, (uint32_t)bsdf_index(bsdfs, s->bsdf));
      put(objs, (uint32_t)0); put(objs, (uint32_t)0);
      put3(objs, s->o); put(objs, s->r);
    } else { std::fprintf(stderr, "[harness] unknown object type\n"); std::exit(3); }
  }
  // Light record: u32 type, u32 is_delta, f32 radiance[3], f32 area, f64 v[12]  (120 bytes)
  uint32_t n_dumped_lights = 0;
  for (StaticScene::SceneLight* l : scene->lights) {
    if (dynamic_cast<StaticScene::EnvironmentLight*>(l)) continue;  // given separately (-e file)
    ++n_dumped_lights;
    uint32_t type = 0xffffffffu;
    float rad[3] = {0, 0, 0}, area = 0;
    Vector3D v[4];
    if (auto* a = dynamic_cast<StaticScene::AreaLight*>(l)) {
      type = 0; rad[0] = a->radiance.r; rad[1] = a->radiance.g; rad[2] = a->radiance.b; area = a->area;
      v[0] = a->position; v[1] = a->direction; v[2] = a->dim_x; v[3] = a->dim_y;
    } else if (auto* p = dynamic_cast<StaticScene::PointLight*>(l)) {
      type = 1; rad[0] = p->radiance.r; rad[1] = p->radiance.g; rad[2] = p->radiance.b; v[0] = p->position;
    } else if (auto* d = dynamic_cast<StaticScene::DirectionalLight*>(l)) {
      type = 2; rad[0] = d->radiance.r; rad[1] = d->radiance.g; rad[2] = d->radiance.b; v[0] = d->dirToLight;
    } else if (auto* h = dynamic_cast<StaticScene::InfiniteHemisphereLight*>(l)) {
      type = 3; rad[0] = h->radiance.r; rad[1] = h->radiance.g; rad[2] = h->radiance.b;
      v[0] = h->sampleToWorld[0]; v[1] = h->sampleToWorld[1]; v[2] = h->sampleToWorld[2];
    } else if (dynamic_cast<StaticScene::EnvironmentLight*>(l)) {
      type = 5;
    } else {
      type = 4;  // Spot/Sphere/Mesh stubs (light.cpp:59-115): no supported sampling
    }
    put(lights, type); put(lights, (uint32_t)(l->is_delta_light() ? 1 : 0));
    put(lights, rad[0]); put(lights, rad[1]); put(lights, rad[2]); put(lights, area);
    for (int i = 0; i < 4; ++i) put3(lights, v[i]);
  }
  std::vector<unsigned char> out;
  const char magic[8] = {'R', 'R', 'T', 'S', 'C', 'N', '1', 0};
  out.insert(out.end(), magic, magic + 8);
  put(out, (uint32_t)bsdfs.size()); put(out, (uint32_t)scene->objects.size());
  put(out, n_dumped_lights); put(out, (uint32_t)0);
  for (BSDF* b : bsdfs) put_bsdf(out, b);
  out.insert(out.end(), objs.begin(), objs.end());
  out.insert(out.end(), lights.begin(), lights.end());
  write_file(path, out);
}

static void dump_camera(const std::string& path, const Camera* c) {
  std::vector<unsigned char> out;
  const char magic[8] = {'R', 'R', 'T', 'C', 'A', 'M', '1', 0};
  out.insert(out.end(), magic, magic + 8);
  put(out, c->hFov); put(out, c->vFov); put(out, c->ar); put(out, c->nClip); put(out, c->fClip);
  put3(out, c->pos); put3(out, c->targetPos);
  put(out, c->phi); put(out, c->theta); put(out, c->r); put(out, c->minR); put(out, c->maxR);
  for (int i = 0; i < 9; ++i) put(out, c->c2w(i / 3, i % 3));  // row-major, as dump_settings
  put(out, (double)c->screenW); put(out, (double)c->screenH); put(out, c->screenDist);
  put(out, c->focalDistance); put(out, c->lensRadius);
  write_file(path, out);
}

// reference BVH, left-first pre-order: per node bbox (min, max), leaf prim range into prim_ids.
static void dump_bvh(const std::string& prefix, StaticScene::Scene* scene, StaticScene::BVHNode* root) {
  // build-order primitive ids: objects in order x get_primitives() order (pathtracer.cpp:310-314)
  std::map<std::pair<const void*, std::vector<size_t>>, std::vector<uint32_t>> tri_ids;
  std::map<const void*, uint32_t> sphere_ids;
  uint32_t next = 0;
  for (StaticScene::SceneObject* o : scene->objects) {
    if (auto* m = dynamic_cast<StaticScene::Mesh*>(o)) {
      for (size_t t = 0; t < m->indices.size() / 3; ++t)
        tri_ids[{m, {m->indices[3 * t], m->indices[3 * t + 1], m->indices[3 * t + 2]}}].push_back(next++);
    } else {
      sphere_ids[o] = next++;
    }
  }
  std::vector<double> boxes;
  std::vector<int32_t> nodes;  // per node: first, count (count 0 = inner), left, right
  std::vector<uint32_t> prims;
  std::map<std::pair<const void*, std::vector<size_t>>, size_t> consumed;
  std::function<int(StaticScene::BVHNode*)> walk = [&](StaticScene::BVHNode* n) -> int {
    int id = (int)(nodes.size() / 4);
    nodes.insert(nodes.end(), {0, 0, -1, -1});
    boxes.insert(boxes.end(), {n->bb.min.x, n->bb.min.y, n->bb.min.z, n->bb.max.x, n->bb.max.y, n->bb.max.z});
    if (n->prims) {
      nodes[4 * id] = (int32_t)prims.size();
      nodes[4 * id + 1] = (int32_t)n->prims->size();
      for (StaticScene::Primitive* p : *n->prims) {
        if (auto* t = dynamic_cast<StaticScene::Triangle*>(p)) {
          auto key = std::make_pair((const void*)t->mesh, std::vector<size_t>{t->v1, t->v2, t->v3});
          auto& ids = tri_ids[key];
          size_t& k = consumed[key];
          prims.push_back(ids.at(k++));
        } else if (auto* s = dynamic_cast<StaticScene::Sphere*>(p)) {
          prims.push_back(sphere_ids.at(s->object));
        }
      }
    } else {
      int l = walk(n->l);
      int r = walk(n->r);
      nodes[4 * id + 2] = l;
      nodes[4 * id + 3] = r;
    }
    return id;
  };
  walk(root);
  size_t nn = nodes.size() / 4;
  harness::write_npy(prefix + "_bvh_boxes.npy", "<f8", {nn, 6}, boxes.data(), boxes.size() * 8);
  harness::write_npy(prefix + "_bvh_nodes.npy", "<i4", {nn, 4}, nodes.data(), nodes.size() * 4);
  harness::write_npy(prefix + "_bvh_prims.npy", "<u4", {prims.size()}, prims.data(), prims.size() * 4);
}

// ------------------------------------------------------------------------------------------
// Application re-enactment (application.cpp), headless only
// ------------------------------------------------------------------------------------------
static DynamicScene::SceneLight* init_light(Collada::LightInfo& light, const Matrix4x4& transform) {
  switch (light.light_type) {  // application.cpp:140-159
    case Collada::LightType::NONE: break;
    case Collada::LightType::AMBIENT: return new DynamicScene::AmbientLight(light);
    case Collada::LightType::DIRECTIONAL: return new DynamicScene::DirectionalLight(light, transform);
    case Collada::LightType::AREA: return new DynamicScene::AreaLight(light, transform);
    case Collada::LightType::POINT: return new DynamicScene::PointLight(light, transform);
    case Collada::LightType::SPOT: return new DynamicScene::SpotLight(light, transform);
    default: break;
  }
  return nullptr;
}

int main(int argc, char** argv) {
  AppConfig config;
  size_t w = 0, h = 0, x = -1, y = 0, dx = 0, dy = 0;
  std::string filename = "ref.png", cam_settings = "", prefix = "ref";
  bool dump_only = false;
  int opt;
  // reference getopt string (main.cpp:88) + S: O: Q
  while ((opt = getopt(argc, argv, "s:l:t:m:e:h:H:f:r:c:a:p:b:d:B:S:O:Q")) != -1) {
    switch (opt) {
      case 'f': filename = optarg; break;
      case 'r': w = atoi(argv[optind - 1]); h = atoi(argv[optind]); optind++; break;
      case 'p':
        x = atoi(argv[optind - 1]); y = atoi(argv[optind]); dx = atoi(argv[optind + 1]); dy = atoi(argv[optind + 2]);
        optind += 3; break;
      case 's': config.pathtracer_ns_aa = atoi(optarg); break;
      case 'l': config.pathtracer_ns_area_light = atoi(optarg); break;
      case 't': config.pathtracer_num_threads = atoi(optarg); break;
      case 'm': config.pathtracer_max_ray_depth = atoi(optarg); break;
      case 'b': config.pathtracer_lensRadius = atof(optarg); break;
      case 'd': config.pathtracer_focalDistance = atof(optarg); break;
      case 'e':
        config.pathtracer_envmap = harness_load_exr(optarg);
        if (!config.pathtracer_envmap) return 1;
        break;
      case 'c': cam_settings = optarg; break;
      case 'a':
        config.pathtracer_samples_per_patch = atoi(argv[optind - 1]);
        config.pathtracer_max_tolerance = atof(argv[optind]); optind++; break;
      case 'H': config.pathtracer_direct_hemisphere_sample = true; optind--; break;
      case 'B':
        global_black_hole.o = Vector3D(atof(argv[optind - 1]), atof(argv[optind]), atof(argv[optind + 1]));
        global_black_hole.r = atof(argv[optind + 2]);
        global_black_hole.r2 = global_black_hole.r * global_black_hole.r;
        global_black_hole.delta_theta = atof(argv[optind + 3]);
        optind += 4; break;
      case 'S': g_seed = strtoull(optarg, nullptr, 0); break;
      case 'O': prefix = optarg; break;
      case 'Q': dump_only = true; break;
      default: std::fprintf(stderr, "bad option\n"); return 1;
    }
  }
  if (optind >= argc) { std::fprintf(stderr, "usage: ref_render [opts] scene.dae\n"); return 1; }
  std::string scene_path = argv[optind];

  Collada::SceneInfo* sceneInfo = new Collada::SceneInfo();
  if (Collada::ColladaParser::load(scene_path.c_str(), sceneInfo) < 0) return 4;

  PathTracer* pt = new PathTracer(config.pathtracer_ns_aa, config.pathtracer_max_ray_depth,
                                  config.pathtracer_ns_area_light, config.pathtracer_ns_diff,
                                  config.pathtracer_ns_glsy, config.pathtracer_ns_refr,
                                  config.pathtracer_num_threads, config.pathtracer_samples_per_patch,
                                  config.pathtracer_max_tolerance, config.pathtracer_envmap,
                                  config.pathtracer_direct_hemisphere_sample, "ref",
                                  config.pathtracer_lensRadius, config.pathtracer_focalDistance);

  // Application::init (application.cpp:90-96): dummy camera configured at 800x600
  Camera camera;
  size_t screenW = 800, screenH = 600;
  {
    Collada::CameraInfo ci;
    ci.hFov = 50; ci.vFov = 35; ci.nClip = 0.01; ci.fClip = 100;
    camera.configure(ci, screenW, screenH);
  }
  // Application::load (application.cpp:219-295)
  std::vector<DynamicScene::SceneLight*> lights;
  std::vector<DynamicScene::SceneObject*> objects;
  Vector3D c_pos = Vector3D(), c_dir = Vector3D();
  for (Collada::Node& node : sceneInfo->nodes) {
    Collada::Instance* instance = node.instance;
    const Matrix4x4& transform = node.transform;
    switch (instance->type) {
      case Collada::Instance::CAMERA: {
        Collada::CameraInfo* c = static_cast<Collada::CameraInfo*>(instance);
        c_pos = (transform * Vector4D(c_pos, 1)).to3D();
        c_dir = (transform * Vector4D(c->view_dir, 1)).to3D().unit();
        camera.configure(*c, screenW, screenH);
        break;
      }
      case Collada::Instance::LIGHT:
        lights.push_back(init_light(static_cast<Collada::LightInfo&>(*instance), transform));
        break;
      case Collada::Instance::SPHERE: {
        const Vector3D& position = (transform * Vector4D(0, 0, 0, 1)).projectTo3D();
        double scale = (transform * Vector4D(1, 0, 0, 0)).to3D().norm();
        objects.push_back(new DynamicScene::Sphere(static_cast<Collada::SphereInfo&>(*instance), position, scale));
        break;
      }
      case Collada::Instance::POLYMESH:
        objects.push_back(new DynamicScene::Mesh(static_cast<Collada::PolymeshInfo&>(*instance), transform));
        break;
      case Collada::Instance::MATERIAL: break;
    }
  }
  DynamicScene::Scene* scene = new DynamicScene::Scene(objects, lights);
  const BBox& bbox = scene->get_bbox();
  if (!bbox.empty()) {
    Vector3D target = bbox.centroid();
    double canonical_view_distance = bbox.extent.norm() / 2 * 1.5;
    double view_distance = canonical_view_distance * 2;
    double min_view_distance = canonical_view_distance / 10.0;
    double max_view_distance = canonical_view_distance * 20.0;
    camera.place(target, acos(c_dir.y), atan2(c_dir.x, c_dir.z), view_distance, min_view_distance,
                 max_view_distance);
  }
  // Application::resize (application.cpp:180-192), EDIT_MODE: no set_frame_size
  if (w && h) { screenW = w; screenH = h; camera.set_screen_size(w, h); }
  if (cam_settings != "") camera.load_settings(cam_settings);

  // Application::render_to_file -> set_up_pathtracer (application.cpp:622-628)
  pt->set_camera(&camera);
  pt->set_scene(scene->get_static_scene());
  pt->set_frame_size(screenW, screenH);

  if (pt->envLight) {  // EnvironmentLight::init accumulates into new double[h]: must have started at zero
    StaticScene::EnvironmentLight* el = pt->envLight;
    const HDRImageBuffer* em = el->envMap;
    double run = 0;
    for (size_t j = 0; j < em->h; ++j) {
      double row = 0;
      for (size_t i = 0; i < em->w; ++i) row += el->pdf_envmap[em->w * j + i];
      run = (j > 0) ? row + run : row;
      if (run != el->marginal_y[j]) {
        std::fprintf(stderr, "[harness] EnvironmentLight::marginal_y[%zu] was not zero-initialised\n", j);
        return 6;
      }
    }
  }
  dump_scene(prefix + ".rrts", pt->scene);
  dump_camera(prefix + ".rrtc", pt->camera);
  dump_bvh(prefix, pt->scene, pt->bvh->root);
  if (dump_only) return 0;

  g_frame_w = pt->sampleBuffer.w;
  g_frame_h = pt->sampleBuffer.h;
  g_pixels.assign(g_frame_w * g_frame_h, PixelRecord{});
  // Cell mode (-p) sizes tile_samples for the cell's 8-pixel tiles but raytrace_tile indexes it
  // by absolute 32-pixel tile coordinates (pathtracer.cpp:256-258 vs :561-579): the increments
  // land past the end of the vector, corrupting the heap (observed aborts at 4K).  The counts are
  // never read for the image, so give the vector enough capacity that the reference's own
  // resize() keeps a buffer the stray increments stay inside.
  pt->tile_samples.reserve((size_t)1 << 22);
  pt->render_to_file(filename, x, y, dx, dy);

  // region actually rendered
  size_t x0 = 0, y0 = 0, rw = g_frame_w, rh = g_frame_h;
  if (x != (size_t)-1) { x0 = x; y0 = y; rw = dx; rh = dy; }
  std::vector<float> rgb(rw * rh * 3);
  std::vector<int32_t> cnt(rw * rh);
  std::vector<uint32_t> draws(rw * rh), bbt(rw * rh), mst(rw * rh);
  size_t missing = 0;
  for (size_t j = 0; j < rh; ++j)
    for (size_t i = 0; i < rw; ++i) {
      const PixelRecord& r = g_pixels[(y0 + j) * g_frame_w + (x0 + i)];
      size_t k = j * rw + i;
      missing += r.done ? 0 : 1;
      rgb[3 * k] = r.rgb[0]; rgb[3 * k + 1] = r.rgb[1]; rgb[3 * k + 2] = r.rgb[2];
      cnt[k] = r.count; draws[k] = r.draws; bbt[k] = r.bbox_tests; mst[k] = r.micro_steps;
    }
  if (missing) { std::fprintf(stderr, "[harness] %zu pixels of the region were not rendered\n", missing); return 5; }
  harness::write_npy(prefix + "_px_rgb.npy", "<f4", {rh, rw, 3}, rgb.data(), rgb.size() * 4);
  harness::write_npy(prefix + "_px_count.npy", "<i4", {rh, rw}, cnt.data(), cnt.size() * 4);
  harness::write_npy(prefix + "_px_draws.npy", "<u4", {rh, rw}, draws.data(), draws.size() * 4);
  harness::write_npy(prefix + "_px_bbox_tests.npy", "<u4", {rh, rw}, bbt.data(), bbt.size() * 4);
  harness::write_npy(prefix + "_px_micro_steps.npy", "<u4", {rh, rw}, mst.data(), mst.size() * 4);
  uint64_t meta[8] = {x0, y0, rw, rh, g_frame_w, g_frame_h, g_seed, (uint64_t)pt->bvh->total_isects};
  harness::write_npy(prefix + "_px_meta.npy", "<u8", {8}, meta, sizeof(meta));
  return 0;
}
