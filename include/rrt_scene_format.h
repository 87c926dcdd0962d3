/* rrt_scene_format.h -- on-disk flattened static scene (.rrts) and camera (.rrtc) records.
 *
 * These files are what the reference's StaticScene / Camera hold after
 * Application::load + set_up_pathtracer (application.cpp:219-295, :622-628;
 * dynamic_scene/scene.cpp:133-145 get_static_scene).  They are produced by the oracle
 * harness (oracle/ref/harness_render.cpp) from the reference itself, and consumed by the
 * product's host loader (rrt_scene_load in include/rrt.h) and by the CPU restatement.
 * All values little-endian; doubles are the reference's exact Vector3D components.
 *
 * .rrts
 *   char     magic[8]  = "RRTSCN1\0"
 *   uint32   n_bsdfs, n_objects, n_lights, reserved
 *   BSDF     bsdfs[n_bsdfs]           64 B each:  uint32 type, uint32 pad, float p[14]
 *              type 0 Diffuse     p[0..2] reflectance                  (bsdf.h:118-133)
 *              type 1 Emission    p[0..2] radiance                     (bsdf.h:184-199)
 *              type 2 Mirror      p[0..2] reflectance                  (bsdf.h:91-106)
 *              type 3 Glass       p[0..2] transmittance, p[3..5] reflectance,
 *                                 p[6] roughness, p[7] ior            (bsdf.h:162-182)
 *              type 4 Microfacet  p[0..2] eta, p[3..5] k, p[6] alpha   (bsdf.h:109-141)
 *              type 5 Refraction  p[0..2] transmittance, p[6] roughness, p[7] ior (stub)
 *   Object   objects[n_objects]       in StaticScene::Scene::objects order (= BVH build order)
 *              uint32 kind (0 mesh, 1 sphere), uint32 bsdf, uint32 a, uint32 b
 *              mesh:   a = n_vertices, b = n_triangles, then
 *                      double positions[a][3], double normals[a][3], uint32 indices[b][3]
 *                      (object.cpp:16-58: triangle t = indices[t], Mesh::get_primitives order)
 *              sphere: double center[3], double radius        (object.cpp:66-80)
 *   Light    lights[n_lights]         120 B each:
 *              uint32 type, uint32 is_delta, float radiance[3], float area, double v[4][3]
 *              type 0 Area         v[0] position, v[1] direction, v[2] dim_x, v[3] dim_y;
 *                                  area = (float)(|dim_x| * |dim_y|)   (light.cpp:74-92)
 *              type 1 Point        v[0] position                       (light.cpp:46-57)
 *              type 2 Directional  v[0] dirToLight                     (light.cpp:11-23)
 *              type 3 InfiniteHemisphere  v[0..2] sampleToWorld columns (light.cpp:27-42)
 *              type 4 unsupported stub (Spot / Sphere / Mesh lights: light.cpp:59-115)
 *              type 5 environment map (needs the envmap payload; not in this format yet)
 *
 * .rrtc  (Camera fields, camera.h; after configure/place/set_screen_size)
 *   char     magic[8] = "RRTCAM1\0"
 *   double   hFov, vFov, ar, nClip, fClip, pos[3], targetPos[3], phi, theta, r, minR, maxR,
 *            c2w[9] (row-major, c2w(i/3, i%3) as Camera::dump_settings), screenW, screenH,
 *            screenDist, focalDistance, lensRadius
 */
#ifndef RRT_SCENE_FORMAT_H
#define RRT_SCENE_FORMAT_H

#define RRT_SCENE_MAGIC "RRTSCN1"
#define RRT_CAMERA_MAGIC "RRTCAM1"
#define RRT_CAMERA_NDOUBLES 30

#endif
