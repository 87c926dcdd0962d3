// rrt_ingest.cpp -- native scene ingest: COLLADA (.dae) -> flattened static scene + the camera
// the reference places for it (include/rrt.h rrt_collada_load), plus the camera-record helpers
// (.rrtc binary, the `-c` text settings format) and the .rrts writer.
//
// Host-only C++ (no HIP).  It reproduces, value for value, what the reference computes between
// reading a .dae file and handing PathTracer its StaticScene and Camera:
//   Collada::ColladaParser::load / parse_node / parse_* (collada/collada.cpp:131-936)
//   Application::load (application.cpp:219-295)  +  Application::init's default camera (:90-96)
//   DynamicScene::Mesh ctor (dynamic_scene/mesh.cpp:17-35) -> HalfedgeMesh::build
//     (halfEdgeMesh.cpp:29-397) with Vertex::computeNormal (halfEdgeMesh.h:492-515)
//   StaticScene::Mesh (static_scene/object.cpp:16-41): vertex labels, one triangle per face
//   DynamicScene::Sphere / lights -> get_static_object / get_static_light
//     (dynamic_scene/sphere.cpp:8-16, *_light.h, static_scene/light.cpp:11-78)
//   Camera::configure / place / compute_position / set_screen_size (camera.cpp:22-119)
//   Camera::load_settings / dump_settings (camera.cpp:138-169)
// The arithmetic keeps the reference's operation order (Matrix4x4 * Vector4D as a column sum,
// 1/w projection, Vector3D::normalize as a multiply by 1./norm), and parses numbers the way
// libstdc++ streams and atof do (strtof for `>> float`, strtod then narrowing for atof).
// Reference quirks kept on purpose: a polygon contributes ONE triangle made of its last, first
// and second vertices (the face's halfedge is the last one built); <scale> writes its z factor
// into the y slot; a <matrix> ends a node's transform list; rotate/translate/scale start from a
// zero matrix; every material instance gets its own BSDF record.
// Deliberate difference: malformed input (which the reference answers with exit(1) or a crash)
// returns RRT_E_INVALID with a message instead.
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "../../include/rrt.h"
#include "../../include/rrt_scene_format.h"
#include "rrt_scene_file.h"

namespace {

constexpr double kPi = 3.14159265358979323;  // CGL misc.h:11
constexpr float kEpsF = 0.00001f;            // CGL misc.h:13

struct IngestError { std::string msg; };
[[noreturn]] void bad(const std::string& m) { throw IngestError{m}; }

// ------------------------------------------------------------------------------- small XML DOM
// Enough of XML for COLLADA: elements, attributes, character data, comments, <? ?>, <!...>,
// CDATA and the predefined entities.  `text` is the character data before the element's first
// child node (tinyxml2's GetText()).
struct XEl {
  std::string name;
  std::vector<std::pair<std::string, std::string>> attrs;
  std::string text;
  bool has_text = false;
  std::vector<XEl*> kids;
  XEl* next = nullptr;  // next sibling element

  const char* attr(const char* k) const {
    for (auto& a : attrs)
      if (a.first == k) return a.second.c_str();
    return nullptr;
  }
  XEl* first(const char* nm = nullptr) const {
    for (XEl* k : kids)
      if (!nm || k->name == nm) return k;
    return nullptr;
  }
  XEl* next_named(const char* nm = nullptr) const {
    for (XEl* s = next; s; s = s->next)
      if (!nm || s->name == nm) return s;
    return nullptr;
  }
};

class XDoc {
 public:
  std::vector<std::unique_ptr<XEl>> pool;
  XEl* root = nullptr;

  void parse(const std::string& s) {
    size_t i = 0, n = s.size();
    std::vector<XEl*> stack;
    bool child_seen = false;  // current element already has a child node (text no longer "first")
    auto decode = [](const std::string& raw) {
      std::string out;
      out.reserve(raw.size());
      for (size_t k = 0; k < raw.size(); ++k) {
        if (raw[k] != '&') { out += raw[k]; continue; }
        size_t e = raw.find(';', k);
        if (e == std::string::npos) { out += raw[k]; continue; }
        std::string ent = raw.substr(k + 1, e - k - 1);
        if (ent == "lt") out += '<';
        else if (ent == "gt") out += '>';
        else if (ent == "amp") out += '&';
        else if (ent == "quot") out += '"';
        else if (ent == "apos") out += '\'';
        else if (!ent.empty() && ent[0] == '#') {
          long cp = (ent.size() > 1 && (ent[1] == 'x' || ent[1] == 'X')) ? std::strtol(ent.c_str() + 2, nullptr, 16)
                                                                          : std::strtol(ent.c_str() + 1, nullptr, 10);
          if (cp < 0x80) out += (char)cp; else out += '?';
        } else { out += raw.substr(k, e - k + 1); }
        k = e;
      }
      return out;
    };
    auto add_text = [&](const std::string& t) {
      if (stack.empty()) return;
      bool blank = t.find_first_not_of(" \t\r\n") == std::string::npos;
      if (blank) return;  // whitespace-only runs are not text nodes
      XEl* top = stack.back();
      if (!child_seen && !top->has_text) { top->text = t; top->has_text = true; }
      child_seen = true;
    };
    while (i < n) {
      if (s[i] != '<') {
        size_t e = s.find('<', i);
        if (e == std::string::npos) e = n;
        add_text(decode(s.substr(i, e - i)));
        i = e;
        continue;
      }
      if (s.compare(i, 4, "<!--") == 0) {
        size_t e = s.find("-->", i + 4);
        if (e == std::string::npos) bad("XML: unterminated comment");
        if (!stack.empty()) child_seen = true;
        i = e + 3;
        continue;
      }
      if (s.compare(i, 9, "<![CDATA[") == 0) {
        size_t e = s.find("]]>", i + 9);
        if (e == std::string::npos) bad("XML: unterminated CDATA");
        add_text(s.substr(i + 9, e - i - 9));
        i = e + 3;
        continue;
      }
      if (s.compare(i, 2, "<?") == 0 || s.compare(i, 2, "<!") == 0) {
        size_t e = s.find('>', i);
        if (e == std::string::npos) bad("XML: unterminated declaration");
        i = e + 1;
        continue;
      }
      if (s.compare(i, 2, "</") == 0) {
        size_t e = s.find('>', i);
        if (e == std::string::npos || stack.empty()) bad("XML: stray end tag");
        std::string nm = s.substr(i + 2, e - i - 2);
        while (!nm.empty() && std::isspace((unsigned char)nm.back())) nm.pop_back();
        if (nm != stack.back()->name) bad("XML: mismatched end tag </" + nm + ">");
        stack.pop_back();
        child_seen = true;
        i = e + 1;
        continue;
      }
      // start tag
      size_t k = i + 1;
      while (k < n && !std::isspace((unsigned char)s[k]) && s[k] != '>' && s[k] != '/') ++k;
      pool.emplace_back(new XEl());
      XEl* el = pool.back().get();
      el->name = s.substr(i + 1, k - i - 1);
      bool self_close = false;
      for (;;) {
        while (k < n && std::isspace((unsigned char)s[k])) ++k;
        if (k >= n) bad("XML: unterminated start tag");
        if (s[k] == '>') { ++k; break; }
        if (s[k] == '/') { self_close = true; k = s.find('>', k); if (k == std::string::npos) bad("XML: bad tag"); ++k; break; }
        size_t a0 = k;
        while (k < n && s[k] != '=' && !std::isspace((unsigned char)s[k])) ++k;
        std::string an = s.substr(a0, k - a0);
        while (k < n && s[k] != '=') ++k;
        ++k;
        while (k < n && std::isspace((unsigned char)s[k])) ++k;
        if (k >= n || (s[k] != '"' && s[k] != '\'')) bad("XML: unquoted attribute");
        char q = s[k];
        size_t v1 = s.find(q, k + 1);
        if (v1 == std::string::npos) bad("XML: unterminated attribute");
        el->attrs.emplace_back(an, decode(s.substr(k + 1, v1 - k - 1)));
        k = v1 + 1;
      }
      if (stack.empty()) {
        if (root) bad("XML: more than one root element");
        root = el;
      } else {
        XEl* parent = stack.back();
        if (!parent->kids.empty()) parent->kids.back()->next = el;
        parent->kids.push_back(el);
      }
      if (!self_close) { stack.push_back(el); child_seen = false; }
      else child_seen = true;
      i = k;
    }
    if (!stack.empty()) bad("XML: unclosed element <" + stack.back()->name + ">");
    if (!root) bad("XML: no root element");
  }
};

// Number scanning like an istringstream over the element text.
struct Scan {
  std::string buf;  // own copy: callers may pass temporaries
  const char* p;
  explicit Scan(std::string s) : buf(std::move(s)), p(buf.c_str()) {}
  bool f32(float& v) {  // `ss >> float` (libstdc++: strtof)
    char* e; float x = std::strtof(p, &e);
    if (e == p) { v = 0; return false; }
    v = x; p = e; return true;
  }
  bool f64(double& v) {
    char* e; double x = std::strtod(p, &e);
    if (e == p) { v = 0; return false; }
    v = x; p = e; return true;
  }
  bool uz(size_t& v) {
    char* e; unsigned long long x = std::strtoull(p, &e, 10);
    if (e == p) { v = 0; return false; }
    v = (size_t)x; p = e; return true;
  }
};
inline float atof_f(const char* s) { return (float)std::atof(s); }  // float field = atof(...)

// ------------------------------------------------------------------------------- CGL arithmetic
struct D3 { double x, y, z; };
inline D3 d3(double x, double y, double z) { return D3{x, y, z}; }
inline D3 operator-(D3 a, D3 b) { return d3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline D3 operator+(D3 a, D3 b) { return d3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline D3 neg(D3 a) { return d3(-a.x, -a.y, -a.z); }
inline D3 cross(D3 u, D3 v) { return d3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x); }
inline double norm(D3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
inline D3 normalized(D3 a) {  // Vector3D::normalize: *this *= (1./norm())
  double c = 1. / norm(a);
  return d3(a.x * c, a.y * c, a.z * c);
}
inline D3 unit(D3 a) {  // Vector3D::unit: rNorm * x
  double r = 1. / std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
  return d3(r * a.x, r * a.y, r * a.z);
}
inline D3 scaled(D3 a, double c) { return d3(a.x * c, a.y * c, a.z * c); }

// 4x4 matrix, M[i][j] = row i, column j.  Default: zero (CGL Matrix4x4's default ctor leaves the
// entries as zero Vector4Ds).
struct M4 {
  double m[4][4] = {};
  static M4 identity() { M4 r; for (int i = 0; i < 4; ++i) r.m[i][i] = 1.; return r; }
  M4 operator*(const M4& B) const {  // C(i,j) = 0. + sum_k A(i,k) B(k,j), k ascending
    M4 C;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        double acc = 0.;
        for (int k = 0; k < 4; ++k) acc += m[i][k] * B.m[k][j];
        C.m[i][j] = acc;
      }
    return C;
  }
  // Matrix4x4 * Vector4D = v0*col0 + v1*col1 + v2*col2 + v3*col3 (left to right)
  void apply(const double v[4], double out[4]) const {
    for (int i = 0; i < 4; ++i) {
      double a = v[0] * m[i][0] + v[1] * m[i][1];
      a = a + v[2] * m[i][2];
      out[i] = a + v[3] * m[i][3];
    }
  }
  D3 to3D(D3 p, double w) const {
    double v[4] = {p.x, p.y, p.z, w}, o[4];
    apply(v, o);
    return d3(o[0], o[1], o[2]);
  }
  D3 project(D3 p) const {  // (M * (p, 1)).projectTo3D(): invW = 1.0 / w
    double v[4] = {p.x, p.y, p.z, 1.0}, o[4];
    apply(v, o);
    double iw = 1.0 / o[3];
    return d3(o[0] * iw, o[1] * iw, o[2] * iw);
  }
};

// ------------------------------------------------------------------------------- COLLADA model
enum class Kind { None, Camera, Light, Sphere, Mesh };
enum class LightKind { None, Ambient, Directional, Area, Point, Spot };

struct Bsdf { uint32_t type = RRT_BSDF_DIFFUSE; float p[14] = {0}; };

struct Instance {
  Kind kind = Kind::None;
  // camera (CameraInfo: float fields)
  float hFov = 0, vFov = 0, nClip = 0, fClip = 0;
  // light (LightInfo defaults, light_info.cpp:5-19)
  LightKind lkind = LightKind::None;
  float spectrum[3] = {1, 1, 1};
  // sphere
  float radius = 0;
  // mesh
  std::vector<D3> vertices;
  std::vector<std::vector<size_t>> polygons;
  // material (sphere / mesh)
  bool has_bsdf = false;
  Bsdf bsdf;
};

struct Node { M4 transform = M4::identity(); Instance inst; };

class Collada {
 public:
  std::vector<Node> nodes;

  void load(const XEl* root) {
    if (root->name != "COLLADA") bad("not a COLLADA file");
    index_ids(root);
    up_fix_ = M4::identity();
    if (XEl* asset = get(root, "asset")) {
      XEl* up = get(asset, "up_axis");
      if (!up) bad("no up_axis in <asset>");
      std::string dir = up->text;
      if (dir == "X_UP") {
        up_fix_.m[0][0] = 0; up_fix_.m[0][1] = 1;
        up_fix_.m[1][0] = 1; up_fix_.m[1][1] = 0;
        up_fix_.m[2][2] = -1;
      } else if (dir == "Z_UP") {
        up_fix_.m[1][1] = 0; up_fix_.m[1][2] = 1;
        up_fix_.m[2][1] = 1; up_fix_.m[2][2] = 0;
        up_fix_.m[0][0] = -1;
      } else if (dir != "Y_UP") {
        bad("invalid up_axis '" + dir + "'");
      }
    }
    XEl* vs = get(root, "scene/instance_visual_scene");
    if (!vs) bad("no <scene>/<instance_visual_scene>");
    current_ = up_fix_;
    for (XEl* n = get(vs, "node"); n; n = n->next_named("node")) node(n);
  }

 private:
  std::map<std::string, XEl*> ids_;
  M4 up_fix_, current_;

  void index_ids(const XEl* e) {
    if (const char* id = e->attr("id")) ids_[id] = const_cast<XEl*>(e);
    for (XEl* k : e->kids) index_ids(k);
  }
  XEl* find_id(const std::string& id) const {
    auto it = ids_.find(id);
    return it == ids_.end() ? nullptr : it->second;
  }
  // ColladaParser::get_element: first-child path walk; a final element with url="#id" resolves
  XEl* get(const XEl* e, const std::string& path) const {
    XEl* cur = const_cast<XEl*>(e);
    size_t a = 0;
    while (cur && a <= path.size()) {
      size_t b = path.find('/', a);
      if (b == std::string::npos) b = path.size();
      cur = cur->first(path.substr(a, b - a).c_str());
      a = b + 1;
    }
    if (cur)
      if (const char* url = cur->attr("url")) cur = find_id(std::string(url + (url[0] ? 1 : 0)));
    return cur;
  }
  XEl* technique_common(const XEl* e) const {
    if (XEl* prof = e->first("profile_COMMON"))
      for (XEl* t = prof->first("technique"); t; t = t->next_named("technique")) {
        const char* sid = t->attr("sid");
        if (sid && std::string(sid) == "common") return t;
      }
    return e->first("technique_common");
  }
  XEl* technique_cgl(const XEl* e) const {
    for (XEl* t = get(e, "extra/technique"); t; t = t->next_named("technique")) {
      const char* pr = t->attr("profile");
      if (pr && std::string(pr) == "CGL") return t;
    }
    return nullptr;
  }
  static const std::string& text_of(const XEl* e, const char* what) {
    if (!e || !e->has_text) bad(std::string("missing text for ") + what);
    return e->text;
  }
  static void spectrum(const std::string& s, float out[3]) {
    Scan sc(s);
    sc.f32(out[0]); sc.f32(out[1]); sc.f32(out[2]);
  }

  void node(XEl* x) {  // parse_node (collada.cpp:234-430)
    Node nd;
    for (XEl* e = x->first(); e; e = e->next) {
      const std::string& nm = e->name;
      if (nm == "matrix") {
        Scan sc(text_of(e, "matrix"));
        M4 mat;
        for (int i = 0; i < 4; ++i)
          for (int j = 0; j < 4; ++j) sc.f64(mat.m[i][j]);
        nd.transform = mat;
        break;
      }
      if (nm == "rotate") {
        M4 r;  // zero matrix; four numbers land in the axis' 2x2 block
        Scan sc(text_of(e, "rotate"));
        const char* sid = e->attr("sid");
        char axis = (sid && *sid) ? sid[std::strlen(sid) - 1] : 0;
        if (axis == 'X') { sc.f64(r.m[1][1]); sc.f64(r.m[1][2]); sc.f64(r.m[2][1]); sc.f64(r.m[2][2]); }
        else if (axis == 'Y') { sc.f64(r.m[0][0]); sc.f64(r.m[2][0]); sc.f64(r.m[0][2]); sc.f64(r.m[2][2]); }
        else if (axis == 'Z') { sc.f64(r.m[0][0]); sc.f64(r.m[0][1]); sc.f64(r.m[1][0]); sc.f64(r.m[1][1]); }
        nd.transform = r * nd.transform;
      }
      if (nm == "translate") {
        M4 t;
        Scan sc(text_of(e, "translate"));
        sc.f64(t.m[0][3]); sc.f64(t.m[1][3]); sc.f64(t.m[2][3]);
        nd.transform = t * nd.transform;
      }
      if (nm == "scale") {
        M4 s;
        Scan sc(text_of(e, "scale"));
        sc.f64(s.m[0][0]); sc.f64(s.m[1][1]); sc.f64(s.m[1][1]);
        nd.transform = s * nd.transform;
      }
    }
    M4 saved = current_;
    nd.transform = current_ * nd.transform;
    current_ = nd.transform;
    for (XEl* c = get(x, "node"); c; c = c->next_named("node")) node(c);
    current_ = saved;

    XEl* cam = get(x, "instance_camera");
    XEl* light = get(x, "instance_light");
    XEl* geom = get(x, "instance_geometry");
    if (cam) {
      camera(cam, nd.inst);
    } else if (light) {
      this->light(light, nd.inst);
    } else if (geom) {
      if (get(geom, "mesh")) {
        mesh(geom, nd.inst);
        bind_material(x, nd.inst);
      } else if (get(geom, "extra")) {
        sphere(geom, nd.inst);
        bind_material(x, nd.inst);
      }
    }
    nodes.push_back(std::move(nd));
  }

  void camera(XEl* x, Instance& c) {  // parse_camera (collada.cpp:432-473)
    c.kind = Kind::Camera;
    XEl* p = get(x, "optics/technique_common/perspective");
    if (!p) bad("camera without <perspective>");
    XEl* xf = p->first("xfov");
    XEl* yf = p->first("yfov");
    XEl* zn = p->first("znear");
    XEl* zf = p->first("zfar");
    c.hFov = xf ? atof_f(text_of(xf, "xfov").c_str()) : 50.0f;
    c.vFov = yf ? atof_f(text_of(yf, "yfov").c_str()) : 35.0f;
    c.nClip = zn ? atof_f(text_of(zn, "znear").c_str()) : 0.001f;
    c.fClip = zf ? atof_f(text_of(zf, "zfar").c_str()) : 1000.0f;
    if (!yf) {
      XEl* ar = get(p, "aspect_ratio");
      if (!ar) bad("camera perspective has neither yfov nor aspect_ratio");
      float aspect = atof_f(text_of(ar, "aspect_ratio").c_str());
      double half = 0.5 * c.hFov;
      c.vFov = (float)(2 * ((std::atan(std::tan(half * (kPi / 180)) / aspect)) * (180 / kPi)));
    }
  }

  void light(XEl* x, Instance& l) {  // parse_light (collada.cpp:475-576)
    l.kind = Kind::Light;
    XEl* tech = technique_cgl(x);
    if (!tech) tech = technique_common(x);
    if (!tech) bad("light without a supported technique");
    XEl* e = tech->first();
    if (!e) return;
    const std::string& type = e->name;
    XEl* color = get(e, "color");
    if (type == "ambient") l.lkind = LightKind::Ambient;
    else if (type == "directional") l.lkind = LightKind::Directional;
    else if (type == "area") l.lkind = LightKind::Area;
    else if (type == "point") {
      l.lkind = LightKind::Point;
      if (!get(e, "constant_attenuation") || !get(e, "linear_attenuation") || !get(e, "quadratic_attenuation"))
        bad("incomplete point light");
    } else if (type == "spot") {
      l.lkind = LightKind::Spot;
      if (!e->first("falloff_angle") || !e->first("falloff_exponent") || !get(e, "constant_attenuation") ||
          !get(e, "linear_attenuation") || !get(e, "quadratic_attenuation"))
        bad("incomplete spot light");
    } else {
      bad("unsupported light type '" + type + "'");
    }
    if (!color) bad("light without <color>");
    spectrum(text_of(color, "color"), l.spectrum);
  }

  void sphere(XEl* x, Instance& s) {  // parse_sphere (collada.cpp:578-601)
    s.kind = Kind::Sphere;
    XEl* tech = technique_cgl(x);
    if (!tech) bad("sphere geometry without a CGL technique");
    XEl* r = get(tech, "sphere/radius");
    if (!r) bad("sphere without radius");
    s.radius = atof_f(text_of(r, "radius").c_str());
  }

  void mesh(XEl* x, Instance& pm) {  // parse_polymesh (collada.cpp:604-850)
    pm.kind = Kind::Mesh;
    XEl* m = x->first("mesh");
    if (!m) bad("geometry without <mesh>");
    std::map<std::string, std::vector<float>> arrays;
    for (XEl* src = m->first("source"); src; src = src->next_named("source")) {
      XEl* fa = src->first("float_array");
      const char* id = src->attr("id");
      if (!fa || !id) continue;
      const char* cnt = fa->attr("count");
      size_t count = cnt ? (size_t)std::strtoll(cnt, nullptr, 10) : 0;
      std::vector<float> v;
      v.reserve(count);
      Scan sc(fa->has_text ? fa->text : std::string());
      float f = 0;
      for (size_t i = 0; i < count; ++i) { sc.f32(f); v.push_back(f); }
      arrays[id] = std::move(v);
    }
    XEl* verts = m->first("vertices");
    if (!verts) bad("mesh without <vertices>");
    const char* vid = verts->attr("id");
    std::string vertices_id = vid ? vid : "";
    std::vector<D3> positions;
    for (XEl* in = verts->first("input"); in; in = in->next_named("input")) {
      const char* sem = in->attr("semantic");
      const char* src = in->attr("source");
      if (!sem || std::string(sem) != "POSITION") continue;
      auto it = arrays.find(src ? src + 1 : "");
      if (it == arrays.end()) bad("undefined POSITION source");
      const std::vector<float>& f = it->second;
      for (size_t i = 0; i + 2 < f.size(); i += 3)
        positions.push_back(d3(f[i], f[i + 1], f[i + 2]));
    }
    XEl* pl = m->first("polylist");
    if (!pl) return;  // (reference: empty polygon list)
    bool has_v = false, has_n = false, has_t = false;
    size_t off_v = 0;
    for (XEl* in = pl->first("input"); in; in = in->next_named("input")) {
      std::string sem = in->attr("semantic") ? in->attr("semantic") : "";
      const char* srcp = in->attr("source");
      std::string src = srcp ? srcp + 1 : "";
      const char* offp = in->attr("offset");
      size_t off = offp ? (size_t)std::strtoll(offp, nullptr, 10) : 0;
      if (sem == "VERTEX") {
        has_v = true; off_v = off;
        if (src != vertices_id) bad("VERTEX input does not name <vertices>");
        pm.vertices = positions;
      } else if (sem == "NORMAL") {
        has_n = true;
        if (!arrays.count(src)) bad("undefined NORMAL source");
      } else if (sem == "TEXCOORD") {
        has_t = true;
        if (!arrays.count(src)) bad("undefined TEXCOORD source");
      }
    }
    const char* cntp = pl->attr("count");
    size_t n_poly = cntp ? (size_t)std::strtoll(cntp, nullptr, 10) : 0;
    size_t stride = (has_v ? 1 : 0) + (has_n ? 1 : 0) + (has_t ? 1 : 0);
    XEl* vc = pl->first("vcount");
    if (!vc) bad("polylist without <vcount>");
    std::vector<size_t> sizes(n_poly);
    size_t n_idx = 0;
    {
      Scan sc(vc->has_text ? vc->text : std::string());
      for (size_t i = 0; i < n_poly; ++i) { sc.uz(sizes[i]); n_idx += sizes[i] * stride; }
    }
    XEl* p = pl->first("p");
    if (!p) bad("polylist without <p>");
    std::vector<size_t> idx(n_idx);
    {
      Scan sc(p->has_text ? p->text : std::string());
      size_t last = 0;
      for (size_t i = 0; i < n_idx; ++i) { if (sc.uz(last)) idx[i] = last; else idx[i] = 0; }
    }
    pm.polygons.assign(n_poly, {});
    if (has_v) {
      size_t k = 0;
      for (size_t i = 0; i < n_poly; ++i)
        for (size_t j = 0; j < sizes[i]; ++j, ++k) pm.polygons[i].push_back(idx[k * stride + off_v]);
    }
  }

  void bind_material(XEl* x, Instance& inst) {  // instance_material -> parse_material (:852-936)
    XEl* im = get(x, "instance_geometry/bind_material/technique_common/instance_material");
    if (!im) return;
    const char* target = im->attr("target");
    if (!target) bad("instance_material without target");
    XEl* mat = find_id(std::string(target + (target[0] ? 1 : 0)));
    if (!mat) bad(std::string("unknown material ") + target);
    XEl* eff = get(mat, "instance_effect");
    if (!eff) bad("material without instance_effect");
    XEl* common = technique_common(eff);
    XEl* cgl = technique_cgl(eff);
    Bsdf b;
    bool set = false;
    auto sp = [&](XEl* parent, const char* what, float* out) {
      XEl* e = get(parent, what);
      spectrum(text_of(e, what), out);
    };
    auto fl = [&](XEl* parent, const char* what) { return atof_f(text_of(get(parent, what), what).c_str()); };
    if (cgl) {
      for (XEl* e = cgl->first(); e; e = e->next) {
        const std::string& t = e->name;
        if (t == "emission") {
          b = Bsdf(); b.type = RRT_BSDF_EMISSION; sp(e, "radiance", b.p); set = true;
        } else if (t == "mirror") {
          b = Bsdf(); b.type = RRT_BSDF_MIRROR; sp(e, "reflectance", b.p); set = true;
        } else if (t == "microfacet") {
          b = Bsdf(); b.type = RRT_BSDF_MICROFACET;
          float alpha = fl(e, "alpha");
          sp(e, "eta", b.p); sp(e, "k", b.p + 3); b.p[6] = alpha; set = true;
        } else if (t == "refraction") {
          b = Bsdf(); b.type = RRT_BSDF_REFRACTION;
          sp(e, "transmittance", b.p); b.p[6] = fl(e, "roughness"); b.p[7] = fl(e, "ior"); set = true;
        } else if (t == "glass") {
          b = Bsdf(); b.type = RRT_BSDF_GLASS;
          sp(e, "transmittance", b.p); sp(e, "reflectance", b.p + 3);
          b.p[6] = fl(e, "roughness"); b.p[7] = fl(e, "ior"); set = true;
        }
      }
      if (!set) bad("CGL material without a supported BSDF");
    } else if (common) {
      b.type = RRT_BSDF_DIFFUSE;
      if (XEl* d = get(common, "phong/diffuse/color")) spectrum(text_of(d, "color"), b.p);
      else { b.p[0] = b.p[1] = b.p[2] = .5f; }
    } else {
      b.type = RRT_BSDF_DIFFUSE; b.p[0] = b.p[1] = b.p[2] = .5f;
    }
    inst.has_bsdf = true;
    inst.bsdf = b;
  }
};

// ------------------------------------------------------------------------------- halfedge mesh
// HalfedgeMesh::build + Vertex::computeNormal restated on index arrays.  Returns the vertex list
// (first-appearance order), its normals and one triangle per face.
struct FlatMesh { std::vector<D3> pos, nrm; std::vector<uint32_t> tri; };

FlatMesh build_halfedge(const std::vector<std::vector<size_t>>& polys, const std::vector<D3>& positions) {
  const int NONE = -1;
  std::map<size_t, int> vert_of;         // input index -> vertex id (vertex ids in creation order)
  std::vector<size_t> degree_in;         // polygons per vertex
  for (const auto& p : polys) {
    if (p.size() < 3) bad("polygon with fewer than three vertices");
    for (size_t a : p) {
      auto it = vert_of.find(a);
      if (it == vert_of.end()) { vert_of.emplace(a, (int)degree_in.size()); degree_in.push_back(1); }
      else degree_in[it->second]++;
    }
    std::vector<size_t> q(p);
    std::sort(q.begin(), q.end());
    if (std::adjacent_find(q.begin(), q.end()) != q.end()) bad("polygon with repeated vertices");
  }
  const size_t nV = degree_in.size(), nF = polys.size();
  std::vector<int> he_next, he_twin, he_vert, he_face;  // face >= nF: boundary loop
  std::vector<int> v_he(nV, NONE), f_he(nF, NONE);
  std::map<std::pair<size_t, size_t>, int> pair_he;
  for (size_t f = 0; f < nF; ++f) {
    const auto& p = polys[f];
    const size_t d = p.size();
    const int base = (int)he_next.size();
    for (size_t i = 0; i < d; ++i) {
      size_t a = p[i], b = p[(i + 1) % d];
      if (pair_he.count({a, b})) bad("non-manifold or inconsistently oriented edge");
      int h = (int)he_next.size();
      he_next.push_back(NONE); he_twin.push_back(NONE);
      he_vert.push_back(vert_of[a]); he_face.push_back((int)f);
      pair_he[{a, b}] = h;
      f_he[f] = h;
      v_he[vert_of[a]] = h;
      auto tw = pair_he.find({b, a});
      if (tw != pair_he.end()) { he_twin[h] = tw->second; he_twin[tw->second] = h; }
    }
    for (size_t i = 0; i < d; ++i) he_next[base + i] = base + (int)((i + 1) % d);
  }
  // boundary vertices: point at a twinless halfedge
  for (size_t v = 0; v < nV; ++v) {
    int h = v_he[v];
    do {
      if (he_twin[h] == NONE) { v_he[v] = h; break; }
      h = he_next[he_twin[h]];
    } while (h != v_he[v]);
  }
  // boundary loops (iterates over halfedges appended during the loop too; those have twins)
  int n_loops = 0;
  for (size_t h = 0; h < he_next.size(); ++h) {
    if (he_twin[h] != NONE) continue;
    const int loop_face = (int)(nF + n_loops++);
    std::vector<int> ring;
    int i = (int)h;
    do {
      int t = (int)he_next.size();
      he_next.push_back(NONE); he_twin.push_back(i);
      he_vert.push_back(he_vert[he_next[i]]); he_face.push_back(loop_face);
      he_twin[i] = t;
      ring.push_back(t);
      i = he_next[i];
      while (i != (int)h && he_twin[i] != NONE) i = he_next[he_twin[i]];
    } while (i != (int)h);
    const size_t d = ring.size();
    for (size_t p = 0; p < d; ++p) he_next[ring[p]] = ring[(p + d - 1) % d];
  }
  for (size_t v = 0; v < nV; ++v) v_he[v] = he_next[he_twin[v_he[v]]];
  auto boundary_face = [&](int h) { return he_face[h] >= (int)nF; };
  for (size_t v = 0; v < nV; ++v) {
    size_t count = 0;
    int h = v_he[v];
    do {
      if (!boundary_face(h)) count++;
      h = he_next[he_twin[h]];
    } while (h != v_he[v]);
    if (count != degree_in[v]) bad("non-manifold vertex");
  }
  if (positions.size() != nV) bad("vertex position count differs from the number of distinct polygon indices");
  FlatMesh out;
  out.pos.resize(nV);
  {
    size_t k = 0;
    for (auto& kv : vert_of) out.pos[kv.second] = positions[k++];  // ascending input index
  }
  out.nrm.resize(nV);
  for (size_t v = 0; v < nV; ++v) {
    const int h0 = v_he[v];
    bool on_boundary = false;
    {
      int h = h0;
      do {
        if (boundary_face(h)) { on_boundary = true; break; }
        h = he_next[he_twin[h]];
      } while (h != h0);
    }
    D3 n = d3(0., 0., 0.);
    const D3 pi = out.pos[v];
    int h = h0;
    do {
      D3 pj = out.pos[he_vert[he_next[h]]];
      D3 pk = out.pos[he_vert[he_next[he_next[h]]]];
      D3 c = cross(pj - pi, pk - pi);
      n.x += c.x; n.y += c.y; n.z += c.z;
      h = on_boundary ? he_twin[he_next[h]] : he_next[he_twin[h]];
    } while (h != h0);
    out.nrm[v] = normalized(n);
  }
  out.tri.reserve(3 * nF);
  for (size_t f = 0; f < nF; ++f) {
    int h = f_he[f];
    out.tri.push_back((uint32_t)he_vert[h]);
    out.tri.push_back((uint32_t)he_vert[he_next[h]]);
    out.tri.push_back((uint32_t)he_vert[he_next[he_next[h]]]);
  }
  return out;
}

// ------------------------------------------------------------------------------- camera
struct Cam {  // the fields of CGL::Camera that .rrtc records
  double hFov = 0, vFov = 0, ar = 0, nClip = 0, fClip = 0;
  D3 pos{}, target{};
  double phi = 0, theta = 0, r = 0, minR = 0, maxR = 0;
  D3 col[3]{};  // c2w columns
  size_t screenW = 0, screenH = 0;
  double screenDist = 0, focalDistance = 0, lensRadius = 0;

  static double rad(double d) { return d * (kPi / 180); }
  static double deg(double r) { return r * (180 / kPi); }
  void configure(float hfov, float vfov, float nclip, float fclip, size_t w, size_t h) {  // camera.cpp:22-40
    screenW = w; screenH = h;
    nClip = nclip; fClip = fclip; hFov = hfov; vFov = vfov;
    double ar1 = std::tan(rad(hFov) / 2) / std::tan(rad(vFov) / 2);
    ar = static_cast<double>(screenW) / screenH;
    if (ar1 < ar) hFov = 2 * deg(std::atan(std::tan(rad(vFov) / 2) * ar));
    else if (ar1 > ar) vFov = 2 * deg(std::atan(std::tan(rad(hFov) / 2) / ar));
    screenDist = ((double)screenH) / (2.0 * std::tan(rad(vFov) / 2));
  }
  void place(D3 tgt, double ph, double th, double rr, double mn, double mx) {  // camera.cpp:42-54
    double r_ = std::min(std::max(rr, mn), mx);
    double phi_ = (std::sin(ph) == 0) ? (ph + kEpsF) : ph;
    target = tgt; phi = phi_; theta = th; r = r_; minR = mn; maxR = mx;
    compute_position();
  }
  void compute_position() {  // camera.cpp:95-119
    double sinPhi = std::sin(phi);
    if (sinPhi == 0) { phi += kEpsF; sinPhi = std::sin(phi); }
    const D3 toCam = d3(r * sinPhi * std::sin(theta), r * std::cos(phi), r * sinPhi * std::cos(theta));
    pos = target + toCam;
    D3 up = d3(0, sinPhi > 0 ? 1 : -1, 0);
    D3 sx = normalized(cross(up, toCam));
    D3 sy = normalized(cross(toCam, sx));
    col[0] = sx; col[1] = sy; col[2] = unit(toCam);
  }
  void set_screen_size(size_t w, size_t h) {  // camera.cpp:68-74
    screenW = w; screenH = h;
    ar = 1.0 * screenW / screenH;
    hFov = 2 * deg(std::atan(((double)screenW) / (2 * screenDist)));
    vFov = 2 * deg(std::atan(((double)screenH) / (2 * screenDist)));
  }
  void to_state(rrt_camera_state* s) const {
    s->hFov = hFov; s->vFov = vFov; s->ar = ar; s->nClip = nClip; s->fClip = fClip;
    s->pos[0] = pos.x; s->pos[1] = pos.y; s->pos[2] = pos.z;
    s->targetPos[0] = target.x; s->targetPos[1] = target.y; s->targetPos[2] = target.z;
    s->phi = phi; s->theta = theta; s->r = r; s->minR = minR; s->maxR = maxR;
    for (int j = 0; j < 3; ++j) {  // row-major c2w(i, j) = component i of column j
      s->c2w[j] = col[j].x; s->c2w[3 + j] = col[j].y; s->c2w[6 + j] = col[j].z;
    }
    s->screenW = (double)screenW; s->screenH = (double)screenH; s->screenDist = screenDist;
    s->focalDistance = focalDistance; s->lensRadius = lensRadius;
  }
};

void set_err(char* err, size_t n, const std::string& m) {
  if (err && n) { std::snprintf(err, n, "%s", m.c_str()); }
}

}  // namespace

// ------------------------------------------------------------------------------- C ABI
extern "C" void rrt_collada_options_default(rrt_collada_options* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->screen_w = 800; o->screen_h = 600;  // Application::init (application.cpp:90-96)
  o->lens_radius = 0.25;                 // AppConfig (application.h:61-62)
  o->focal_distance = 4.7;
}

extern "C" int rrt_collada_load(const char* path, const rrt_collada_options* opt, rrt_scene_file** scene_out,
                                rrt_camera_state* cam_out, char* err, size_t err_len) {
  if (!path || !scene_out) { set_err(err, err_len, "null argument"); return RRT_E_INVALID; }
  *scene_out = nullptr;
  rrt_collada_options o;
  if (opt) o = *opt; else rrt_collada_options_default(&o);
  if (o.screen_w == 0 || o.screen_h == 0) { set_err(err, err_len, "screen size must be positive"); return RRT_E_INVALID; }
  std::string text;
  {
    FILE* f = std::fopen(path, "rb");
    if (!f) { set_err(err, err_len, std::string("cannot open ") + path); return RRT_E_IO; }
    char buf[1 << 16];
    size_t got;
    while ((got = std::fread(buf, 1, sizeof(buf), f)) > 0) text.append(buf, got);
    std::fclose(f);
  }
  try {
    XDoc doc;
    doc.parse(text);
    Collada dae;
    dae.load(doc.root);

    std::unique_ptr<rrt_scene_file> sc(new rrt_scene_file());
    // Application::init: default camera, then Application::load over the nodes
    Cam cam;
    cam.configure(50, 35, 0.01f, 100, 800, 600);
    D3 c_dir = d3(0, 0, 0);
    struct Box { D3 mn{INFINITY, INFINITY, INFINITY}, mx{-INFINITY, -INFINITY, -INFINITY};
      void add(D3 p) {
        mn.x = std::min(mn.x, p.x); mn.y = std::min(mn.y, p.y); mn.z = std::min(mn.z, p.z);
        mx.x = std::max(mx.x, p.x); mx.y = std::max(mx.y, p.y); mx.z = std::max(mx.z, p.z);
      } } bbox;
    // scene-wide bbox = expand(object bbox) in object order; std::min/max over boxes equals the
    // union over every point, so the per-object boxes are folded point by point here.
    for (const Node& nd : dae.nodes) {
      const Instance& in = nd.inst;
      const M4& T = nd.transform;
      switch (in.kind) {
        case Kind::None:
          break;  // (the reference dereferences a null instance here)
        case Kind::Camera: {
          c_dir = unit(T.to3D(d3(0, 0, -1), 1));
          cam.configure(in.hFov, in.vFov, in.nClip, in.fClip, 800, 600);
          break;
        }
        case Kind::Light: {
          rrt_light_desc L;
          std::memset(&L, 0, sizeof(L));
          const D3 li_pos = d3(0, 0, 0), li_dir = d3(0, 0, -1), li_up = d3(0, 1, 0);
          auto put = [&](int k, D3 v) { L.v[k][0] = v.x; L.v[k][1] = v.y; L.v[k][2] = v.z; };
          switch (in.lkind) {
            case LightKind::Ambient:
              L.type = RRT_LIGHT_HEMISPHERE; L.is_delta = 0;
              std::memcpy(L.radiance, in.spectrum, sizeof(L.radiance));
              put(0, d3(1, 0, 0)); put(1, d3(0, 0, -1)); put(2, d3(0, 1, 0));
              break;
            case LightKind::Directional: {
              D3 dir = normalized(neg(T.to3D(li_dir, 1)));
              L.type = RRT_LIGHT_DIRECTIONAL; L.is_delta = 1;
              std::memcpy(L.radiance, in.spectrum, sizeof(L.radiance));
              put(0, neg(unit(dir)));
              break;
            }
            case LightKind::Area: {
              D3 p = T.to3D(li_pos, 1);
              D3 dir = normalized(T.to3D(li_dir, 1) - p);
              D3 dx = T.to3D(cross(li_up, li_dir), 1) - p;
              D3 dy = T.to3D(li_up, 1) - p;
              L.type = RRT_LIGHT_AREA; L.is_delta = 0;
              std::memcpy(L.radiance, in.spectrum, sizeof(L.radiance));
              L.area = (float)(norm(dx) * norm(dy));
              put(0, p); put(1, dir); put(2, dx); put(3, dy);
              break;
            }
            case LightKind::Point:
              L.type = RRT_LIGHT_POINT; L.is_delta = 1;
              std::memcpy(L.radiance, in.spectrum, sizeof(L.radiance));
              put(0, T.to3D(li_pos, 1));
              break;
            case LightKind::Spot:
              L.type = 4; L.is_delta = 1;  // SpotLight: no sampling (light.cpp:61-69)
              break;
            case LightKind::None:
              bad("light node without a light type");
          }
          sc->lights.push_back(L);
          break;
        }
        case Kind::Sphere: {
          rrt_object_desc ob;
          std::memset(&ob, 0, sizeof(ob));
          D3 c = T.project(d3(0, 0, 0));
          double scale = norm(T.to3D(d3(1, 0, 0), 0));
          double r = in.radius * scale;
          ob.kind = RRT_OBJ_SPHERE;
          ob.center[0] = c.x; ob.center[1] = c.y; ob.center[2] = c.z; ob.radius = r;
          ob.bsdf = (uint32_t)sc->bsdfs.size();
          rrt_bsdf_desc b;
          std::memset(&b, 0, sizeof(b));
          if (in.has_bsdf) { b.type = in.bsdf.type; std::memcpy(b.params, in.bsdf.p, sizeof(b.params)); }
          else { b.type = RRT_BSDF_DIFFUSE; b.params[0] = b.params[1] = b.params[2] = .5f; }
          sc->bsdfs.push_back(b);
          sc->objects.push_back(ob);
          bbox.add(d3(c.x - r, c.y - r, c.z - r));
          bbox.add(d3(c.x + r, c.y + r, c.z + r));
          break;
        }
        case Kind::Mesh: {
          std::vector<D3> v(in.vertices.size());
          for (size_t i = 0; i < v.size(); ++i) v[i] = T.project(in.vertices[i]);
          FlatMesh fm = build_halfedge(in.polygons, v);
          rrt_object_desc ob;
          std::memset(&ob, 0, sizeof(ob));
          ob.kind = RRT_OBJ_MESH;
          ob.n_vertices = (uint32_t)fm.pos.size();
          ob.n_triangles = (uint32_t)(fm.tri.size() / 3);
          ob.bsdf = (uint32_t)sc->bsdfs.size();
          rrt_bsdf_desc b;
          std::memset(&b, 0, sizeof(b));
          if (in.has_bsdf) { b.type = in.bsdf.type; std::memcpy(b.params, in.bsdf.p, sizeof(b.params)); }
          else { b.type = RRT_BSDF_DIFFUSE; b.params[0] = b.params[1] = b.params[2] = .5f; }
          sc->bsdfs.push_back(b);
          std::vector<double> P(3 * fm.pos.size()), N(3 * fm.pos.size());
          for (size_t i = 0; i < fm.pos.size(); ++i) {
            P[3 * i] = fm.pos[i].x; P[3 * i + 1] = fm.pos[i].y; P[3 * i + 2] = fm.pos[i].z;
            N[3 * i] = fm.nrm[i].x; N[3 * i + 1] = fm.nrm[i].y; N[3 * i + 2] = fm.nrm[i].z;
            bbox.add(fm.pos[i]);
          }
          sc->dbl.push_back(std::move(P));
          sc->dbl.push_back(std::move(N));
          sc->idx.push_back(std::move(fm.tri));
          sc->objects.push_back(ob);
          break;
        }
      }
    }
    sc->finalize();
    if (bbox.mn.x > bbox.mx.x || bbox.mn.y > bbox.mx.y || bbox.mn.z > bbox.mx.z)
      bad("scene has no geometry (empty bounding box): no camera placement");
    // Application::load camera placement (application.cpp:265-290)
    D3 ext = bbox.mx - bbox.mn;
    D3 target = d3(bbox.mn.x + bbox.mx.x, bbox.mn.y + bbox.mx.y, bbox.mn.z + bbox.mx.z);
    target = scaled(target, 1.0 / 2);  // BBox::centroid: (min + max) / 2 via operator/ (rc = 1.0/c)
    double canonical = norm(ext) / 2 * 1.5;
    cam.place(target, std::acos(c_dir.y), std::atan2(c_dir.x, c_dir.z), canonical * 2, canonical / 10.0,
              canonical * 20.0);
    // Application::resize in windowless mode, then PathTracer::set_camera's lens parameters
    cam.set_screen_size(o.screen_w, o.screen_h);
    cam.lensRadius = o.lens_radius;
    cam.focalDistance = o.focal_distance;
    if (cam_out) cam.to_state(cam_out);
    *scene_out = sc.release();
    return RRT_OK;
  } catch (const IngestError& e) {
    set_err(err, err_len, std::string(path) + ": " + e.msg);
    return RRT_E_INVALID;
  }
}

// Camera::dump_settings / load_settings text format (camera.cpp:138-169).
extern "C" int rrt_camera_settings_load(const char* path, rrt_camera_state* s) {
  if (!path || !s) return RRT_E_INVALID;
  FILE* f = std::fopen(path, "rb");
  if (!f) return RRT_E_IO;
  std::string t;
  char buf[4096];
  size_t got;
  while ((got = std::fread(buf, 1, sizeof(buf), f)) > 0) t.append(buf, got);
  std::fclose(f);
  Scan sc(t);
  double* d[] = {&s->hFov, &s->vFov, &s->ar, &s->nClip, &s->fClip, &s->pos[0], &s->pos[1], &s->pos[2],
                 &s->targetPos[0], &s->targetPos[1], &s->targetPos[2], &s->phi, &s->theta, &s->r, &s->minR, &s->maxR};
  bool ok = true;
  for (double* p : d) ok = ok && sc.f64(*p);
  for (int i = 0; i < 9; ++i) ok = ok && sc.f64(s->c2w[i]);
  size_t w = 0, h = 0;
  ok = ok && sc.uz(w) && sc.uz(h);
  s->screenW = (double)w; s->screenH = (double)h;
  ok = ok && sc.f64(s->screenDist) && sc.f64(s->focalDistance) && sc.f64(s->lensRadius);
  return ok ? RRT_OK : RRT_E_IO;
}

extern "C" int rrt_camera_settings_save(const char* path, const rrt_camera_state* s) {
  if (!path || !s) return RRT_E_INVALID;
  FILE* f = std::fopen(path, "wb");
  if (!f) return RRT_E_IO;
  // ostream's default formatting: %g with 6 significant digits
  std::fprintf(f, "%g %g %g %g %g\n", s->hFov, s->vFov, s->ar, s->nClip, s->fClip);
  for (int i = 0; i < 3; ++i) std::fprintf(f, "%g ", s->pos[i]);
  for (int i = 0; i < 3; ++i) std::fprintf(f, "%g ", s->targetPos[i]);
  std::fprintf(f, "\n%g %g %g %g %g\n", s->phi, s->theta, s->r, s->minR, s->maxR);
  for (int i = 0; i < 9; ++i) std::fprintf(f, "%g ", s->c2w[i]);
  std::fprintf(f, "\n%zu %zu %g\n%g %g\n", (size_t)s->screenW, (size_t)s->screenH, s->screenDist, s->focalDistance,
               s->lensRadius);
  std::fclose(f);
  return RRT_OK;
}

extern "C" int rrt_camera_state_file_load(const char* path, rrt_camera_state* s) {
  if (!path || !s) return RRT_E_INVALID;
  FILE* f = std::fopen(path, "rb");
  if (!f) return RRT_E_IO;
  char magic[8];
  double d[RRT_CAMERA_NDOUBLES];
  bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, RRT_CAMERA_MAGIC, 8) == 0 &&
            std::fread(d, 1, sizeof(d), f) == sizeof(d);
  std::fclose(f);
  if (!ok) return RRT_E_IO;
  static_assert(sizeof(rrt_camera_state) == RRT_CAMERA_NDOUBLES * sizeof(double), "rrtc record layout");
  std::memcpy(s, d, sizeof(d));
  return RRT_OK;
}

extern "C" int rrt_camera_state_file_save(const char* path, const rrt_camera_state* s) {
  if (!path || !s) return RRT_E_INVALID;
  FILE* f = std::fopen(path, "wb");
  if (!f) return RRT_E_IO;
  bool ok = std::fwrite(RRT_CAMERA_MAGIC, 1, 8, f) == 8 && std::fwrite(s, 1, sizeof(*s), f) == sizeof(*s);
  std::fclose(f);
  return ok ? RRT_OK : RRT_E_IO;
}

extern "C" int rrt_camera_state_desc(const rrt_camera_state* s, rrt_camera_desc* out) {
  if (!s || !out) return RRT_E_INVALID;
  std::memset(out, 0, sizeof(*out));
  out->hFov = s->hFov; out->vFov = s->vFov; out->nClip = s->nClip; out->fClip = s->fClip;
  for (int i = 0; i < 3; ++i) out->pos[i] = s->pos[i];
  std::memcpy(out->c2w, s->c2w, sizeof(out->c2w));
  out->lensRadius = s->lensRadius; out->focalDistance = s->focalDistance;
  return RRT_OK;
}

// .rrts writer (layout: include/rrt_scene_format.h)
extern "C" int rrt_scene_file_save(const char* path, const rrt_scene_desc* s) {
  if (!path || !s) return RRT_E_INVALID;
  FILE* f = std::fopen(path, "wb");
  if (!f) return RRT_E_IO;
  bool ok = true;
  auto w = [&](const void* p, size_t n) { ok = ok && std::fwrite(p, 1, n, f) == n; };
  w(RRT_SCENE_MAGIC, 8);
  uint32_t hdr[4] = {s->n_bsdfs, s->n_objects, s->n_lights, 0};
  w(hdr, 16);
  for (uint32_t i = 0; i < s->n_bsdfs; ++i) {
    uint32_t tp[2] = {s->bsdfs[i].type, 0};
    w(tp, 8); w(s->bsdfs[i].params, 56);
  }
  for (uint32_t i = 0; i < s->n_objects; ++i) {
    const rrt_object_desc& o = s->objects[i];
    if (o.kind == RRT_OBJ_MESH) {
      uint32_t oh[4] = {o.kind, o.bsdf, o.n_vertices, o.n_triangles};
      w(oh, 16);
      w(o.positions, (size_t)o.n_vertices * 24);
      w(o.normals, (size_t)o.n_vertices * 24);
      w(o.indices, (size_t)o.n_triangles * 12);
    } else {
      uint32_t oh[4] = {o.kind, o.bsdf, 0, 0};
      w(oh, 16);
      double sp[4] = {o.center[0], o.center[1], o.center[2], o.radius};
      w(sp, 32);
    }
  }
  for (uint32_t i = 0; i < s->n_lights; ++i) {
    const rrt_light_desc& l = s->lights[i];
    uint32_t th[2] = {l.type, l.is_delta};
    float fv[4] = {l.radiance[0], l.radiance[1], l.radiance[2], l.area};
    w(th, 8); w(fv, 16); w(l.v, 96);
  }
  std::fclose(f);
  return ok ? RRT_OK : RRT_E_IO;
}
