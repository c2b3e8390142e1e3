// rt_host.cpp -- host side of the MI355X ray-traversal library: Tucano-semantics scene ingest, the
// reference's flat box partition (which defines closest-hit tie-breaking and the per-face box
// predicate), the traversal BVH build, camera setup, PPM output and the host-only C ABI entry points.
//
// Reference semantics restated here (file:line in plindhorst/Ray-Tracing-Project):
//   OBJ/MTL ingest      tucano/utils/objimporter.hpp:81-351, tucano/utils/mtlIO.hpp:36-140
//   normalisation       tucano/mesh.hpp:592-628, tucano/model.hpp:102-105,169-173
//   face normals        tucano/mesh.hpp:448-482
//   flat box partition  src/BoundingBox.cpp:41-161, src/flyscene.cpp:399-428
//   camera              tucano/camera.hpp:115-118,155-173,263-266; tucano/utils/flycamera.hpp:76-202
//   PPM writer          tucano/utils/ppmIO.hpp:135-156
#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <future>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "rt_scene.h"

using rt::f3;

namespace rt {
static thread_local std::string g_err;
static std::atomic<bool> g_debug_env{false};
void set_debug_env(bool on) { g_debug_env.store(on); }
const char* debug_env(const char* name) { return g_debug_env.load(std::memory_order_relaxed) ? getenv(name) : nullptr; }

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
}
}  // namespace rt

extern "C" const char* rt_last_error(void) { return rt::g_err.c_str(); }
extern "C" int rt_version(void) { return RT_API_VERSION; }

// =====================================================================================================
// Ingest (Tucano::MeshImporter semantics)
// =====================================================================================================
namespace {

void mtl_default(rt_material& m) {  // Tucano::Material::Mtl defaults (materials/mtl.hpp:22-40)
  for (int k = 0; k < 3; k++) { m.ka[k] = 0.3f; m.kd[k] = 0.5f; m.ks[k] = 1.0f; }
  m.shininess = 10.0f;
  m.optical_density = 0.0f;
  m.dissolve = 1.0f;
}

std::string path_name(const std::string& s) {  // getPathName (mtlIO.hpp:36-40)
  size_t found = s.find_last_of("/\\");
  return s.substr(0, found + 1);
}

void erase_crlf(std::string& s) {
  s.erase(std::remove(s.begin(), s.end(), '\n'), s.end());
  s.erase(std::remove(s.begin(), s.end(), '\r'), s.end());
}

// MaterialImporter::loadMTL (mtlIO.hpp:49-140): tokens split on single spaces, atof values
bool load_mtl(rt_mesh* m, const std::string& filename) {
  std::ifstream in(filename.c_str(), std::ios::in);
  if (!in) return false;
  for (std::string line; std::getline(in, line);) {
    std::stringstream ss(line);
    if (ss.str().empty()) continue;
    std::string s;
    std::vector<std::string> tok;
    while (std::getline(ss, s, ' ')) tok.push_back(s);
    if (tok.empty() || tok[0] == "#") continue;
    if (tok[0] == "newmtl") {
      rt_material mt;
      mtl_default(mt);
      m->mats.push_back(mt);
      std::string nm = tok.size() > 1 ? tok[1] : std::string();
      erase_crlf(nm);
      m->mat_names.push_back(nm);
      continue;
    }
    if (m->mats.empty()) continue;  // reference: materials.back() on an empty vector (UB); ignored
    rt_material& cur = m->mats.back();
    auto f = [&](size_t i) { return i < tok.size() ? (float)atof(tok[i].c_str()) : 0.0f; };
    if (tok[0] == "Ns") cur.shininess = f(1);
    else if (tok[0] == "Ka") { cur.ka[0] = f(1); cur.ka[1] = f(2); cur.ka[2] = f(3); }
    else if (tok[0] == "Kd") { cur.kd[0] = f(1); cur.kd[1] = f(2); cur.kd[2] = f(3); }
    else if (tok[0] == "Ks") { cur.ks[0] = f(1); cur.ks[1] = f(2); cur.ks[2] = f(3); }
    else if (tok[0] == "Ni") cur.optical_density = f(1);
    else if (tok[0] == "d") cur.dissolve = f(1);
  }
  if (m->mats.empty()) {  // "if no mtllib then just create a default material"
    rt_material mt;
    mtl_default(mt);
    m->mats.push_back(mt);
    m->mat_names.push_back("");
  }
  return true;
}

// istringstream >> float for the numeric tokens of v/vn lines (num_get -> strtof on the prefix)
int parse_floats(const char* s, const char* end, float* out, int n) {
  for (int k = 0; k < n; k++) {
    while (s < end && (*s == ' ' || *s == '\t' || *s == '\r' || *s == '\v' || *s == '\f')) s++;
    if (s >= end) return k;
    char* e;
    out[k] = strtof(s, &e);
    if (e == s) return k;
    s = e;
  }
  return n;
}

// Mesh::loadVertices bounding box / scale / centre (mesh.hpp:592-628); std::max/min argument order
void load_vertices(rt_mesh* m) {
  size_t nv = m->v4.size() / 4;
  m->scale = 1.0f;
  m->center[0] = m->center[1] = m->center[2] = 0.0f;
  if (nv == 0) return;
  const float* v = m->v4.data();
  float xMax = v[0], xMin = v[0], yMax = v[1], yMin = v[1], zMax = v[2], zMin = v[2];
  for (size_t i = 0; i < nv; i++) {
    const float* p = v + 4 * i;
    xMax = rt::smax(p[0], xMax); yMax = rt::smax(p[1], yMax); zMax = rt::smax(p[2], zMax);
    xMin = rt::smin(p[0], xMin); yMin = rt::smin(p[1], yMin); zMin = rt::smin(p[2], zMin);
  }
  float ext = rt::smax(rt::smax(std::fabs(xMax - xMin), std::fabs(yMax - yMin)), std::fabs(zMax - zMin));
  m->scale = (float)(1.0 / (double)ext);
  m->center[0] = (float)((double)(xMax + xMin) / 2.0);
  m->center[1] = (float)((double)(yMax + yMin) / 2.0);
  m->center[2] = (float)((double)(zMax + zMin) / 2.0);
}

// computeNormals (objimporter.hpp:81-106)
void compute_normals(rt_mesh* m, const std::vector<std::vector<uint32_t>>& groups) {
  size_t nv = m->v4.size() / 4;
  m->vn3.assign(3 * nv, 0.0f);
  auto V = [&](uint32_t i) { return f3{m->v4[4 * i], m->v4[4 * i + 1], m->v4[4 * i + 2]}; };
  for (const auto& g : groups)
    for (size_t i = 0; i + 2 < g.size(); i += 3) {
      f3 v0 = rt::normalized(rt::sub(V(g[i + 1]), V(g[i])));
      f3 v1 = rt::normalized(rt::sub(V(g[i + 2]), V(g[i])));
      f3 n = rt::normalized(rt::cross(v0, v1));
      for (int k = 0; k < 3; k++) {
        float* d = &m->vn3[3 * g[i + k]];
        d[0] = d[0] + n.x; d[1] = d[1] + n.y; d[2] = d[2] + n.z;
      }
    }
  for (size_t i = 0; i < nv; i++) {
    f3 n = rt::normalized(f3{m->vn3[3 * i], m->vn3[3 * i + 1], m->vn3[3 * i + 2]});
    m->vn3[3 * i] = n.x; m->vn3[3 * i + 1] = n.y; m->vn3[3 * i + 2] = n.z;
  }
}

// createFaces (mesh.hpp:448-482), normalizeModelMatrix + getShapeModelMatrix (model.hpp)
int finish_mesh(rt_mesh* m, const std::vector<std::vector<uint32_t>>& groups, const std::vector<int32_t>& gmat,
                bool have_vn) {
  const size_t nv = m->v4.size() / 4;
  // validate every index group before anything indexes with it (computeNormals included: the
  // reference reads and writes out of bounds here)
  if (nv > 0)
    for (const auto& ix : groups) {
      if (ix.size() % 3 != 0) {
        rt::set_error("index group of %zu indices is not a multiple of 3 (reference reads out of bounds)", ix.size());
        return RT_ERR_INVALID;
      }
      for (uint32_t id : ix)
        if (id >= nv) { rt::set_error("face vertex index %u out of range", id + 1); return RT_ERR_INVALID; }
    }
  load_vertices(m);
  if (!have_vn && nv > 0) compute_normals(m, groups);  // no vertices: no faces either (below)
  m->fidx.clear(); m->fn3.clear(); m->fmat.clear();
  auto V = [&](uint32_t i) { return f3{m->v4[4 * i], m->v4[4 * i + 1], m->v4[4 * i + 2]}; };
  if (nv > 0)
    for (size_t g = 0; g < groups.size(); g++) {
      const auto& ix = groups[g];
      for (size_t i = 0; i < ix.size(); i += 3) {
        for (int k = 0; k < 3; k++) m->fidx.push_back(ix[i + k]);
        m->fmat.push_back(gmat[g]);
        f3 v1 = rt::normalized(rt::sub(V(ix[i + 2]), V(ix[i])));
        f3 v0 = rt::normalized(rt::sub(V(ix[i + 1]), V(ix[i])));
        f3 n = rt::normalized(rt::cross(v0, v1));
        m->fn3.push_back(n.x); m->fn3.push_back(n.y); m->fn3.push_back(n.z);
      }
    }
  float shape[16], model[16];
  rt::identity4(shape);
  rt::scale4(shape, m->scale);
  rt::translate4(shape, f3{-m->center[0], -m->center[1], -m->center[2]});
  rt::identity4(model);
  rt::affmul(model, shape, m->M);
  return RT_OK;
}

}  // namespace

extern "C" int rt_mesh_load_obj(const char* path, rt_mesh** out) {
  if (!path || !out) { rt::set_error("rt_mesh_load_obj: null argument"); return RT_ERR_INVALID; }
  *out = nullptr;
  FILE* f = fopen(path, "rb");
  if (!f) { rt::set_error("Cannot open %s", path); return RT_ERR_IO; }
  std::string buf;
  fseek(f, 0, SEEK_END);
  long len = ftell(f);
  fseek(f, 0, SEEK_SET);
  buf.resize(len > 0 ? (size_t)len : 0);
  if (len > 0 && fread(&buf[0], 1, (size_t)len, f) != (size_t)len) { fclose(f); rt::set_error("read error %s", path); return RT_ERR_IO; }
  fclose(f);

  auto m = new rt_mesh();
  const std::string dir = path_name(path);
  std::vector<std::vector<uint32_t>> groups(1);
  std::vector<int32_t> gmat(1, -1);
  std::vector<float> norms;
  int32_t current_mat = -1;
  size_t pos = 0;
  while (pos < buf.size()) {  // std::getline(in, line)
    size_t nl = buf.find('\n', pos);
    if (nl == std::string::npos) nl = buf.size();
    const char* ls = buf.data() + pos;
    const char* le = buf.data() + nl;
    size_t L = nl - pos;
    pos = nl + 1;
    if (L >= 6 && !strncmp(ls, "mtllib", 6)) {
      if (L < 7) { delete m; rt::set_error("malformed mtllib line"); return RT_ERR_INVALID; }
      std::string fn = dir + std::string(ls + 7, le);
      erase_crlf(fn);
      load_mtl(m, fn);
    } else if (L >= 6 && !strncmp(ls, "usemtl", 6)) {
      if (!groups.back().empty()) { groups.emplace_back(); gmat.push_back(-1); }
      if (L < 7) { delete m; rt::set_error("malformed usemtl line"); return RT_ERR_INVALID; }
      std::string nm(ls + 7, le);
      erase_crlf(nm);
      for (size_t i = 0; i < m->mat_names.size(); i++)
        if (m->mat_names[i] == nm) current_mat = (int32_t)i;
      gmat.back() = current_mat;
    } else if (L >= 2 && ls[0] == 'v' && ls[1] == ' ') {
      float v[3] = {0, 0, 0};
      parse_floats(ls + 2, le, v, 3);
      m->v4.insert(m->v4.end(), {v[0], v[1], v[2], 1.0f});
    } else if (L >= 2 && ls[0] == 'v' && ls[1] == 'n') {
      float n[3] = {0, 0, 0};
      if (L >= 3) parse_floats(ls + 3, le, n, 3);
      norms.insert(norms.end(), {n[0], n[1], n[2]});
    } else if (L >= 2 && ls[0] == 'f' && ls[1] == ' ') {
      const char* p = ls + 2;
      while (p < le) {
        while (p < le && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\v' || *p == '\f')) p++;
        if (p >= le) break;
        const char* e = p;
        while (e < le && !(*e == ' ' || *e == '\t' || *e == '\r' || *e == '\v' || *e == '\f')) e++;
        long vid = strtol(std::string(p, e).c_str(), nullptr, 10);  // stoi(element before '/')
        groups.back().push_back((uint32_t)(vid - 1));
        p = e;
      }
    }
  }
  const size_t nv = m->v4.size() / 4;
  const bool have_vn = norms.size() == 3 * nv;
  if (have_vn) m->vn3 = norms;
  // only non-empty index groups become index buffers (objimporter.hpp:312-319)
  std::vector<std::vector<uint32_t>> g2;
  std::vector<int32_t> m2;
  for (size_t g = 0; g < groups.size(); g++)
    if (!groups[g].empty()) { g2.push_back(std::move(groups[g])); m2.push_back(gmat[g]); }
  int rc = finish_mesh(m, g2, m2, have_vn);
  if (rc) { delete m; return rc; }
  *out = m;
  return RT_OK;
}

extern "C" int rt_mesh_from_arrays(int32_t nv, const float* v3, const float* vn3, int32_t ng, const int32_t* gcount,
                                   const uint32_t* idx, const int32_t* gmat, int32_t nm, const rt_material* mats,
                                   rt_mesh** out) {
  if (!out || nv < 0 || ng < 0 || (nv && !v3) || (ng && (!gcount || !gmat))) {
    rt::set_error("rt_mesh_from_arrays: invalid arguments");
    return RT_ERR_INVALID;
  }
  *out = nullptr;
  auto m = new rt_mesh();
  m->v4.resize(4 * (size_t)nv);
  for (int32_t i = 0; i < nv; i++) {
    m->v4[4 * i] = v3[3 * i]; m->v4[4 * i + 1] = v3[3 * i + 1]; m->v4[4 * i + 2] = v3[3 * i + 2]; m->v4[4 * i + 3] = 1.0f;
  }
  if (vn3) m->vn3.assign(vn3, vn3 + 3 * (size_t)nv);
  for (int32_t i = 0; i < nm; i++) { m->mats.push_back(mats[i]); m->mat_names.push_back("material_" + std::to_string(i)); }
  std::vector<std::vector<uint32_t>> groups(ng);
  std::vector<int32_t> gm(ng);
  size_t off = 0;
  for (int32_t g = 0; g < ng; g++) {
    if (gcount[g] < 0) { delete m; rt::set_error("negative group size"); return RT_ERR_INVALID; }
    groups[g].assign(idx + off, idx + off + gcount[g]);
    gm[g] = gmat[g];
    if (gm[g] >= nm) { delete m; rt::set_error("group material %d out of range", gm[g]); return RT_ERR_INVALID; }
    off += (size_t)gcount[g];
  }
  int rc = finish_mesh(m, groups, gm, vn3 != nullptr);
  if (rc) { delete m; return rc; }
  *out = m;
  return RT_OK;
}

extern "C" void rt_mesh_destroy(rt_mesh* m) { delete m; }

extern "C" int rt_mesh_get_desc(const rt_mesh* m, rt_mesh_desc* d) {
  if (!m || !d) { rt::set_error("rt_mesh_get_desc: null argument"); return RT_ERR_INVALID; }
  d->n_vertices = (int32_t)(m->v4.size() / 4);
  d->vertices = m->v4.data();
  d->vertex_normals = m->vn3.data();
  d->n_faces = (int32_t)m->fmat.size();
  d->face_vertex_ids = m->fidx.data();
  d->face_normals = m->fn3.data();
  d->face_material_ids = m->fmat.data();
  d->n_materials = (int32_t)m->mats.size();
  d->materials = m->mats.data();
  memcpy(d->shape_model_matrix, m->M, 64);
  return RT_OK;
}

// =====================================================================================================
// Synthetic soup, PPM, camera
// =====================================================================================================
static inline uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static inline float u01(uint64_t& s) { return (float)(splitmix64(s) >> 40) * (1.0f / 16777216.0f); }

extern "C" void rt_generate_soup(int32_t n, uint64_t seed, float* v) {
  uint64_t s = seed;
  for (int32_t t = 0; t < n; t++) {
    float c[3];
    for (int k = 0; k < 3; k++) c[k] = u01(s) - 0.5f;
    for (int j = 0; j < 3; j++)
      for (int k = 0; k < 3; k++) {
        float off = (u01(s) * 2.0f - 1.0f) * 0.01f;
        v[9 * (size_t)t + 3 * j + k] = c[k] + off;
      }
  }
}

// (int)(255*c) with x86 cvttss2si semantics for out-of-range / NaN (0x80000000)
static inline int to_int_x86(float x) {
  if (!(x >= -2147483648.0f && x < 2147483648.0f)) return INT_MIN;
  return (int)x;
}

extern "C" int rt_write_ppm(const char* path, const float* rgb, int32_t W, int32_t H) {
  if (!path || !rgb || W <= 0 || H <= 0) { rt::set_error("rt_write_ppm: invalid arguments"); return RT_ERR_INVALID; }
  FILE* f = fopen(path, "wb");
  if (!f) { rt::set_error("cannot write %s", path); return RT_ERR_IO; }
  std::string out;
  out.reserve((size_t)W * H * 12 + 64);
  out += "P3\n" + std::to_string(W) + " " + std::to_string(H) + "\n255\n";
  char tmp[64];
  for (int32_t j = 0; j < H; j++) {
    for (int32_t i = 0; i < W; i++) {
      const float* c = rgb + 3 * ((size_t)j * W + i);
      int n = snprintf(tmp, sizeof tmp, "%d %d %d ", std::min(255, to_int_x86(255 * c[0])),
                       std::min(255, to_int_x86(255 * c[1])), std::min(255, to_int_x86(255 * c[2])));
      out.append(tmp, (size_t)n);
    }
    out += "\n";
  }
  size_t wr = fwrite(out.data(), 1, out.size(), f);
  fclose(f);
  if (wr != out.size()) { rt::set_error("short write %s", path); return RT_ERR_IO; }
  return RT_OK;
}

// writePPMImage's text for 8-bit values (same bytes as rt_write_ppm when every value is in 0..255),
// without per-number formatting calls: a table of the 256 "%d " strings
extern "C" int rt_write_ppm_rgb8(const char* path, const uint8_t* rgb8, int32_t W, int32_t H) {
  if (!path || !rgb8 || W <= 0 || H <= 0) { rt::set_error("rt_write_ppm_rgb8: invalid arguments"); return RT_ERR_INVALID; }
  struct Tab {
    char s[256][5];  // "255 " plus the terminator
    uint8_t len[256];
    Tab() {
      for (int v = 0; v < 256; v++) len[v] = (uint8_t)snprintf(s[v], sizeof s[v], "%d ", v);
    }
  };
  static const Tab t;  // thread-safe one-time initialisation
  const auto& tab = t.s;
  const auto& len = t.len;
  std::string out;
  out.reserve((size_t)W * H * 12 + 64);
  out += "P3\n" + std::to_string(W) + " " + std::to_string(H) + "\n255\n";
  for (int32_t j = 0; j < H; j++) {
    const uint8_t* row = rgb8 + (size_t)j * W * 3;
    for (int32_t i = 0; i < 3 * W; i++) out.append(tab[row[i]], len[row[i]]);
    out += "\n";
  }
  FILE* f = fopen(path, "wb");
  if (!f) { rt::set_error("cannot write %s", path); return RT_ERR_IO; }
  const size_t wr = fwrite(out.data(), 1, out.size(), f);
  fclose(f);
  if (wr != out.size()) { rt::set_error("short write %s", path); return RT_ERR_IO; }
  return RT_OK;
}

// ---------------------------------------------------------------------------------------------------
// Lights
// ---------------------------------------------------------------------------------------------------
// glibc rand(): TYPE_3 additive feedback generator, r[i] = r[i-31] + r[i-3] (mod 2^32) after a
// Park-Miller seeding of r[0..30], r[31..33] = r[0..2] and 310 discarded outputs; rand() = r[i] >> 1.
// The state is the ring of the last 34 values.
extern "C" void rt_rand_seed(rt_rand_state* st, uint32_t seed) {
  if (!st) return;
  uint32_t r[344];
  r[0] = seed ? seed : 1u;
  for (int i = 1; i < 31; i++) {
    const int64_t w = (16807LL * (int64_t)(int32_t)r[i - 1]) % 2147483647LL;
    r[i] = (uint32_t)(w < 0 ? w + 2147483647LL : w);
  }
  for (int i = 31; i < 34; i++) r[i] = r[i - 31];
  for (int i = 34; i < 344; i++) r[i] = r[i - 31] + r[i - 3];
  for (int i = 310; i < 344; i++) st->r[i % 34] = r[i];
  st->k = 344 % 34;
}

extern "C" int32_t rt_rand(rt_rand_state* st) {
  const uint32_t k = st->k;  // slot of r[i - 34]; r[i - 31] is k + 3, r[i - 3] is k + 31 (mod 34)
  const uint32_t v = st->r[(k + 3) % 34] + st->r[(k + 31) % 34];
  st->r[k] = v;
  st->k = (k + 1) % 34;
  return (int32_t)(v >> 1);
}

extern "C" int32_t rt_lights_spherical(const rt_light* centre, float radius, int32_t n_points, rt_rand_state* rng,
                                       rt_light* out) {
  if (!centre || !out || n_points < 0) { rt::set_error("rt_lights_spherical: invalid arguments"); return RT_ERR_INVALID; }
  rt_rand_state local;
  if (!rng) { rt_rand_seed(&local, 1); rng = &local; }
  const float div = (float)(n_points + 1);
  float col[3];
  for (int k = 0; k < 3; k++) col[k] = centre->color[k] / div;  // light.second / (nLightpoints + 1)
  for (int32_t i = 0; i < n_points; i++) {
    float off[3];
    for (int k = 0; k < 3; k++) {  // -radius + (rand() / (RAND_MAX / (radius * 2))), x then y then z
      const float q = (float)2147483647 / (radius * 2);
      off[k] = -radius + ((float)rt_rand(rng) / q);
    }
    for (int k = 0; k < 3; k++) {
      out[i].position[k] = centre->position[k] + off[k];
      out[i].color[k] = col[k];
    }
    out[i].kind = RT_LIGHT_POINT;
  }
  for (int k = 0; k < 3; k++) {
    out[n_points].position[k] = centre->position[k];
    out[n_points].color[k] = col[k];  // light.second /= (Nlights + 1)
  }
  out[n_points].kind = RT_LIGHT_POINT;
  return n_points + 1;
}

// Camera::screenToWorld (camera.hpp:155-173) of a (float) screen position
static f3 screen_to_world(const rt_camera* c, float px, float py) {
  f3 nc;
  nc.x = (float)(2.0 * (double)(px - c->viewport[0]) / (double)c->viewport[2] - 1.0);
  nc.y = (float)(1.0 - 2.0 * (double)(py - c->viewport[1]) / (double)c->viewport[3]);
  nc.z = -1.0f;
  const float persp = (float)((double)1.0f / tan((double)(c->fovy / 2.0f) * (M_PI / 180.0)));
  const float scale = (float)(1.0 / (double)persp);
  nc.x = nc.x * (c->aspect_ratio * scale);
  nc.y = nc.y * scale;
  float vinv[16];
  rt::affinv(c->view_matrix, vinv);
  return rt::affv3(vinv, nc);
}

// Camera::getCenter (camera.hpp:115-118): view.linear().inverse() * (-view.translation())
static f3 camera_center(const rt_camera* c) {
  float L[9], Li[9];
  rt::linear_of(c->view_matrix, L);
  rt::m3inv(L, Li);
  return rt::m3v3(Li, f3{-c->view_matrix[12], -c->view_matrix[13], -c->view_matrix[14]});
}

extern "C" void rt_light_directional(const rt_camera* c, const float color[3], rt_light* out) {
  // screenToWorld(Vector2f(viewport(2) / 2, viewport(3) / 2)): the point itself is stored
  const f3 w = screen_to_world(c, c->viewport[2] / 2, c->viewport[3] / 2);
  out->position[0] = w.x; out->position[1] = w.y; out->position[2] = w.z;
  for (int k = 0; k < 3; k++) out->color[k] = color[k];
  out->kind = RT_LIGHT_DIRECTIONAL;
}

// createDebugRay (flyscene.cpp:129-173) without the GL cylinders: the camera ray through the mouse
// position, its traceRay colour, and the chain of reflections. As the reference, every segment gets the
// first ray's colour, each reflection reflects the *first* direction about the new hit's interpolated
// normal, and a miss ends the chain with a 10-unit segment. All ray queries run on the device.
extern "C" int rt_debug_ray(rt_scene* s, const rt_camera* cam, const rt_light* lights, int32_t n_lights, float mouse_x,
                            float mouse_y, int32_t max_depth, rt_ray_segment* out, int32_t* n_out) {
  if (!s || !cam || !out || !n_out || max_depth < 1) { rt::set_error("rt_debug_ray: invalid arguments"); return RT_ERR_INVALID; }
  *n_out = 0;
  const f3 origin = camera_center(cam);
  const f3 dir = rt::normalized(rt::sub(screen_to_world(cam, mouse_x, mouse_y), origin));
  float o[3] = {origin.x, origin.y, origin.z}, d[3] = {dir.x, dir.y, dir.z}, rgb[3];
  int rc = rt_trace_color(s, 1, o, d, lights, n_lights, rgb, nullptr, nullptr);
  if (rc) return rc;
  for (int32_t i = 1; i <= max_depth; i++) {
    int32_t face;
    float t, P[3], N[3];
    if ((rc = rt_trace_closest_normal(s, 1, o, d, &face, &t, P, N))) return rc;
    rt_ray_segment& g = out[i - 1];
    memcpy(g.origin, o, 12);
    memcpy(g.direction, d, 12);
    memcpy(g.color, rgb, 12);
    *n_out = i;
    if (t == INFINITY) {
      g.length = 10.0f;
      return RT_OK;
    }
    g.length = t;
    if (i != max_depth) {
      const f3 dn = rt::reflect(dir, f3{N[0], N[1], N[2]});
      const f3 start = rt::offset(f3{P[0], P[1], P[2]}, dn, 0.001f);
      o[0] = start.x; o[1] = start.y; o[2] = start.z;
      d[0] = dn.x; d[1] = dn.y; d[2] = dn.z;
    }
  }
  return RT_OK;
}

extern "C" void rt_camera_flycam(int32_t W, int32_t H, float dx, float dy, float dz, rt_camera* c) {
  // Flycamera::translate (flycamera.hpp:196-202), yaw = identity at rotation_Y_axis = 0
  const float I9[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  const float speed = 0.05f;  // flycamera.hpp:107
  f3 yv = rt::m3v3(I9, f3{-dx, -dy, dz});
  f3 tv{0.0f + yv.x * speed, 0.0f + yv.y * speed, 0.0f + yv.z * speed};
  // updateViewMatrix (flycamera.hpp:166-191) at zero rotation
  rt::identity4(c->view_matrix);
  rt::translate4(c->view_matrix, f3{0.0f, 0.0f, -2.0f});
  rt::translate4(c->view_matrix, tv);
  c->viewport[0] = 0.0f; c->viewport[1] = 0.0f; c->viewport[2] = (float)W; c->viewport[3] = (float)H;
  c->fovy = 60.0f;                     // flyscene.cpp:14
  c->aspect_ratio = (float)W / (float)H;
}

extern "C" void rt_scene_opts_default(rt_scene_opts* o) {
  memset(o, 0, sizeof *o);
  o->device = -1;
  o->min_faces = 300;       // flyscene.hpp:168
  o->max_boxes = INT32_MAX; // flyscene.hpp:169
  o->leaf_size = 0;
  o->frames_in_flight = 4;
  o->builder = RT_BUILDER_SBVH_GPU;  // host RT_BUILDER_SBVH when there is no device
  o->box_builder = RT_BOXES_GPU;     // host partition when there is no device (same boxes and order)
  for (int k = 0; k < 3; k++) { o->default_material.ka[k] = 0.2f; o->background[k] = 0.9f; }
  o->default_material.kd[0] = 0.9f; o->default_material.kd[1] = 0.9f; o->default_material.kd[2] = 0.0f;
  o->default_material.shininess = 0.0f;
  o->default_material.dissolve = 0.0f;
}

// =====================================================================================================
// Reference flat box partition (BoundingBox.cpp / flyscene.cpp:399-428)
// =====================================================================================================
namespace rt {
namespace {
// The partition is a sequence of passes; within a pass every box that still qualifies is split (with
// axis retries) independently of the others, and the boxes it creates are appended in box order. So a
// pass runs its boxes in parallel and appends the results in order: the same boxes, face lists and
// order as the sequential reference loop. Vertex coordinates are copied per face (9 floats, face
// order) so the passes stream instead of gathering from the shared vertex array.
struct BoxBuilder {
  const float* fv;  // [nf][3 vertices][3] object-space coordinates (v / w is not taken: Tucano uses x,y,z)
  const float* V(int32_t face, int k) const { return fv + 9 * (size_t)face + 3 * k; }

  static void reshape(RefBox& b) { for (int k = 0; k < 3; k++) b.shape[k] = b.high[k] - b.low[k]; }

  bool has_face(const RefBox& b, int32_t face) const {  // hasFace / hasVertex (inclusive)
    for (int k = 0; k < 3; k++) {
      const float* v = V(face, k);
      if (!(v[0] >= b.low[0] && v[0] <= b.high[0] && v[1] >= b.low[1] && v[1] <= b.high[1] &&
            v[2] >= b.low[2] && v[2] <= b.high[2]))
        return false;
    }
    return true;
  }
  void fit(RefBox& b) const {  // fitFaces: first-vertex init, if/else-if min/max
    if (b.faces.empty()) return;
    const float* t = V(b.faces[0], 0);
    float mn[3] = {t[0], t[1], t[2]}, mx[3] = {t[0], t[1], t[2]};
    for (int32_t face : b.faces)
      for (int j = 0; j < 3; j++) {
        const float* v = V(face, j);
        for (int a = 0; a < 3; a++) {
          if (v[a] < mn[a]) mn[a] = v[a];
          else if (v[a] > mx[a]) mx[a] = v[a];
        }
      }
    for (int a = 0; a < 3; a++) { b.low[a] = mn[a]; b.high[a] = mx[a]; }
    reshape(b);
  }
  float average(const RefBox& b, int axis) const {  // averageVertexCoord: sequential float sum
    float avg = 0.0f;
    for (int32_t face : b.faces) {
      avg += V(face, 0)[axis];
      avg += V(face, 1)[axis];
      avg += V(face, 2)[axis];
    }
    avg /= (float)(b.faces.size() * 3);
    return avg;
  }
  // splitBox: 1 = split, `out` receives the new box; 0 = axis failed (returned `this`); -1 = nullptr
  int split(RefBox& b, RefBox& out) const {
    float oldLow[3], oldHigh[3];
    memcpy(oldLow, b.low, 12);
    memcpy(oldHigh, b.high, 12);
    const float w = b.shape[0], h = b.shape[1], d = b.shape[2];
    int choice;
    if ((w >= h || b.failed[1]) && (w >= d || b.failed[2]) && !b.failed[0]) choice = 0;
    else if ((h >= w || b.failed[0]) && (h >= d || b.failed[2]) && !b.failed[1]) choice = 1;
    else if (!(b.failed[0] && b.failed[1] && b.failed[2])) choice = 2;
    else return -1;
    b.high[choice] = average(b, choice);
    reshape(b);
    std::vector<int32_t> inside, outside;  // outsideFaces: stable partition
    inside.reserve(b.faces.size());
    for (int32_t face : b.faces) (has_face(b, face) ? inside : outside).push_back(face);
    if (inside.empty() || outside.empty()) {
      b.faces = inside.empty() ? std::move(outside) : std::move(inside);
      b.failed[choice] = true;
      memcpy(b.low, oldLow, 12);
      memcpy(b.high, oldHigh, 12);
      reshape(b);
      return 0;
    }
    b.faces = std::move(inside);
    b.failed[0] = b.failed[1] = b.failed[2] = false;
    out = RefBox();
    out.faces = std::move(outside);
    fit(out);
    fit(b);
    return 1;
  }
};
}  // namespace

void build_ref_boxes(HostScene& hs, const float* v4, int32_t min_faces, int32_t max_boxes) {
  hs.boxes.clear();
  std::vector<float> fv(9 * (size_t)hs.nf);
  for (int32_t f = 0; f < hs.nf; f++)
    for (int k = 0; k < 3; k++) memcpy(&fv[9 * (size_t)f + 3 * k], v4 + 4 * (size_t)hs.fidx[3 * (size_t)f + k], 12);
  BoxBuilder bb{fv.data()};
  RefBox b0;
  b0.faces.resize(hs.nf);
  for (int32_t i = 0; i < hs.nf; i++) b0.faces[i] = i;
  hs.boxes.push_back(std::move(b0));
  bb.fit(hs.boxes[0]);
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  bool notDone = true;
  while (notDone && (int64_t)hs.boxes.size() < (int64_t)max_boxes) {
    notDone = false;
    const size_t ncur = hs.boxes.size();
    std::vector<size_t> todo;
    for (size_t bi = 0; bi < ncur; bi++) {
      const RefBox& b = hs.boxes[bi];
      if ((int64_t)b.faces.size() > min_faces && (!b.failed[0] || !b.failed[1] || !b.failed[2])) todo.push_back(bi);
    }
    if (todo.empty()) break;
    notDone = true;
    std::vector<RefBox> created(todo.size());
    std::vector<char> made(todo.size(), 0);
    auto work = [&](size_t i) {
      RefBox& b = hs.boxes[todo[i]];
      int r = bb.split(b, created[i]);
      while (r == 0) r = bb.split(b, created[i]);
      made[i] = r == 1;
    };
    // larger boxes first across the workers (the first passes hold few, huge boxes)
    std::atomic<size_t> cursor{0};
    std::vector<size_t> order(todo.size());
    for (size_t i = 0; i < order.size(); i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
      return hs.boxes[todo[a]].faces.size() > hs.boxes[todo[b]].faces.size();
    });
    const unsigned nth = (unsigned)std::min<size_t>(hw, todo.size());
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nth; t++)
      th.emplace_back([&]() { for (size_t k; (k = cursor.fetch_add(1)) < order.size();) work(order[k]); });
    for (size_t k; (k = cursor.fetch_add(1)) < order.size();) work(order[k]);
    for (auto& t : th) t.join();
    // the reference appends each new box right after splitting, i.e. in box order within the pass
    for (size_t i = 0; i < todo.size(); i++)
      if (made[i]) hs.boxes.push_back(std::move(created[i]));
  }
  assign_box_ranks(hs);
}

void assign_box_ranks(HostScene& hs) {
  hs.face_rank.assign(hs.nf, 0);
  hs.face_box.assign(hs.nf, 0);
  uint32_t rank = 0;
  for (size_t bi = 0; bi < hs.boxes.size(); bi++)
    for (int32_t face : hs.boxes[bi].faces) {
      hs.face_rank[face] = rank++;
      hs.face_box[face] = (uint32_t)bi;
    }
}

// =====================================================================================================
// Traversal BVH: binned SAH BVH2 over world-space triangle bounds, 64-byte nodes in DFS order.
// Child boxes are padded outward so node culling is conservative with respect to the reference's
// (rounded) triangle test: a triangle the reference accepts is never behind a culled box.
// =====================================================================================================
namespace {
struct Prim {
  float lo[3], hi[3], c[3];
  uint32_t id;  // face index
};
struct Aabb {
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const float* l, const float* h) {
    for (int k = 0; k < 3; k++) { lo[k] = std::min(lo[k], l[k]); hi[k] = std::max(hi[k], h[k]); }
  }
  void growp(const float* p) { grow(p, p); }
  void merge(const Aabb& o) { grow(o.lo, o.hi); }
  float area() const {
    float d[3];
    for (int k = 0; k < 3; k++) d[k] = std::max(0.0f, hi[k] - lo[k]);
    return 2.0f * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
  }
};

// one more concurrent subtree task if fewer than `cap` run (the build order and result do not depend on it)
static bool take_task(std::atomic<int>& live, unsigned cap) {
  if (live.fetch_add(1) < (int)cap) return true;
  live.fetch_sub(1);
  return false;
}

// Binned SAH over the working array of primitives (partitioned in place, so a subtree's primitives are
// contiguous and become the leaf order). Large ranges bin and bound in parallel chunks (min/max/count
// merges are order-independent, so the splits do not depend on the thread count); subtrees above
// 16k primitives build as separate tasks.
struct BvhBuilder {
  std::vector<Prim>& prims;
  std::vector<Node64>& nodes;
  std::atomic<uint32_t> next{0};
  int leaf_size;
  float pad;
  unsigned hw = 1;
  std::atomic<int> max_depth{0}, leaves{0};
  // concurrent subtree tasks of this build, at most hw (a torchrun job builds one scene per rank on the
  // same host: without a bound each rank would start ~250 threads at once)
  std::atomic<int> tasks{0};
  static constexpr int kBins = 32;
  static constexpr float kIsect = 1.0f;
  // node-visit cost relative to one triangle test (RT_SAH_TRAV, A/B knob). 0.7: once the packet node
  // step had lost its SALU overhead (order bits, byte handles) a node became cheaper than a triangle
  // test; measured C3 7,440 -> 7,810 Mrays/s (0.3-0.5 within 2% of 0.7, 1.5 -11%), bunny +1-2%
  float kTrav = 0.7f;

  void set_child(Node64& n, int which, const Aabb& b, uint32_t h) const {
    float lo[3], hi[3];
    for (int k = 0; k < 3; k++) { lo[k] = b.lo[k] - pad; hi[k] = b.hi[k] + pad; }
    if (which == 0) {
      n.c0lx = lo[0]; n.c0hx = hi[0]; n.c0ly = lo[1]; n.c0hy = hi[1]; n.c0lz = lo[2]; n.c0hz = hi[2];
      n.child0 = h;
    } else {
      n.c1lx = lo[0]; n.c1hx = hi[0]; n.c1ly = lo[1]; n.c1hy = hi[1]; n.c1lz = lo[2]; n.c1hz = hi[2];
      n.child1 = h;
    }
  }

  // run f(chunk_begin, chunk_end, chunk_index) over [b, e) in up to `hw` parallel chunks
  template <typename F>
  int chunked(uint32_t b, uint32_t e, F&& f) const {
    const uint32_t n = e - b;
    const int T = n >= 65536 ? (int)std::min<unsigned>(hw, 16) : 1;
    if (T == 1) { f(b, e, 0); return 1; }
    std::vector<std::thread> th;
    for (int t = 1; t < T; t++)
      th.emplace_back([&, t]() { f(b + (uint32_t)((uint64_t)n * t / T), b + (uint32_t)((uint64_t)n * (t + 1) / T), t); });
    f(b, b + (uint32_t)((uint64_t)n / T), 0);
    for (auto& x : th) x.join();
    return T;
  }

  struct Bins {
    Aabb box[3][kBins];
    uint32_t cnt[3][kBins];
  };

  // builds [b,e); returns the handle and the (unpadded) bounds of the subtree
  uint32_t build(uint32_t b, uint32_t e, int depth, Aabb& box) {
    const uint32_t n = e - b;
    Aabb cb;
    {
      Aabb pb[16], pc[16];
      const int T = chunked(b, e, [&](uint32_t lo, uint32_t hi, int t) {
        Aabb a, c;  // thread-local, stored once (no false sharing on pb / pc)
        for (uint32_t i = lo; i < hi; i++) { a.grow(prims[i].lo, prims[i].hi); c.growp(prims[i].c); }
        pb[t] = a;
        pc[t] = c;
      });
      box = Aabb();
      for (int t = 0; t < T; t++) { box.merge(pb[t]); cb.merge(pc[t]); }
    }
    int md = max_depth.load();
    while (depth > md && !max_depth.compare_exchange_weak(md, depth)) {}
    auto make_leaf_h = [&]() { leaves++; return make_leaf(b, n); };
    if (n == 1) return make_leaf_h();
    // choose split
    int axis = -1;
    uint32_t mid = b;
    float best_cost = INFINITY;
    float ext[3];
    for (int k = 0; k < 3; k++) ext[k] = cb.hi[k] - cb.lo[k];
    const bool force_median = depth >= kMaxDepth - 20;
    if (!force_median) {
      int best_bin = -1;
      float sc[3];
      for (int k = 0; k < 3; k++) sc[k] = ext[k] > 0.0f ? kBins / ext[k] : 0.0f;
      // one pass bins all three axes
      std::vector<Bins> part(n >= 65536 ? std::min<unsigned>(hw, 16) : 1);
      for (Bins& pbn : part) memset(pbn.cnt, 0, sizeof pbn.cnt);
      const int T = chunked(b, e, [&](uint32_t lo, uint32_t hi, int t) {
        Bins& B = part[t];
        for (uint32_t i = lo; i < hi; i++) {
          const Prim& p = prims[i];
          for (int k = 0; k < 3; k++) {
            if (!(ext[k] > 0.0f)) continue;
            const int bi = std::min(kBins - 1, (int)((p.c[k] - cb.lo[k]) * sc[k]));
            B.box[k][bi].grow(p.lo, p.hi);
            B.cnt[k][bi]++;
          }
        }
      });
      for (int t = 1; t < T; t++)
        for (int k = 0; k < 3; k++)
          for (int i = 0; i < kBins; i++) { part[0].box[k][i].merge(part[t].box[k][i]); part[0].cnt[k][i] += part[t].cnt[k][i]; }
      const Bins& bins = part[0];
      for (int k = 0; k < 3; k++) {
        if (!(ext[k] > 0.0f)) continue;
        float right_area[kBins];
        uint32_t right_cnt[kBins];
        Aabb acc;
        uint32_t c = 0;
        for (int i = kBins - 1; i > 0; i--) {
          acc.merge(bins.box[k][i]);
          c += bins.cnt[k][i];
          right_area[i] = acc.area();
          right_cnt[i] = c;
        }
        Aabb lacc;
        uint32_t lc = 0;
        for (int i = 0; i < kBins - 1; i++) {
          lacc.merge(bins.box[k][i]);
          lc += bins.cnt[k][i];
          if (lc == 0 || right_cnt[i + 1] == 0) continue;
          float cost = lacc.area() * lc + right_area[i + 1] * right_cnt[i + 1];
          if (cost < best_cost) { best_cost = cost; axis = k; best_bin = i; }
        }
      }
      const float parent_area = std::max(box.area(), 1e-30f);
      const float split_cost = kTrav + kIsect * best_cost / parent_area;
      if ((int)n <= leaf_size && (axis < 0 || (float)n * kIsect <= split_cost)) return make_leaf_h();
      if (axis >= 0) {
        const float s = sc[axis];
        const float lo = cb.lo[axis];
        auto it = std::partition(prims.begin() + b, prims.begin() + e, [&](const Prim& p) {
          return std::min(kBins - 1, (int)((p.c[axis] - lo) * s)) <= best_bin;
        });
        mid = (uint32_t)(it - prims.begin());
      }
    } else if ((int)n <= leaf_size) {
      return make_leaf_h();
    }
    if (axis < 0 || mid == b || mid == e) {
      // degenerate centroids or forced: object median along the widest centroid axis
      if ((int)n <= kMaxLeaf && !(ext[0] > 0 || ext[1] > 0 || ext[2] > 0)) return make_leaf_h();
      int k = (ext[0] >= ext[1] && ext[0] >= ext[2]) ? 0 : (ext[1] >= ext[2] ? 1 : 2);
      mid = b + n / 2;
      std::nth_element(prims.begin() + b, prims.begin() + mid, prims.begin() + e,
                       [&](const Prim& x, const Prim& y) { return x.c[k] < y.c[k]; });
    }
    const uint32_t me = next.fetch_add(1);
    Aabb lb, rb;
    uint32_t lh, rh;
    if (n > 4096 && depth < 16 && take_task(tasks, hw)) {
      auto fut = std::async(std::launch::async, [&]() { return build(b, mid, depth + 1, lb); });
      rh = build(mid, e, depth + 1, rb);
      lh = fut.get();
      tasks.fetch_sub(1);
    } else {
      lh = build(b, mid, depth + 1, lb);
      rh = build(mid, e, depth + 1, rb);
    }
    Node64 nd{};
    set_child(nd, 0, lb, lh);
    set_child(nd, 1, rb, rh);
    nodes[me] = nd;
    return me;
  }
};

// Spatial-split BVH (SBVH: object splits as above, plus splits of the space that cut triangles
// straddling the plane into two references with clipped bounds; the host builder's default when
// RT_BUILDER_SBVH). A triangle referenced by several leaves is tested more than once, with
// identical (t, rank), so the (t, rank) argmin, hence every result, is unchanged; culling stays
// conservative because each reference's box bounds the part of the triangle it stands for (clip
// points in double, rounded outward) and every child box is padded as before.
struct SbvhBuilder {
  const HostScene& hs;
  std::vector<Node64>& nodes;                      // sized to the node capacity
  std::vector<std::vector<uint32_t>> leaf_lists;   // face ids per leaf, sized to the leaf capacity
  std::atomic<uint32_t> next{0}, nleaf{0};
  std::atomic<int64_t> refs{0};  // references made (statistics); the budget itself is per subtree
  int leaf_size = 4;
  float pad = 0.0f, kTrav = 0.7f, alpha = 1e-5f, root_area = 1.0f;
  std::atomic<int> max_depth{0};
  std::atomic<int> tasks{0};  // concurrent subtree tasks, at most hw (as BvhBuilder)
  static constexpr int kBins = 32;
  static constexpr float kIsect = 1.0f;

  void verts(uint32_t f, double v[3][3]) const {
    for (int j = 0; j < 3; j++) {
      const f3& w = bound_vert(hs, f, j);
      v[j][0] = w.x; v[j][1] = w.y; v[j][2] = w.z;
    }
  }
  static float down(double x) { float f = (float)x; return (double)f > x ? std::nextafter(f, -INFINITY) : f; }
  static float up(double x) { float f = (float)x; return (double)f < x ? std::nextafter(f, INFINITY) : f; }
  // bounds of (triangle f) within [a, b] on axis k, intersected with `within`; false if empty
  bool clip(uint32_t f, int k, float a, float b, const Prim& within, Prim& out) const {
    double v[3][3];
    verts(f, v);
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    auto add = [&](const double* q) {
      for (int i = 0; i < 3; i++) { lo[i] = std::min(lo[i], q[i]); hi[i] = std::max(hi[i], q[i]); }
    };
    for (int j = 0; j < 3; j++) {
      const double* p = v[j];
      const double* q = v[(j + 1) % 3];
      if (p[k] >= a && p[k] <= b) add(p);
      for (double pl : {(double)a, (double)b}) {
        if ((p[k] < pl && q[k] > pl) || (p[k] > pl && q[k] < pl)) {
          const double t = (pl - p[k]) / (q[k] - p[k]);
          double x[3];
          for (int i = 0; i < 3; i++) x[i] = p[i] + t * (q[i] - p[i]);
          x[k] = pl;
          add(x);
        }
      }
    }
    out.id = f;
    for (int i = 0; i < 3; i++) {
      out.lo[i] = std::max(down(lo[i]), within.lo[i]);
      out.hi[i] = std::min(up(hi[i]), within.hi[i]);
      if (i == k) { out.lo[i] = std::max(out.lo[i], a); out.hi[i] = std::min(out.hi[i], b); }
      if (!(out.lo[i] <= out.hi[i])) return false;
      out.c[i] = 0.5f * (out.lo[i] + out.hi[i]);
    }
    return true;
  }

  void set_child(Node64& n, int which, const Aabb& b, uint32_t h) const {
    float lo[3], hi[3];
    for (int k = 0; k < 3; k++) { lo[k] = b.lo[k] - pad; hi[k] = b.hi[k] + pad; }
    if (which == 0) {
      n.c0lx = lo[0]; n.c0hx = hi[0]; n.c0ly = lo[1]; n.c0hy = hi[1]; n.c0lz = lo[2]; n.c0hz = hi[2];
      n.child0 = h;
    } else {
      n.c1lx = lo[0]; n.c1hx = hi[0]; n.c1ly = lo[1]; n.c1hy = hi[1]; n.c1lz = lo[2]; n.c1hz = hi[2];
      n.child1 = h;
    }
  }
  uint32_t leaf(std::vector<Prim>& r) {
    const uint32_t li = nleaf.fetch_add(1);
    std::vector<uint32_t>& ids = leaf_lists[li];
    ids.reserve(r.size());
    for (const Prim& p : r) ids.push_back(p.id);
    const uint32_t n = (uint32_t)r.size();
    std::vector<Prim>().swap(r);
    return make_leaf(li, n);  // leaf index for now; triangle slots are assigned depth first afterwards
  }

  unsigned hw = 1;
  // f(begin, end, chunk) over [0, n) in up to 16 contiguous chunks (one below 64k references); the
  // per-chunk partial results are merged in chunk order, so nothing depends on the thread count
  template <typename F>
  int chunked(uint32_t n, F&& f) const {
    const int T = n >= 65536 ? (int)std::min<unsigned>(hw, 16) : 1;
    if (T == 1) { f(0u, n, 0); return 1; }
    std::vector<std::thread> th;
    for (int t = 1; t < T; t++)
      th.emplace_back([&, t]() { f((uint32_t)((uint64_t)n * t / T), (uint32_t)((uint64_t)n * (t + 1) / T), t); });
    f(0u, (uint32_t)((uint64_t)n / T), 0);
    for (auto& x : th) x.join();
    return T;
  }
  struct Bins {
    Aabb box[3][kBins];
    uint32_t cnt[3][kBins], cnt2[3][kBins];
    void clear() { memset(cnt, 0, sizeof cnt); memset(cnt2, 0, sizeof cnt2); for (auto& a : box) for (Aabb& b : a) b = Aabb(); }
    void merge(const Bins& o) {
      for (int k = 0; k < 3; k++)
        for (int i = 0; i < kBins; i++) { box[k][i].merge(o.box[k][i]); cnt[k][i] += o.cnt[k][i]; cnt2[k][i] += o.cnt2[k][i]; }
    }
  };
  // best plane of binned boxes on axis k: left of plane i = bins 0..i (counted by cnt), right = bins
  // i+1.. (counted by cnt2 for spatial bins, cnt otherwise)
  static void sweep(const Bins& B, int k, bool spatial, float& best, int& axis, int& bin, Aabb* lbest, Aabb* rbest) {
    const uint32_t* rcnt = spatial ? B.cnt2[k] : B.cnt[k];
    Aabb racc[kBins];
    uint32_t rc[kBins];
    Aabb acc;
    uint32_t c = 0;
    for (int i = kBins - 1; i > 0; i--) { acc.merge(B.box[k][i]); c += rcnt[i]; racc[i] = acc; rc[i] = c; }
    Aabb lacc;
    uint32_t lc = 0;
    for (int i = 0; i < kBins - 1; i++) {
      lacc.merge(B.box[k][i]);
      lc += B.cnt[k][i];
      if (lc == 0 || rc[i + 1] == 0) continue;
      const float cost = lacc.area() * lc + racc[i + 1].area() * rc[i + 1];
      if (cost < best) {
        best = cost; axis = k; bin = i;
        if (lbest) { *lbest = lacc; *rbest = racc[i + 1]; }
      }
    }
  }

  // builds the subtree over `r` (consumed); returns its handle and the bounds of its references.
  // budget: references this subtree may add by spatial splits. Each split spends what it duplicates and
  // hands the rest to its children in proportion to their reference counts, so the tree (which splits
  // are taken) never depends on the order the parallel subtree tasks run in.
  uint32_t build(std::vector<Prim>& r, int depth, Aabb& box, int64_t budget) {
    const uint32_t n = (uint32_t)r.size();
    Aabb cb;
    box = Aabb();
    {
      Aabb pb[16], pc[16];
      const int T = chunked(n, [&](uint32_t b, uint32_t e, int t) {
        Aabb a, c;  // thread-local, stored once
        for (uint32_t i = b; i < e; i++) { a.grow(r[i].lo, r[i].hi); c.growp(r[i].c); }
        pb[t] = a;
        pc[t] = c;
      });
      for (int t = 0; t < T; t++) { box.merge(pb[t]); cb.merge(pc[t]); }
    }
    int md = max_depth.load();
    while (depth > md && !max_depth.compare_exchange_weak(md, depth)) {}
    if (n == 1) return leaf(r);
    const bool forced = depth >= kMaxDepth - 20;
    const float parent_area = std::max(box.area(), 1e-30f);
    const int TB = n >= 65536 ? (int)std::min<unsigned>(hw, 16) : 1;
    std::vector<Bins> part((size_t)TB);
    // object split: binned SAH over reference centroids
    int o_axis = -1, o_bin = -1;
    float o_cost = INFINITY;
    Aabb o_lb, o_rb;
    float ext[3], sc[3];
    for (int k = 0; k < 3; k++) { ext[k] = cb.hi[k] - cb.lo[k]; sc[k] = ext[k] > 0.0f ? kBins / ext[k] : 0.0f; }
    auto obin = [&](const Prim& p, int k) { return std::min(kBins - 1, (int)((p.c[k] - cb.lo[k]) * sc[k])); };
    if (!forced) {
      for (Bins& B : part) B.clear();
      const int T = chunked(n, [&](uint32_t b, uint32_t e, int t) {
        Bins& B = part[t];
        for (uint32_t i = b; i < e; i++)
          for (int k = 0; k < 3; k++) {
            if (!(ext[k] > 0.0f)) continue;
            const int bi = obin(r[i], k);
            B.box[k][bi].grow(r[i].lo, r[i].hi);
            B.cnt[k][bi]++;
          }
      });
      for (int t = 1; t < T; t++) part[0].merge(part[t]);
      for (int k = 0; k < 3; k++)
        if (ext[k] > 0.0f) sweep(part[0], k, false, o_cost, o_axis, o_bin, &o_lb, &o_rb);
    }
    // spatial split, tried when the object split's children overlap by more than alpha of the root:
    // kBins slabs per axis; a reference enters the bin of its low end, exits the bin of its high end,
    // and adds the bounds of its clipped part to every bin it spans
    int s_axis = -1, s_bin = -1;
    float s_cost = INFINITY;
    float pl[3][kBins + 1];
    float ov = 0.0f;
    if (o_axis >= 0) {
      float d[3];
      for (int k = 0; k < 3; k++) d[k] = std::max(0.0f, std::min(o_lb.hi[k], o_rb.hi[k]) - std::max(o_lb.lo[k], o_rb.lo[k]));
      ov = 2.0f * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
    }
    if (!forced && budget > 0 && (o_axis < 0 || ov > alpha * root_area)) {
      float w[3];
      for (int k = 0; k < 3; k++) {
        w[k] = (box.hi[k] - box.lo[k]) / kBins;
        for (int i = 0; i <= kBins; i++) pl[k][i] = box.lo[k] + w[k] * i;
        pl[k][kBins] = box.hi[k];
      }
      auto sbin = [&](float x, int k) {
        int bi = std::min(kBins - 1, std::max(0, (int)((x - box.lo[k]) / w[k])));
        while (bi > 0 && x < pl[k][bi]) bi--;
        while (bi < kBins - 1 && x >= pl[k][bi + 1]) bi++;
        return bi;
      };
      for (Bins& B : part) B.clear();
      const int T = chunked(n, [&](uint32_t b, uint32_t e, int t) {
        Bins& B = part[t];
        for (uint32_t i = b; i < e; i++) {
          const Prim& p = r[i];
          for (int k = 0; k < 3; k++) {
            if (!(w[k] > 0.0f)) continue;
            const int b0 = sbin(p.lo[k], k), b1 = sbin(p.hi[k], k);
            B.cnt[k][b0]++;
            B.cnt2[k][b1]++;
            if (b0 == b1) { B.box[k][b0].grow(p.lo, p.hi); continue; }
            for (int bi = b0; bi <= b1; bi++) {
              Prim q;
              if (clip(p.id, k, std::max(pl[k][bi], p.lo[k]), std::min(pl[k][bi + 1], p.hi[k]), p, q)) B.box[k][bi].grow(q.lo, q.hi);
            }
          }
        }
      });
      for (int t = 1; t < T; t++) part[0].merge(part[t]);
      for (int k = 0; k < 3; k++)
        if (w[k] > 0.0f) sweep(part[0], k, true, s_cost, s_axis, s_bin, nullptr, nullptr);
    }
    const float best = std::min(o_cost, s_cost);
    if (!forced && (int)n <= leaf_size && (best == INFINITY || (float)n * kIsect <= kTrav + kIsect * best / parent_area))
      return leaf(r);
    if (forced && (int)n <= leaf_size) return leaf(r);
    std::vector<Prim> L, R;
    bool spatial = s_axis >= 0 && s_cost < o_cost;
    const float s_pos = spatial ? pl[s_axis][s_bin + 1] : 0.0f;
    if (spatial) {
      // the references this split adds are reserved against the budget first (a hard bound on the
      // reference count, hence on the leaf and node storage); without room it is an object split
      std::vector<int64_t> cnt((size_t)TB, 0);
      const int T = chunked(n, [&](uint32_t b, uint32_t e, int t) {
        int64_t k = 0;  // thread-local
        for (uint32_t i = b; i < e; i++) k += r[i].lo[s_axis] < s_pos && r[i].hi[s_axis] > s_pos;
        cnt[t] = k;
      });
      int64_t straddle = 0;
      for (int t = 0; t < T; t++) straddle += cnt[t];
      if (straddle > budget) spatial = false;
      else {
        budget -= straddle;
        refs += straddle;
      }
    }
    if (spatial || o_axis >= 0) {
      std::vector<std::vector<Prim>> pL((size_t)TB), pR((size_t)TB);
      const int k = spatial ? s_axis : o_axis;
      const int T = chunked(n, [&](uint32_t b, uint32_t e, int t) {
        std::vector<Prim>& l = pL[t];
        std::vector<Prim>& rr = pR[t];
        for (uint32_t i = b; i < e; i++) {
          const Prim& p = r[i];
          if (!spatial) { (obin(p, k) <= o_bin ? l : rr).push_back(p); continue; }
          if (p.hi[k] <= s_pos) { l.push_back(p); continue; }
          if (p.lo[k] >= s_pos) { rr.push_back(p); continue; }
          Prim ql, qr;
          const bool hl = clip(p.id, k, p.lo[k], s_pos, p, ql), hr = clip(p.id, k, s_pos, p.hi[k], p, qr);
          if (hl && hr) { l.push_back(ql); rr.push_back(qr); }
          else if (hl) l.push_back(ql);
          else if (hr) rr.push_back(qr);
          else (p.c[k] < s_pos ? l : rr).push_back(p);
        }
      });
      for (int t = 0; t < T; t++) {
        L.insert(L.end(), pL[t].begin(), pL[t].end());
        R.insert(R.end(), pR[t].begin(), pR[t].end());
      }
    }
    if (L.empty() || R.empty()) {
      L.clear();
      R.clear();
      // degenerate centroids or forced: object median along the widest centroid axis
      if ((int)n <= kMaxLeaf && !(ext[0] > 0 || ext[1] > 0 || ext[2] > 0)) return leaf(r);
      const int k = (ext[0] >= ext[1] && ext[0] >= ext[2]) ? 0 : (ext[1] >= ext[2] ? 1 : 2);
      std::nth_element(r.begin(), r.begin() + n / 2, r.end(), [&](const Prim& x, const Prim& y) { return x.c[k] < y.c[k]; });
      L.assign(r.begin(), r.begin() + n / 2);
      R.assign(r.begin() + n / 2, r.end());
    }
    std::vector<Prim>().swap(r);
    const uint32_t me = next.fetch_add(1);
    const int64_t bl = (int64_t)((double)budget * (double)L.size() / (double)(L.size() + R.size())), br = budget - bl;
    Aabb lb, rb;
    uint32_t lh, rh;
    if (n > 4096 && depth < 16 && take_task(tasks, hw)) {
      auto fut = std::async(std::launch::async, [&]() { return build(L, depth + 1, lb, bl); });
      rh = build(R, depth + 1, rb, br);
      lh = fut.get();
      tasks.fetch_sub(1);
    } else {
      lh = build(L, depth + 1, lb, bl);
      rh = build(R, depth + 1, rb, br);
    }
    Node64 nd{};
    set_child(nd, 0, lb, lh);
    set_child(nd, 1, rb, rh);
    nodes[me] = nd;
    return me;
  }
};
}  // namespace

// f(begin, end, chunk) over [0, n) in hardware_concurrency() contiguous chunks (one when n is small)
template <typename F>
static int parallel_chunks(size_t n, F&& f) {
  const int T = n >= 65536 ? (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency())) : 1;
  std::vector<std::thread> th;
  for (int t = 1; t < T; t++) th.emplace_back([&, t]() { f(n * t / T, n * (t + 1) / T, t); });
  f(0, n / T, 0);
  for (auto& x : th) x.join();
  return T;
}

// [0, n) in contiguous chunks on up to 16 threads (one below 64k items): f(begin, end)
void parallel_for(size_t n, const std::function<void(size_t, size_t)>& f) {
  parallel_chunks(n, [&](size_t b, size_t e, int) { f(b, e); });
}

// A face whose interpolated normal (interpolateNormal, flyscene.cpp:594-599) can never be the zero
// vector for a point that passed the inside test: its area A (same expression the kernel uses) is a
// positive normal number and every unit vertex normal leans into the face normal (n.nk >= 0.5). Then
// n.(sum_k nk a_k / A) >= 0.5 (sum a_k)/A >= 0.5 (sub-areas of a point in the plane sum to >= A),
// far above rounding, so norm() != 0 and the reference never rejects the face for it; when A would
// overflow the blend, the result is NaN, which the reference also accepts (NaN != 0).
static bool safe_normal(const HostScene& hs, uint32_t f) {
  const f3& w0 = hs.wv[hs.fidx[3 * f]];
  const f3& w1 = hs.wv[hs.fidx[3 * f + 1]];
  const f3& w2 = hs.wv[hs.fidx[3 * f + 2]];
  const f3 e0 = sub(w1, w0), e2 = sub(w0, w2);
  const float A = norm(cross(e0, neg(e2))) / 2;
  if (!(A > 1e-30f) || !std::isfinite(A)) return false;
  const f3& n = hs.fnn[f];
  for (int k = 0; k < 3; k++) {
    const f3& nk = hs.vnn[hs.fidx[3 * f + k]];
    if (!std::isfinite(nk.x) || !std::isfinite(nk.y) || !std::isfinite(nk.z)) return false;
    if (std::fabs(sqnorm(nk) - 1.0f) > 1e-3f) return false;
    if (!(dot(n, nk) >= 0.5f)) return false;
  }
  return true;
}

// conservative padding of every BVH child box: covers the reference's rounding of P = o + t d and of
// the inclusive edge tests for ray origins within ~16 scene extents (DESIGN.md "Exactness of culling")
float bvh_pad(const float lo[3], const float hi[3]) {
  float ext = 0.0f, mag = 0.0f;
  for (int k = 0; k < 3; k++) {
    ext = std::max(ext, hi[k] - lo[k]);
    mag = std::max(mag, std::max(std::fabs(lo[k]), std::fabs(hi[k])));
  }
  return 2e-5f * std::max(std::max(ext, mag), 1e-3f);
}

// the static pad the builders gave every box: bvh_pad of the triangles' bounds (the builders' `world`)
float scene_static_pad(const HostScene& hs) {
  // per-chunk bounds merged afterwards: min / max skip NaN coordinates the same way in any order
  float plo[16][3], phi[16][3];
  for (int t = 0; t < 16; t++)
    for (int k = 0; k < 3; k++) { plo[t][k] = INFINITY; phi[t][k] = -INFINITY; }
  const int T = parallel_chunks(hs.tris.size(), [&](size_t b, size_t e, int t) {
    float l[3] = {INFINITY, INFINITY, INFINITY}, h[3] = {-INFINITY, -INFINITY, -INFINITY};  // thread-local (no false sharing)
    for (size_t i = b; i < e; i++)
      for (int j = 0; j < 3; j++) {
        const f3& w = bound_vert(hs, hs.tris[i].face, j);
        const float v[3] = {w.x, w.y, w.z};
        for (int k = 0; k < 3; k++) { l[k] = std::min(l[k], v[k]); h[k] = std::max(h[k], v[k]); }
      }
    for (int k = 0; k < 3; k++) { plo[t][k] = l[k]; phi[t][k] = h[k]; }
  });
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int t = 0; t < T; t++)
    for (int k = 0; k < 3; k++) { lo[k] = std::min(lo[k], plo[t][k]); hi[k] = std::max(hi[k], phi[t][k]); }
  return hs.tris.empty() ? 0.0f : bvh_pad(lo, hi);
}

void world_bounds(const HostScene& hs, float lo[3], float hi[3]) {
  Aabb parts[16];
  const std::vector<f3>& pts = hs.av.empty() ? hs.wv : hs.av;
  const int T = parallel_chunks(pts.size(), [&](size_t b, size_t e, int t) {
    Aabb a;  // thread-local, stored once (adjacent per-thread slots written per item share cache lines)
    for (size_t i = b; i < e; i++) {
      const float c[3] = {pts[i].x, pts[i].y, pts[i].z};
      a.growp(c);
    }
    parts[t] = a;
  });
  Aabb w;
  for (int t = 0; t < T; t++) w.merge(parts[t]);
  for (int k = 0; k < 3; k++) { lo[k] = w.lo[k]; hi[k] = w.hi[k]; }
}

// Reference-box certificates (TriRec64::box kBoxCertBit). The accept path's box fast path (rt_device.hip
// accept_candidate) accepts a candidate lane whose object-space hit point X = Minv p lies inside the
// face's reference box by m_k = 1e-5 ((hi - lo) + |lo| + |hi| + |o2_k|) per axis, o2 the ray's
// object-space origin -- margins far above the rounding of the reference's intersectBox
// (flyscene.cpp:484-507), so the reference accepts too. A face is certified when that fast path must
// succeed for every hit point its edge tests can accept, for any ray whose |o2|_inf <= Ro =
// cert_origin_max: its three object-space vertices lie inside the box by m_k(Ro) + delta_k, where
// delta_k = 1e-5 ((hi - lo) + |lo| + |hi|) + 4e-4 diam covers how far a hit point the reference's
// inclusive float edge tests accept can lie outside the triangle (at most a few ulp of |p - w| over
// sin(theta_min / 2), here <= 0.01 diam -- only triangles whose smallest angle has sin(theta/2) >= 0.01
// are certified) and the rounding of M / Minv (a similarity) and of X. Uncertified faces and rays
// beyond Ro take the fast path and, where it fails, the exact test, as before.
bool model_is_similarity(const float* M);
float cert_origin_max(const HostScene& hs) {
  if (!model_is_similarity(hs.M)) return 0.0f;  // no certificates (box_certified needs Ro > 0)
  float R = 0.0f;
  for (float v : hs.ov3) R = std::max(R, std::fabs(v));  // NaN coordinates are skipped by max
  return std::isfinite(R) ? 16.0f * R : 0.0f;
}

// The argument above holds for the triangle the edge tests actually accept on, which is the world
// triangle only when the face normal they use (hs.fnn, the caller's face_normals, never transformed by M)
// is the world triangle's own normal: with a tilted normal n the accepted region is the triangle projected
// along n onto n's plane, whose vertices move by up to diam * sin(angle(n, geometric normal)). And Minv
// must be a similarity for object-space distances to be world distances over one scale. So a
// model matrix whose linear part is not a uniform scale times a rotation certifies nothing
// (model_is_similarity), and a face certifies only if its normal is within kCertNormalSin of the world
// triangle's normal, with that projection offset (2 diam sin) added to the margin.
constexpr double kCertNormalSin = 1e-3;
bool model_is_similarity(const float* M) {
  double c[3][3], n2[3];
  for (int j = 0; j < 3; j++) {
    for (int k = 0; k < 3; k++) c[j][k] = M[4 * j + k];  // column j of the column-major linear part
    n2[j] = c[j][0] * c[j][0] + c[j][1] * c[j][1] + c[j][2] * c[j][2];
    if (!std::isfinite(n2[j]) || !(n2[j] > 0.0)) return false;
  }
  for (int j = 0; j < 3; j++) {
    if (std::fabs(n2[j] - n2[0]) > 1e-5 * n2[0]) return false;
    const int i = (j + 1) % 3;
    const double d = c[j][0] * c[i][0] + c[j][1] * c[i][1] + c[j][2] * c[i][2];
    if (std::fabs(d) > 1e-5 * n2[0]) return false;
  }
  return M[3] == 0.0f && M[7] == 0.0f && M[11] == 0.0f && M[15] == 1.0f;
}

// sin of the angle between the face normal the edge tests use and the world triangle's normal (2 on
// degenerate or non-finite input: never certified)
static double face_normal_tilt(const HostScene& hs, uint32_t f) {
  double w[3][3];
  for (int j = 0; j < 3; j++) {
    const f3& p = hs.wv[hs.fidx[3 * f + j]];
    w[j][0] = p.x; w[j][1] = p.y; w[j][2] = p.z;
  }
  const double a[3] = {w[1][0] - w[0][0], w[1][1] - w[0][1], w[1][2] - w[0][2]};
  const double c[3] = {w[2][0] - w[0][0], w[2][1] - w[0][1], w[2][2] - w[0][2]};
  const double g[3] = {a[1] * c[2] - a[2] * c[1], a[2] * c[0] - a[0] * c[2], a[0] * c[1] - a[1] * c[0]};
  const f3& nf = hs.fnn[f];
  const double n[3] = {nf.x, nf.y, nf.z};
  const double gg = g[0] * g[0] + g[1] * g[1] + g[2] * g[2], nn = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
  if (!std::isfinite(gg) || !std::isfinite(nn) || !(gg > 0.0) || !(nn > 0.0)) return 2.0;
  const double x[3] = {g[1] * n[2] - g[2] * n[1], g[2] * n[0] - g[0] * n[2], g[0] * n[1] - g[1] * n[0]};
  const double dn = g[0] * n[0] + g[1] * n[1] + g[2] * n[2];
  if (!(dn > 0.0)) return 2.0;  // opposite orientation: the edge tests' inside is the other side
  return std::sqrt((x[0] * x[0] + x[1] * x[1] + x[2] * x[2]) / (gg * nn));
}

// The edge tests (flyscene.cpp:580-590) accept P when n.(e_k x (P - w_k)) >= 0 for the three world edges,
// n the object-space face normal; P = o + t d lies on n's plane n.x = dist (:459-465). Adding multiples of
// n to e_k or P - w_k leaves those triple products unchanged, so the accepted set is the world triangle
// projected along n onto that plane, p_k = w_k - ((n.w_k - dist) / n.n) n -- the world triangle itself
// only when n is its normal. A face whose normal tilts by more than kBoundTilt (offsets above 1e-6 of
// its diameter, well inside the static pad's rounding allowance) is bounded by that projection; an
// untilted scene keeps hs.av empty and its builds unchanged. (A normal facing away from the triangle
// accepts nothing beyond rounding; its projection still bounds that.)
constexpr double kBoundTilt = 1e-6;
void accept_region(HostScene& hs) {
  hs.av.clear();
  std::atomic<bool> any{false};
  parallel_chunks((size_t)hs.nf, [&](size_t b, size_t e, int) {
    for (size_t f = b; f < e && !any.load(std::memory_order_relaxed); f++)
      if (!(face_normal_tilt(hs, (uint32_t)f) <= kBoundTilt)) any = true;
  });
  if (!any) return;
  hs.av.resize(3 * (size_t)hs.nf);
  parallel_chunks((size_t)hs.nf, [&](size_t b, size_t e, int) {
    for (size_t f = b; f < e; f++) {
      const f3& nf = hs.fnn[f];
      const double n[3] = {nf.x, nf.y, nf.z}, nn = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
      const bool tilted = !(face_normal_tilt(hs, (uint32_t)f) <= kBoundTilt);
      for (int j = 0; j < 3; j++) {
        const f3& w = hs.wv[hs.fidx[3 * f + j]];
        f3& p = hs.av[3 * f + j];
        p = w;
        if (!tilted || !(nn > 0.0) || !std::isfinite(nn)) continue;
        const double s = (n[0] * w.x + n[1] * w.y + n[2] * w.z - (double)hs.fdist[f]) / nn;
        p = f3{(float)(w.x - s * n[0]), (float)(w.y - s * n[1]), (float)(w.z - s * n[2])};
      }
    }
  });
}

static bool box_certified(const HostScene& hs, uint32_t f, float Ro) {
  if (!(Ro > 0.0f) || hs.ov3.empty()) return false;
  const double tilt = face_normal_tilt(hs, f);
  if (!(tilt <= kCertNormalSin)) return false;
  const RefBox& b = hs.boxes[hs.face_box[f]];
  double v[3][3];
  for (int j = 0; j < 3; j++)
    for (int k = 0; k < 3; k++) {
      v[j][k] = hs.ov3[3 * (size_t)hs.fidx[3 * f + j] + k];
      if (!std::isfinite(v[j][k])) return false;
    }
  // edge lengths and the smallest angle (law of cosines, in double)
  double L[3];
  for (int j = 0; j < 3; j++) {
    const double* a = v[j];
    const double* c = v[(j + 1) % 3];
    L[j] = std::sqrt((c[0] - a[0]) * (c[0] - a[0]) + (c[1] - a[1]) * (c[1] - a[1]) + (c[2] - a[2]) * (c[2] - a[2]));
  }
  const double diam = std::max(L[0], std::max(L[1], L[2]));
  if (!(diam > 0.0)) return false;
  for (int j = 0; j < 3; j++) {  // angle opposite edge j: between edges j+1 and j+2
    const double a = L[(j + 1) % 3], c = L[(j + 2) % 3], o = L[j];
    if (!(a > 0.0 && c > 0.0)) return false;
    const double cosv = std::min(1.0, std::max(-1.0, (a * a + c * c - o * o) / (2.0 * a * c)));
    const double s_half = std::sqrt(std::max(0.0, (1.0 - cosv) / 2.0));  // sin(theta / 2)
    if (!(s_half >= 0.01)) return false;
  }
  for (int k = 0; k < 3; k++) {
    const double lo = b.low[k], hi = b.high[k];
    if (!std::isfinite(lo) || !std::isfinite(hi)) return false;
    const double S = (hi - lo) + std::fabs(lo) + std::fabs(hi);
    const double need = 1e-5 * (S + Ro) + 1e-30 + 1e-5 * S + 4e-4 * diam + 2.0 * tilt * diam;
    for (int j = 0; j < 3; j++)
      if (!(v[j][k] - lo >= need && hi - v[j][k] >= need)) return false;
  }
  return true;
}

// the flag bits of face f's triangle records (kSafeNormalBit, kBoxCertBit): derived from the geometry
// alone, so the scene cache loader recomputes them instead of trusting the file
uint32_t tri_flags(const HostScene& hs, uint32_t f, float Ro) {
  return (safe_normal(hs, f) ? kSafeNormalBit : 0u) | (box_certified(hs, f, Ro) ? kBoxCertBit : 0u);
}

// exact-test record of face f (the kernels' TriRec64)
static void tri_record(const HostScene& hs, uint32_t f, TriRec64& r, float Ro) {
  const f3& n = hs.fnn[f];
  const f3& w0 = hs.wv[hs.fidx[3 * f]];
  const f3& w1 = hs.wv[hs.fidx[3 * f + 1]];
  const f3& w2 = hs.wv[hs.fidx[3 * f + 2]];
  r.nx = n.x; r.ny = n.y; r.nz = n.z; r.dist = hs.fdist[f];
  r.w0x = w0.x; r.w0y = w0.y; r.w0z = w0.z;
  r.w1x = w1.x; r.w1y = w1.y; r.w1z = w1.z;
  r.w2x = w2.x; r.w2y = w2.y; r.w2z = w2.z;
  r.rank = hs.face_rank[f];
  r.face = f;
  r.box = hs.face_box[f] | tri_flags(hs, f, Ro);
}

void face_records(const HostScene& hs, std::vector<TriRec64>& out) {
  out.resize(hs.nf);
  const float Ro = cert_origin_max(hs);
  parallel_chunks((size_t)hs.nf, [&](size_t b, size_t e, int) {
    for (size_t f = b; f < e; f++) tri_record(hs, (uint32_t)f, out[f], Ro);
  });
}

// the GPU builders bound the records' vertices: with a tilted normal anywhere (hs.av non-empty) they get
// the accept-region vertices, and world_records puts the world vertices back into the built leaf order
static void set_verts(TriRec64& r, const f3& w0, const f3& w1, const f3& w2) {
  r.w0x = w0.x; r.w0y = w0.y; r.w0z = w0.z;
  r.w1x = w1.x; r.w1y = w1.y; r.w1z = w1.z;
  r.w2x = w2.x; r.w2y = w2.y; r.w2z = w2.z;
}
static void bound_records(const HostScene& hs, std::vector<TriRec64>& recs) {
  if (hs.av.empty()) return;
  parallel_chunks(recs.size(), [&](size_t b, size_t e, int) {
    for (size_t i = b; i < e; i++) {
      TriRec64& r = recs[i];
      set_verts(r, bound_vert(hs, r.face, 0), bound_vert(hs, r.face, 1), bound_vert(hs, r.face, 2));
    }
  });
}
// the device builders take scenes whose culling bounds are finite and well inside the float range (their
// bin arithmetic, Morton codes and surface areas stay finite); anything else is built on the host
static bool device_buildable(const std::vector<TriRec64>& recs) {
  std::atomic<bool> ok{true};
  parallel_chunks(recs.size(), [&](size_t b, size_t e, int) {
    for (size_t i = b; i < e && ok.load(std::memory_order_relaxed); i++) {
      const TriRec64& r = recs[i];
      const float v[9] = {r.w0x, r.w0y, r.w0z, r.w1x, r.w1y, r.w1z, r.w2x, r.w2y, r.w2z};
      for (float x : v)
        if (!(std::fabs(x) <= 1e30f)) ok = false;  // NaN fails too
    }
  });
  return ok.load();
}
static void world_records(HostScene& hs) {
  if (hs.av.empty()) return;
  parallel_chunks(hs.tris.size(), [&](size_t b, size_t e, int) {
    for (size_t i = b; i < e; i++) {
      TriRec64& r = hs.tris[i];
      const uint32_t* v = &hs.fidx[3 * (size_t)r.face];
      set_verts(r, hs.wv[v[0]], hs.wv[v[1]], hs.wv[v[2]]);
    }
  });
}

// Traversal-order hint of a node for waves whose rays share one direction octant (bit k of the octant:
// axis k negative): bit `oct` set = visit child 1 first. Split-axis rule: along the axis on which the
// children's centres are furthest apart, the child on the ray's entry side comes first. Only the visit
// order depends on it, never a result (every needed child is still visited).
uint32_t octant_order(const Node64& nd) {
  const float c0[3] = {nd.c0lx + nd.c0hx, nd.c0ly + nd.c0hy, nd.c0lz + nd.c0hz};
  const float c1[3] = {nd.c1lx + nd.c1hx, nd.c1ly + nd.c1hy, nd.c1lz + nd.c1hz};
  int axis = 0;
  float best = -1.0f;
  for (int k = 0; k < 3; k++) {
    const float sep = std::fabs(c1[k] - c0[k]);
    if (sep > best) best = sep, axis = k;
  }
  const bool c1_low = c1[axis] < c0[axis];
  uint32_t bits = 0;
  for (uint32_t oct = 0; oct < 8; oct++) {
    const bool negative = (oct >> axis) & 1u;
    if (c1_low != negative) bits |= 1u << oct;
  }
  return bits;
}

// interior nodes re-laid out depth-first (near child first) from `root`; unreferenced nodes dropped;
// sets hs.nodes, hs.root = 0, hs.depth (levels of interior nodes + the leaf level)
// Sibling-pair layout (RT_NODE_LAYOUT=pairs, A/B): the two interior children of a node occupy one
// 128-B aligned pair of records (one L2 line on MI355X), depth first over the pairs; a node with one
// interior child leaves the second record of its pair empty (never referenced). Root at 0, record 1 empty.
static void relayout_pairs(HostScene& hs, const std::vector<Node64>& tmp, uint32_t root) {
  Node64 empty;
  memset(&empty, 0, sizeof empty);
  empty.c0lx = empty.c0ly = empty.c0lz = empty.c1lx = empty.c1ly = empty.c1lz = INFINITY;
  empty.c0hx = empty.c0hy = empty.c0hz = empty.c1hx = empty.c1hy = empty.c1hz = -INFINITY;
  empty.child0 = empty.child1 = make_leaf(0, 1);
  std::vector<uint32_t> remap(tmp.size(), UINT32_MAX);
  std::vector<uint32_t> slot_src{root, UINT32_MAX};  // record index -> source node (UINT32_MAX = empty)
  remap[root] = 0;
  std::vector<std::pair<uint32_t, int>> st{{root, 1}};
  int depth = 0;
  while (!st.empty()) {
    const auto [n, d] = st.back();
    st.pop_back();
    depth = std::max(depth, d + 1);
    const Node64& nd = tmp[n];
    const bool i0 = !is_leaf(nd.child0), i1 = !is_leaf(nd.child1);
    if (!i0 && !i1) continue;
    const uint32_t base = (uint32_t)slot_src.size();
    slot_src.push_back(UINT32_MAX);
    slot_src.push_back(UINT32_MAX);
    uint32_t k = base;
    if (i0) { remap[nd.child0] = k; slot_src[k++] = nd.child0; }
    if (i1) { remap[nd.child1] = k; slot_src[k++] = nd.child1; }
    if (i1) st.push_back({nd.child1, d + 1});
    if (i0) st.push_back({nd.child0, d + 1});
  }
  hs.nodes.resize(slot_src.size());
  hs.leaves = 0;
  for (size_t i = 0; i < slot_src.size(); i++) {
    if (slot_src[i] == UINT32_MAX) { hs.nodes[i] = empty; continue; }
    Node64 nd = tmp[slot_src[i]];
    if (!is_leaf(nd.child0)) nd.child0 = remap[nd.child0];
    if (!is_leaf(nd.child1)) nd.child1 = remap[nd.child1];
    hs.leaves += (int)is_leaf(nd.child0) + (int)is_leaf(nd.child1);
    nd.pad0 = octant_order(nd);
    hs.nodes[i] = nd;
  }
  hs.root = 0;
  hs.depth = depth;
}

void relayout_dfs(HostScene& hs, const std::vector<Node64>& tmp, uint32_t root) {
  const char* layout_env = debug_env("RT_NODE_LAYOUT");
  const bool pairs = layout_env && !strcmp(layout_env, "pairs");
  if (pairs) { relayout_pairs(hs, tmp, root); return; }
  const size_t N = tmp.size();
  std::vector<uint32_t> remap(N, UINT32_MAX), order;
  int depth = 0;
  // Every builder allocates a node's children after the node itself (child index > parent index). Then the
  // pre-order position follows from subtree sizes in two streaming sweeps over tmp: sizes from the back,
  // positions (and levels) from the front -- pos(child0) = pos + 1, pos(child1) = pos + 1 + size(child0) --
  // the order the explicit-stack walk below gives, without its dependent random accesses (1M-node trees:
  // ~5x faster). Any child at a lower index than its parent takes the walk.
  bool forward = root < N;
  std::vector<uint32_t> size(N, 1);
  for (size_t i = N; forward && i-- > 0;) {
    const Node64& nd = tmp[i];
    for (uint32_t c : {nd.child0, nd.child1}) {
      if (is_leaf(c)) continue;
      if (c <= i || c >= N) { forward = false; break; }
      size[i] += size[c];
    }
  }
  if (forward) {
    std::vector<uint8_t> lev(N, 0);
    remap[root] = 0;
    lev[root] = 1;
    order.assign(size[root], UINT32_MAX);
    for (size_t i = root; i < N; i++) {
      const uint32_t p = remap[i];
      if (p == UINT32_MAX) continue;  // not reachable from root
      order[p] = (uint32_t)i;
      depth = std::max(depth, lev[i] + 1);
      const Node64& nd = tmp[i];
      uint32_t next = p + 1;
      for (uint32_t c : {nd.child0, nd.child1}) {
        if (is_leaf(c)) continue;
        remap[c] = next;
        lev[c] = (uint8_t)std::min(lev[i] + 1, 255);
        next += size[c];
      }
    }
  } else {
    std::fill(remap.begin(), remap.end(), UINT32_MAX);
    std::vector<std::pair<uint32_t, int>> st{{root, 1}};
    while (!st.empty()) {
      const auto [n, d] = st.back();
      st.pop_back();
      remap[n] = (uint32_t)order.size();
      order.push_back(n);
      depth = std::max(depth, d + 1);
      const Node64& nd = tmp[n];
      if (!is_leaf(nd.child1)) st.push_back({nd.child1, d + 1});
      if (!is_leaf(nd.child0)) st.push_back({nd.child0, d + 1});
    }
  }
  hs.nodes.resize(order.size());
  int leaves[16] = {};
  const int T = parallel_chunks(order.size(), [&](size_t b, size_t e, int t) {
    int lv = 0;  // thread-local count (no false sharing on leaves[])
    for (size_t i = b; i < e; i++) {
      Node64 nd = tmp[order[i]];
      if (!is_leaf(nd.child0)) nd.child0 = remap[nd.child0];
      if (!is_leaf(nd.child1)) nd.child1 = remap[nd.child1];
      lv += (int)is_leaf(nd.child0) + (int)is_leaf(nd.child1);
      nd.pad0 = octant_order(nd);
      hs.nodes[i] = nd;
    }
    leaves[t] = lv;
  });
  hs.root = 0;
  hs.depth = depth;
  hs.leaves = 0;
  for (int t = 0; t < T; t++) hs.leaves += leaves[t];
}

// SBVH build (SbvhBuilder) from the face references; leaves get their triangle slots depth first (the
// order the DFS re-layout visits them), so the result does not depend on the build's thread timing
static void build_sbvh(HostScene& hs, int leaf_size, std::vector<Prim>& prims, const Aabb& world, float alpha) {
  const char* budget_env = debug_env("RT_SBVH_BUDGET");
  const float budget = budget_env ? (float)atof(budget_env) : 0.5f;
  const int64_t cap = std::min<int64_t>((int64_t)hs.nf + (int64_t)(budget * hs.nf) + 1, (int64_t)kMaxFaces);
  std::vector<Node64> tmp((size_t)cap);
  SbvhBuilder B{hs, tmp};
  B.hw = std::max(1u, std::thread::hardware_concurrency());
  B.leaf_lists.resize((size_t)cap);
  B.refs = hs.nf;
  B.leaf_size = std::max(1, std::min(leaf_size, kMaxLeaf));
  if (const char* e = debug_env("RT_SAH_TRAV")) B.kTrav = std::max(0.05f, (float)atof(e));
  B.pad = bvh_pad(world.lo, world.hi);
  B.alpha = alpha;
  B.root_area = std::max(world.area(), 1e-30f);
  Aabb rootb;
  const auto tb0 = std::chrono::steady_clock::now();
  uint32_t root = B.build(prims, 0, rootb, cap - hs.nf);
  uint32_t nn = B.next.load();
  if (is_leaf(root)) {
    Node64 nd{};
    B.set_child(nd, 0, rootb, root);
    nd.c1lx = nd.c1ly = nd.c1lz = INFINITY;
    nd.c1hx = nd.c1hy = nd.c1hz = -INFINITY;
    nd.child1 = make_leaf(0, 1);  // never hit; slot 0 exists after the assignment below
    tmp[0] = nd;
    nn = 1;
    root = 0;
  }
  tmp.resize(nn);
  // triangle slots in depth-first leaf order (child 0 first)
  std::vector<uint32_t> order;
  std::vector<uint32_t> st{root};
  while (!st.empty()) {
    Node64& nd = tmp[st.back()];
    st.pop_back();
    uint32_t* hc[2] = {&nd.child0, &nd.child1};
    for (int c = 0; c < 2; c++) {
      const uint32_t h = *hc[c];
      if (!is_leaf(h)) continue;
      if ((c ? nd.c1lx : nd.c0lx) > (c ? nd.c1hx : nd.c0hx)) continue;  // the never-hit sentinel
      const std::vector<uint32_t>& ids = B.leaf_lists[leaf_first(h)];
      *hc[c] = make_leaf((uint32_t)order.size(), leaf_count(h));
      order.insert(order.end(), ids.begin(), ids.end());
    }
    if (!is_leaf(nd.child1)) st.push_back(nd.child1);
    if (!is_leaf(nd.child0)) st.push_back(nd.child0);
  }
  relayout_dfs(hs, tmp, root);
  hs.leaves = (int)B.nleaf.load();
  hs.tris.resize(order.size());
  const float Ro = cert_origin_max(hs);
  parallel_chunks(order.size(), [&](size_t sb, size_t se, int) {
    for (size_t i = sb; i < se; i++) tri_record(hs, order[i], hs.tris[i], Ro);
  });
  if (debug_env("RT_TIMING")) {
    size_t cert = 0;
    for (const TriRec64& t : hs.tris) cert += (t.box & kBoxCertBit) != 0;
    fprintf(stderr, "[rt] sbvh build %.1f ms: %zu references for %d faces, %u nodes, %zu references box-certified\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb0).count(), order.size(),
            hs.nf, nn, cert);
  }
}

void build_bvh(HostScene& hs, int leaf_size, bool spatial) {
  hs.nodes.clear();
  hs.tris.clear();
  hs.depth = 0;
  hs.leaves = 0;
  if (hs.nf == 0) { hs.root = 0; return; }
  std::vector<Prim> prims(hs.nf);
  Aabb wparts[16];
  const int TW = parallel_chunks((size_t)hs.nf, [&](size_t b, size_t e, int t) {
    Aabb wa;  // thread-local, stored once
    for (size_t f = b; f < e; f++) {
      Prim& p = prims[f];
      p.id = (uint32_t)f;
      for (int k = 0; k < 3; k++) { p.lo[k] = INFINITY; p.hi[k] = -INFINITY; }
      for (int j = 0; j < 3; j++) {
        const f3& w = bound_vert(hs, (uint32_t)f, j);
        const float c[3] = {w.x, w.y, w.z};
        for (int k = 0; k < 3; k++) { p.lo[k] = std::min(p.lo[k], c[k]); p.hi[k] = std::max(p.hi[k], c[k]); }
      }
      for (int k = 0; k < 3; k++) p.c[k] = 0.5f * (p.lo[k] + p.hi[k]);
      wa.grow(p.lo, p.hi);
    }
    wparts[t] = wa;
  });
  Aabb world;
  for (int t = 0; t < TW; t++) world.merge(wparts[t]);
  // spatial splits (RT_BUILDER_SBVH): alpha 1e-3 keeps the gain of 1e-5..1e-7 (the same node / triangle
  // counts within 0.2%) at less than half the build time (profiles/ab/r02_sbvh_sweep.txt)
  constexpr float kSbvhAlpha = 1e-3f;
  if (spatial && hs.nf > 1) { build_sbvh(hs, leaf_size, prims, world, kSbvhAlpha); return; }
  std::vector<Node64> tmp((size_t)std::max(hs.nf, 1));
  BvhBuilder B{prims, tmp};
  B.hw = std::max(1u, std::thread::hardware_concurrency());
  B.leaf_size = std::max(1, std::min(leaf_size, kMaxLeaf));
  if (const char* e = debug_env("RT_SAH_TRAV")) B.kTrav = std::max(0.05f, (float)atof(e));
  B.pad = bvh_pad(world.lo, world.hi);
  Aabb rootb;
  const bool timing = debug_env("RT_TIMING") != nullptr;
  auto tb0 = std::chrono::steady_clock::now();
  uint32_t root = B.build(0, (uint32_t)hs.nf, 0, rootb);
  if (timing) fprintf(stderr, "[rt] bvh recursive build %.1f ms\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb0).count());
  uint32_t nn = B.next.load();
  if (is_leaf(root)) {  // whole scene in one leaf: wrap in a node whose second child never hits
    Node64 nd{};
    B.set_child(nd, 0, rootb, root);
    nd.c1lx = nd.c1ly = nd.c1lz = INFINITY;
    nd.c1hx = nd.c1hy = nd.c1hz = -INFINITY;
    nd.child1 = make_leaf(0, 1);
    tmp[0] = nd;
    nn = 1;
    root = 0;
  }
  tmp.resize(nn);
  relayout_dfs(hs, tmp, root);
  hs.leaves = B.leaves.load();
  // triangle records in leaf order
  hs.tris.resize(hs.nf);
  const float Ro = cert_origin_max(hs);
  parallel_chunks((size_t)hs.nf, [&](size_t sb, size_t se, int) {
    for (size_t s = sb; s < se; s++) tri_record(hs, prims[s].id, hs.tris[s], Ro);
  });
}

// GPU LBVH (rt_build.hip) + host depth-first re-layout; false (with nothing changed) if the device
// build is not possible, in which case the caller builds on the host
bool build_bvh_gpu(HostScene& hs, int device, int leaf_size, double* gpu_ms) {
  if (hs.nf <= leaf_size || hs.nf < 2) return false;
  float lo[3], hi[3];
  world_bounds(hs, lo, hi);
  std::vector<TriRec64> recs;
  face_records(hs, recs);
  bound_records(hs, recs);
  if (!device_buildable(recs)) return false;
  std::vector<Node64> tmp;
  std::vector<TriRec64> tris;
  if (gpu_build_lbvh(device, recs, lo, hi, std::max(1, std::min(leaf_size, kMaxLeaf)), bvh_pad(lo, hi), tmp, tris,
                     gpu_ms) != RT_OK)
    return false;
  HostScene trial;
  relayout_dfs(trial, tmp, 0);
  if (trial.depth > kMaxDepth + 2) return false;  // too deep for the wave stack: host SAH instead
  hs.nodes = std::move(trial.nodes);
  hs.root = 0;
  hs.depth = trial.depth;
  hs.leaves = trial.leaves;
  hs.tris = std::move(tris);
  world_records(hs);
  return true;
}

// GPU PLOC (rt_build.hip gpu_build_ploc) + host layout: the device returns the clustered binary tree
// (n - 1 interior nodes, root n - 2) with the SAH collapse flags; here its kept interior nodes get
// pre-order indices, every collapsed subtree / single triangle becomes a leaf whose triangles take
// consecutive slots in depth-first order (child 0 first), and relayout_dfs re-lays out the nodes as for the
// host builders. false (nothing changed) when the device build is impossible or the tree too deep.
// clusters searched either side: on the C3 soup a wider search gives a worse tree (radius 4 / 16 / 32: SAH
// cost 506 / 513 / 517, C3 8.3 / 7.0 / 6.3 Grays/s, profiles/ab/r04_builders.txt), so 4, not the paper's ~25
constexpr int kPlocRadius = 4;
constexpr float kPlocTrav = 0.7f;     // node-step cost relative to a triangle test (as the host builders)
bool build_bvh_ploc(HostScene& hs, int device, int leaf_size, double* gpu_ms) {
  if (hs.nf < 2) return false;
  float lo[3], hi[3];
  world_bounds(hs, lo, hi);
  std::vector<TriRec64> recs;
  face_records(hs, recs);
  bound_records(hs, recs);
  if (!device_buildable(recs)) return false;
  std::vector<int32_t> child;
  std::vector<float> box;
  std::vector<uint8_t> leaf;
  int iters = 0;
  const int lb = std::max(1, std::min(leaf_size, kMaxLeaf));
  int radius = kPlocRadius, rule = 0;
  float trav = kPlocTrav;
  if (const char* e = debug_env("RT_PLOC_RADIUS")) radius = std::max(1, std::min(32, atoi(e)));
  if (const char* e = debug_env("RT_PLOC_TRAV")) trav = std::max(0.05f, (float)atof(e));
  if (const char* e = debug_env("RT_PLOC_RULE")) rule = atoi(e);
  if (gpu_build_ploc(device, recs, lo, hi, lb, radius, trav, child, box, leaf, gpu_ms, &iters, rule) != RT_OK)
    return false;
  const int n = hs.nf, ni = n - 1, root = n - 2;
  const float pad = bvh_pad(lo, hi);
  // pre-order walk (child 0 first): kept interior nodes get tmp indices, leaves get their slots
  std::vector<uint32_t> handle_int((size_t)ni, 0), handle_tri((size_t)n, 0);
  std::vector<int32_t> kept;  // tmp index -> PLOC node
  std::vector<TriRec64> tris;
  tris.reserve((size_t)n);
  std::vector<int32_t> st{root}, sub;
  auto tri_of = [&](int32_t c) { return (uint32_t)~c; };
  while (!st.empty()) {
    const int32_t c = st.back();
    st.pop_back();
    if (c < 0) {  // a single-triangle leaf
      handle_tri[tri_of(c)] = make_leaf((uint32_t)tris.size(), 1u);
      tris.push_back(recs[tri_of(c)]);
    } else if (leaf[(size_t)c] && c != root) {  // a collapsed subtree: its triangles in depth-first order
      const uint32_t first = (uint32_t)tris.size();
      sub.assign(1, c);
      while (!sub.empty()) {
        const int32_t q = sub.back();
        sub.pop_back();
        if (q < 0) { tris.push_back(recs[tri_of(q)]); continue; }
        sub.push_back(child[2 * (size_t)q + 1]);
        sub.push_back(child[2 * (size_t)q]);
      }
      handle_int[(size_t)c] = make_leaf(first, (uint32_t)tris.size() - first);
    } else {
      handle_int[(size_t)c] = (uint32_t)kept.size();
      kept.push_back(c);
      st.push_back(child[2 * (size_t)c + 1]);
      st.push_back(child[2 * (size_t)c]);
    }
  }
  std::vector<Node64> tmp(kept.size());
  for (size_t k = 0; k < kept.size(); k++) {
    const int32_t q = kept[k];
    Node64 nd{};
    for (int side = 0; side < 2; side++) {
      const int32_t c = child[2 * (size_t)q + side];
      float b[6];
      uint32_t h;
      if (c < 0) {
        const TriRec64& t = recs[tri_of(c)];
        b[0] = std::min(std::min(t.w0x, t.w1x), t.w2x); b[3] = std::max(std::max(t.w0x, t.w1x), t.w2x);
        b[1] = std::min(std::min(t.w0y, t.w1y), t.w2y); b[4] = std::max(std::max(t.w0y, t.w1y), t.w2y);
        b[2] = std::min(std::min(t.w0z, t.w1z), t.w2z); b[5] = std::max(std::max(t.w0z, t.w1z), t.w2z);
        h = handle_tri[tri_of(c)];
      } else {
        for (int j = 0; j < 6; j++) b[j] = box[6 * (size_t)c + j];
        h = handle_int[(size_t)c];
      }
      float* o = side ? &nd.c1lx : &nd.c0lx;  // lx hx ly hy lz hz
      o[0] = b[0] - pad; o[1] = b[3] + pad; o[2] = b[1] - pad; o[3] = b[4] + pad; o[4] = b[2] - pad; o[5] = b[5] + pad;
      (side ? nd.child1 : nd.child0) = h;
    }
    tmp[k] = nd;
  }
  HostScene trial;
  relayout_dfs(trial, tmp, 0);
  if (trial.depth > kMaxDepth + 2) return false;  // too deep for the wave stack: host SAH instead
  if (debug_env("RT_TIMING")) fprintf(stderr, "[rt] ploc: %d iterations, %zu nodes, depth %d\n", iters, tmp.size(), trial.depth);
  hs.nodes = std::move(trial.nodes);
  hs.root = 0;
  hs.depth = trial.depth;
  hs.leaves = trial.leaves;
  hs.tris = std::move(tris);
  world_records(hs);
  return true;
}

// GPU top-down binned SAH (rt_build.hip gpu_build_sah) + host layout: interior node 0 is the root, child
// handles are node ids or leaf handles over the returned slot order; the host pads the boxes and re-lays
// the nodes out depth first. false (nothing changed) when the device build is impossible or too deep.
bool build_bvh_sah_gpu(HostScene& hs, int device, int leaf_size, bool spatial, double* gpu_ms) {
  if (hs.nf < 2) return false;
  PhaseTimer pt("sbvh-gpu");
  float lo[3], hi[3];
  world_bounds(hs, lo, hi);
  std::vector<TriRec64> recs;
  face_records(hs, recs);
  bound_records(hs, recs);
  if (!device_buildable(recs)) return false;
  pt.mark("records");
  std::vector<uint32_t> nchild, slot_face;
  std::vector<float> ncb;
  int levels = 0;
  float trav = 0.7f;
  if (const char* e = debug_env("RT_SAH_TRAV")) trav = std::max(0.05f, (float)atof(e));
  float budget = 0.5f;  // as the host SBVH (rt_host.cpp build_sbvh)
  if (const char* e = debug_env("RT_SBVH_BUDGET")) budget = std::max(0.0f, (float)atof(e));
  constexpr float kSbvhGpuAlpha = 1e-3f;  // the host SBVH's overlap threshold (build_bvh)
  if (gpu_build_sah(device, recs, lo, hi, std::max(1, std::min(leaf_size, kMaxLeaf)), trav, spatial, budget, kSbvhGpuAlpha,
                    nchild, ncb, slot_face, gpu_ms, &levels) != RT_OK)
    return false;
  pt.mark("gpu_build_sah");
  const size_t nn = nchild.size() / 2;
  const float pad = bvh_pad(lo, hi);
  std::vector<Node64> tmp(nn);
  std::atomic<bool> bad{false};
  parallel_chunks(nn, [&](size_t kb, size_t ke, int) {
    for (size_t k = kb; k < ke; k++) {
      Node64 nd{};
      for (int side = 0; side < 2; side++) {
        const float* b = &ncb[12 * k + 6 * side];  // lo xyz, hi xyz
        const uint32_t h = nchild[2 * k + side];
        if (!is_leaf(h) && h >= nn) bad = true;
        float* o = side ? &nd.c1lx : &nd.c0lx;  // lx hx ly hy lz hz
        o[0] = b[0] - pad; o[1] = b[3] + pad; o[2] = b[1] - pad; o[3] = b[4] + pad; o[4] = b[2] - pad; o[5] = b[5] + pad;
        (side ? nd.child1 : nd.child0) = h;
      }
      tmp[k] = nd;
    }
  });
  if (bad) return false;
  pt.mark("nodes");
  HostScene trial;
  relayout_dfs(trial, tmp, 0);
  if (trial.depth > kMaxDepth + 2) return false;  // too deep for the wave stack: host SAH instead
  pt.mark("relayout");
  if (debug_env("RT_TIMING"))
    fprintf(stderr, "[rt] %s: %d levels, %zu nodes, %zu references, depth %d\n", spatial ? "sbvh-gpu" : "sah-gpu", levels, nn,
            slot_face.size(), trial.depth);
  std::vector<TriRec64> tris(slot_face.size());
  parallel_chunks(slot_face.size(), [&](size_t b, size_t e, int) {
    for (size_t sl = b; sl < e; sl++) tris[sl] = recs[slot_face[sl]];
  });
  hs.nodes = std::move(trial.nodes);
  hs.root = 0;
  hs.depth = trial.depth;
  hs.leaves = trial.leaves;
  hs.tris = std::move(tris);
  pt.mark("tris");
  world_records(hs);
  pt.mark("world_records");
  return true;
}

// ---------------------------------------------------------------------------------------------------
// 4-wide collapse: each wide node takes a binary node's two children and keeps opening the interior
// child with the largest surface area until it has four children (or only leaves remain). Child
// boxes (already padded) are quantised outward to 8 bits on a per-node, per-axis power-of-two grid.
// ---------------------------------------------------------------------------------------------------
namespace {
struct WChild {
  float lo[3], hi[3];
  uint32_t h;
};

void child_box(const Node64& n, int c, WChild& w) {
  if (c == 0) {
    w.lo[0] = n.c0lx; w.hi[0] = n.c0hx; w.lo[1] = n.c0ly; w.hi[1] = n.c0hy; w.lo[2] = n.c0lz; w.hi[2] = n.c0hz;
    w.h = n.child0;
  } else {
    w.lo[0] = n.c1lx; w.hi[0] = n.c1hx; w.lo[1] = n.c1ly; w.hi[1] = n.c1hy; w.lo[2] = n.c1lz; w.hi[2] = n.c1hz;
    w.h = n.child1;
  }
}

float warea(const WChild& w) {
  float d[3];
  for (int k = 0; k < 3; k++) d[k] = std::max(0.0f, w.hi[k] - w.lo[k]);
  return d[0] * d[1] + d[1] * d[2] + d[2] * d[0];
}

void quantize(Node4Q& q, const WChild* ch, int n) {
  float L[3] = {INFINITY, INFINITY, INFINITY}, U[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int c = 0; c < n; c++)
    for (int k = 0; k < 3; k++) { L[k] = std::min(L[k], ch[c].lo[k]); U[k] = std::max(U[k], ch[c].hi[k]); }
  uint8_t eb[3];
  double scale[3];
  for (int k = 0; k < 3; k++) {
    const double ext = (double)U[k] - (double)L[k];
    int e = -100;
    if (ext > 0) {
      e = (int)std::ceil(std::log2(ext / 255.0));
      while (std::ldexp(255.0, e) < ext) e++;
      e = std::max(e, -100);
    }
    eb[k] = (uint8_t)(e + 127);
    scale[k] = std::ldexp(1.0, e);
  }
  q.ox = L[0]; q.oy = L[1]; q.oz = L[2];
  q.ex = eb[0]; q.ey = eb[1]; q.ez = eb[2];
  q.valid = 0;
  uint32_t* ql[3] = {&q.qlx, &q.qly, &q.qlz};
  uint32_t* qh[3] = {&q.qhx, &q.qhy, &q.qhz};
  for (int k = 0; k < 3; k++) { *ql[k] = 0; *qh[k] = 0; }
  const double org[3] = {q.ox, q.oy, q.oz};
  for (int c = 0; c < 4; c++) {
    if (c >= n) { q.child[c] = 0; continue; }
    q.valid |= (uint8_t)(1u << c);
    q.child[c] = ch[c].h;
    for (int k = 0; k < 3; k++) {
      double a = std::floor(((double)ch[c].lo[k] - org[k]) / scale[k]);
      double b = std::ceil(((double)ch[c].hi[k] - org[k]) / scale[k]);
      a = std::min(std::max(a, 0.0), 255.0);
      b = std::min(std::max(b, 0.0), 255.0);
      while (a > 0 && org[k] + a * scale[k] > (double)ch[c].lo[k]) a -= 1;
      while (b < 255 && org[k] + b * scale[k] < (double)ch[c].hi[k]) b += 1;
      *ql[k] |= (uint32_t)a << (8 * c);
      *qh[k] |= (uint32_t)b << (8 * c);
    }
  }
  q.pad0 = q.pad1 = 0;
}

uint32_t collapse(const std::vector<Node64>& bin, uint32_t n2, std::vector<Node4Q>& out, int depth, int& maxd) {
  maxd = std::max(maxd, depth);
  WChild ch[4];
  int n = 2;
  child_box(bin[n2], 0, ch[0]);
  child_box(bin[n2], 1, ch[1]);
  // drop the never-hit sentinel child of a single-leaf root (inverted box)
  if (ch[1].lo[0] > ch[1].hi[0]) n = 1;
  while (n < 4) {
    int best = -1;
    float ba = -1.0f;
    for (int c = 0; c < n; c++)
      if (!is_leaf(ch[c].h) && warea(ch[c]) > ba) { ba = warea(ch[c]); best = c; }
    if (best < 0) break;
    const Node64& sub = bin[ch[best].h];
    WChild a, b;
    child_box(sub, 0, a);
    child_box(sub, 1, b);
    ch[best] = a;
    ch[n++] = b;
  }
  const uint32_t me = (uint32_t)out.size();
  out.emplace_back();
  uint32_t handles[4];
  for (int c = 0; c < n; c++)
    handles[c] = is_leaf(ch[c].h) ? ch[c].h : collapse(bin, ch[c].h, out, depth + 1, maxd);
  for (int c = 0; c < n; c++) ch[c].h = handles[c];
  quantize(out[me], ch, n);
  return me;
}
}  // namespace

void build_bvh4(HostScene& hs) {
  hs.nodes4.clear();
  hs.depth4 = 0;
  if (hs.nodes.empty()) return;
  hs.nodes4.reserve(hs.nodes.size() / 2 + 1);
  int maxd = 0;
  collapse(hs.nodes, hs.root, hs.nodes4, 0, maxd);
  hs.depth4 = maxd + 1;
}
// (the wide traversal pushes at most 3 entries per level and writes up to 3 slots past the top)

// ---------------------------------------------------------------------------------------------------
// fp32 4-wide tree (Node128 on the device): the same collapse as above (each wide node opens the interior
// child of largest surface area until it has four children), with the BVH2 child boxes kept exactly --
// they are already padded, so culling stays conservative -- and, per ray-direction octant, the children's
// near-to-far order. Order rule (the binary tree's octant_order, pairwise): of two children, along the
// axis on which their centres are furthest apart, the one on the ray's entry side of that axis comes
// first (insertion sort; only the visit order depends on it, never a result).
// ---------------------------------------------------------------------------------------------------
namespace {
bool wide_before(const float* a, const float* b, uint32_t oct) {
  int axis = 0;
  float best = -1.0f;
  for (int k = 0; k < 3; k++) {
    const float sep = std::fabs((b[2 * k] + b[2 * k + 1]) - (a[2 * k] + a[2 * k + 1]));
    if (sep > best) best = sep, axis = k;
  }
  const float ca = a[2 * axis] + a[2 * axis + 1], cb = b[2 * axis] + b[2 * axis + 1];
  return ((oct >> axis) & 1u) ? ca > cb : ca < cb;
}

uint32_t collapse_wide(const std::vector<Node64>& bin, uint32_t n2, std::vector<Wide4>& out, int depth, int& maxd) {
  maxd = std::max(maxd, depth);
  WChild ch[4];
  int n = 2;
  child_box(bin[n2], 0, ch[0]);
  child_box(bin[n2], 1, ch[1]);
  if (ch[1].lo[0] > ch[1].hi[0]) n = 1;  // the never-hit sentinel child of a single-leaf root
  while (n < 4) {
    int best = -1;
    float ba = -1.0f;
    for (int c = 0; c < n; c++)
      if (!is_leaf(ch[c].h) && warea(ch[c]) > ba) { ba = warea(ch[c]); best = c; }
    if (best < 0) break;
    const Node64& sub = bin[ch[best].h];
    WChild a, b;
    child_box(sub, 0, a);
    child_box(sub, 1, b);
    ch[best] = a;
    ch[n++] = b;
  }
  const uint32_t me = (uint32_t)out.size();
  out.emplace_back();
  uint32_t handles[4];
  for (int c = 0; c < n; c++)
    handles[c] = is_leaf(ch[c].h) ? ch[c].h : collapse_wide(bin, ch[c].h, out, depth + 1, maxd);
  Wide4& w = out[me];
  memset(&w, 0, sizeof w);
  w.n = (uint8_t)n;
  for (int c = 0; c < 4; c++) {
    for (int k = 0; k < 3; k++) {
      w.box[c][2 * k] = c < n ? ch[c].lo[k] : INFINITY;
      w.box[c][2 * k + 1] = c < n ? ch[c].hi[k] : -INFINITY;
    }
    w.child[c] = c < n ? handles[c] : kWideEmpty;
  }
  for (uint32_t oct = 0; oct < 8; oct++) {
    uint8_t* o = w.order[oct];
    for (int c = 0; c < 4; c++) o[c] = (uint8_t)c;
    for (int i = 1; i < n; i++)  // insertion sort of the occupied slots; empty slots stay last
      for (int j = i; j > 0 && wide_before(w.box[o[j]], w.box[o[j - 1]], oct); j--) std::swap(o[j], o[j - 1]);
  }
  return me;
}
}  // namespace

void build_wide(HostScene& hs) {
  hs.wide.clear();
  hs.depth_wide = 0;
  if (hs.nodes.empty() || is_leaf(hs.root)) return;
  hs.wide.reserve(hs.nodes.size() / 2 + 1);
  int maxd = 0;
  collapse_wide(hs.nodes, hs.root, hs.wide, 0, maxd);
  hs.depth_wide = maxd + 1;
  if (3 * hs.depth_wide + 4 > kStackW) {  // too deep for the wave stack: binary traversal only
    hs.wide.clear();
    hs.depth_wide = 0;
  }
}

}  // namespace rt

// =====================================================================================================
// Scene creation (host preparation + device upload)
// =====================================================================================================
extern "C" int rt_scene_create(const rt_mesh_desc* d, const rt_scene_opts* opts, rt_scene** out) {
  if (!d || !out) { rt::set_error("rt_scene_create: null argument"); return RT_ERR_INVALID; }
  *out = nullptr;
  if (d->n_vertices < 0 || d->n_faces < 0 || (d->n_faces && (!d->face_vertex_ids || !d->face_normals || !d->face_material_ids)) ||
      (d->n_vertices && (!d->vertices || !d->vertex_normals))) {
    rt::set_error("rt_scene_create: invalid mesh description");
    return RT_ERR_INVALID;
  }
  // leaf handles hold the first triangle slot in 27 bits (the all-ones handle is the traversal's pop
  // marker) and records are addressed by 32-bit byte offsets (kMaxFaces, rt_internal.h)
  static_assert(rt::kMaxFaces < rt::kLeafFirstMask - rt::kMaxLeaf, "leaf handle range");
  if ((int64_t)d->n_faces > (int64_t)rt::kMaxFaces) {
    rt::set_error("rt_scene_create: %d faces exceed the %u-face limit", d->n_faces, rt::kMaxFaces);
    return RT_ERR_INVALID;
  }
  auto t0 = std::chrono::steady_clock::now();
  auto s = new rt_scene();
  if (opts) s->opts = *opts; else rt_scene_opts_default(&s->opts);
  if (s->opts.min_faces <= 0) s->opts.min_faces = 300;
  s->opts.frames_in_flight = std::max(1, std::min(s->opts.frames_in_flight, (int32_t)rt_scene::kMaxSlots));
  if (s->opts.max_boxes <= 0) s->opts.max_boxes = INT32_MAX;
  if (s->opts.device == RT_DEVICE_NONE && s->opts.n_devices != 0) {
    delete s;
    rt::set_error("rt_scene_create: a host-only scene (RT_DEVICE_NONE) lists no devices");
    return RT_ERR_INVALID;
  }
  if (s->opts.device != RT_DEVICE_NONE) {  // device list -> opts.device = devices[0] (builds and uploads there)
    const int rc = rt::resolve_devices(s->opts);
    if (rc) { delete s; return rc; }
  }
  const int leaf = s->opts.leaf_size > 0 ? s->opts.leaf_size : 4;
  // the device's first-use initialisation overlaps the host preparation below (joined before the first
  // device step, or on any return)
  struct Joiner {
    std::thread t;
    ~Joiner() { if (t.joinable()) t.join(); }
  } warm;
  if (s->opts.device != RT_DEVICE_NONE) {
    const int wdev = s->opts.device >= 0 ? s->opts.device : rt::current_device();
    if (wdev >= 0) {
      try {
        warm.t = std::thread(rt::device_warmup, wdev);
      } catch (const std::exception&) {
        // no helper thread (resource limits): the device initialises at its first use instead
      }
    }
  }
  rt::HostScene& hs = s->hs;
  hs.nv = d->n_vertices;
  hs.nf = d->n_faces;
  memcpy(hs.M, d->shape_model_matrix, 64);
  rt::affinv(hs.M, hs.Minv);
  rt::linear_of(hs.Minv, hs.MS);
  hs.fidx.assign(d->face_vertex_ids, d->face_vertex_ids + 3 * (size_t)hs.nf);
  hs.fmat.assign(d->face_material_ids, d->face_material_ids + hs.nf);
  hs.mats.assign(d->materials, d->materials + d->n_materials);
  for (int32_t f = 0; f < hs.nf; f++) {
    for (int k = 0; k < 3; k++)
      if (hs.fidx[3 * f + k] >= (uint32_t)hs.nv) {
        delete s;
        rt::set_error("face %d references vertex %u of %d", f, hs.fidx[3 * f + k], hs.nv);
        return RT_ERR_INVALID;
      }
    if (hs.fmat[f] >= d->n_materials || hs.fmat[f] < -1) {
      delete s;
      rt::set_error("face %d has material id %d (n_materials %d)", f, hs.fmat[f], d->n_materials);
      return RT_ERR_INVALID;
    }
  }
  // hoisted per-vertex / per-face invariants (same expressions as flyscene.cpp:449-450,459,574-577,599)
  hs.wv.resize(hs.nv);
  hs.vnn.resize(hs.nv);
  hs.ov3.resize(3 * (size_t)hs.nv);
  rt::parallel_for((size_t)hs.nv, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; i++) {
      const float* v = d->vertices + 4 * i;
      memcpy(&hs.ov3[3 * i], v, 12);
      hs.wv[i] = rt::affv3(hs.M, f3{v[0] / v[3], v[1] / v[3], v[2] / v[3]});
      const float* n = d->vertex_normals + 3 * i;
      hs.vnn[i] = rt::normalized(f3{n[0], n[1], n[2]});
    }
  });
  hs.fnn.resize(hs.nf);
  hs.fdist.resize(hs.nf);
  rt::parallel_for((size_t)hs.nf, [&](size_t b, size_t e) {
    for (size_t f = b; f < e; f++) {
      const float* n = d->face_normals + 3 * f;
      hs.fnn[f] = rt::normalized(f3{n[0], n[1], n[2]});
      hs.fdist[f] = rt::dot(hs.fnn[f], hs.wv[hs.fidx[3 * f]]);
    }
  });
  rt::accept_region(hs);
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
  if (warm.t.joinable()) warm.t.join();
  s->prep_ms = ms_since(t0);
  auto t1 = clk::now();
  bool boxes_done = false;
  if (s->opts.box_builder == RT_BOXES_GPU && s->opts.device != RT_DEVICE_NONE && hs.nf > 0) {  // (a face-less scene: host)
    int dev = s->opts.device;
    if (dev < 0) dev = rt::current_device();
    bool nonfinite = false;
    if (dev >= 0) {
      const int rc = rt::gpu_build_ref_boxes(dev, hs, d->vertices, s->opts.min_faces, s->opts.max_boxes,
                                             &s->boxes_gpu_ms, &nonfinite);
      if (rc) { delete s; return rc; }
      if (!nonfinite) {
        rt::PhaseTimer pr("boxes-gpu");
        rt::assign_box_ranks(hs);
        pr.mark("box_ranks");
        boxes_done = true;
        s->box_builder_used = RT_BOXES_GPU;
      }
    }
  }
  if (!boxes_done) rt::build_ref_boxes(hs, d->vertices, s->opts.min_faces, s->opts.max_boxes);
  s->boxes_ms = ms_since(t1);
  if (rt::debug_env("RT_TIMING"))
    fprintf(stderr, "[rt] boxes %.1f ms (%s, device %.1f ms), %zu boxes\n", s->boxes_ms,
            s->box_builder_used == RT_BOXES_GPU ? "gpu" : "host", s->boxes_gpu_ms, hs.boxes.size());
  auto t2 = clk::now();
  bool built = false;
  if ((s->opts.builder == RT_BUILDER_SAH_GPU || s->opts.builder == RT_BUILDER_SBVH_GPU) && s->opts.device != RT_DEVICE_NONE) {
    int dev = s->opts.device;
    if (dev < 0) dev = rt::current_device();
    built = dev >= 0 && rt::build_bvh_sah_gpu(hs, dev, leaf, s->opts.builder == RT_BUILDER_SBVH_GPU, &s->bvh_gpu_ms);
    if (built) s->builder_used = s->opts.builder;
  }
  if (s->opts.builder == RT_BUILDER_PLOC_GPU && s->opts.device != RT_DEVICE_NONE) {
    int dev = s->opts.device;
    if (dev < 0) dev = rt::current_device();
    built = dev >= 0 && rt::build_bvh_ploc(hs, dev, leaf, &s->bvh_gpu_ms);
    if (built) s->builder_used = RT_BUILDER_PLOC_GPU;
  }
  if (s->opts.builder == RT_BUILDER_LBVH_GPU && s->opts.device != RT_DEVICE_NONE) {
    int dev = s->opts.device;
    if (dev < 0) dev = rt::current_device();
    // LBVH default leaf bound 1: the Morton tree's small subtrees are poor leaves (measured at 1M tris:
    // 1 -> 97% of the SAH tree's traversal rate, 4 -> 85%)
    const int lb_leaf = s->opts.leaf_size > 0 ? s->opts.leaf_size : 1;
    built = dev >= 0 && rt::build_bvh_gpu(hs, dev, lb_leaf, &s->bvh_gpu_ms);
    if (built) s->builder_used = RT_BUILDER_LBVH_GPU;
  }
  if (!built) {  // host build: spatial splits for either SBVH builder, binned SAH for the rest
    const bool spatial = s->opts.builder == RT_BUILDER_SBVH || s->opts.builder == RT_BUILDER_SBVH_GPU;
    rt::build_bvh(hs, leaf, spatial);
    s->builder_used = spatial ? RT_BUILDER_SBVH : RT_BUILDER_SAH;
    if (rt::debug_env("RT_TIMING")) fprintf(stderr, "[rt] build_bvh %.1f ms\n", ms_since(t2));
    rt::build_bvh4(hs);
  }
  if (s->opts.wide_tree) rt::build_wide(hs);  // fp32 4-wide collapse of the binary tree (PRIMARY packets)
  s->bvh_ms = ms_since(t2);
  if (3 * hs.depth4 + 4 > rt::kStack4) hs.nodes4.clear();  // too deep for the wide stack: binary traversal
  if (hs.depth > rt::kMaxDepth + 2) {  // the wave stack holds 64 entries
    delete s;
    rt::set_error("BVH depth %d exceeds the traversal stack", hs.depth);
    return RT_ERR_UNSUPPORTED;
  }
  s->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (s->opts.device != RT_DEVICE_NONE) {
    auto t3 = clk::now();
    int rc = rt::device_upload(s);
    if (rc) { delete s; return rc; }
    s->upload_ms = ms_since(t3);
    if (s->opts.n_devices > 1 && (rc = rt::device_replicate(s))) { delete s; return rc; }
  }
  *out = s;
  return RT_OK;
}

extern "C" void rt_scene_destroy(rt_scene* s) {
  delete s;  // ~rt_scene releases the device replicas and this scene's device state (rt_device.hip)
}

extern "C" int rt_scene_get_info(const rt_scene* s, rt_scene_info* o) {
  if (!s || !o) { rt::set_error("rt_scene_get_info: null argument"); return RT_ERR_INVALID; }
  o->n_faces = s->hs.nf;
  o->n_vertices = s->hs.nv;
  o->n_ref_boxes = (int32_t)s->hs.boxes.size();
  o->bvh_nodes = (int32_t)s->hs.nodes.size();
  o->bvh_leaves = s->hs.leaves;
  o->bvh_depth = s->hs.depth;
  o->device_bytes = s->device_bytes;
  for (const auto& r : s->replicas) o->device_bytes += r->device_bytes;
  o->n_devices = s->device == RT_DEVICE_NONE ? 0 : 1 + (int32_t)s->replicas.size();
  o->replicate_ms = s->replicate_ms;
  o->build_ms = s->build_ms;
  o->device = s->device;
  o->prep_ms = s->prep_ms;
  o->boxes_ms = s->boxes_ms;
  o->bvh_ms = s->bvh_ms;
  o->upload_ms = s->upload_ms;
  o->builder = s->builder_used;
  o->bvh_gpu_ms = s->bvh_gpu_ms;
  o->box_builder = s->box_builder_used;
  o->boxes_gpu_ms = s->boxes_gpu_ms;
  {
    // the wide tree is uploaded only where its record offsets fit below kLeafBit (record_layout)
    uint64_t wb = 0;
    rt::record_layout(s->hs.nodes.size(), s->hs.tris.size(), s->hs.wide.size(), &wb);
    o->wide_nodes = wb ? (int32_t)s->hs.wide.size() : 0;
  }
  o->wide_depth = s->hs.depth_wide;
  return RT_OK;
}

// BoundingBox::setRandomColor (BoundingBox.cpp:163-165) per box in creation order. The three rand() calls
// are constructor arguments, whose evaluation order C++ leaves open; the reference built with g++ (this
// image's compiler, and x86-64 MSVC alike) evaluates them right to left: a box's first call is its blue
// channel (tests/golden/boxcolor_kat.bin, generated from that expression by oracle/boxcolor_kat.cpp).
extern "C" int rt_box_colors_random(int32_t n_boxes, rt_rand_state* rng, float* out3) {
  if (n_boxes < 0 || (n_boxes && !out3)) { rt::set_error("rt_box_colors_random: bad arguments"); return RT_ERR_INVALID; }
  rt_rand_state local;
  if (!rng) { rt_rand_seed(&local, 1); rng = &local; }
  for (int64_t b = 0; b < (int64_t)n_boxes; b++)
    for (int k = 2; k >= 0; k--) out3[3 * b + k] = (float)rt_rand(rng) / (float)2147483647;
  return RT_OK;
}

extern "C" int rt_scene_set_box_colors(rt_scene* s, const float* colors3) {
  if (!s) { rt::set_error("rt_scene_set_box_colors: null scene"); return RT_ERR_INVALID; }
  const int32_t nb = (int32_t)s->hs.boxes.size();
  std::vector<float> c(3 * (size_t)nb);
  if (colors3) memcpy(c.data(), colors3, c.size() * 4);
  else rt_box_colors_random(nb, nullptr, c.data());
  // frames in flight may still read the per-face table: it is rebuilt at the next box-colour frame,
  // after the scene's streams have drained (rt_device.hip: ensure_face_boxcolor)
  for (auto& r : s->replicas) {  // every device of a multi-device scene renders with the same colours
    r->box_colors = c;
    r->face_boxcolor_valid = false;
  }
  s->box_colors.swap(c);
  s->face_boxcolor_valid = false;
  return RT_OK;
}

extern "C" int rt_scene_ref_boxes(const rt_scene* s, float* bounds6, int32_t* counts, int32_t* face_order) {
  if (!s) { rt::set_error("rt_scene_ref_boxes: null scene"); return RT_ERR_INVALID; }
  size_t off = 0;
  for (size_t i = 0; i < s->hs.boxes.size(); i++) {
    const rt::RefBox& b = s->hs.boxes[i];
    if (bounds6) { memcpy(bounds6 + 6 * i, b.low, 12); memcpy(bounds6 + 6 * i + 3, b.high, 12); }
    if (counts) counts[i] = (int32_t)b.faces.size();
    if (face_order) memcpy(face_order + off, b.faces.data(), sizeof(int32_t) * b.faces.size());
    off += b.faces.size();
  }
  return RT_OK;
}

// =====================================================================================================
// Verification hook: Eigen-order primitives on the host (op codes: oracle/eigen_kat.cpp)
// =====================================================================================================
#include "rt_kat.h"

extern "C" int rt_debug_math_host(int32_t op, int32_t n, const float* in, float* out) {
  static const int in_len[] = {6, 3, 6, 12, 19, 20, 9, 16, 4, 6, 6, 6, 6, 13, 3, 16, 24, 2};
  static const int out_len[] = {1, 3, 3, 3, 3, 4, 9, 16, 16, 3, 3, 3, 3, 3, 1, 3, 3, 1};
  if (op < 0 || op > 17 || n < 0 || !in || !out) { rt::set_error("rt_debug_math_host: bad op"); return RT_ERR_INVALID; }
  for (int32_t k = 0; k < n; k++)
    if (rt::debug_math_case(op, in + (size_t)k * in_len[op], out + (size_t)k * out_len[op])) return RT_ERR_INVALID;
  return RT_OK;
}

// ---------------------------------------------------------------------------------------------------
// Acceleration-structure validation (rt_debug_validate_bvh)
// ---------------------------------------------------------------------------------------------------
namespace {
struct VBox {
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void add(const VBox& b) {
    for (int k = 0; k < 3; k++) { lo[k] = std::min(lo[k], b.lo[k]); hi[k] = std::max(hi[k], b.hi[k]); }
  }
  bool inside(const double* l, const double* h) const {
    for (int k = 0; k < 3; k++)
      if (lo[k] <= hi[k] && (lo[k] < l[k] || hi[k] > h[k])) return false;
    return true;
  }
};

struct Validator {
  const rt::HostScene& hs;
  std::vector<int> seen2, seen4;
  int64_t bad = 0;
  // a tree without duplicated references must hold every triangle whole inside every ancestor box;
  // a spatial-split tree (more records than faces) holds each reference's part: its content is the
  // triangle's bounds cut to the path's boxes, and coverage() checks that the faces' leaf regions
  // together cover every face
  bool strict = true;
  std::vector<std::vector<VBox>> regions;  // per face: the path-intersected boxes of its leaves (split trees)
  // the box of the triangle the culling must bound (rt::bound_vert: the accept region)
  VBox tri_box(const rt::TriRec64& t) const {
    VBox b;
    for (int j = 0; j < 3; j++) {
      const rt::f3& w = rt::bound_vert(hs, t.face, j);
      const double v[3] = {w.x, w.y, w.z};
      for (int k = 0; k < 3; k++) { b.lo[k] = std::min(b.lo[k], v[k]); b.hi[k] = std::max(b.hi[k], v[k]); }
    }
    return b;
  }
  VBox leaf(uint32_t h, std::vector<int>& seen, const VBox& region, bool record) {
    VBox b;
    for (uint32_t i = rt::leaf_first(h); i < rt::leaf_first(h) + rt::leaf_count(h); i++) {
      if (i >= hs.tris.size()) { bad++; continue; }
      seen[i]++;
      VBox t = tri_box(hs.tris[i]);
      if (!strict) {
        for (int k = 0; k < 3; k++) { t.lo[k] = std::max(t.lo[k], region.lo[k]); t.hi[k] = std::min(t.hi[k], region.hi[k]); }
        if (t.lo[0] > t.hi[0] || t.lo[1] > t.hi[1] || t.lo[2] > t.hi[2]) { bad++; continue; }  // reference outside its region
        if (record && hs.tris[i].face < regions.size()) regions[hs.tris[i].face].push_back(region);
      }
      b.add(t);
    }
    return b;
  }
  static VBox cut(const VBox& a, const double* l, const double* u) {
    VBox r;
    for (int k = 0; k < 3; k++) { r.lo[k] = std::max(a.lo[k], l[k]); r.hi[k] = std::min(a.hi[k], u[k]); }
    return r;
  }
  VBox bin(uint32_t n, int d, int64_t& depth, const VBox& region) {
    depth = std::max<int64_t>(depth, d + 1);
    const rt::Node64& nd = hs.nodes[n];
    VBox all;
    for (int c = 0; c < 2; c++) {
      const uint32_t h = c ? nd.child1 : nd.child0;
      if ((c ? nd.c1lx : nd.c0lx) > (c ? nd.c1hx : nd.c0hx)) continue;  // never-hit sentinel child
      const double l[3] = {c ? nd.c1lx : nd.c0lx, c ? nd.c1ly : nd.c0ly, c ? nd.c1lz : nd.c0lz};
      const double u[3] = {c ? nd.c1hx : nd.c0hx, c ? nd.c1hy : nd.c0hy, c ? nd.c1hz : nd.c0hz};
      const VBox sub = cut(region, l, u);
      const VBox b = rt::is_leaf(h) ? leaf(h, seen2, sub, true) : bin(h, d + 1, depth, sub);
      if (!b.inside(l, u)) bad++;
      all.add(b);
    }
    return all;
  }
  VBox wide(uint32_t n, int d, int64_t& depth, const VBox& region) {
    depth = std::max<int64_t>(depth, d + 1);
    const rt::Node4Q& nd = hs.nodes4[n];
    const double org[3] = {nd.ox, nd.oy, nd.oz};
    const uint8_t e[3] = {nd.ex, nd.ey, nd.ez};
    const uint32_t ql[3] = {nd.qlx, nd.qly, nd.qlz}, qh[3] = {nd.qhx, nd.qhy, nd.qhz};
    VBox all;
    for (int c = 0; c < 4; c++) {
      if (!((nd.valid >> c) & 1)) continue;
      const uint32_t h = nd.child[c];
      double l[3], u[3];
      for (int k = 0; k < 3; k++) {
        // the device's cell size: the float with biased exponent e (2^(e-127))
        const double sc = std::ldexp(1.0, (int)e[k] - 127);
        l[k] = org[k] + ((ql[k] >> (8 * c)) & 255u) * sc;
        u[k] = org[k] + ((qh[k] >> (8 * c)) & 255u) * sc;
      }
      const VBox sub = cut(region, l, u);
      const VBox b = rt::is_leaf(h) ? leaf(h, seen4, sub, false) : wide(h, d + 1, depth, sub);
      if (!b.inside(l, u)) bad++;
      all.add(b);
    }
    return all;
  }
  // the fp32 4-wide tree (device Node128): its boxes are the binary tree's, copied; every octant order
  // a permutation of the slots with the occupied ones first
  std::vector<int> seenw;
  VBox widef(uint32_t n, int d, int64_t& depth, const VBox& region) {
    depth = std::max<int64_t>(depth, d + 1);
    if (n >= hs.wide.size()) { bad++; return VBox{}; }
    const rt::Wide4& w = hs.wide[n];
    for (int o = 0; o < 8; o++) {
      int mask = 0;
      for (int k = 0; k < 4; k++) {
        mask |= 1 << w.order[o][k];
        if ((k < w.n) != (w.order[o][k] < w.n)) bad++;
      }
      if (mask != 15) bad++;
    }
    VBox all;
    for (int c = 0; c < w.n; c++) {
      const uint32_t h = w.child[c];
      const double l[3] = {w.box[c][0], w.box[c][2], w.box[c][4]}, u[3] = {w.box[c][1], w.box[c][3], w.box[c][5]};
      const VBox sub = cut(region, l, u);
      const VBox b = rt::is_leaf(h) ? leaf(h, seenw, sub, false) : widef(h, d + 1, depth, sub);
      if (!b.inside(l, u)) bad++;
      all.add(b);
    }
    return all;
  }
  // split trees: points of every face on a barycentric grid (vertices, edges, interior) each lie in
  // one of that face's leaf regions
  void coverage() {
    constexpr int G = 8;
    for (uint32_t f = 0; f < (uint32_t)hs.nf; f++) {
      const std::vector<VBox>& rs = regions[f];
      if (rs.empty()) { bad++; continue; }
      const rt::f3& a = rt::bound_vert(hs, f, 0);
      const rt::f3& b = rt::bound_vert(hs, f, 1);
      const rt::f3& c = rt::bound_vert(hs, f, 2);
      for (int i = 0; i <= G; i++)
        for (int j = 0; i + j <= G; j++) {
          const double s = (double)i / G, t = (double)j / G, r = 1.0 - s - t;
          const double p[3] = {r * a.x + s * b.x + t * c.x, r * a.y + s * b.y + t * c.y, r * a.z + s * b.z + t * c.z};
          bool in = false;
          for (const VBox& q : rs) {
            in = true;
            for (int k = 0; k < 3; k++) in = in && p[k] >= q.lo[k] && p[k] <= q.hi[k];
            if (in) break;
          }
          if (!in) bad++;
        }
    }
  }
};
}  // namespace

extern "C" int rt_debug_record_layout(int64_t n_nodes, int64_t n_tris, int64_t n_wide, int64_t out[2]) {
  if (!out || n_nodes < 0 || n_tris < 0 || n_wide < 0) { rt::set_error("rt_debug_record_layout: bad argument"); return RT_ERR_INVALID; }
  uint64_t wb = 0;
  out[0] = (int64_t)rt::record_layout((uint64_t)n_nodes, (uint64_t)n_tris, (uint64_t)n_wide, &wb);
  out[1] = (int64_t)wb;
  return RT_OK;
}

extern "C" int rt_debug_scene_flags(const rt_scene* s, int64_t counts[3], float* cert_origin_max, uint32_t* face_flags) {
  if (!s || !counts) { rt::set_error("rt_debug_scene_flags: null argument"); return RT_ERR_INVALID; }
  counts[0] = (int64_t)s->hs.tris.size();
  counts[1] = counts[2] = 0;
  if (face_flags) memset(face_flags, 0, sizeof(uint32_t) * (size_t)s->hs.nf);
  for (const rt::TriRec64& t : s->hs.tris) {
    counts[1] += (t.box & rt::kSafeNormalBit) != 0;
    counts[2] += (t.box & rt::kBoxCertBit) != 0;
    if (face_flags && t.face < (uint32_t)s->hs.nf) face_flags[t.face] |= t.box & (rt::kSafeNormalBit | rt::kBoxCertBit);
  }
  if (cert_origin_max) *cert_origin_max = rt::cert_origin_max(s->hs);
  return RT_OK;
}

extern "C" int rt_debug_tree_cost(const rt_scene* s, double k_trav, double out[4]) {
  if (!s || !out) { rt::set_error("rt_debug_tree_cost: null argument"); return RT_ERR_INVALID; }
  const rt::HostScene& hs = s->hs;
  for (int k = 0; k < 4; k++) out[k] = 0.0;
  if (hs.nodes.empty()) return RT_OK;
  auto area = [](const float* b) {  // lx hx ly hy lz hz
    const double dx = (double)b[1] - b[0], dy = (double)b[3] - b[2], dz = (double)b[5] - b[4];
    return dx < 0 || dy < 0 || dz < 0 ? 0.0 : dx * dy + dy * dz + dz * dx;
  };
  double inner = 0.0, leafc = 0.0, leaves = 0.0, tris = 0.0;
  std::vector<std::pair<uint32_t, double>> st{{hs.root, -1.0}};
  double root_area = 0.0;
  while (!st.empty()) {
    const auto [h, a] = st.back();
    st.pop_back();
    if (rt::is_leaf(h)) {
      leafc += a * rt::leaf_count(h);
      leaves += 1;
      tris += rt::leaf_count(h);
      continue;
    }
    const rt::Node64& nd = hs.nodes[h];
    const float* b0 = &nd.c0lx;
    const float* b1 = &nd.c1lx;
    double an = a;
    if (an < 0) {  // the root: the union of its children's boxes
      float u[6];
      for (int k = 0; k < 3; k++) {
        u[2 * k] = std::min(b0[2 * k], b1[2 * k]);
        u[2 * k + 1] = std::max(b0[2 * k + 1], b1[2 * k + 1]);
      }
      an = root_area = area(u);
    }
    inner += an;
    st.push_back({nd.child0, area(b0)});
    st.push_back({nd.child1, area(b1)});
  }
  if (!(root_area > 0)) return RT_OK;
  out[0] = (k_trav * inner + leafc) / root_area;  // SAH cost in triangle tests per random ray
  out[1] = inner / root_area;                      // expected node visits (interior) per random ray
  out[2] = leafc / root_area;                      // expected triangle tests per random ray
  out[3] = leaves > 0 ? tris / leaves : 0.0;       // mean leaf size
  return RT_OK;
}

extern "C" int rt_debug_validate_bvh(const rt_scene* s, int64_t info[7]) {
  if (!s || !info) { rt::set_error("rt_debug_validate_bvh: null argument"); return RT_ERR_INVALID; }
  const rt::HostScene& hs = s->hs;
  Validator v{hs, std::vector<int>(hs.tris.size()), std::vector<int>(hs.tris.size())};
  v.strict = hs.tris.size() == (size_t)hs.nf;
  if (!v.strict) v.regions.resize((size_t)hs.nf);
  for (int k = 0; k < 7; k++) info[k] = 0;
  info[0] = (int64_t)hs.nodes.size();
  info[2] = (int64_t)hs.nodes4.size();
  const VBox everywhere = [] {
    VBox b;
    for (int k = 0; k < 3; k++) { b.lo[k] = -INFINITY; b.hi[k] = INFINITY; }
    return b;
  }();
  if (!hs.nodes.empty()) v.bin(hs.root, 0, info[1], everywhere);
  if (!hs.nodes4.empty()) v.wide(0, 0, info[3], everywhere);
  if (!v.strict && !hs.nodes.empty()) v.coverage();
  int64_t wide_depth = 0, wide_once = 0;
  v.seenw.assign(hs.tris.size(), 0);
  if (!hs.wide.empty()) {
    v.widef(0, 0, wide_depth, everywhere);
    if (wide_depth != hs.depth_wide || 3 * wide_depth + 4 > rt::kStackW) v.bad++;
  }
  for (size_t i = 0; i < hs.tris.size(); i++) {
    info[4] += v.seen2[i] == 1;
    info[5] += v.seen4[i] == 1;
    wide_once += v.seenw[i] == 1;
  }
  info[6] = v.bad;
  const bool ok = v.bad == 0 && info[4] == (int64_t)hs.tris.size() &&
                  (hs.nodes4.empty() || info[5] == (int64_t)hs.tris.size()) &&
                  (hs.wide.empty() || wide_once == (int64_t)hs.tris.size());
  if (!ok) { rt::set_error("acceleration structure check failed (%lld violations)", (long long)v.bad); return RT_ERR_INVALID; }
  return RT_OK;
}
