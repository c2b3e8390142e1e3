// Host-side AddressSanitizer / UBSan harness (CPU only; tools/asan/run.sh builds it): drives the host
// entry points of the C ABI -- OBJ ingest (valid and malformed files), host-only scene creation with
// both box builders' host path, the BVH validator, the binary scene cache (save, load, and every
// truncation / byte flip of a small file), PPM writers, lights and camera helpers -- so that heap
// errors in the host code surface as sanitizer reports instead of later crashes.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt/rt_api.h"

static int g_fail = 0;
#define EXPECT(c)                                                          \
  do {                                                                     \
    if (!(c)) { std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); g_fail++; } \
  } while (0)

static std::string tmpdir() {
  const char* t = std::getenv("TMPDIR");
  return std::string(t ? t : "/tmp");
}

static void write_file(const std::string& p, const std::string& s) {
  FILE* f = std::fopen(p.c_str(), "wb");
  std::fwrite(s.data(), 1, s.size(), f);
  std::fclose(f);
}

static std::string read_file(const std::string& p) {
  std::string s;
  FILE* f = std::fopen(p.c_str(), "rb");
  if (!f) return s;
  std::fseek(f, 0, SEEK_END);
  s.resize((size_t)std::ftell(f));
  std::fseek(f, 0, SEEK_SET);
  if (!s.empty() && std::fread(&s[0], 1, s.size(), f) != s.size()) s.clear();
  std::fclose(f);
  return s;
}

static void malformed_objs() {
  const std::string p = tmpdir() + "/rt_asan_bad.obj";
  const char* cases[] = {
      "v 0 0 0\nv 1 0 0\nf 1 2\n",                  // not a multiple of 3
      "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 9\n",       // index past the end (computeNormals path)
      "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 0 1 2\n",       // index 0 -> -1
      "v 0 0 0\nv 1 0 0\nv 0 1 0\nf -1 2 3\n",      // negative
      "f 1 2 3\n",                                  // faces without vertices
      "v 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\nf 1 2 3\n",  // #vn != #v
      "mtllib\n",                                   // malformed mtllib
      "usemtl\n",                                   // malformed usemtl
      "v 1e40 -1e40 nan\nv 1 0 0\nv 0 1 0\nf 1 2 3\n",
      "v\nvn\nf\n",
      "",
  };
  for (const char* c : cases) {
    write_file(p, c);
    rt_mesh* m = nullptr;
    int rc = rt_mesh_load_obj(p.c_str(), &m);
    if (rc == RT_OK) {
      rt_mesh_desc d;
      EXPECT(rt_mesh_get_desc(m, &d) == RT_OK);
      rt_mesh_destroy(m);
    } else {
      EXPECT(m == nullptr);
    }
  }
  rt_mesh* m = nullptr;
  EXPECT(rt_mesh_load_obj((tmpdir() + "/rt_asan_missing.obj").c_str(), &m) != RT_OK);
}

static void from_arrays() {
  const float v[9] = {0, 0, 0, 1, 0, 0, 0, 1, 0};
  const uint32_t bad[3] = {0, 1, 7};
  const int32_t gc[1] = {3}, gm[1] = {-1};
  rt_mesh* m = nullptr;
  EXPECT(rt_mesh_from_arrays(3, v, nullptr, 1, gc, bad, gm, 0, nullptr, &m) != RT_OK);
  const uint32_t good[3] = {0, 1, 2};
  EXPECT(rt_mesh_from_arrays(3, v, nullptr, 1, gc, good, gm, 0, nullptr, &m) == RT_OK);
  rt_mesh_destroy(m);
  const int32_t gneg[1] = {-3};
  EXPECT(rt_mesh_from_arrays(3, v, nullptr, 1, gneg, good, gm, 0, nullptr, &m) != RT_OK);
}

static void scene_roundtrip(const std::string& obj, int box_builder) {
  rt_mesh* m = nullptr;
  if (rt_mesh_load_obj(obj.c_str(), &m) != RT_OK) { std::fprintf(stderr, "skip %s\n", obj.c_str()); return; }
  rt_mesh_desc d;
  EXPECT(rt_mesh_get_desc(m, &d) == RT_OK);
  rt_scene_opts o;
  rt_scene_opts_default(&o);
  o.device = RT_DEVICE_NONE;
  o.box_builder = box_builder;
  rt_scene* s = nullptr;
  EXPECT(rt_scene_create(&d, &o, &s) == RT_OK);
  if (!s) { rt_mesh_destroy(m); return; }
  int64_t info[7];
  EXPECT(rt_debug_validate_bvh(s, info) == RT_OK);
  rt_scene_info si;
  EXPECT(rt_scene_get_info(s, &si) == RT_OK);
  std::vector<float> b6(6 * (size_t)si.n_ref_boxes);
  std::vector<int32_t> cnt(si.n_ref_boxes), order(si.n_faces);
  EXPECT(rt_scene_ref_boxes(s, b6.data(), cnt.data(), order.data()) == RT_OK);
  const std::string p = tmpdir() + "/rt_asan.rtscene", q = tmpdir() + "/rt_asan_bad.rtscene";
  EXPECT(rt_scene_save(s, p.c_str()) == RT_OK);
  rt_scene* l = nullptr;
  EXPECT(rt_scene_load(p.c_str(), &o, &l) == RT_OK);
  if (l) rt_scene_destroy(l);
  // damaged copies: every truncation length on a coarse grid and single-bit flips across the file
  const std::string raw = read_file(p);
  const size_t step = raw.size() / 97 + 1;
  for (size_t n = 0; n < raw.size(); n += step) {
    write_file(q, raw.substr(0, n));
    l = nullptr;
    if (rt_scene_load(q.c_str(), &o, &l) == RT_OK) rt_scene_destroy(l);
  }
  for (size_t i = 0; i < raw.size(); i += step) {
    std::string c = raw;
    c[i] ^= 0x10;
    write_file(q, c);
    l = nullptr;
    if (rt_scene_load(q.c_str(), &o, &l) == RT_OK) rt_scene_destroy(l);
  }
  rt_scene_destroy(s);
  rt_mesh_destroy(m);
}

static void misc() {
  const int W = 7, H = 5;
  std::vector<float> rgb(3 * W * H, 0.5f);
  std::vector<uint8_t> rgb8(3 * W * H, 200);
  EXPECT(rt_write_ppm((tmpdir() + "/rt_asan.ppm").c_str(), rgb.data(), W, H) == RT_OK);
  EXPECT(rt_write_ppm_rgb8((tmpdir() + "/rt_asan8.ppm").c_str(), rgb8.data(), W, H) == RT_OK);
  rt_rand_state st;
  rt_rand_seed(&st, 1);
  for (int i = 0; i < 1000; i++) (void)rt_rand(&st);
  rt_camera cam;
  rt_camera_flycam(64, 48, 0.0f, 0.0f, 20.0f, &cam);
  rt_light c;
  std::memset(&c, 0, sizeof c);
  c.position[0] = 1.0f; c.color[0] = c.color[1] = c.color[2] = 1.0f;
  std::vector<rt_light> out(9);
  (void)rt_lights_spherical(&c, 0.5f, 8, &st, out.data());
  const float col[3] = {1, 1, 1};
  rt_light_directional(&cam, col, &out[0]);
  std::vector<float> soup(9 * 1000);
  rt_generate_soup(1000, 12345, soup.data());
}

int main(int argc, char** argv) {
  const std::string scenes = argc > 1 ? argv[1] : "scenes";
  malformed_objs();
  from_arrays();
  for (const char* n : {"cube.obj", "testding.obj", "dodgeColorTest.obj"})
    for (int bb : {RT_BOXES_HOST}) scene_roundtrip(scenes + "/" + n, bb);
  misc();
  std::printf("host_asan: %s (%d failed expectations)\n", g_fail ? "FAILED" : "ok", g_fail);
  return g_fail ? 1 : 0;
}
