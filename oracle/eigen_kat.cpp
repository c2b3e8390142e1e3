// eigen_kat.cpp -- TEST INFRASTRUCTURE (oracle pinning), never shipped or linked by the product.
//
// Generates known-answer vectors for every Eigen 3.3.7 float expression the reference hot path
// evaluates, by running those expressions through the Eigen headers VENDORED in the reference
// (/root/reference/dependencies/eigen/include, the exact version the reference compiles against).
// The output file (tests/golden/eigen_kat.bin) pins the op order / rounding of:
//   - oracle/rt_oracle.c   (CPU restatement used as the parity checker), and
//   - ray-tracing-project_amd/csrc/rt_math.h  (host + device arithmetic of the product).
//
// Why this exists: Eigen's fixed-size reductions are NOT left-associative. A Vector3f dot()
// reduces as x0 + (x1 + x2) (redux_novec_unroller halving, Redux.h), while Matrix4f*Vector4f
// accumulates column packets left to right. Bit parity with the reference needs the exact order.
//
// Expressions mirrored (reference call sites):
//   DOT/NORMALIZED/NORM/CROSS     src/flyscene.cpp:450,453,459,463,558,587-599 (Dot.h, OrthoMethods.h)
//   M3V3                          src/flyscene.cpp:490  (MS * dir)
//   AFF_V3                        src/flyscene.cpp:449,489,574-576 (Affine3f * Vector3f)
//   M4V4                          Transform.h:1372-1392 (T.matrix() * [v;1])
//   M3INV / AFF_INV               src/flyscene.cpp:486 (getShapeModelMatrix().inverse()), camera.hpp:170
//   SHAPE                         tucano/model.hpp:102-105,169-173 (scale(s).translate(-c), I*shape)
//   OFFSET_001 / OFFSET_003       src/flyscene.cpp:362 (P + 0.001*r), :512 (P + 0.003*L)
//   REFLECT                       src/flyscene.cpp:480-482
//   PHONG_R                       src/flyscene.cpp:557
//   NRM_INTERP                    src/flyscene.cpp:599
//   CENTER                        tucano/camera.hpp:115-118
//   SCREEN                        tucano/camera.hpp:155-173,263-266
//
// Build: oracle/Makefile target `eigen_kat` (only where /root/reference exists). Output binary goes
// to oracle/_ref/ (git-ignored); the generated fixture is committed.
#include <Eigen/Dense>
#include <Eigen/Geometry>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

using Eigen::Affine3f;
using Eigen::Matrix3f;
using Eigen::Matrix4f;
using Eigen::Vector3f;
using Eigen::Vector4f;

enum {
  OP_DOT = 0, OP_NORMALIZED, OP_CROSS, OP_M3V3, OP_AFF_V3, OP_M4V4, OP_M3INV, OP_AFF_INV,
  OP_SHAPE, OP_OFFSET_001, OP_OFFSET_003, OP_REFLECT, OP_PHONG_R, OP_NRM_INTERP, OP_NORM,
  OP_CENTER, OP_SCREEN, OP_COUNT
};

static std::mt19937 rng(20261015);
static float uni(float lo, float hi) { return std::uniform_real_distribution<float>(lo, hi)(rng); }
static float wild() {
  // mix of magnitudes and exact specials, so zero handling and signs get exercised
  int k = std::uniform_int_distribution<int>(0, 15)(rng);
  if (k == 0) return 0.0f;
  if (k == 1) return -0.0f;
  if (k == 2) return 1.0f;
  if (k < 6) return uni(-1e-3f, 1e-3f);
  if (k < 9) return uni(-100.f, 100.f);
  return uni(-1.f, 1.f);
}

struct Section {
  int op, n, in_len, out_len;
  std::vector<float> in, out;
};

static Vector3f v3(const float* p) { return Vector3f(p[0], p[1], p[2]); }

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "eigen_kat.bin";
  const int N = 2000;
  std::vector<Section> secs;
  auto add = [&](int op, int in_len, int out_len) -> Section& {
    secs.push_back(Section{op, N, in_len, out_len, {}, {}});
    secs.back().in.resize((size_t)N * in_len);
    secs.back().out.resize((size_t)N * out_len);
    return secs.back();
  };

  { Section& s = add(OP_DOT, 6, 1);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 6]; for (int i = 0; i < 6; i++) a[i] = wild();
      s.out[k] = v3(a).dot(v3(a + 3)); } }
  { Section& s = add(OP_NORMALIZED, 3, 3);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 3]; for (int i = 0; i < 3; i++) a[i] = (k % 50 == 0) ? 0.f : wild();
      Vector3f r = v3(a).normalized(); memcpy(&s.out[k * 3], r.data(), 12); } }
  { Section& s = add(OP_CROSS, 6, 3);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 6]; for (int i = 0; i < 6; i++) a[i] = wild();
      Vector3f r = v3(a).cross(v3(a + 3)); memcpy(&s.out[k * 3], r.data(), 12); } }
  { Section& s = add(OP_M3V3, 12, 3);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 12]; for (int i = 0; i < 12; i++) a[i] = wild();
      Matrix3f M; memcpy(M.data(), a, 36); Vector3f r = M * v3(a + 9); memcpy(&s.out[k * 3], r.data(), 12); } }
  { Section& s = add(OP_AFF_V3, 19, 3);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 19]; for (int i = 0; i < 19; i++) a[i] = wild();
      a[3] = a[7] = a[11] = 0.f; a[15] = 1.f;
      Affine3f T; memcpy(T.matrix().data(), a, 64); Vector3f r = T * v3(a + 16); memcpy(&s.out[k * 3], r.data(), 12); } }
  { Section& s = add(OP_M4V4, 20, 4);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 20]; for (int i = 0; i < 20; i++) a[i] = wild();
      Matrix4f M; memcpy(M.data(), a, 64); Vector4f v(a[16], a[17], a[18], a[19]); Vector4f r = M * v;
      memcpy(&s.out[k * 4], r.data(), 16); } }
  { Section& s = add(OP_M3INV, 9, 9);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 9];
      if (k % 3 == 0) { float d = uni(0.1f, 3.f); for (int i = 0; i < 9; i++) a[i] = (i % 4 == 0) ? d : 0.f; }
      else for (int i = 0; i < 9; i++) a[i] = uni(-2.f, 2.f);
      Matrix3f M; memcpy(M.data(), a, 36); Matrix3f r = M.inverse(); memcpy(&s.out[k * 9], r.data(), 36); } }
  { Section& s = add(OP_AFF_INV, 16, 16);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 16];
      Affine3f T = Affine3f::Identity();
      if (k % 2 == 0) { T.scale(uni(0.2f, 5.f)); T.translate(Vector3f(uni(-2, 2), uni(-2, 2), uni(-2, 2))); }
      else { for (int i = 0; i < 3; i++) for (int j = 0; j < 4; j++) T.matrix()(i, j) = uni(-2.f, 2.f); }
      memcpy(a, T.matrix().data(), 64);
      Affine3f r = T.inverse(); memcpy(&s.out[k * 16], r.matrix().data(), 64); } }
  { Section& s = add(OP_SHAPE, 4, 16);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 4];
      a[0] = (k % 7 == 0) ? 1.0f : 1.0f / uni(0.01f, 20.f);
      for (int i = 1; i < 4; i++) a[i] = (k % 11 == 0) ? 0.5f : uni(-10.f, 10.f);
      Affine3f shape = Affine3f::Identity(); shape.scale(a[0]); shape.translate(-v3(a + 1));
      Affine3f model = Affine3f::Identity(); Affine3f r = model * shape;
      memcpy(&s.out[k * 16], r.matrix().data(), 64); } }
  { Section& s = add(OP_OFFSET_001, 6, 3);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 6]; for (int i = 0; i < 6; i++) a[i] = uni(-1.5f, 1.5f);
      Vector3f p = v3(a), r = v3(a + 3); Vector3f o = p + (0.001 * r); memcpy(&s.out[k * 3], o.data(), 12); } }
  { Section& s = add(OP_OFFSET_003, 6, 3);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 6]; for (int i = 0; i < 6; i++) a[i] = uni(-1.5f, 1.5f);
      Vector3f p = v3(a), L = v3(a + 3); Vector3f o = p + 0.003 * (L); memcpy(&s.out[k * 3], o.data(), 12); } }
  { Section& s = add(OP_REFLECT, 6, 3);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 6]; for (int i = 0; i < 6; i++) a[i] = uni(-1.f, 1.f);
      Vector3f d = v3(a), n = v3(a + 3);
      Vector3f r = (d - 2 * (d.dot(n) * n)).normalized(); memcpy(&s.out[k * 3], r.data(), 12); } }
  { Section& s = add(OP_PHONG_R, 6, 3);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 6]; for (int i = 0; i < 6; i++) a[i] = uni(-1.f, 1.f);
      Vector3f L = v3(a), nn = v3(a + 3);
      Vector3f r = (L - 2 * (nn.dot(L)) * nn); memcpy(&s.out[k * 3], r.data(), 12); } }
  { Section& s = add(OP_NRM_INTERP, 13, 3);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 13]; for (int i = 0; i < 9; i++) a[i] = (k % 40 == 0) ? 0.f : wild();
      a[9] = uni(0.f, 1e-3f); a[10] = uni(0.f, 1e-3f); a[11] = uni(0.f, 1e-3f); a[12] = uni(1e-5f, 2e-3f);
      float area0 = a[9], area1 = a[10], area2 = a[11], area = a[12];
      Vector3f r = (v3(a).normalized() * area1 / area + v3(a + 3).normalized() * area2 / area +
                    v3(a + 6).normalized() * area0 / area).normalized();
      memcpy(&s.out[k * 3], r.data(), 12); } }
  { Section& s = add(OP_NORM, 3, 1);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 3]; for (int i = 0; i < 3; i++) a[i] = wild();
      s.out[k] = v3(a).norm() / 2; } }
  { Section& s = add(OP_CENTER, 16, 3);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 16];
      Affine3f V = Affine3f::Identity();
      if (k % 2 == 0) V.translate(Vector3f(uni(-3, 3), uni(-3, 3), uni(-3, 3)));
      else { V.rotate(Eigen::AngleAxisf(uni(-3.f, 3.f), Vector3f(uni(-1, 1), uni(-1, 1), uni(-1, 1)).normalized()));
             V.translate(Vector3f(uni(-3, 3), uni(-3, 3), uni(-3, 3))); }
      memcpy(a, V.matrix().data(), 64);
      Vector3f c = V.linear().inverse() * (-V.translation()); memcpy(&s.out[k * 3], c.data(), 12); } }
  { // screenToWorld: in = view[16], raster x, y, viewport[4], fovy, aspect  (23 floats)
    Section& s = add(OP_SCREEN, 24, 3);
    for (int k = 0; k < N; k++) { float* a = &s.in[k * 24];
      Affine3f V = Affine3f::Identity();
      if (k % 2 == 1) V.rotate(Eigen::AngleAxisf(uni(-3.f, 3.f), Vector3f(uni(-1, 1), uni(-1, 1), uni(-1, 1)).normalized()));
      V.translate(Vector3f(uni(-1, 1), uni(-1, 1), uni(-4, 0)));
      memcpy(a, V.matrix().data(), 64);
      float W = (float)std::uniform_int_distribution<int>(1, 4096)(rng);
      float H = (float)std::uniform_int_distribution<int>(1, 4096)(rng);
      a[16] = (float)std::uniform_int_distribution<int>(0, (int)W - 1)(rng);
      a[17] = (float)std::uniform_int_distribution<int>(0, (int)H - 1)(rng);
      a[18] = 0.f; a[19] = 0.f; a[20] = W; a[21] = H;
      a[22] = (k % 3 == 0) ? 60.0f : uni(10.f, 120.f);
      a[23] = W / (float)H;
      Eigen::Vector4f viewport(a[18], a[19], a[20], a[21]);
      float fovy = a[22], aspect_ratio = a[23];
      Eigen::Vector2f raster(a[16], a[17]);
      Vector3f norm_coords = Vector3f(2.0 * (raster[0] - viewport[0]) / viewport[2] - 1.0,
                                      1.0 - 2.0 * (raster[1] - viewport[1]) / viewport[3], -1.0);
      float persp = (float)1.0f / tan((fovy / 2.0f) * (M_PI / 180.0f));
      float scale = 1.0 / persp;
      norm_coords[0] *= aspect_ratio * scale;
      norm_coords[1] *= scale;
      Vector3f w = V.inverse() * norm_coords;
      memcpy(&s.out[k * 3], w.data(), 12); } }

  FILE* f = fopen(path, "wb");
  if (!f) { perror(path); return 1; }
  const uint32_t magic = 0x4B54414Bu; // "KATK"
  const uint32_t count = (uint32_t)secs.size();
  fwrite(&magic, 4, 1, f); fwrite(&count, 4, 1, f);
  for (auto& s : secs) {
    int32_t hdr[4] = {s.op, s.n, s.in_len, s.out_len};
    fwrite(hdr, 4, 4, f);
    fwrite(s.in.data(), 4, s.in.size(), f);
    fwrite(s.out.data(), 4, s.out.size(), f);
  }
  fclose(f);
  printf("wrote %zu sections x %d cases to %s\n", secs.size(), N, path);
  return 0;
}
