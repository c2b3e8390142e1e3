// tucano_kat.cpp -- TEST INFRASTRUCTURE (oracle pinning), never shipped or linked by the product.
//
// Known answers for the camera and model-matrix expressions of the reference path, computed by the
// reference's OWN Tucano code, compiled here unmodified from
// /root/reference/dependencies/tucano (+ its vendored Eigen and GLEW headers):
//   CENTER  Tucano::Camera::getCenter            tucano/camera.hpp:115-118
//   SCREEN  Tucano::Camera::screenToWorld        tucano/camera.hpp:155-173 (+ setViewport :302-305,
//           setPerspectiveMatrix :433-448 for fovy / aspect ratio, getPerspectiveScale :263-266)
//   SHAPE   Tucano::Model::normalizeModelMatrix  tucano/model.hpp:169-173, getShapeModelMatrix :102-105
// The inputs are those of the same sections of tests/golden/eigen_kat.bin (oracle/eigen_kat.cpp); the
// outputs are written to tests/golden/tucano_kat.bin in the same format, and the tests hold the oracle,
// the product's host math and its gfx950 kernels to them (tests/test_oracle_pinning.py).
//
// Only the protected state those members read is set, through thin subclasses (view_matrix for the
// camera; objectCenter / normalization_scale, which Tucano::Mesh fills when loading, for the model):
// every computed value comes from the reference's member functions. Not covered: Tucano::Flycamera
// (flycamera.hpp) -- its CoordinateAxes member draws with OpenGL, so the class cannot be constructed
// without a GL context; rt_camera_flycam restates its translate / updateViewMatrix.
//
// Build (oracle/Makefile target tucano_kat, only where /root/reference exists): g++ against the vendored
// headers, GLEW_NO_GLU (GLEW's own switch: no GLU header is in this image), no GL library linked -- the
// link fails on any undefined symbol, so none of the GL-bound code is instantiated.
#include <tucano/camera.hpp>
#include <tucano/model.hpp>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

namespace {

enum { OP_SHAPE = 8, OP_CENTER = 15, OP_SCREEN = 16 };  // eigen_kat.cpp op codes

struct KatCamera : Tucano::Camera {
  void set_view(const float* m16) { std::memcpy(view_matrix.matrix().data(), m16, 64); }
};

struct KatModel : Tucano::Model {
  void set_shape(float scale, const float* center) {
    normalization_scale = scale;
    objectCenter = Eigen::Vector3f(center[0], center[1], center[2]);
  }
};

struct Section {
  int32_t op, n, in_len, out_len;
  std::vector<float> in, out;
};

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: tucano_kat <eigen_kat.bin> <tucano_kat.bin>\n");
    return 2;
  }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) { std::perror(argv[1]); return 1; }
  uint32_t magic = 0, count = 0;
  if (std::fread(&magic, 4, 1, f) != 1 || std::fread(&count, 4, 1, f) != 1 || magic != 0x4B54414Bu) {
    std::fprintf(stderr, "%s: not a KAT file\n", argv[1]);
    return 1;
  }
  std::vector<Section> out;
  int differ = 0;
  for (uint32_t s = 0; s < count; s++) {
    Section sec;
    if (std::fread(&sec.op, 4, 4, f) != 4) return 1;
    sec.in.resize((size_t)sec.n * sec.in_len);
    sec.out.resize((size_t)sec.n * sec.out_len);
    if (std::fread(sec.in.data(), 4, sec.in.size(), f) != sec.in.size()) return 1;
    if (std::fread(sec.out.data(), 4, sec.out.size(), f) != sec.out.size()) return 1;
    if (sec.op != OP_SHAPE && sec.op != OP_CENTER && sec.op != OP_SCREEN) continue;
    std::vector<float> ref(sec.out.size());
    for (int k = 0; k < sec.n; k++) {
      const float* a = &sec.in[(size_t)k * sec.in_len];
      float* o = &ref[(size_t)k * sec.out_len];
      if (sec.op == OP_CENTER) {
        KatCamera cam;
        cam.set_view(a);
        const Eigen::Vector3f c = cam.getCenter();
        std::memcpy(o, c.data(), 12);
      } else if (sec.op == OP_SCREEN) {
        // in: view[16], raster x, y, viewport[4], fovy, aspect (eigen_kat.cpp OP_SCREEN)
        KatCamera cam;
        cam.set_view(a);
        cam.setViewport(Eigen::Vector4f(a[18], a[19], a[20], a[21]));
        cam.setPerspectiveMatrix(a[22], a[23], 0.1f, 100.0f);
        const Eigen::Vector3f w = cam.screenToWorld(Eigen::Vector2f(a[16], a[17]));
        std::memcpy(o, w.data(), 12);
      } else {
        // in: normalization scale, object centre (eigen_kat.cpp OP_SHAPE); model matrix identity
        KatModel m;
        m.set_shape(a[0], a + 1);
        m.normalizeModelMatrix();
        const Eigen::Affine3f sm = m.getShapeModelMatrix();
        std::memcpy(o, sm.matrix().data(), 64);
      }
    }
    for (size_t i = 0; i < ref.size(); i++) {
      uint32_t x, y;
      std::memcpy(&x, &ref[i], 4);
      std::memcpy(&y, &sec.out[i], 4);
      differ += x != y;
    }
    sec.out = ref;
    out.push_back(std::move(sec));
  }
  std::fclose(f);
  FILE* g = std::fopen(argv[2], "wb");
  if (!g) { std::perror(argv[2]); return 1; }
  const uint32_t n = (uint32_t)out.size();
  std::fwrite(&magic, 4, 1, g);
  std::fwrite(&n, 4, 1, g);
  for (const Section& s : out) {
    std::fwrite(&s.op, 4, 4, g);
    std::fwrite(s.in.data(), 4, s.in.size(), g);
    std::fwrite(s.out.data(), 4, s.out.size(), g);
  }
  std::fclose(g);
  std::printf("wrote %u sections (CENTER, SCREEN, SHAPE) to %s; %d values differ from %s\n", n, argv[2], differ, argv[1]);
  return 0;
}
