// flyscene.hpp -- GL-free mirror of the reference's render-to-image entry point
// (src/flyscene.hpp:22-186). It keeps the reference's call shape -- initialize(w, h), getCamera(),
// the public `lights` vector and raytraceScene(w, h) writing result.ppm -- and replaces the
// 20-thread CPU traceRay loop (flyscene.cpp:250-314) with one rt_render() call on the GPU.
// Only the ray-tracing state is mirrored; the OpenGL preview, debug rays and stdin light prompts
// are out of scope.
#pragma once
#include <string>
#include <utility>
#include <vector>

#include "rt/rt_api.h"

namespace fly {

struct Vec3 {
  float x, y, z;
};

// Tucano::Flycamera subset used by the ray tracer (tucano/utils/flycamera.hpp:41-317) at zero
// rotation: translate() accumulates translation_vector exactly as the reference does.
class Flycamera {
 public:
  void reset();
  void translate(float dx, float dy, float dz);  // flycamera.hpp:196-202
  void updateViewMatrix();                       // flycamera.hpp:166-191 (rotation_X/Y = 0)
  void setPerspectiveMatrix(float fovy, float aspect) { fovy_ = fovy; aspect_ = aspect; }
  void setViewport(float w, float h) { vp_[2] = w; vp_[3] = h; }
  rt_camera camera() const;
  int viewportWidth() const { return (int)vp_[2]; }
  int viewportHeight() const { return (int)vp_[3]; }

 private:
  float tv_[3] = {0, 0, 0};
  float view_[16];
  float vp_[4] = {0, 0, 0, 0};
  float fovy_ = 60.0f, aspect_ = 1.0f;
  const float speed_ = 0.05f;
};

class Flyscene {
 public:
  Flyscene() = default;
  ~Flyscene();
  Flyscene(const Flyscene&) = delete;
  Flyscene& operator=(const Flyscene&) = delete;

  // flyscene.cpp:9-64: projection (fovy 60, aspect w/h), viewport, OBJ load + normalisation,
  // default light (-0.5, 2, 3) white, acceleration structures (reference boxes + BVH, on the GPU)
  void initialize(int width, int height, const std::string& obj_path = "resources/models/dodgeColorTest.obj",
                  int device = -1);
  // flyscene.cpp:250-297: render the current view (all W x H pixels) and write result.ppm.
  // Returns the device kernel time in milliseconds (negative on failure; message on stderr).
  double raytraceScene(int width = 0, int height = 0);

  Flycamera* getCamera() { return &flycamera; }

  // light sources for ray tracing (flyscene.hpp:132)
  std::vector<std::pair<Vec3, Vec3>> lights;
  int mode = RT_MODE_FULL;               // the reference traceRay (max_depth 2, shadows); RT_MODE_BOX_COLORS =
                                         // RENDER_BOUNDINGBOX_COLORED_TRIANGLES (flyscene.hpp:166) with the
                                         // boxes' setRandomColor colours of a fresh process
  std::string output = "result.ppm";
  std::vector<float> last_image;         // [H][W][3] float frame (kept only when the 8-bit path was inexact)
  std::string cache_path;                // binary scene cache: loaded if present, written after a build
  int builder = RT_BUILDER_SAH;          // RT_BUILDER_LBVH_GPU: build the BVH on the GPU
  int box_builder = RT_BOXES_HOST;       // RT_BOXES_GPU: build the reference box partition on the GPU
  std::vector<int> devices;              // several GPUs render every frame (rt_scene_opts.devices); empty: the
                                         // `device` of initialize(); {RT_DEVICES_ALL}: every visible GPU

 private:
  Flycamera flycamera;
  rt_mesh* mesh_ = nullptr;
  rt_scene* scene_ = nullptr;
};

}  // namespace fly
