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
  // what initialize() built (rt_scene_get_info of the scene) and how long it took (OBJ load + scene setup, or
  // the cache load), for the CLI's report; false before a successful initialize()
  bool sceneInfo(rt_scene_info* out) const { return scene_ && rt_scene_get_info(scene_, out) == RT_OK; }
  double setupSeconds() const { return setup_s_; }   // OBJ load + rt_scene_create (or the cache load)
  double buildSeconds() const { return build_s_; }   // rt_scene_create alone (boxes, BVH, upload)

  // light sources for ray tracing (flyscene.hpp:132)
  std::vector<std::pair<Vec3, Vec3>> lights;
  int mode = RT_MODE_FULL;               // the reference traceRay (max_depth 2, shadows); RT_MODE_BOX_COLORS =
                                         // RENDER_BOUNDINGBOX_COLORED_TRIANGLES (flyscene.hpp:166) with the
                                         // boxes' setRandomColor colours of a fresh process
  std::string output = "result.ppm";
  std::vector<float> last_image;         // [H][W][3] float frame (kept only when the 8-bit path was inexact)
  std::string cache_path;                // binary scene cache: loaded if present, written after a build
  // acceleration structures: the library default (rt_scene_opts_default), the configuration every bench number
  // is measured on -- SAH with spatial splits built on the device (RT_BUILDER_SBVH_GPU) and the reference box
  // partition on the device (RT_BOXES_GPU); RT_BUILDER_SBVH / RT_BOXES_HOST build the same tree and boxes on the
  // host (seconds for 1M faces), RT_BUILDER_SAH the host binned SAH tree (~5% slower traversal)
  int builder = RT_BUILDER_SBVH_GPU;
  int box_builder = RT_BOXES_GPU;
  std::vector<int> devices;              // several GPUs render every frame (rt_scene_opts.devices); empty: the
                                         // `device` of initialize(); {RT_DEVICES_ALL}: every visible GPU

 private:
  Flycamera flycamera;
  rt_mesh* mesh_ = nullptr;
  rt_scene* scene_ = nullptr;
  double setup_s_ = 0.0, build_s_ = 0.0;
};

}  // namespace fly
