// flyscene.cpp -- see flyscene.hpp. Reference: src/flyscene.cpp:9-64 (initialize), :250-297
// (raytraceScene); tucano/utils/flycamera.hpp (camera); all hot-path work happens in librtamd.
#include "flyscene.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>

#include "../csrc/rt_math.h"

namespace fly {

void Flycamera::reset() {
  tv_[0] = tv_[1] = tv_[2] = 0.0f;
  updateViewMatrix();
}

void Flycamera::translate(float dx, float dy, float dz) {
  const float I9[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};  // AngleAxisf(rotation_Y_axis = 0, UnitY)
  const rt::f3 yv = rt::m3v3(I9, rt::f3{-dx, -dy, dz});
  tv_[0] = tv_[0] + yv.x * speed_;
  tv_[1] = tv_[1] + yv.y * speed_;
  tv_[2] = tv_[2] + yv.z * speed_;
}

void Flycamera::updateViewMatrix() {
  rt::identity4(view_);
  rt::translate4(view_, rt::f3{0.0f, 0.0f, -2.0f});  // default_translation
  rt::translate4(view_, rt::f3{tv_[0], tv_[1], tv_[2]});
}

rt_camera Flycamera::camera() const {
  rt_camera c;
  memcpy(c.view_matrix, view_, sizeof view_);
  memcpy(c.viewport, vp_, sizeof vp_);
  c.fovy = fovy_;
  c.aspect_ratio = aspect_;
  return c;
}

Flyscene::~Flyscene() {
  rt_scene_destroy(scene_);
  rt_mesh_destroy(mesh_);
}

void Flyscene::initialize(int width, int height, const std::string& obj_path, int device) {
  flycamera.setPerspectiveMatrix(60.0f, width / (float)height);
  flycamera.setViewport((float)width, (float)height);
  flycamera.reset();
  lights.push_back({Vec3{-0.5f, 2.0f, 3.0f}, Vec3{1.0f, 1.0f, 1.0f}});
  rt_scene_opts o;
  rt_scene_opts_default(&o);
  o.device = device;
  o.builder = builder;
  o.box_builder = box_builder;
  if (devices.size() == 1 && devices[0] == RT_DEVICES_ALL) {
    o.n_devices = RT_DEVICES_ALL;
  } else if (!devices.empty()) {
    o.n_devices = (int32_t)std::min(devices.size(), (size_t)RT_MAX_DEVICES);
    for (int32_t k = 0; k < o.n_devices; k++) o.devices[k] = devices[k];
  }
  const auto t0 = std::chrono::steady_clock::now();
  auto done = [&] { setup_s_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
  // a scene cache skips OBJ parsing and every build
  if (!cache_path.empty() && rt_scene_load(cache_path.c_str(), &o, &scene_) == RT_OK) { done(); return; }
  if (rt_mesh_load_obj(obj_path.c_str(), &mesh_) != RT_OK) {
    fprintf(stderr, "%s\n", rt_last_error());  // reference: "Cannot open", empty mesh
    return;
  }
  rt_mesh_desc d;
  rt_mesh_get_desc(mesh_, &d);
  const auto t1 = std::chrono::steady_clock::now();
  const int rc = rt_scene_create(&d, &o, &scene_);
  build_s_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
  if (rc != RT_OK) {
    fprintf(stderr, "%s\n", rt_last_error());
    return;
  }
  done();
  if (!cache_path.empty() && rt_scene_save(scene_, cache_path.c_str()) != RT_OK) fprintf(stderr, "%s\n", rt_last_error());
}

double Flyscene::raytraceScene(int width, int height) {
  if (!scene_) { fprintf(stderr, "raytraceScene: no scene\n"); return -1.0; }
  if (width == 0 || height == 0) {
    width = flycamera.viewportWidth();
    height = flycamera.viewportHeight();
  }
  flycamera.updateViewMatrix();
  rt_camera cam = flycamera.camera();
  std::vector<rt_light> ls(lights.size());
  for (size_t i = 0; i < lights.size(); i++) {
    ls[i] = rt_light{{lights[i].first.x, lights[i].first.y, lights[i].first.z},
                     {lights[i].second.x, lights[i].second.y, lights[i].second.z}};
  }
  rt_frame fr{width, height, mode, 0, 1, 0, 0};
  rt_stats st;
  printf("ray tracing ...\n");
  const auto t0 = std::chrono::steady_clock::now();
  // render, then the 8-bit frame (3 B/px over PCIe); the float frame only when some value falls outside
  // the PPM's 0..255 (NaN / negative colours), where writePPMImage's own numbers are reproduced from it
  if (rt_render(scene_, &cam, ls.data(), (int32_t)ls.size(), &fr, nullptr, &st) != RT_OK) {
    fprintf(stderr, "%s\n", rt_last_error());
    return -1.0;
  }
  std::vector<uint8_t> rgb8((size_t)width * height * 3);
  int32_t exact = 0;
  int rc = rt_frame_download_rgb8(scene_, (int64_t)width * height, rgb8.data(), &exact);
  if (rc == RT_OK && exact) {
    rc = rt_write_ppm_rgb8(output.c_str(), rgb8.data(), width, height);
  } else if (rc == RT_OK) {
    last_image.assign((size_t)width * height * 3, 0.0f);
    rc = rt_frame_download(scene_, (int64_t)width * height, last_image.data(), nullptr, nullptr);
    if (rc == RT_OK) rc = rt_write_ppm(output.c_str(), last_image.data(), width, height);
  }
  if (rc != RT_OK) fprintf(stderr, "%s\n", rt_last_error());
  const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf(" ray tracing done! \n\nTime it took to render(in seconds): %.6f (kernel %.3f ms)\n", wall, st.kernel_ms);
  return st.kernel_ms;
}

}  // namespace fly
