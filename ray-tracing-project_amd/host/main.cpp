// main.cpp -- headless stand-in for the reference's src/main.cpp key-'T' path (main.cpp:68-69):
// initialize a Flyscene, optionally move the Flycamera, ray trace, write the PPM.
//   rt_render_cli <scene.obj> [W H] [--primary] [--dz N] [--out result.ppm] [--device D] [--cache file]
//                 [--host-build] [--lbvh] [--gpu-boxes] [--box-colors] [--devices all|D0,D1,...]
// The scene is built as the library's default (rt_scene_opts_default: the SBVH and the reference box partition
// on the device, the configuration the benchmarks measure); --host-build builds the same tree and boxes on the
// host instead, --lbvh the device LBVH. The scene setup time and the builders that ran are printed.
// --devices: render every frame on several GPUs of this process (rt_scene_opts.n_devices / devices; the
// reference renders one frame in one process too, flyscene.cpp:266-289)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>
#include <vector>

#include "flyscene.hpp"

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s scene.obj [W H] [--primary] [--dz N] [--out file.ppm] [--device D] [--cache file] [--host-build] [--lbvh] [--gpu-boxes] [--box-colors] [--devices all|D0,D1,...]\n",
            argv[0]);
    return 2;
  }
  std::string obj = argv[1], out = "result.ppm", cache;
  int builder = RT_BUILDER_SBVH_GPU, box_builder = RT_BOXES_GPU;
  int W = 1000, H = 1000, device = -1, mode = RT_MODE_FULL;
  float dz = 0.0f;
  int pos = 0;
  std::vector<int> devices;  // empty: one device; {-1}: every visible device
  for (int i = 2; i < argc; i++) {
    if (!strcmp(argv[i], "--primary")) mode = RT_MODE_PRIMARY;
    else if (!strcmp(argv[i], "--box-colors")) mode = RT_MODE_BOX_COLORS;
    else if (!strcmp(argv[i], "--dz") && i + 1 < argc) dz = (float)atof(argv[++i]);
    else if (!strcmp(argv[i], "--out") && i + 1 < argc) out = argv[++i];
    else if (!strcmp(argv[i], "--device") && i + 1 < argc) device = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--cache") && i + 1 < argc) cache = argv[++i];
    else if (!strcmp(argv[i], "--lbvh")) builder = RT_BUILDER_LBVH_GPU;
    else if (!strcmp(argv[i], "--host-build")) { builder = RT_BUILDER_SBVH; box_builder = RT_BOXES_HOST; }
    else if (!strcmp(argv[i], "--gpu-boxes")) box_builder = RT_BOXES_GPU;
    else if (!strcmp(argv[i], "--devices") && i + 1 < argc) {
      const std::string list = argv[++i];
      if (list == "all") {
        devices = {RT_DEVICES_ALL};
      } else {
        for (size_t b = 0; b <= list.size();) {
          const size_t e = std::min(list.find(',', b), list.size());
          if (e > b) devices.push_back(atoi(list.substr(b, e - b).c_str()));
          b = e + 1;
        }
      }
    }
    else if (pos == 0) { W = atoi(argv[i]); pos++; }
    else if (pos == 1) { H = atoi(argv[i]); pos++; }
  }
  fly::Flyscene scene;
  scene.cache_path = cache;
  scene.builder = builder;
  scene.box_builder = box_builder;
  scene.devices = devices;
  scene.initialize(W, H, obj, device);
  rt_scene_info info;
  if (scene.sceneInfo(&info)) {
    static const char* names[] = {"sah-host", "lbvh-gpu", "sbvh-host", "ploc-gpu", "sah-gpu", "sbvh-gpu"};
    printf("scene setup: %.3f s, rt_scene_create %.3f s (%d faces; builder %s, boxes %s, %d device(s))\n",
           scene.setupSeconds(), scene.buildSeconds(), info.n_faces,
           info.builder >= 0 && info.builder <= 5 ? names[info.builder] : "?", info.box_builder == RT_BOXES_GPU ? "gpu" : "host",
           info.n_devices);
  }
  scene.mode = mode;
  scene.output = out;
  if (dz != 0.0f) scene.getCamera()->translate(0.0f, 0.0f, dz);
  return scene.raytraceScene() < 0 ? 1 : 0;
}
