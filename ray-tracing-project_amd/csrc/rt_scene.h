// rt_scene.h -- internal definitions of rt_mesh / rt_scene (host + device halves).
#pragma once
#include <chrono>
#include <cstdio>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rt/rt_api.h"
#include "rt_internal.h"

struct rt_mesh {
  std::vector<float> v4;       // [nv][4]
  std::vector<float> vn3;      // [nv][3]
  std::vector<uint32_t> fidx;  // [nf][3]
  std::vector<float> fn3;      // [nf][3]
  std::vector<int32_t> fmat;   // [nf]
  std::vector<rt_material> mats;
  std::vector<std::string> mat_names;
  float scale = 1.0f, center[3] = {0, 0, 0};
  float M[16];
};

namespace rt {

struct RefBox {
  float low[3], high[3], shape[3];
  bool failed[3] = {false, false, false};
  std::vector<int32_t> faces;
};

// One node of the fp32 4-wide tree before upload (device_upload lays out the eight octant copies)
struct Wide4 {
  float box[4][6];       // child boxes (lo.x hi.x lo.y hi.y lo.z hi.z), copied from the BVH2 node records
  uint32_t child[4];     // wide-node index (interior) or leaf handle; slots >= n unused
  uint8_t n;             // children (2..4; 1 only for a single-leaf root)
  uint8_t order[8][4];   // per direction octant: child slots near to far
};

struct HostScene {
  int32_t nv = 0, nf = 0;
  std::vector<f3> wv;        // world vertices  (M * v)
  std::vector<float> ov3;    // object-space vertices [nv][3] (Mesh::getVertex, BoundingBox::hasFace)
  std::vector<f3> vnn;       // normalised vertex normals
  std::vector<f3> fnn;       // normalised face normals
  std::vector<float> fdist;  // facenormal.dot(vert0)
  // Accept-region vertices [nf][3]: where a face normal is tilted against its world triangle (a rotating
  // or non-uniformly scaling model matrix: the reference keeps object-space normals), the hit points the
  // edge tests accept lie on the triangle projected along that normal onto its plane, not on the world
  // triangle; the builders bound those (accept_region). Empty when every face is untilted.
  std::vector<f3> av;
  std::vector<uint32_t> fidx;
  std::vector<int32_t> fmat;
  std::vector<rt_material> mats;
  float M[16], Minv[16], MS[9];
  std::vector<RefBox> boxes;
  std::vector<uint32_t> face_rank, face_box;
  // BVH
  std::vector<Node64> nodes;
  std::vector<Node4Q> nodes4;  // 4-wide collapse of `nodes`, quantised boxes (A/B variant)
  std::vector<Wide4> wide;     // 4-wide collapse of `nodes`, fp32 boxes (default PRIMARY tree); root = 0
  int32_t depth_wide = 0;
  std::vector<TriRec64> tris;  // leaf order
  uint32_t root = 0;
  int32_t depth = 0, leaves = 0, depth4 = 0;
};

void build_ref_boxes(HostScene& hs, const float* v4, int32_t min_faces, int32_t max_boxes);
// the same partition on the GPU (rt_boxes.hip); *nonfinite: some vertex coordinate is not finite and
// nothing was built (the caller uses the host builder)
int gpu_build_ref_boxes(int device, HostScene& hs, const float* v4, int32_t min_faces, int32_t max_boxes,
                        double* gpu_ms, bool* nonfinite);
// face_rank / face_box from hs.boxes (boxes in creation order, faces in in-box order)
void assign_box_ranks(HostScene& hs);
void build_bvh(HostScene& hs, int leaf_size, bool spatial);  // spatial: SBVH (RT_BUILDER_SBVH)
bool build_bvh_gpu(HostScene& hs, int device, int leaf_size, double* gpu_ms);
bool build_bvh_ploc(HostScene& hs, int device, int leaf_size, double* gpu_ms);
int gpu_build_ploc(int device, const std::vector<TriRec64>& face_recs, const float lo[3], const float hi[3],
                   int leaf_size, int radius, float k_trav, std::vector<int32_t>& child2, std::vector<float>& box6,
                   std::vector<uint8_t>& leaf, double* gpu_ms, int* iterations, int rule);
int gpu_build_sah(int device, const std::vector<TriRec64>& face_recs, const float lo[3], const float hi[3],
                  int leaf_size, float k_trav, bool spatial, float budget, float alpha, std::vector<uint32_t>& nchild,
                  std::vector<float>& ncb, std::vector<uint32_t>& slot_face, double* gpu_ms, int* levels);
bool build_bvh_sah_gpu(HostScene& hs, int device, int leaf_size, bool spatial, double* gpu_ms);
int gpu_build_lbvh(int device, const std::vector<TriRec64>& face_recs, const float lo[3], const float hi[3],
                   int leaf_size, float pad, std::vector<Node64>& nodes, std::vector<TriRec64>& tris, double* gpu_ms);
// [0, n) in contiguous chunks on up to 16 host threads: f(begin, end) (rt_host.cpp)
void parallel_for(size_t n, const std::function<void(size_t, size_t)>& f);
// the device's scene-construction stream (rt_device.hip; created once, never destroyed)
void* build_stream(int device);  // a hipStream_t
// first-use initialisation of the device (its build stream, a first allocation); thread-safe (rt_device.hip)
void device_warmup(int device);
// host <-> device copies of large pageable buffers through pinned staging (rt_device.hip)
int h2d(void* dst, const void* src, size_t bytes);
int d2h(void* dst, const void* src, size_t bytes);
void build_bvh4(HostScene& hs);
void build_wide(HostScene& hs);
float bvh_pad(const float lo[3], const float hi[3]);
// fills hs.av (see HostScene::av) from wv / fnn / fdist; leaves it empty when no face needs it
void accept_region(HostScene& hs);
// vertex j of the triangle the culling boxes must bound for face f
inline const f3& bound_vert(const HostScene& hs, uint32_t f, int j) {
  return hs.av.empty() ? hs.wv[hs.fidx[3 * (size_t)f + j]] : hs.av[3 * (size_t)f + j];
}
float scene_static_pad(const HostScene& hs);
float cert_origin_max(const HostScene& hs);
uint32_t tri_flags(const HostScene& hs, uint32_t f, float Ro);  // kSafeNormalBit | kBoxCertBit of face f
void set_error(const char* fmt, ...);
// Diagnostic / A/B environment knobs (RT_KERNEL_VARIANT, RT_SPLIT_K, RT_SPLIT_KP, RT_SPLIT_KP_ANY, RT_XCD_RUN, RT_LDS_PAD, RT_LPT_REFRESH, RT_LPT_MOVED, RT_LPT_DILATE, RT_LPT_PRED, RT_LPT_DILW, RT_ASM_DEVICE, RT_SLOT_POOL, RT_HWQ_GPU_CAP, RT_SAH_TRAV,
// RT_SBVH_BUDGET, RT_NODE_LAYOUT, RT_PLOC_RADIUS, RT_PLOC_TRAV, RT_PLOC_RULE, RT_TIMING): getenv(name) once rt_debug_env_knobs(1) has been called,
// else nullptr -- the product library's behaviour never depends on the caller's environment otherwise.
const char* debug_env(const char* name);
void set_debug_env(bool on);
// RT_TIMING phase log (debug knobs only): mark(name) prints the ms since the previous mark (or construction)
struct PhaseTimer {
  const char* scope;
  bool on;
  std::chrono::steady_clock::time_point t;
  explicit PhaseTimer(const char* sc) : scope(sc), on(debug_env("RT_TIMING") != nullptr), t(std::chrono::steady_clock::now()) {}
  void mark(const char* name) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    fprintf(stderr, "[rt] %s/%s %.1f ms\n", scope, name, std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
};

}  // namespace rt

namespace rt {
struct EnqueueWorker;  // rt_device.hip: a host thread that queues one replica's share of each frame
}

struct rt_scene {
  rt_scene_opts opts;
  // the host scene; shared with the scene's device replicas (one HostScene per rt_scene_create)
  std::shared_ptr<rt::HostScene> hsp;
  rt::HostScene& hs;
  rt_scene() : hsp(std::make_shared<rt::HostScene>()), hs(*hsp) {}
  explicit rt_scene(std::shared_ptr<rt::HostScene> shared) : hsp(std::move(shared)), hs(*hsp) {}
  ~rt_scene();  // releases the replicas and this scene's device state (rt_device.hip)
  rt_scene(const rt_scene&) = delete;
  rt_scene& operator=(const rt_scene&) = delete;
  // Multi-device scenes (rt_scene_opts.n_devices > 1): this scene is device 0's replica; replicas[k - 1]
  // renders on opts.devices[k] with its own copy of the device data (peer copies of this scene's buffers)
  // and its own frame slots. A frame's tiles are split over the replicas as shards (rt_device.hip
  // render_multi); each replica packs its tiles and copies them into pinned host memory for assembly.
  std::vector<std::unique_ptr<rt_scene>> replicas;
  bool is_replica = false;  // a replica of another scene (its box colours are set through that scene only)
  // one enqueue worker per replica of replicas (started at the first multi-device frame, stopped before the
  // replicas are released): each replica's launches of a frame are queued by its own host thread
  std::vector<std::shared_ptr<rt::EnqueueWorker>> workers;
  struct Assembly {
    void* d_pack = nullptr;  // device: this replica's tiles of the last frame, packed (rt_device.hip)
    void* h_pack = nullptr;  // pinned host copy of it
    size_t bytes = 0;        // capacity of both
  } asm_buf;
  // Device-side assembly of a multi-device scene's frame (rt_device.hip assemble_device; this scene = device 0):
  // every replica's packed tiles land in d_gather (peer copies over xGMI), one kernel places them into d_frame,
  // and one pinned copy brings the frame to the host
  struct DevAssembly {
    void* d_gather = nullptr;  // device 0: the replicas' packed slices, one after the other
    size_t gather_bytes = 0;
    void* d_frame = nullptr;   // device 0: the assembled frame (+16 B: the 8-bit frame's exactness flag)
    size_t frame_bytes = 0;
    void* h_frame = nullptr;   // pinned host copy of d_frame
    size_t h_bytes = 0;
    static constexpr int kChunks = 8;
    void* ev_chunk[kChunks] = {};  // device 0: the device-to-host copy of each chunk has landed
  } dasm;
  void* asm_ev = nullptr;  // this replica's packed slice has reached device 0 (an event of this replica's device)
  std::vector<rt_stats> last_device_stats;  // per replica, from the last rt_synchronize of a multi-device scene
  // device buffer sizes (peer replication copies these)
  size_t nodes_bytes = 0, nodes4_bytes = 0, fshade_bytes = 0, refbox_bytes = 0, mats_bytes = 0;
  double replicate_ms = 0.0;
  double build_ms = 0.0, prep_ms = 0.0, boxes_ms = 0.0, bvh_ms = 0.0, upload_ms = 0.0, bvh_gpu_ms = 0.0, boxes_gpu_ms = 0.0;
  int32_t box_builder_used = 0;
  int32_t builder_used = 0;
  int32_t device = RT_DEVICE_NONE;
  // device state (rt_device.hip)
  void* stream = nullptr;        // = slots[0].stream (ray-list queries, uploads)
  std::vector<void*> ev_pool;   // event pairs, one per render launch since the last synchronize
  size_t ev_used = 0;
  rt::Node64* d_nodes = nullptr;
  rt::Node4Q* d_nodes4 = nullptr;
  rt::TriRec64* d_tris = nullptr;
  uint32_t wide_base = 0, wide_copy_bytes = 0;  // fp32 4-wide tree in d_nodes (DevScene), 0: none
  float static_pad = 0.0f;  // the pad every BVH box carries (DevScene::static_pad)
  float cert_origin_max = 0.0f;  // DevScene::cert_origin_max (cert_origin_max(hs))
  float* d_fshade = nullptr;  // per-face shading record: three unit vertex normals + material (float4 x 3)
  float* d_refbox = nullptr;
  // RT_MODE_BOX_COLORS: the boxes' colours and, per face id, the sum of the colours of the boxes that
  // hasFace() it (float4; computed on the device when the colours changed)
  std::vector<float> box_colors;  // [n_boxes][3]; empty = not set yet
  float* d_face_boxcolor = nullptr;
  bool face_boxcolor_valid = false;
  rt::DevMat* d_mats = nullptr;
  unsigned long long* d_stats = nullptr;
  uint32_t* d_pf_check = nullptr;  // RT_CHECK_PREFETCH debug build: out-of-range prefetch sites (DevScene::pf_check)
  int64_t device_bytes = 0;
  // frames in flight: each slot has its own stream and frame buffers (grown on demand)
  struct FrameSlot {
    void* stream = nullptr;
    bool dedicated_queue = false;  // the stream has a hardware queue of its own (rt_device.hip slot_stream)
    float* d_rgb = nullptr;
    int32_t* d_face = nullptr;
    float* d_t = nullptr;
    uint2* d_hits = nullptr;
    size_t fb_pixels = 0;
    uint8_t* d_rgb8 = nullptr;  // 8-bit output frame (+ a 4-byte anomaly flag after it)
    size_t rgb8_pixels = 0;
    void* d_full = nullptr;  // FULL stage-pipeline hand-off buffers
    size_t full_pixels = 0;
    void* last_done = nullptr;  // event after this slot's latest frame (since the last synchronize)
    uint32_t* d_queue = nullptr;  // persistent-threads variant: 8 per-XCD work counters
    uint32_t* d_timeline = nullptr;  // RT_FRAME_TIMELINE records (8 words per wave)
    size_t timeline_waves = 0;
    uint32_t* d_wave_stats = nullptr;  // RT_FRAME_WAVE_STATS records (8 words per logical wave)
    size_t wave_stats_waves = 0;
  };
  // Longest-first dispatch of lone frames (rt_device.hip render_one): the per-wave costs of a recording frame
  // and the order k_order_lpt computed from them, valid for frames with the same key. One map per scene, not
  // per frame slot: only a frame alone on the GPU reads or writes it, and such a frame is queued after every
  // earlier frame (and its sort) has finished, so consecutive lone frames share it whatever slot they take
  // (round 6: per-slot maps made synchronous frames of a 4-slot scene use a map recorded 4-32 frames earlier).
  struct LptMap {
    uint32_t* d_cost = nullptr;
    uint32_t* d_order = nullptr;
    size_t waves = 0;
    int64_t key[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    bool valid = false;     // d_order holds an order for frames of key
    int age = 0;            // lone frames dispatched with that order since it was computed
    float view[16] = {0};   // the camera of the frame whose costs made the order
    float prev_view[16] = {0};  // the camera of the scene's previous lone frame (motion test)
    uint32_t* d_cost_dil = nullptr;  // a moving camera's costs dilated over neighbouring waves (FrameParams::cost_dil)
    bool dilated_map = false;        // the order was sorted from dilated costs
    int64_t sorts = 0, frames = 0, dilated = 0;  // lone frames dispatched longest-first / that re-sorted / dilated
  } lpt;
  static constexpr int kMaxSlots = 4;
  FrameSlot slots[kMaxSlots];
  int n_slots = 1, next_slot = 0, last_slot = 0;
  uint32_t band_rot = 0;  // frames in flight: rotation of the XCDs' frame bands (FrameParams::xcd_rot)
  int32_t last_W = 0, last_H = 0, last_flags = 0, last_shard_index = 0, last_shard_count = 1;
  int64_t last_rays = 0, last_total_rays = 0;
  int64_t rays_key[4] = {-1, -1, -1, -1}, rays_of_key = 0;  // primary rays of a frame shape (W, H, shard)
  int64_t last_timeline_waves = 0;  // waves recorded by the last RT_FRAME_TIMELINE frame
  int64_t last_wave_stats_waves = 0;  // logical waves of the last RT_FRAME_WAVE_STATS frame
  bool pending = false;
};

namespace rt {
int device_upload(rt_scene* s);
// Multi-device scenes: validates opts.n_devices / opts.devices (RT_DEVICES_ALL -> every visible device)
// and writes the resolved list; n_devices 0 or 1 means a single-device scene (rt_device.hip)
int resolve_devices(rt_scene_opts& o);
// after device_upload of s (device opts.devices[0]): one replica per further listed device, its device
// data peer-copied from s's (rt_device.hip)
int device_replicate(rt_scene* s);
int current_device();  // -1 without a GPU
void device_release(rt_scene* s);
}  // namespace rt
