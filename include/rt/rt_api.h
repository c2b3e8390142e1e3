/* rt_api.h -- C ABI of the MI355X-native ray-traversal library (librtamd.so).
 *
 * Drop-in boundary for the reference's CPU render path (plindhorst/Ray-Tracing-Project):
 *   Flyscene::raytraceScene(int width, int height)      src/flyscene.hpp:65, src/flyscene.cpp:250-297
 *     -> traceRayThread (ray generation)                 src/flyscene.cpp:299-314
 *     -> traceRay / calculateMinimumFace / shadow / calculateColor   src/flyscene.cpp:317-614
 * The GL-free Flyscene mirror (ray-tracing-project_amd/host/flyscene.hpp) keeps initialize(w,h) and
 * raytraceScene(w,h) and calls rt_render() for the whole frame, then writes result.ppm with
 * rt_write_ppm() (= Tucano::ImageImporter::writePPMImage, tucano/utils/ppmIO.hpp:135-156).
 *
 * Conventions: plain C types only; every call returns 0 (RT_OK) or a negative rt_status; the message
 * of the last failure on the calling thread is rt_last_error(). No exceptions cross the ABI. A scene
 * handle is used from one host thread at a time. The caller owns every input array and output buffer;
 * the library copies the scene to the device at rt_scene_create(). There is no CPU fallback: every
 * render/trace entry point runs the gfx950 kernels and fails with RT_ERR_NO_DEVICE without a GPU.
 */
#ifndef RT_API_H
#define RT_API_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_API_VERSION 4  /* 4: multi-device scenes (rt_scene_opts.n_devices/devices, rt_synchronize_devices);
                             3: rt_stats.wave_node_bytes, RT_BUILDER_SBVH */

typedef enum rt_status {
  RT_OK = 0,
  RT_ERR_INVALID = -1,   /* bad argument / malformed input */
  RT_ERR_IO = -2,        /* file could not be opened / written */
  RT_ERR_NOMEM = -3,     /* host or device allocation failed */
  RT_ERR_HIP = -4,       /* HIP runtime error (message in rt_last_error) */
  RT_ERR_NO_DEVICE = -5, /* no GPU, or the scene was created host-only */
  RT_ERR_UNSUPPORTED = -6
} rt_status;

/* Tucano::Material::Mtl fields the ray tracer reads (tucano/materials/mtl.hpp:22-40) */
typedef struct rt_material {
  float ka[3], kd[3], ks[3];
  float shininess;        /* Ns */
  float optical_density;  /* Ni */
  float dissolve;         /* d  */
} rt_material;

/* ---------------------------------------------------------------------------------------------
 * Host-side scene ingest with Tucano semantics (no GPU needed)
 * ------------------------------------------------------------------------------------------- */
typedef struct rt_mesh rt_mesh;

/* Tucano::MeshImporter::loadObjFile (tucano/utils/objimporter.hpp:117-351) + Mesh::normalizeModelMatrix
 * (tucano/model.hpp:169-173), as Flyscene::initialize does (src/flyscene.cpp:18-22). */
int rt_mesh_load_obj(const char* path, rt_mesh** out);
/* Same ingest from memory: v3 [nv][3]; vn3 [nv][3] or NULL (then normals are computed as
 * computeNormals, objimporter.hpp:81-106); index groups as usemtl groups (group_index_counts are
 * index counts, multiples of 3); materials [n_materials]. */
int rt_mesh_from_arrays(int32_t n_vertices, const float* v3, const float* vn3, int32_t n_groups,
                        const int32_t* group_index_counts, const uint32_t* indices,
                        const int32_t* group_material, int32_t n_materials,
                        const rt_material* materials, rt_mesh** out);
void rt_mesh_destroy(rt_mesh* m);

/* Borrowed view of a prepared mesh, in the layout Flyscene holds after initialize(). */
typedef struct rt_mesh_desc {
  int32_t n_vertices;
  const float* vertices;            /* [n_vertices][4] object space, w = 1 (Mesh::vertices, mesh.hpp:292) */
  const float* vertex_normals;      /* [n_vertices][3] (Mesh::normals, mesh.hpp:293)              */
  int32_t n_faces;
  const uint32_t* face_vertex_ids;  /* [n_faces][3] (Face::vertex_ids, mesh.hpp:242)              */
  const float* face_normals;        /* [n_faces][3] (Face::normal, mesh.hpp:245; createFaces :475-477) */
  const int32_t* face_material_ids; /* [n_faces] (Face::material_id), -1 = none                   */
  int32_t n_materials;
  const rt_material* materials;     /* Flyscene::materials (flyscene.hpp:151)                     */
  float shape_model_matrix[16];     /* Mesh::getShapeModelMatrix(), column-major (model.hpp:102-105) */
} rt_mesh_desc;

int rt_mesh_get_desc(const rt_mesh* m, rt_mesh_desc* out);

/* Deterministic synthetic triangle soup used by the C3/C4 workloads: n_tris triangles, unshared
 * vertices v3_out [3*n_tris][3]; SplitMix64(seed); centres U[-0.5,0.5)^3, vertex jitter U[-0.01,0.01)^3. */
void rt_generate_soup(int32_t n_tris, uint64_t seed, float* v3_out);

/* Tucano::ImageImporter::writePPMImage (tucano/utils/ppmIO.hpp:135-156): P3, row 0 first,
 * min(255, (int)(255*c)). rgb is [H][W][3]. */
int rt_write_ppm(const char* path, const float* rgb, int32_t width, int32_t height);
/* The same P3 text from 8-bit values (rt_frame_download_rgb8); byte-identical to rt_write_ppm whenever
 * that download reported exact = 1. */
int rt_write_ppm_rgb8(const char* path, const uint8_t* rgb8, int32_t width, int32_t height);

/* ---------------------------------------------------------------------------------------------
 * Scene (device-resident acceleration structure)
 * ------------------------------------------------------------------------------------------- */
#define RT_DEVICE_NONE (-2) /* host-only scene: preparation + inspection, no upload, no rendering */

typedef struct rt_scene_opts {
  int32_t device;         /* HIP device ordinal; -1 = current device; RT_DEVICE_NONE = host only */
  int32_t min_faces;      /* Flyscene::MIN_FACES (flyscene.hpp:168), default 300 */
  int32_t max_boxes;      /* Flyscene::MAX_BOXES (flyscene.hpp:169), default INT32_MAX */
  int32_t leaf_size;      /* BVH leaf size bound (1..16), 0 = default (4 for SAH, 1 for the GPU LBVH) */
  rt_material default_material; /* Flyscene::ka/kd/ks/shininess defaults (flyscene.hpp:179-184) */
  float background[3];    /* Flyscene::BACKGROUND_COLOR (flyscene.hpp:175) */
  int32_t frames_in_flight; /* rt_render_async frames that may execute concurrently (1..4, default 4):
                             * each in-flight frame has its own stream and frame buffers; frames stay
                             * independent and rt_frame_download returns the most recent one. A frame
                             * alone on the GPU is dispatched longest-first from an earlier frame's wave
                             * costs (small scenes also split their costliest waves); results never
                             * depend on the dispatch order */
  int32_t builder;          /* the traversal tree's builder (results never depend on it):
                             * RT_BUILDER_SBVH_GPU (rt_scene_opts_default: SAH with spatial splits built on
                             * the device, 1M faces ~0.1 s of kernels; host RT_BUILDER_SBVH without a device or
                             * when the tree would be too deep), RT_BUILDER_SBVH (the same tree quality on the
                             * host; 1M faces 2-5 s), RT_BUILDER_SAH (host binned SAH without
                             * splits: ~4x faster build, ~5% slower traversal) or RT_BUILDER_LBVH_GPU
                             * (Morton/radix-sort/Karras build on the device in milliseconds;
                             * falls back to RT_BUILDER_SAH when the tree would be too deep) or
                             * RT_BUILDER_PLOC_GPU (parallel locally-ordered clustering on the
                             * device in milliseconds; same fallback) or RT_BUILDER_SAH_GPU (the host
                             * binned-SAH algorithm run top-down on the device, one level per round of
                             * launches; same fallback) or RT_BUILDER_SBVH_GPU (the same with the host
                             * SBVH's spatial splits; same fallback) */
  int32_t box_builder;      /* the reference box partition (generateBoundingBoxes): RT_BOXES_GPU (default since
                             * round 4; host-only scenes use the host builder) or RT_BOXES_HOST (parallel
                             * passes on the host); RT_BOXES_GPU (one launch per pass,
                             * one workgroup per box; identical boxes and face order; scenes with
                             * non-finite vertex coordinates use the host builder) */
  int32_t wide_tree;        /* 1: also build the fp32 4-wide tree (eight per-octant copies of 128-B nodes in
                             * HBM: ~8x the binary tree's node bytes) and walk it for PRIMARY packets whose
                             * rays share a direction octant. 0 (default): the binary tree only -- measured
                             * equal speed at a quarter of the memory. Results are
                             * identical either way (API 3) */
  /* Multi-device rendering in one process (API 4; SURVEY 8(b) b2 / 8(e) e1 -- the reference's frame
   * driver is one process, flyscene.cpp:266-289): n_devices > 1 renders every frame on the listed HIP
   * devices together. The scene is built once (on devices[0]) and replicated to every other listed
   * device by peer copy over xGMI; each frame's 16x16 tiles are split into 64x64-pixel super-tiles
   * interleaved over the devices (the rt_frame shard layout: device k of D renders shard
   * shard_index + shard_count * k of shard_count * D), each device renders on its own streams, and the
   * frame is assembled in the caller's buffer from each device's tiles (packed on the device, copied
   * through pinned host memory by a host worker per device): no collective. Entries may repeat (two
   * replicas sharing one GPU). n_devices 0 (default) or 1: one device, `device` (n_devices 1: devices[0]);
   * RT_DEVICES_ALL: every visible device. Results are bit-identical to a one-device render. Ray-list
   * queries (rt_trace_*), diagnostics and rt_frame_pack_shard_rgb8 use devices[0] only. */
  int32_t n_devices;
  int32_t devices[16];      /* RT_MAX_DEVICES */
} rt_scene_opts;

#define RT_MAX_DEVICES 16
#define RT_DEVICES_ALL (-1)

#define RT_BUILDER_SAH 0
#define RT_BUILDER_LBVH_GPU 1
#define RT_BUILDER_SBVH 2
#define RT_BUILDER_PLOC_GPU 3
#define RT_BUILDER_SAH_GPU 4
#define RT_BUILDER_SBVH_GPU 5
#define RT_BOXES_HOST 0
#define RT_BOXES_GPU 1

void rt_scene_opts_default(rt_scene_opts* o);

typedef struct rt_scene rt_scene;

/* Builds the reference's flat box partition (generateBoundingBoxes, flyscene.cpp:399-428, whose box
 * order defines closest-hit tie-breaking) and the traversal BVH, then uploads both. At most 2^25 - 1
 * faces (node and triangle records are addressed by 32-bit byte offsets); more: RT_ERR_INVALID. */
int rt_scene_create(const rt_mesh_desc* mesh, const rt_scene_opts* opts, rt_scene** out);
void rt_scene_destroy(rt_scene* s);

typedef struct rt_scene_info {
  int32_t n_faces, n_vertices, n_ref_boxes;
  int32_t bvh_nodes, bvh_leaves, bvh_depth;
  int64_t device_bytes;
  double build_ms;        /* host preparation (boxes + BVH) */
  int32_t device;         /* RT_DEVICE_NONE for host-only scenes */
  double prep_ms;         /* phases of rt_scene_create: per-vertex / per-face invariants, */
  double boxes_ms;        /* the reference box partition, */
  double bvh_ms;          /* the BVH build(s), */
  double upload_ms;       /* the device upload */
  int32_t builder;        /* the builder actually used (RT_BUILDER_*) */
  double bvh_gpu_ms;      /* device time of the LBVH kernels (RT_BUILDER_LBVH_GPU) */
  int32_t box_builder;    /* the box partition builder actually used (RT_BOXES_*) */
  double boxes_gpu_ms;    /* device time of the GPU box partition (RT_BOXES_GPU) */
  int32_t wide_nodes;     /* fp32 4-wide nodes per octant copy (0: no wide tree) (API 3) */
  int32_t wide_depth;     /* its depth */
  int32_t n_devices;      /* devices rendering the scene's frames (API 4; 1 for a single-device scene,
                             0 host-only); device_bytes sums over them */
  double replicate_ms;    /* time to replicate the device data to devices[1..] (0: one device) */
} rt_scene_info;

int rt_scene_get_info(const rt_scene* s, rt_scene_info* out);

/* Binary scene cache: rt_scene_save writes everything rt_scene_create derived from
 * the mesh (object and world vertices, unit normals, the reference box partition and its face order, the BVHs and
 * triangle records; versioned, with a content hash); rt_scene_load restores it and uploads it without
 * OBJ parsing or any build. The build parameters (min_faces, max_boxes, leaf_size) come from the file;
 * device, frames_in_flight, default_material and background from opts (NULL = defaults). A truncated,
 * corrupt or foreign file fails with RT_ERR_IO. Renders of a loaded scene equal the original's bit for
 * bit. */
int rt_scene_save(const rt_scene* s, const char* path);
int rt_scene_load(const char* path, const rt_scene_opts* opts, rt_scene** out);
/* reference boxes: bounds6 [n][6] (low xyz, high xyz, object space), counts [n], face_order [n_faces]
 * (faces in reference iteration order: box creation order, then in-box order). NULL = skip. */
int rt_scene_ref_boxes(const rt_scene* s, float* bounds6, int32_t* counts, int32_t* face_order);

/* ---------------------------------------------------------------------------------------------
 * Camera, lights, frames
 * ------------------------------------------------------------------------------------------- */
typedef struct rt_camera {
  float view_matrix[16]; /* Camera::view_matrix (Affine3f), column-major (tucano/camera.hpp) */
  float viewport[4];     /* Camera::viewport: x, y, width, height */
  float fovy;            /* degrees */
  float aspect_ratio;
} rt_camera;

/* Flycamera default pose (eye (0,0,2), tucano/utils/flycamera.hpp:76-86) after translate(dx,dy,dz)
 * and updateViewMatrix(), with Flyscene::initialize's projection (fovy 60, aspect W/H, viewport). */
void rt_camera_flycam(int32_t width, int32_t height, float dx, float dy, float dz, rt_camera* out);

typedef struct rt_light {
  float position[3]; /* point: Flyscene::lights[i].first (flyscene.hpp:132); directional: the vector the
                        reference stores as get<0>(dirLights[i]) (flyscene.hpp:135) and uses as the light
                        direction as is (calculateColor, flyscene.cpp:610-612) */
  float color[3];    /* Flyscene::lights[i].second / get<1>(dirLights[i]) */
  int32_t kind;      /* RT_LIGHT_POINT or RT_LIGHT_DIRECTIONAL */
} rt_light;

#define RT_LIGHT_POINT 0
#define RT_LIGHT_DIRECTIONAL 1
/* calculateColor sums every point light (in order), then every directional light (in order); the
 * library applies that order whatever the order of the array. */
#define RT_MAX_LIGHTS 32

/* Light helpers. The reference draws sphere jitter from the C library's rand()
 * without seeding it (flyscene.cpp:529-538); rt_rand_state reproduces glibc's rand() (TYPE_3 additive
 * feedback generator, RAND_MAX 2^31-1), so seed 1 gives the sequence of a fresh reference process. */
typedef struct rt_rand_state {
  uint32_t r[34];
  uint32_t k;
} rt_rand_state;
void rt_rand_seed(rt_rand_state* st, uint32_t seed);
int32_t rt_rand(rt_rand_state* st);
/* Flyscene::sphericalLight + addLight('s') (flyscene.cpp:212-239, 529-538): n_points jittered point lights
 * (offset (-r + rand()/(RAND_MAX/(2r))) per axis, x then y then z) each with colour/(n_points+1), then the
 * centre light with colour/(n_points+1); writes n_points + 1 lights to out and returns that count. */
int32_t rt_lights_spherical(const rt_light* centre, float radius, int32_t n_points, rt_rand_state* rng, rt_light* out);
/* addLight('d') (flyscene.cpp:242-246): the "direction" the reference stores is screenToWorld(viewport
 * centre), a point (a point used as a direction); kind = RT_LIGHT_DIRECTIONAL. */
void rt_light_directional(const rt_camera* cam, const float color[3], rt_light* out);

enum { RT_MODE_PRIMARY = 0, RT_MODE_FULL = 1, RT_MODE_BOX_COLORS = 2 };

typedef struct rt_frame {
  int32_t width, height;
  int32_t mode;        /* RT_MODE_PRIMARY: closest hit + unshadowed Phong (traceRay at depth limit 1);
                          RT_MODE_FULL: reference traceRay as-is (shadow per light + 1 reflection);
                          RT_MODE_BOX_COLORS: traceRay with RENDER_BOUNDINGBOX_COLORED_TRIANGLES set
                          (flyscene.hpp:166, flyscene.cpp:334-348): a hit pixel is the sum of the colours
                          of every reference box that hasFace() the closest face, unclamped, no shading,
                          shadows or reflection (a miss: the background); colours: rt_scene_set_box_colors */
  int32_t shard_index; /* this device renders its share of the frame's 16x16-pixel tiles: with
                          shard_count > 1 the tiles are grouped into 4x4-tile super-tiles (64x64 pixels;
                          row-major over the frame, partial at the right / bottom edges) and super-tile s
                          belongs to shard s % shard_count (an XCD's concurrent waves then trace
                          neighbouring pixels); rt_frame_shard_tiles lists them */
  int32_t shard_count; /* 1 = whole frame */
  int32_t flags;       /* RT_FRAME_* */
  int32_t max_depth;   /* traceRay's recursion limit (Flyscene::max_depth, flyscene.hpp:142; the reference
                          fixes 2): 0 = the mode's own (PRIMARY 1, FULL 2); 1..RT_MAX_TRACE_DEPTH = trace
                          that many levels (primary hit + max_depth-1 reflection bounces), with shadow rays
                          in FULL mode and without in PRIMARY mode. The FULL/2 and PRIMARY/1 cases run the
                          tuned kernels; other depths one generic kernel (same arithmetic, same bits).
                          RT_MODE_BOX_COLORS returns before any reflection, so every depth >= 1 renders
                          the same frame there (0 and 1..16 accepted, one kernel). */
} rt_frame;

#define RT_MAX_TRACE_DEPTH 16

#define RT_FRAME_WRITE_HITS 1 /* also record per-pixel face index and t (rt_frame_download) */
#define RT_FRAME_STATS 2      /* counting run: per-ray node visits / triangle tests (slower) */
#define RT_FRAME_TIMELINE 4   /* diagnostics: each wave of the render kernel records its start / end clocks
                                 and the CU it ran on (rt_debug_timeline); PRIMARY and FULL kernels */
#define RT_FRAME_WAVE_STATS 8 /* diagnostics, with RT_FRAME_STATS: each wave of the counting run also records its own
                                 counts (rt_debug_wave_stats) */

typedef struct rt_stats {
  double kernel_ms;         /* device time of the render kernels since the previous rt_synchronize,
                               summed over launches (HIP events on the scene's stream) */
  int64_t launches;         /* render launches covered by kernel_ms */
  double trace_kernel_ms;   /* part of kernel_ms spent in the traversal kernel (PRIMARY: first of the
                               two kernels of a frame; FULL: the whole single kernel) */
  int64_t primary_rays;     /* pixels traced by this call */
  int64_t total_rays;       /* primary + shadow + reflection rays issued */
  int64_t hits;             /* primary rays that hit */
  int64_t node_visits;      /* RT_FRAME_STATS: sum over rays of interior nodes whose box the ray hit */
  int64_t tri_tests;        /* RT_FRAME_STATS: sum over rays of triangle tests */
  int64_t wave_node_fetches;/* RT_FRAME_STATS: node records fetched (once per wave) */
  int64_t wave_tri_fetches; /* RT_FRAME_STATS: triangle records fetched (once per wave) */
  int64_t wave_node_bytes;  /* RT_FRAME_STATS: bytes of the node records fetched (64 per binary record,
                               128 per fp32 4-wide record; API 3) */
} rt_stats;

/* Renders the frame (this shard's tiles) on the scene's device and copies it into out_rgb
 * ([H][W][3], row 0 = top, untouched outside this shard). Synchronous. */
int rt_render(rt_scene* s, const rt_camera* cam, const rt_light* lights, int32_t n_lights,
              const rt_frame* frame, float* out_rgb, rt_stats* stats);

/* Device-resident variant for benchmarking: renders into the scene's device frame buffer and returns
 * without synchronising; rt_synchronize() waits and fills the stats of the last render. */
int rt_render_async(rt_scene* s, const rt_camera* cam, const rt_light* lights, int32_t n_lights,
                    const rt_frame* frame);
int rt_synchronize(rt_scene* s, rt_stats* stats);
/* rt_synchronize with the figures of every device of a multi-device scene (API 4): per_device[k] (k <
 * capacity, may be NULL) = device k's own stats (its kernel_ms, primary_rays, ...). In *stats (may be
 * NULL) ray counts and counters are summed over the devices and kernel_ms / trace_kernel_ms are the
 * maximum over the devices (the frames' critical path); launches are per device. Returns the number of
 * devices (>= 1) or a negative rt_status. rt_synchronize(s, st) == rt_synchronize_devices(s, st, 0, NULL). */
int rt_synchronize_devices(rt_scene* s, rt_stats* stats, int32_t capacity, rt_stats* per_device);
/* copies the last frame from the device: rgb [H][W][3]; face [H][W] (-1 miss) and t [H][W] need
 * RT_FRAME_WRITE_HITS. NULL = skip. capacity_pixels: the pixels each given buffer holds; smaller than
 * the last frame's W x H -> RT_ERR_INVALID, nothing written. */
int rt_frame_download(rt_scene* s, int64_t capacity_pixels, float* rgb, int32_t* face, float* t);
/* Output path: the last frame converted on the device to writePPMImage's 8-bit
 * values min(255, (int)(255*c)) and downloaded at 3 B/px. *exact (may be NULL) = 1 when every value
 * was in 0..255, i.e. the bytes are exactly the PPM's numbers; 0 when some colour was NaN or negative
 * (clamped to 0 here; rt_frame_download + rt_write_ppm reproduce the reference's text then).
 * capacity_pixels: pixels the buffer holds (3 bytes each), checked as in rt_frame_download. */
int rt_frame_download_rgb8(rt_scene* s, int64_t capacity_pixels, uint8_t* rgb8, int32_t* exact);

/* Multi-GPU frame assembly (f3). Each rank's slice holds the 8-bit values of its own 16x16 tiles
 * (rt_frame.shard_index/shard_count of its last frame) in shard tile order, rt_frame_shard_bytes() long
 * (equal for all ranks, so one RCCL gather / all-gather of the slices brings the frame to one GPU);
 * rt_frame_unpack_shards_rgb8 turns the concatenated slices into the H x W x 3 frame. Both pointers are
 * device memory on the scene's / the given device (e.g. torch tensors' data_ptr()); both calls return
 * after their device work is complete, and the caller orders any earlier writes to those buffers made on
 * other streams (the library's streams do not synchronise with the legacy default stream). */
int64_t rt_frame_shard_bytes(int32_t width, int32_t height, int32_t shard_count);
/* The 16x16 tiles shard shard_index of shard_count renders, in its slot order (the order of its packed
 * slice; slots of super-tile tiles outside the frame are skipped here and zero in the slice): writes the
 * first min(n, capacity) as tiles_xy [..][2] = (tile x, tile y) (NULL = count only) and returns n, the
 * shard's tile count (0 for invalid arguments). */
int32_t rt_frame_shard_tiles(int32_t width, int32_t height, int32_t shard_index, int32_t shard_count, int32_t* tiles_xy,
                             int32_t capacity);
int rt_frame_pack_shard_rgb8(rt_scene* s, void* dst_device);
int rt_frame_unpack_shards_rgb8(const void* packed_device, int32_t shard_count, int32_t width, int32_t height,
                                void* frame_device, int32_t device);

/* Box colours of RT_MODE_BOX_COLORS. The reference draws them in generateBoundingBoxes when its
 * RENDER_BOUNDINGBOX_COLORED_TRIANGLES flag is set (flyscene.cpp:422-427): BoundingBox::setRandomColor
 * per box in creation order, colour = Vector3f(rand() / (float)RAND_MAX, x3) (BoundingBox.cpp:163-165).
 * rt_box_colors_random reproduces that sequence from rng (NULL = seed 1: a fresh reference process,
 * whose first rand() calls these are) into out3 [n_boxes][3], with the constructor's arguments
 * evaluated right to left as the reference's g++ (and x86-64 MSVC) build does: each box's first
 * rand() call is its blue channel, the third its red (C++ leaves the order unspecified; pinned by
 * tests/golden/boxcolor_kat.bin from that expression compiled here). Callers of another compiler's
 * order pass their own colours to rt_scene_set_box_colors. rt_scene_set_box_colors gives the scene
 * its colours ([n_ref_boxes][3]; NULL = rt_box_colors_random(n_ref_boxes, NULL)); a scene that renders
 * RT_MODE_BOX_COLORS without them gets the NULL colours. The per-face sums are computed on the device
 * at the first box-colour frame after the colours change (one pass over faces x boxes). */
int rt_box_colors_random(int32_t n_boxes, rt_rand_state* rng, float* out3);
int rt_scene_set_box_colors(rt_scene* s, const float* colors3);

/* calculateMinimumFace (flyscene.cpp:373-396) for n rays on the device: face -1 = miss (t = +inf) */
int rt_trace_closest(rt_scene* s, int32_t n, const float* origins3, const float* dirs3, int32_t* face,
                     float* t, float* P3);
/* shadow(P, L) (flyscene.cpp:510-526) for n rays on the device: blocked 1/0 */
int rt_trace_shadow(rt_scene* s, int32_t n, const float* P3, const float* L3, int32_t* blocked);
/* calculateMinimumFace plus interpolateNormal at the hit (N [n][3], zero on a miss) */
int rt_trace_closest_normal(rt_scene* s, int32_t n, const float* o3, const float* d3, int32_t* face, float* t,
                            float* P3, float* N3);
/* traceRay(o, d, 0) (flyscene.cpp:317-371, max_depth 2 with shadows: the FULL frame's colour path) for
 * arbitrary rays: colour rgb [n][3], first-hit face (-1 miss) and t (NULL = skip). */
int rt_trace_color(rt_scene* s, int32_t n, const float* o3, const float* d3, const rt_light* lights, int32_t n_lights,
                   float* rgb3, int32_t* face, float* t);

/* createDebugRay (flyscene.cpp:129-173) without the GL cylinders: the camera ray through a
 * (float) mouse position and its reflection chain, up to max_depth segments; every segment carries the
 * first ray's traceRay colour; a miss ends the chain with a 10-unit segment. *n_out = segments written. */
typedef struct rt_ray_segment {
  float origin[3], direction[3];
  float length;
  float color[3];
} rt_ray_segment;
int rt_debug_ray(rt_scene* s, const rt_camera* cam, const rt_light* lights, int32_t n_lights, float mouse_x, float mouse_y,
                 int32_t max_depth, rt_ray_segment* out, int32_t* n_out);

/* ---------------------------------------------------------------------------------------------
 * Misc
 * ------------------------------------------------------------------------------------------- */
int rt_device_count(void);       /* 0 when no GPU is visible */
int rt_version(void);            /* RT_API_VERSION */
/* "librtamd api <N> gfx950 sources <hash>": the build's identity. rt_source_hash() is the hash alone:
 * SHA-256 (first 16 hex digits) of the product sources this library was built from (the csrc/ .hip,
 * .cpp and .h files and include/rt/rt_api.h, concatenated in sorted path order), so a record can show that
 * the binary it ran matches the tree it came from. */
const char* rt_version_string(void);
const char* rt_source_hash(void);
const char* rt_last_error(void); /* thread-local */

/* Verification hooks (tests only; never used by the render path): evaluate the Eigen-order float
 * primitives of rt_math.h on the host (rt_debug_math_host) or in a gfx950 kernel
 * (rt_debug_math_device) for n known-answer cases of op (tests/golden/eigen_kat.bin; op 17 = the
 * specular term's pow, in {x, y} -> out {pow}, checked against the host C library). */
int rt_debug_math_host(int32_t op, int32_t n, const float* in, float* out);
int rt_debug_math_device(int32_t op, int32_t n, const float* in, float* out);

/* Host-side check of the scene's acceleration structures (tests only): every triangle lies inside
 * each ancestor box of the binary tree, of the 4-wide quantised tree and of the fp32 4-wide tree (whose
 * per-octant child orders must be permutations), and every triangle record sits in exactly one leaf of
 * each. info[0..6] = binary nodes, binary depth, quantised nodes, quantised depth, triangles reached
 * (binary), triangles reached (quantised), violations (all three trees). RT_OK iff sound. */
int rt_debug_validate_bvh(const rt_scene* s, int64_t info[7]);
/* Surface-area cost of the binary tree (host data, tests and A/B only): out[0] = k_trav * (interior
 * node area sum) + (triangle-weighted leaf area sum), over the root's area -- the SAH estimate of the
 * node steps and triangle tests of a random ray; out[1] = its node term, out[2] = its triangle term,
 * out[3] = the mean leaf size. */
int rt_debug_tree_cost(const rt_scene* s, double k_trav, double out[4]);
/* Record layout of the device node allocation for a scene of n_nodes binary nodes, n_tris triangle
 * records and n_wide fp32 4-wide nodes per octant copy (host only, no device): out[0] = allocation bytes
 * (0: records exceed 4 GiB), out[1] = byte offset of the wide copies (0: the wide tree is dropped because
 * a wide record offset would reach 2^31, the leaf-handle bit). */
int rt_debug_record_layout(int64_t n_nodes, int64_t n_tris, int64_t n_wide, int64_t out[2]);
/* The accept path's shortcuts (host data, no device needed): counts[0] = triangle records, counts[1] =
 * those whose interpolated normal is certified non-zero, counts[2] = those with a reference-box
 * certificate; *cert_origin_max (may be NULL) = the object-space origin range (max norm) within which
 * certified faces skip the box predicate; face_flags (may be NULL, else n_faces entries) = per face the
 * OR of its records' flag bits (0x80000000 safe normal, 0x40000000 box certificate). */
int rt_debug_scene_flags(const rt_scene* s, int64_t counts[3], float* cert_origin_max, uint32_t* face_flags);

/* Kernel-variant override (tests and A/B measurements only; default 0 = the measured-best kernels).
 * Bits of the product library: 4 / 512 / 1536 tile orders, 8192 / 16384 FULL megakernel builds, 32768
 * PRIMARY as trace + shade kernels, 65536 the generic traceRay kernel, 131072 / 262144 / 524288
 * longest-first dispatch knobs, 2097152 PRIMARY packets on the binary tree. Bits of the variants library
 * only (make variants -> librtamd_variants.so; the product library's rt_render returns
 * RT_ERR_UNSUPPORTED for them): 1 VGPR wave stack, 2 4-wide quantised BVH (scenes of the host builders,
 * which also build that tree), 16 FULL as a stage pipeline (whole frames only: a sharded frame returns
 * RT_ERR_UNSUPPORTED) (+32/64/128 per-lane traversal in its reflection / secondary-shadow / primary-shadow
 * stages), 256 two
 * rays per lane, 2048 persistent threads (+4096 no stealing), 1048576 two packets per wave. Every
 * variant renders the same bits. Returns the previous value. */
int rt_debug_set_variant(int32_t v);
/* Diagnostics: on = 1 lets the library read its A/B and diagnostic environment knobs (RT_KERNEL_VARIANT,
 * RT_SPLIT_K, RT_SPLIT_KP, RT_SPLIT_KP_ANY, RT_TIMELINE_SPLIT, RT_XCD_RUN, RT_LDS_PAD, RT_LPT_REFRESH, RT_LPT_MOVED,
 * RT_LPT_DILATE, RT_LPT_PRED, RT_LPT_DILW, RT_ASM_DEVICE, RT_SLOT_POOL, RT_HWQ_GPU_CAP, RT_SAH_TRAV, RT_SBVH_BUDGET, RT_NODE_LAYOUT, RT_PLOC_RADIUS, RT_PLOC_TRAV, RT_PLOC_RULE, RT_TIMING); by default
 * (and after on = 0) it ignores the process environment, so a drop-in's trees, kernels and dispatch never
 * depend on it. Turning it on also takes RT_KERNEL_VARIANT as the current kernel variant. */
int rt_debug_env_knobs(int32_t on);

/* Wave timeline of the last frame rendered with RT_FRAME_TIMELINE (diagnostics): per wave, in dispatch
 * order (workgroup id), 8 words: shader-clock s_memtime at start (lo, hi) and end (lo, hi), the
 * constant 100 MHz s_memrealtime at start and end (low 32 bits), HW_ID, and XCC_ID << 28 | the logical
 * wave (tile * 4 + quarter) the block traced. *n_waves = waves of
 * that frame; capacity_waves smaller than that -> RT_ERR_INVALID. */
int rt_debug_timeline(rt_scene* s, int64_t capacity_waves, uint32_t* out8, int64_t* n_waves);

/* Raw counters of the last RT_FRAME_STATS frame (diagnostics), out[0..n): 0 node visits, 1 triangle tests,
 * 2 wave node fetches, 3 wave triangle fetches, 4 primary rays, 5 hits, 6 total rays, 7 wave stack pops,
 * 8 pops at which no lane that wanted the entry still could reach it before its closest hit (closest-hit
 * traversal only); 48..63: the FULL kernel's packet walks by phase (csrc/rt_kernels.h ST_PW .. ST_PH); entries past
 * the last counter are 0. */
int rt_debug_counters(rt_scene* s, int64_t n, int64_t* out);

/* Per-wave counts of the last frame rendered with RT_FRAME_STATS | RT_FRAME_WAVE_STATS (diagnostics), indexed by
 * logical wave (tile * 4 + quarter), 8 words each: PRIMARY node steps, triangle tests, hit lanes, 0 x 5; FULL the
 * node steps of its four packet phases (primary, shadows of the primary hits, reflection, shadows of the
 * reflection hits), then their triangle tests. *n_waves = the frame's logical waves; capacity_waves smaller than
 * that -> RT_ERR_INVALID. */
int rt_debug_wave_stats(rt_scene* s, int64_t capacity_waves, uint32_t* out8, int64_t* n_waves);

/* Longest-first dispatch of lone frames (diagnostics): out3[0] = lone frames dispatched with the scene's cost
 * map since the scene was created, out3[1] = of them, frames that re-sorted the map from their own wave costs
 * (a new frame shape, every 8th frame, or a camera moved since the map's frame), out3[2] = 1 when a valid map is
 * held. Device 0's replica for a multi-device scene. */
int rt_debug_lpt_stats(const rt_scene* s, int64_t* out3);

#ifdef __cplusplus
}
#endif
#endif /* RT_API_H */
