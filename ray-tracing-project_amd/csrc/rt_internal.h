// rt_internal.h -- shared host/device data layout of the MI355X ray-traversal library.
//
// HBM layout (one copy per device; all arrays 16-byte aligned, read-only during a frame):
//   nodes    Node64[n_nodes]       BVH2 interior nodes: both children's padded AABBs + child handles
//                                  (one 64-B record = one s_load_dwordx16 per wave per visit)
//   tris     TriRec64[n_faces]     exact-test data in BVH leaf order: unit face normal, plane distance,
//                                  world vertices, reference rank / face id / reference box id
//   fshade   float4[3*n_slots]     per triangle slot (BVH leaf order): the three normalised vertex normals (interpolateNormal,
//                                  flyscene.cpp:599) + material id; read by the final hit (one 48-B gather)
//   refbox   float4[2*n_boxes]     reference flat boxes, object space (BoundingBox::low/high)
//   mats     float4[3*n_mats]      ka|Ns, kd|-, ks|- per material
// Frame buffers: rgb float[H][W][3]; optional face int32[H][W], t float[H][W]; stats counters.
#pragma once
#include <cstdint>
#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#else
struct uint2 { unsigned int x, y; };
#endif

#include "rt_math.h"

namespace rt {

constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kLeafCountShift = 27;          // 4 bits: count - 1 (1..16 triangles)
constexpr uint32_t kLeafFirstMask = (1u << 27) - 1;  // first triangle slot (< 134M)
constexpr int kMaxLeaf = 16;
// Node and triangle records are addressed by 32-bit byte offsets from one base (scalar loads with an
// SGPR offset; nodes and triangles share one allocation), so nodes + triangles < 2^26 records: with
// at most n_faces - 1 interior nodes that is n_faces < 2^25
constexpr uint32_t kMaxFaces = (1u << 25) - 1;
constexpr int kMaxDepth = 60;  // wave stack holds 64 entries; occupancy <= depth
// TriRec64::box bit 31: the triangle's interpolated normal can never be the zero vector (see
// rt_host.cpp safe_normal()), so calculateDistance's norm()==0 rejection never fires for it
constexpr uint32_t kSafeNormalBit = 0x80000000u;
// TriRec64::box bit 30: reference-box certificate (rt_host.cpp box_certified()): for a ray whose
// object-space origin lies within DevScene::cert_origin_max (max norm), every hit point the reference's
// edge tests accept on this face lies inside the face's reference box by more than the box fast path's
// margin, so intersectBox accepts and the accept path skips the box predicate
constexpr uint32_t kBoxCertBit = 0x40000000u;
constexpr uint32_t kBoxIndexMask = 0x3FFFFFFFu;  // TriRec64::box without its flag bits

// Record layout of the one node allocation: binary nodes, then triangle records (together < 4 GiB, so
// one 32-bit byte offset reaches any record; binary interior handles = node index * 64 < 2^31 since there
// are fewer interior nodes than references), then -- 128-B aligned -- the fp32 4-wide tree's eight octant
// copies. A wide interior handle is the byte offset of its record, and bit 31 marks a leaf handle
// (kLeafBit), so the wide copies are placed only if every wide record offset stays below 2^31 (ADVICE r3:
// a record at or above 2 GiB would read as a leaf); otherwise the binary tree serves alone.
// Returns the allocation's bytes (0: the records exceed 4 GiB); *wide_base = 0 when the wide tree is dropped.
inline uint64_t record_layout(uint64_t n_nodes, uint64_t n_tris, uint64_t n_wide, uint64_t* wide_base) {
  const uint64_t bytes = (n_nodes + n_tris) * 64;
  *wide_base = 0;
  if (bytes > 0xFFFFFFFFull) return 0;
  const uint64_t wb = (bytes + 127) & ~(uint64_t)127, wide_bytes = 8 * n_wide * 128;
  if (n_wide == 0 || wb + wide_bytes > (uint64_t)kLeafBit) return bytes;
  *wide_base = wb;
  return wb + wide_bytes;
}

RT_HD bool is_leaf(uint32_t h) { return (h & kLeafBit) != 0; }
RT_HD uint32_t leaf_first(uint32_t h) { return h & kLeafFirstMask; }
RT_HD uint32_t leaf_count(uint32_t h) { return ((h >> kLeafCountShift) & 15u) + 1u; }
RT_HD uint32_t make_leaf(uint32_t first, uint32_t count) {
  return kLeafBit | ((count - 1u) << kLeafCountShift) | first;
}

// Shard tiling (rt_frame.shard_index / shard_count): the frame is cut into 16x16-pixel tiles, grouped
// into S x S super-tiles (S = super); super-tile s (row-major over the frame) belongs to shard s % count,
// and shard i's L-th tile is tile k = L % S^2 (row-major) of its (L / S^2)-th super-tile. S = 1: tile t
// goes to shard t % count. Tiles of a super-tile that fall outside the frame are still enumerated (their
// pixels are inactive), so every shard has ceil(n_super / count) * S^2 slots.
constexpr int kShardSuperTile = 4;  // super-tile width (tiles) of a split frame
RT_HD int shard_super_count(int tiles_x, int tiles_y, int S) { return ((tiles_x + S - 1) / S) * ((tiles_y + S - 1) / S); }
RT_HD int shard_tile_slots(int tiles_x, int tiles_y, int S, int index, int count) {
  const int ns = shard_super_count(tiles_x, tiles_y, S);
  return ns > index ? (ns - index + count - 1) / count * S * S : 0;
}
RT_HD void shard_tile_xy(int tiles_x, int S, int index, int count, int L, int& tx, int& ty) {
  if (S <= 1) {
    const int t = index + L * count;
    tx = t % tiles_x;
    ty = t / tiles_x;
    return;
  }
  const int S2 = S * S, j = L / S2, k = L - j * S2;
  const int s = index + j * count, sx_n = (tiles_x + S - 1) / S;
  tx = (s % sx_n) * S + k % S;
  ty = (s / sx_n) * S + k / S;
}

struct alignas(16) Node64 {
  // child 0: lo.x hi.x lo.y hi.y | lo.z hi.z ; child 1: lo.x hi.x | lo.y hi.y lo.z hi.z
  float c0lx, c0hx, c0ly, c0hy;
  float c0lz, c0hz, c1lx, c1hx;
  float c1ly, c1hy, c1lz, c1hz;
  uint32_t child0, child1, pad0, pad1;
};
static_assert(sizeof(Node64) == 64, "node record must be 64 bytes");

// 4-wide node, one 64-B record: the four children's boxes quantised to 8 bits on a per-node grid
// (origin + q * 2^e per axis, rounded outward -> conservative), plus the four child handles.
struct alignas(16) Node4Q {
  float ox, oy, oz;        // grid origin
  uint8_t ex, ey, ez;      // biased exponents: cell size 2^(e-127) per axis
  uint8_t valid;           // bit c: child c present
  uint32_t qlx, qhx, qly, qhy, qlz, qhz;  // byte c = child c's low / high cell index per axis
  uint32_t child[4];       // child handles (internal node index or leaf handle)
  uint32_t pad0, pad1;
};
static_assert(sizeof(Node4Q) == 64, "wide node record must be 64 bytes");
constexpr int kStack4 = 128;  // per-wave stack entries of the 4-wide traversal (needs 3 * depth4 + 4)

// 4-wide node with exact fp32 child boxes (the default PRIMARY tree): one 128-B record, fetched per wave
// with two s_load_dwordx16. The tree is stored once per ray-direction octant (8 copies), each copy with
// every node's children in that octant's near-to-far order, so the traversal of a wave whose rays share
// an octant visits the nearest hit child next and pushes the others farthest-first without sorting.
struct alignas(128) Node128 {
  float box[4][6];     // child c: lo.x hi.x lo.y hi.y lo.z hi.z (padded BVH2 boxes); empty slot: lo +inf, hi -inf
  uint32_t child[4];   // interior: byte offset of the child's record (same copy) from the scene-record base;
                       // leaf: leaf handle; empty slot: kWideEmpty (never entered by a certified ray)
  uint32_t pf[4];      // byte offset of what the child's visit reads first (its record, or a leaf's first
                       // triangle record): scalar-cache prefetch; empty slot: this record
};
static_assert(sizeof(Node128) == 128, "wide node record must be 128 bytes");
constexpr uint32_t kWideEmpty = 0xFFFFFFFFu;  // = the traversal's pop marker: an entered empty slot pops
constexpr int kStackW = 128;  // wave stack entries of the fp32 4-wide traversal (3 per level + 4 headroom)

struct alignas(16) TriRec64 {
  float nx, ny, nz, dist;  // face.normal.normalized(), facenormal.dot(vert0)  (flyscene.cpp:450,459)
  float w0x, w0y, w0z, w1x;
  float w1y, w1z, w2x, w2y;
  float w2z;
  uint32_t rank;  // position in the reference's (box, in-box) iteration order: tie-break key
  uint32_t face;  // original mesh face index
  uint32_t box;   // reference box holding the face (intersectBox predicate) | kSafeNormalBit | kBoxCertBit
};
static_assert(sizeof(TriRec64) == 64, "triangle record must be 64 bytes");

struct alignas(16) DevMat {
  float ka[3], ns;
  float kd[3], pad0;
  float ks[3], pad1;
};

struct Light {
  float p[3], c[3];
  int32_t kind;  // RT_LIGHT_POINT / RT_LIGHT_DIRECTIONAL
};

// Device scene view (pointers stay wave-uniform: SGPRs)
struct DevScene {
  const Node64* nodes;
  const Node4Q* nodes4;
  uint32_t root4;
  int32_t n_nodes4;
  // fp32 4-wide tree (Node128), in the same allocation as `nodes`/`tris`: copy o's root record at byte
  // offset wide_base + o * wide_copy_bytes from `nodes`; wide_base == 0: no wide tree (binary traversal)
  uint32_t wide_base, wide_copy_bytes;
  float static_pad;        // the pad every BVH box carries (setup_cull adds a ray's own pad beyond it)
  const TriRec64* tris;
  const float* fshade;     // float4 x 3 per triangle slot: unit vertex normals (n0 .w = material id bits)
  const float* refbox;     // 2 float4 per box
  const DevMat* mats;
  uint32_t root;           // root handle; n_nodes == 0 -> empty scene
  int32_t n_nodes;
  float Minv[16];          // getShapeModelMatrix().inverse() (object-space hit point for the box fast path)
  float cert_origin_max;   // kBoxCertBit holds for rays whose object-space origin has max norm <= this
  // Byte ranges of the scalar prefetches (checked only in the RT_CHECK_PREFETCH debug build, `make pfcheck`):
  // node / child-prefetch offsets from `nodes` stay below rec_bytes (binary nodes + triangle records),
  // leaf-prefetch offsets from `tris` below tri_bytes, wide-tree offsets from `nodes` below all_bytes; a
  // violation sets bit <site> of *pf_check (and the load reads offset 0 instead)
  uint32_t rec_bytes, tri_bytes, all_bytes;
  uint32_t* pf_check;
};

// hit information handed between FULL stage kernels (32 B); face == 0xFFFFFFFF: no hit
struct HitState {
  float px, py, pz;
  float nx, ny, nz;
  int32_t mat;
  uint32_t face;
};
// a ray handed between stages (32 B)
struct RayRec {
  float ox, oy, oz;
  float dx, dy, dz;
  uint32_t pad0, pad1;
};

// Per-launch parameters (kernel argument, ~1 KB)
struct FrameParams {
  DevScene sc;
  float Minv[16];          // getShapeModelMatrix().inverse()  (flyscene.cpp:486)
  float MS[9];             // its linear block                  (flyscene.cpp:487)
  DevMat defmat;           // Flyscene sticky defaults (flyscene.hpp:179-182)
  float bg[3];
  // camera (reproduces Camera::screenToWorld, camera.hpp:155-173)
  float vinv[16];          // view_matrix.inverse()
  float eye[3];            // getCenter()
  float eye_obj[3];        // Minv * eye (object-space origin of every primary ray's box test)
  float vp[4];             // viewport
  float xscale, yscale;    // aspect_ratio * scale, scale
  // lights
  int32_t n_lights;
  Light lights[32];
  // frame
  int32_t W, H, tiles_x, tiles_y;  // tiles = 16x16 pixel blocks (one 256-thread block each)
  int32_t xcd_remap;
  int32_t xcd_rot;            // chunked XCD order: XCD x takes the runs of XCD x + xcd_rot (mod 8)
  int32_t shard_index, shard_count, n_tiles_shard;
  int32_t super_tile;         // S of shard_tile_xy (1: tile t -> shard t % count)
  int32_t mode, flags;
  int32_t max_depth;          // k_render_depth: traceRay's recursion limit (flyscene.hpp:142)
  int32_t shadows;            // k_render_depth: shadow() per light (FULL) or not (PRIMARY)
  float* rgb;
  int32_t* face_out;
  float* t_out;
  unsigned long long* stats;  // [8] counters (RT_FRAME_STATS)
  uint2* hits;                // [H][W] (t bits, triangle slot): PRIMARY trace -> shade hand-off
  // FULL as a wavefront pipeline (per-pixel hand-off records between the stage kernels)
  HitState* state0;           // [H][W] primary hit point / normal / material
  HitState* state1;           // [H][W] reflection hit
  RayRec* refl;               // [H][W] reflection ray (origin, direction)
  uint2* hits1;               // [H][W] reflection closest hit (t bits, slot)
  uint32_t* blk0;             // [H][W] per-light shadow bits of the primary hit
  uint32_t* blk1;             // [H][W] per-light shadow bits of the reflection hit
  uint32_t* list0;            // pixels whose primary ray hit, compacted in wave order (tile-coherent)
  uint32_t* list1;            // pixels whose reflection ray hit, compacted in list0 order
  uint32_t* wcount0;          // per primary wave: number of hit lanes (written by k_trace_primary)
  uint32_t* wcount1;          // per list0 wave: number of reflection hits (written by k_full_refl)
  uint32_t* woff0;            // exclusive prefix sums of wcount0 / wcount1 (k_scan_counts)
  uint32_t* woff1;
  uint32_t* counters;         // [0] = |list0|, [1] = |list1|
  int32_t n_waves_max;        // list waves of the worst case (every pixel listed)
  uint32_t* timeline;         // RT_FRAME_TIMELINE: 8 words per wave (rt_debug_timeline), else null
  // dispatch order of the one-wave render kernels (longest waves first, from an earlier frame's costs):
  // order[blockIdx] = the logical wave (tile * 4 + quarter) this block traces; null = the default
  // chunked-XCD order. cost[logical wave] receives the wave's duration in shader cycles (null = off).
  const uint32_t* order;
  uint32_t* cost;
  // a moving camera's cost map (whole frames, rt_device.hip render_one): each wave also raises cost_dil over the
  // (2 dil_r + 1)^2 waves around it in the frame's wave grid (atomic max), so the next frame's order sees each
  // wave's neighbourhood maximum; null = off
  uint32_t* cost_dil;
  int32_t dil_r;
  int32_t dil_w;  // the ring's cost = cost - (cost >> dil_w)
  // pred: each wave raises cost_dil around the wave where its primary hit point is expected in the next frame
  // instead of around itself (rt_kernels.h pred_mark / wave_clock_end): pred_proj = (a, b, c, e), a pixel's
  // view-space ray direction (a px + b, c py + e, -1); pred_step = the camera's last step as a view-space
  // translation (V_n V_(n-1)^-1), applied once more; 0 = off
  int32_t pred;
  float pred_proj[4];
  float pred_step[3];
  // RT_FRAME_WAVE_STATS (a counting frame, diagnostics): 8 words per logical wave (rt_debug_wave_stats)
  uint32_t* wave_stats;
  // k_render_full with an order: the first split_k logical waves of the order (the costliest of an
  // earlier frame) run as four 16-lane sub-waves each (blocks 0 .. 4 split_k - 1), the rest whole; the
  // grid is then (logical waves + 3 split_k) blocks. 0 = off.
  int32_t split_k;
  const float* face_boxcolor;  // RT_MODE_BOX_COLORS: [n_faces][4] summed box colours per face id
};

// Ray-list query parameters (rt_trace_closest / rt_trace_shadow)
struct RayParams {
  const float* o;  // [n][3]
  const float* d;  // [n][3]
  int32_t n;
  int32_t* face;
  float* t;
  float* P;
  int32_t* blocked;
  float* N;        // [n][3] interpolated normal at the closest hit (optional)
  float* rgb;      // [n][3] traceRay colour (rt_trace_color)
};

}  // namespace rt
