// rt_build.hip -- GPU BVH builders (SURVEY.md 8(f) f2 "LBVH/PLOC").
// LBVH: Morton codes of the triangle centroids, a device radix sort (hipCUB), Karras' parallel radix-tree
// construction (one thread per interior node), bottom-up bounds with agent-scope acquire/release
// counters, then one Node64 per interior node with subtrees of <= leaf_size triangles collapsed into leaf
// handles. Build time is milliseconds instead of the host SAH's ~1 s at 1M triangles; the tree is
// lower-quality (no SAH), traded for build speed.
// PLOC (Meister & Bittner, "Parallel Locally-Ordered Clustering for Bounding Volume Hierarchy
// Construction", TVCG 2018): the Morton-sorted triangles are clusters; every iteration each cluster finds
// its nearest neighbour (smallest surface area of the merged box) among the `radius` clusters either side
// in Morton order, mutual nearest neighbours merge into a new interior node, and the cluster array is
// compacted in order -- until one cluster is left. Agglomerative clustering by surface area gives trees of
// SAH quality at GPU speed. A bottom-up SAH pass (same costs as the host builders: triangle 1, node step
// 0.7) then marks the subtrees of <= leaf_size triangles that are cheaper as one leaf; the host lays the
// tree out depth first (rt_host.cpp build_bvh_ploc). Child boxes get the same conservative padding as the
// host builders either way, so traversal stays exact.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <vector>

#include "rt_scene.h"

#define BCHECK(expr)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) {                                                                   \
      rt::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
      return RT_ERR_HIP;                                                                      \
    }                                                                                         \
  } while (0)

namespace rt {
namespace {

__device__ __forceinline__ uint32_t expand10(uint32_t v) {  // 10 bits -> every third bit
  v &= 1023u;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

struct Box6 {
  float lo[3], hi[3];
};

__device__ __forceinline__ Box6 tri_box(const TriRec64& t) {
  Box6 b;
  b.lo[0] = fminf(fminf(t.w0x, t.w1x), t.w2x); b.hi[0] = fmaxf(fmaxf(t.w0x, t.w1x), t.w2x);
  b.lo[1] = fminf(fminf(t.w0y, t.w1y), t.w2y); b.hi[1] = fmaxf(fmaxf(t.w0y, t.w1y), t.w2y);
  b.lo[2] = fminf(fminf(t.w0z, t.w1z), t.w2z); b.hi[2] = fmaxf(fmaxf(t.w0z, t.w1z), t.w2z);
  return b;
}

// key = 30-bit Morton code of the centroid (scene box quantised to 1024^3) << 32 | face slot: unique
__global__ void k_morton(const TriRec64* rec, int n, float3 lo, float3 scale, uint64_t* keys) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Box6 b = tri_box(rec[i]);
  uint32_t q[3];
  const float l[3] = {lo.x, lo.y, lo.z}, s[3] = {scale.x, scale.y, scale.z};
  for (int k = 0; k < 3; k++) {
    const float c = 0.5f * (b.lo[k] + b.hi[k]);
    const float f = (c - l[k]) * s[k];
    q[k] = (uint32_t)fminf(fmaxf(f, 0.0f), 1023.0f);
  }
  const uint32_t m = (expand10(q[0]) << 2) | (expand10(q[1]) << 1) | expand10(q[2]);
  keys[i] = ((uint64_t)m << 32) | (uint32_t)i;
}

__device__ __forceinline__ int delta(const uint64_t* k, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  return __clzll((long long)(k[i] ^ k[j]));
}

// Karras 2012, one thread per interior node i in [0, n-1): range [first, last], split, children.
// child encoding: >= 0 interior node, < 0: ~leaf index (a single sorted primitive)
__global__ void k_karras(const uint64_t* keys, int n, int2* range, int2* child, int* parent_int, int* parent_leaf) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n - 1) return;
  const int d = (delta(keys, n, i, i + 1) - delta(keys, n, i, i - 1)) >= 0 ? 1 : -1;
  const int dmin = delta(keys, n, i, i - d);
  int lmax = 2;
  while (delta(keys, n, i, i + lmax * d) > dmin) lmax *= 2;
  int l = 0;
  for (int t = lmax / 2; t >= 1; t /= 2)
    if (delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
  const int j = i + l * d;
  const int dnode = delta(keys, n, i, j);
  int s = 0, t = l;
  do {
    t = (t + 1) >> 1;
    if (delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
  } while (t > 1);
  const int gamma = i + s * d + min(d, 0);
  const int first = min(i, j), last = max(i, j);
  const int left = (first == gamma) ? ~gamma : gamma;
  const int right = (last == gamma + 1) ? ~(gamma + 1) : gamma + 1;
  range[i] = make_int2(first, last);
  child[i] = make_int2(left, right);
  if (left >= 0) parent_int[left] = i; else parent_leaf[gamma] = i;
  if (right >= 0) parent_int[right] = i; else parent_leaf[gamma + 1] = i;
}

__global__ void k_leaf_boxes(const uint64_t* keys, const TriRec64* rec, int n, Box6* pbox) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  pbox[i] = tri_box(rec[(uint32_t)keys[i]]);
}

__device__ __forceinline__ Box6 join(const Box6& a, const Box6& b) {
  Box6 r;
  for (int k = 0; k < 3; k++) { r.lo[k] = fminf(a.lo[k], b.lo[k]); r.hi[k] = fmaxf(a.hi[k], b.hi[k]); }
  return r;
}

// bottom-up interior bounds: the second child to finish computes its parent (agent-scope acq/rel)
__global__ void k_bottom_up(const int2* child, const int* parent_int, const int* parent_leaf, const Box6* pbox,
                            Box6* nbox, int* flags, int n) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  int node = parent_leaf[k];
  while (node >= 0) {
    const int arrived = __hip_atomic_fetch_add(&flags[node], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (arrived == 0) return;  // the sibling subtree is not done: it will continue from here
    const int2 c = child[node];
    const Box6 a = c.x >= 0 ? nbox[c.x] : pbox[~c.x];
    const Box6 b = c.y >= 0 ? nbox[c.y] : pbox[~c.y];
    nbox[node] = join(a, b);
    __atomic_thread_fence(__ATOMIC_RELEASE);
    node = node == 0 ? -1 : parent_int[node];
  }
}

__device__ __forceinline__ uint32_t child_handle(int c, const int2* range, int leaf_size) {
  if (c < 0) return make_leaf((uint32_t)~c, 1u);
  const int2 r = range[c];
  const int cnt = r.y - r.x + 1;
  if (cnt <= leaf_size) return make_leaf((uint32_t)r.x, (uint32_t)cnt);
  return (uint32_t)c;
}

__global__ void k_emit_nodes(const int2* child, const int2* range, const Box6* pbox, const Box6* nbox, Node64* out,
                             int n, int leaf_size, float pad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n - 1) return;
  const int2 c = child[i];
  const Box6 a = c.x >= 0 ? nbox[c.x] : pbox[~c.x];
  const Box6 b = c.y >= 0 ? nbox[c.y] : pbox[~c.y];
  Node64 nd;
  nd.c0lx = a.lo[0] - pad; nd.c0hx = a.hi[0] + pad; nd.c0ly = a.lo[1] - pad; nd.c0hy = a.hi[1] + pad;
  nd.c0lz = a.lo[2] - pad; nd.c0hz = a.hi[2] + pad;
  nd.c1lx = b.lo[0] - pad; nd.c1hx = b.hi[0] + pad; nd.c1ly = b.lo[1] - pad; nd.c1hy = b.hi[1] + pad;
  nd.c1lz = b.lo[2] - pad; nd.c1hz = b.hi[2] + pad;
  nd.child0 = child_handle(c.x, range, leaf_size);
  nd.child1 = child_handle(c.y, range, leaf_size);
  nd.pad0 = nd.pad1 = 0;
  out[i] = nd;
}

__global__ void k_emit_tris(const uint64_t* keys, const TriRec64* rec, TriRec64* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = rec[(uint32_t)keys[i]];
}


// ---------------------------------------------------------------------------------------------------
// PLOC
// ---------------------------------------------------------------------------------------------------
struct Cluster {
  Box6 b;
  int id;  // >= 0: interior node, < 0: ~face (index of the face record)
  int pad;
};

__device__ __forceinline__ float half_area(const Box6& b) {
  const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
  return dx * dy + dy * dz + dz * dx;
}

__global__ void k_ploc_init(const uint64_t* keys, const TriRec64* rec, int n, Cluster* cl, Box6* tbox) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t f = (uint32_t)keys[i];
  Cluster c;
  c.b = tri_box(rec[f]);
  c.id = ~(int)f;
  c.pad = 0;
  cl[i] = c;
  tbox[f] = c.b;
}

// nearest neighbour of every cluster among the `radius` clusters either side in Morton order (surface
// area of the merged box; ties to the smaller index, so the pair that is smallest under (area, lower
// index, higher index) is always mutual and every iteration merges at least once). One block of
// kPlocBlock clusters stages its window [first - radius, first + kPlocBlock + radius) in LDS.
constexpr int kPlocBlock = 256, kPlocMaxRadius = 32;
__global__ __launch_bounds__(kPlocBlock) void k_ploc_nn(const Cluster* cl, int n, int radius, int* nn) {
  __shared__ Box6 win[kPlocBlock + 2 * kPlocMaxRadius];
  const int first = (int)blockIdx.x * kPlocBlock;
  const int lo = first - radius, cnt = kPlocBlock + 2 * radius;
  for (int k = (int)threadIdx.x; k < cnt; k += kPlocBlock) {
    const int g = lo + k;
    if (g >= 0 && g < n) win[k] = cl[g].b;
  }
  __syncthreads();
  const int i = first + (int)threadIdx.x;
  if (i >= n) return;
  const Box6 bi = win[i - lo];
  float best = INFINITY;
  int bj = -1;
  const int j0 = max(0, i - radius), j1 = min(n - 1, i + radius);
  for (int j = j0; j <= j1; j++) {
    if (j == i) continue;
    const float d = half_area(join(bi, win[j - lo]));
    if (d < best) { best = d; bj = j; }  // ascending j: the first minimum is the smaller index
  }
  nn[i] = bj;
}

// per cluster: merge flag (the lower index of a mutual pair) in the high word, keep flag (not the higher
// index of a mutual pair) in the low word -- one exclusive scan gives both output positions
__global__ void k_ploc_flags(const int* nn, int n, uint64_t* flags) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int j = nn[i];
  const bool mutual = j >= 0 && nn[j] == i;
  const uint64_t merge = (mutual && i < j) ? 1u : 0u, keep = (mutual && j < i) ? 0u : 1u;
  flags[i] = (merge << 32) | keep;
}

// the merged clusters become interior nodes node_base + (their merge rank); the survivors move to their
// compacted position (Morton order kept)
__global__ void k_ploc_merge(const Cluster* cl, const int* nn, const uint64_t* flags, const uint64_t* pos, int n,
                             int node_base, Cluster* out, int2* child, Box6* nbox, int* parent_int, int* parent_leaf) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t f = flags[i];
  if (!(f & 0xFFFFFFFFull)) return;  // merged into its lower-index partner
  Cluster c = cl[i];
  if (f >> 32) {
    const int node = node_base + (int)(pos[i] >> 32);
    const Cluster o = cl[nn[i]];
    child[node] = make_int2(c.id, o.id);
    if (c.id >= 0) parent_int[c.id] = node; else parent_leaf[~c.id] = node;
    if (o.id >= 0) parent_int[o.id] = node; else parent_leaf[~o.id] = node;
    c.b = join(c.b, o.b);
    nbox[node] = c.b;
    c.id = node;
  }
  out[(uint32_t)pos[i]] = c;
}

// bottom-up SAH collapse of the finished tree (one thread per face, the second child to finish computes
// its parent, agent-scope acquire/release as k_bottom_up): per node its triangle count and cost, and
// `leaf` = the subtree becomes one leaf (<= leaf_size triangles and no costlier than the split). Costs in
// units of one triangle test: a leaf n * A, an interior node k_trav * A + C(child 0) + C(child 1), A the
// node's (half) surface area -- the host builders' cost model (triangle 1, node step 0.7).
__global__ void k_ploc_collapse(const int2* child, const int* parent_int, const int* parent_leaf, const Box6* nbox,
                                const Box6* tbox, int* flags, int* count, float* cost, uint8_t* leaf, int n,
                                int leaf_size, float k_trav, int rule) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  int node = parent_leaf[k];
  while (node >= 0) {
    const int arrived = __hip_atomic_fetch_add(&flags[node], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (arrived == 0) return;  // the sibling subtree is not done: it continues from here
    const int2 c = child[node];
    const int na = c.x >= 0 ? count[c.x] : 1, nb = c.y >= 0 ? count[c.y] : 1;
    const float ca = c.x >= 0 ? cost[c.x] : half_area(tbox[~c.x]);
    const float cb = c.y >= 0 ? cost[c.y] : half_area(tbox[~c.y]);
    const float A = half_area(nbox[node]);
    const int m = na + nb;
    // rule 1 (A/B): the top-down builders' greedy test, children priced as leaves (n_c * A_c)
    const float pa = rule == 1 && c.x >= 0 ? (float)na * half_area(nbox[c.x]) : ca;
    const float pb = rule == 1 && c.y >= 0 ? (float)nb * half_area(nbox[c.y]) : cb;
    const float split = k_trav * A + (m <= leaf_size ? pa + pb : ca + cb), as_leaf = (float)m * A;
    const bool lf = m <= leaf_size && as_leaf <= split;
    count[node] = m;
    cost[node] = lf ? as_leaf : split;
    leaf[node] = lf ? 1 : 0;
    __atomic_thread_fence(__ATOMIC_RELEASE);
    node = parent_int[node];
  }
}
}  // namespace

// face_recs: one TriRec64 per face in face order. Outputs interior nodes in Karras order (root 0; nodes
// whose whole range became a leaf of their parent are left unreferenced) and the triangle records in
// leaf (Morton) order.
int gpu_build_lbvh(int device, const std::vector<TriRec64>& face_recs, const float lo[3], const float hi[3],
                   int leaf_size, float pad, std::vector<Node64>& nodes, std::vector<TriRec64>& tris, double* gpu_ms) {
  const int n = (int)face_recs.size();
  if (n < 2) { set_error("gpu_build_lbvh: needs at least 2 triangles"); return RT_ERR_INVALID; }
  BCHECK(hipSetDevice(device));
  hipStream_t st;
  st = (hipStream_t)build_stream(device);
  if (!st) return RT_ERR_HIP;
  struct Guard {
    hipStream_t st;
    std::vector<void*> bufs;
    std::vector<hipEvent_t> evs;  // released on every return (the fallback paths included)
    ~Guard() {
      (void)hipStreamSynchronize(st);
      for (void* b : bufs) (void)hipFree(b);
      for (hipEvent_t e : evs) (void)hipEventDestroy(e);
    }
  } g{st, {}, {}};
  auto alloc = [&](void** p, size_t bytes) -> hipError_t {
    hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 16));
    if (e == hipSuccess) g.bufs.push_back(*p);
    return e;
  };
  TriRec64 *d_rec = nullptr, *d_tris = nullptr;
  uint64_t *d_k0 = nullptr, *d_k1 = nullptr;
  int2 *d_range = nullptr, *d_child = nullptr;
  int *d_pint = nullptr, *d_pleaf = nullptr, *d_flags = nullptr;
  Box6 *d_pbox = nullptr, *d_nbox = nullptr;
  Node64* d_nodes = nullptr;
  BCHECK(alloc((void**)&d_rec, (size_t)n * sizeof(TriRec64)));
  BCHECK(alloc((void**)&d_tris, (size_t)n * sizeof(TriRec64)));
  BCHECK(alloc((void**)&d_k0, (size_t)n * 8));
  BCHECK(alloc((void**)&d_k1, (size_t)n * 8));
  BCHECK(alloc((void**)&d_range, (size_t)n * sizeof(int2)));
  BCHECK(alloc((void**)&d_child, (size_t)n * sizeof(int2)));
  BCHECK(alloc((void**)&d_pint, (size_t)n * 4));
  BCHECK(alloc((void**)&d_pleaf, (size_t)n * 4));
  BCHECK(alloc((void**)&d_flags, (size_t)n * 4));
  BCHECK(alloc((void**)&d_pbox, (size_t)n * sizeof(Box6)));
  BCHECK(alloc((void**)&d_nbox, (size_t)n * sizeof(Box6)));
  BCHECK(alloc((void**)&d_nodes, (size_t)n * sizeof(Node64)));
  if (int rc = h2d(d_rec, face_recs.data(), (size_t)n * sizeof(TriRec64))) return rc;  // pinned staging
  BCHECK(hipMemsetAsync(d_flags, 0, (size_t)n * 4, st));
  hipEvent_t e0, e1;
  BCHECK(hipEventCreate(&e0));
  g.evs.push_back(e0);
  BCHECK(hipEventCreate(&e1));
  g.evs.push_back(e1);
  BCHECK(hipEventRecord(e0, st));
  const int B = 256, G = (n + B - 1) / B;
  float3 flo = make_float3(lo[0], lo[1], lo[2]), fsc;
  fsc.x = hi[0] > lo[0] ? 1024.0f / (hi[0] - lo[0]) : 0.0f;
  fsc.y = hi[1] > lo[1] ? 1024.0f / (hi[1] - lo[1]) : 0.0f;
  fsc.z = hi[2] > lo[2] ? 1024.0f / (hi[2] - lo[2]) : 0.0f;
  hipLaunchKernelGGL(k_morton, dim3(G), dim3(B), 0, st, (const TriRec64*)d_rec, n, flo, fsc, d_k0);
  size_t tb = 0;
  BCHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, d_k0, d_k1, n, 0, 64, st));
  void* d_tmp = nullptr;
  BCHECK(alloc(&d_tmp, tb));
  BCHECK(hipcub::DeviceRadixSort::SortKeys(d_tmp, tb, d_k0, d_k1, n, 0, 64, st));
  hipLaunchKernelGGL(k_karras, dim3(G), dim3(B), 0, st, (const uint64_t*)d_k1, n, d_range, d_child, d_pint, d_pleaf);
  hipLaunchKernelGGL(k_leaf_boxes, dim3(G), dim3(B), 0, st, (const uint64_t*)d_k1, (const TriRec64*)d_rec, n, d_pbox);
  hipLaunchKernelGGL(k_bottom_up, dim3(G), dim3(B), 0, st, (const int2*)d_child, (const int*)d_pint, (const int*)d_pleaf,
                     (const Box6*)d_pbox, d_nbox, d_flags, n);
  hipLaunchKernelGGL(k_emit_nodes, dim3(G), dim3(B), 0, st, (const int2*)d_child, (const int2*)d_range,
                     (const Box6*)d_pbox, (const Box6*)d_nbox, d_nodes, n, leaf_size, pad);
  hipLaunchKernelGGL(k_emit_tris, dim3(G), dim3(B), 0, st, (const uint64_t*)d_k1, (const TriRec64*)d_rec, d_tris, n);
  BCHECK(hipGetLastError());
  BCHECK(hipEventRecord(e1, st));
  nodes.resize((size_t)n - 1);
  tris.resize(n);
  BCHECK(hipStreamSynchronize(st));
  if (int rc = d2h(nodes.data(), d_nodes, (size_t)(n - 1) * sizeof(Node64))) return rc;  // pinned staging
  if (int rc = d2h(tris.data(), d_tris, (size_t)n * sizeof(TriRec64))) return rc;
  float ms = 0.0f;
  BCHECK(hipEventElapsedTime(&ms, e0, e1));
  if (gpu_ms) *gpu_ms = ms;
  return RT_OK;
}

// PLOC (see the top of the file). face_recs: one TriRec64 per face. Outputs the n - 1 interior nodes
// (root n - 2): children (>= 0 interior node, < 0 ~face), boxes, the SAH collapse flag per node; the
// host lays the tree out (rt_host.cpp build_bvh_ploc). RT_ERR_INVALID when the clustering cannot finish
// (an iteration without a merge: non-finite boxes), so the caller builds on the host instead.
int gpu_build_ploc(int device, const std::vector<TriRec64>& face_recs, const float lo[3], const float hi[3],
                   int leaf_size, int radius, float k_trav, std::vector<int32_t>& child2, std::vector<float>& box6,
                   std::vector<uint8_t>& leaf, double* gpu_ms, int* iterations, int rule) {
  const int n = (int)face_recs.size();
  if (n < 2) { set_error("gpu_build_ploc: needs at least 2 triangles"); return RT_ERR_INVALID; }
  radius = std::max(1, std::min(radius, kPlocMaxRadius));
  BCHECK(hipSetDevice(device));
  hipStream_t st;
  st = (hipStream_t)build_stream(device);
  if (!st) return RT_ERR_HIP;
  struct Guard {
    hipStream_t st;
    std::vector<void*> bufs;
    std::vector<hipEvent_t> evs;  // released on every return (the fallback paths included)
    ~Guard() {
      (void)hipStreamSynchronize(st);
      for (void* b : bufs) (void)hipFree(b);
      for (hipEvent_t e : evs) (void)hipEventDestroy(e);
    }
  } g{st, {}, {}};
  auto alloc = [&](void** p, size_t bytes) -> hipError_t {
    hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 16));
    if (e == hipSuccess) g.bufs.push_back(*p);
    return e;
  };
  TriRec64* d_rec = nullptr;
  uint64_t *d_k0 = nullptr, *d_k1 = nullptr, *d_flags = nullptr, *d_pos = nullptr;
  Cluster *d_ca = nullptr, *d_cb = nullptr;
  Box6 *d_tbox = nullptr, *d_nbox = nullptr;
  int2* d_child = nullptr;
  int *d_nn = nullptr, *d_pint = nullptr, *d_pleaf = nullptr, *d_cflags = nullptr, *d_count = nullptr;
  float* d_cost = nullptr;
  uint8_t* d_leaf = nullptr;
  BCHECK(alloc((void**)&d_rec, (size_t)n * sizeof(TriRec64)));
  BCHECK(alloc((void**)&d_k0, (size_t)n * 8));
  BCHECK(alloc((void**)&d_k1, (size_t)n * 8));
  BCHECK(alloc((void**)&d_flags, (size_t)n * 8));
  BCHECK(alloc((void**)&d_pos, (size_t)n * 8));
  BCHECK(alloc((void**)&d_ca, (size_t)n * sizeof(Cluster)));
  BCHECK(alloc((void**)&d_cb, (size_t)n * sizeof(Cluster)));
  BCHECK(alloc((void**)&d_tbox, (size_t)n * sizeof(Box6)));
  BCHECK(alloc((void**)&d_nbox, (size_t)n * sizeof(Box6)));
  BCHECK(alloc((void**)&d_child, (size_t)n * sizeof(int2)));
  BCHECK(alloc((void**)&d_nn, (size_t)n * 4));
  BCHECK(alloc((void**)&d_pint, (size_t)n * 4));
  BCHECK(alloc((void**)&d_pleaf, (size_t)n * 4));
  BCHECK(alloc((void**)&d_cflags, (size_t)n * 4));
  BCHECK(alloc((void**)&d_count, (size_t)n * 4));
  BCHECK(alloc((void**)&d_cost, (size_t)n * 4));
  BCHECK(alloc((void**)&d_leaf, (size_t)n));
  if (int rc = h2d(d_rec, face_recs.data(), (size_t)n * sizeof(TriRec64))) return rc;  // pinned staging
  BCHECK(hipMemsetAsync(d_pint, 0xFF, (size_t)n * 4, st));  // the root's parent: -1
  BCHECK(hipMemsetAsync(d_cflags, 0, (size_t)n * 4, st));
  hipEvent_t e0, e1;
  BCHECK(hipEventCreate(&e0));
  g.evs.push_back(e0);
  BCHECK(hipEventCreate(&e1));
  g.evs.push_back(e1);
  BCHECK(hipEventRecord(e0, st));
  const int B = 256, G = (n + B - 1) / B;
  float3 flo = make_float3(lo[0], lo[1], lo[2]), fsc;
  fsc.x = hi[0] > lo[0] ? 1024.0f / (hi[0] - lo[0]) : 0.0f;
  fsc.y = hi[1] > lo[1] ? 1024.0f / (hi[1] - lo[1]) : 0.0f;
  fsc.z = hi[2] > lo[2] ? 1024.0f / (hi[2] - lo[2]) : 0.0f;
  hipLaunchKernelGGL(k_morton, dim3(G), dim3(B), 0, st, (const TriRec64*)d_rec, n, flo, fsc, d_k0);
  size_t tb = 0, tscan = 0;
  BCHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, d_k0, d_k1, n, 0, 64, st));
  BCHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tscan, d_flags, d_pos, n, st));
  void* d_tmp = nullptr;
  BCHECK(alloc(&d_tmp, std::max(tb, tscan)));
  BCHECK(hipcub::DeviceRadixSort::SortKeys(d_tmp, tb, d_k0, d_k1, n, 0, 64, st));
  hipLaunchKernelGGL(k_ploc_init, dim3(G), dim3(B), 0, st, (const uint64_t*)d_k1, (const TriRec64*)d_rec, n, d_ca, d_tbox);
  BCHECK(hipGetLastError());
  int N = n, base = 0, iters = 0;
  Cluster *cur = d_ca, *nxt = d_cb;
  while (N > 1) {
    const int g = (N + kPlocBlock - 1) / kPlocBlock;
    hipLaunchKernelGGL(k_ploc_nn, dim3(g), dim3(kPlocBlock), 0, st, (const Cluster*)cur, N, radius, d_nn);
    hipLaunchKernelGGL(k_ploc_flags, dim3(g), dim3(kPlocBlock), 0, st, (const int*)d_nn, N, d_flags);
    BCHECK(hipcub::DeviceScan::ExclusiveSum(d_tmp, tscan, d_flags, d_pos, N, st));
    hipLaunchKernelGGL(k_ploc_merge, dim3(g), dim3(kPlocBlock), 0, st, (const Cluster*)cur, (const int*)d_nn,
                       (const uint64_t*)d_flags, (const uint64_t*)d_pos, N, base, nxt, d_child, d_nbox, d_pint, d_pleaf);
    BCHECK(hipGetLastError());
    uint64_t tail[2];
    BCHECK(hipMemcpyAsync(&tail[0], d_pos + (N - 1), 8, hipMemcpyDeviceToHost, st));
    BCHECK(hipMemcpyAsync(&tail[1], d_flags + (N - 1), 8, hipMemcpyDeviceToHost, st));
    BCHECK(hipStreamSynchronize(st));
    const uint64_t tot = tail[0] + tail[1];
    const int merges = (int)(tot >> 32), keeps = (int)(tot & 0xFFFFFFFFull);
    if (merges == 0 || keeps != N - merges) { set_error("gpu_build_ploc: clustering stalled (non-finite boxes?)"); return RT_ERR_INVALID; }
    base += merges;
    N = keeps;
    std::swap(cur, nxt);
    iters++;
  }
  if (base != n - 1) { set_error("gpu_build_ploc: %d interior nodes for %d faces", base, n); return RT_ERR_INVALID; }
  hipLaunchKernelGGL(k_ploc_collapse, dim3(G), dim3(B), 0, st, (const int2*)d_child, (const int*)d_pint,
                     (const int*)d_pleaf, (const Box6*)d_nbox, (const Box6*)d_tbox, d_cflags, d_count, d_cost, d_leaf, n,
                     std::max(1, std::min(leaf_size, kMaxLeaf)), k_trav, rule);
  BCHECK(hipGetLastError());
  BCHECK(hipEventRecord(e1, st));
  child2.resize(2 * (size_t)(n - 1));
  box6.resize(6 * (size_t)(n - 1));
  leaf.resize((size_t)(n - 1));
  BCHECK(hipStreamSynchronize(st));
  if (int rc = d2h(child2.data(), d_child, (size_t)(n - 1) * sizeof(int2))) return rc;  // pinned staging
  if (int rc = d2h(box6.data(), d_nbox, (size_t)(n - 1) * sizeof(Box6))) return rc;
  if (int rc = d2h(leaf.data(), d_leaf, (size_t)(n - 1))) return rc;
  float ms = 0.0f;
  BCHECK(hipEventElapsedTime(&ms, e0, e1));
  if (gpu_ms) *gpu_ms = ms;
  if (iterations) *iterations = iters;
  return RT_OK;
}


// ---------------------------------------------------------------------------------------------------
// Top-down binned SAH on the GPU, with or without spatial splits (RT_BUILDER_SAH_GPU / RT_BUILDER_SBVH_GPU):
// the host builders' algorithms (32 centroid bins per axis, cost k_trav * A + sum(n_side * A_side), a leaf
// when <= leaf_size references and no costlier; SBVH: 32 spatial bins per axis tried when the object
// split's children overlap by more than alpha of the root, straddling triangles clipped to both sides,
// duplication bounded by a per-subtree budget divided in proportion to the children) run breadth first,
// one level of the tree per round of launches. References keep their Morton order inside every node's
// contiguous range (stable partition), so small tasks stay coherent. Per level:
//   (1) every active task's box and centroid bounds: a segmented wave reduction over its contiguous
//       positions, one atomic per segment and wave;
//   (2) tasks above kSahSmall references: centroid bins (ordered-uint atomics; a block whose 256 positions
//       belong to one task bins in LDS first); one thread per task sweeps them (phase A) and flags the
//       tasks whose object split overlaps enough for a spatial split, which then bin their references'
//       clipped parts (SBVH only);
//   (3) one thread per task decides: the cheaper of the object and spatial split for big tasks, an exact
//       sweep over the sorted centroids (<= kSahSmall) for small ones, the position median when the
//       centroids are degenerate or the depth nears the stack bound; a leaf takes a leaf id, a split its
//       node and two child tasks;
//   (4) every position's sides (left, right or both for a clipped straddler) and two exclusive scans give
//       every output position; the child tasks get their ranges; (5) one scatter writes the next level.
// Leaves are resolved to slot ranges at the end (their references move while others duplicate).
// ---------------------------------------------------------------------------------------------------
namespace {
constexpr int kSahBins = 32, kSahSmall = 16, kSahBlock = 256;
constexpr int kObjW = 7, kSpW = 8;  // words per object bin (box lo, hi as ordered uints; count) / spatial bin (+ exits)

struct SahTask {
  uint32_t begin, count;  // reference range at this level
  int32_t parent_slot;    // 2 * parent node + side, -1 for the root
  int32_t big;            // object-bin block (count > kSahSmall) or -1
  int32_t sp;             // spatial-bin block or -1
  int32_t child;          // first child task of the next level; -1: a leaf (bin = its leaf id)
  int32_t axis, bin;      // >= 0: object split (last left bin); -1: position median (bin = left count);
                          // -2: sides from the exact sweep; 3..5: spatial split on axis - 3 at `plane`
  float plane;
  int32_t budget;         // references this subtree may add by spatial splits
  float o_cost;           // phase A: the best object split
  int32_t o_axis, o_bin;
  uint32_t o_nl;
};

__device__ __forceinline__ uint32_t f2o(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float o2f(uint32_t u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u); }
__device__ __forceinline__ float cen(const Box6& b, int k) { return 0.5f * (b.lo[k] + b.hi[k]); }
__device__ __forceinline__ float sah_area(const float* lo, const float* hi) {
  const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
  return dx * dy + dy * dz + dz * dx;
}
// bin index, clamped explicitly (a NaN or out-of-range product lands in bin 0 / the last bin, never outside)
__device__ __forceinline__ int sah_bin(float c, float lo, float sc) {
  const float x = (c - lo) * sc;
  return x >= 1.0f ? (x < (float)kSahBins ? (int)x : kSahBins - 1) : 0;
}
__device__ __forceinline__ bool is_lo_word(int k) { return k < 3 || (k >= 6 && k < 9); }

// spatial bin planes of a task box on axis k: pl(i) = lo + w * i, pl(kSahBins) = hi (as the host builder)
__device__ __forceinline__ float sp_plane(const Box6& b, int k, int i) {
  const float w = (b.hi[k] - b.lo[k]) / kSahBins;
  return i >= kSahBins ? b.hi[k] : b.lo[k] + w * i;
}
__device__ __forceinline__ int sp_bin(const Box6& b, int k, float x) {
  const float w = (b.hi[k] - b.lo[k]) / kSahBins, q = (x - b.lo[k]) / w;
  int bi = q >= 1.0f ? (q < (float)kSahBins ? (int)q : kSahBins - 1) : 0;
  while (bi > 0 && x < sp_plane(b, k, bi)) bi--;
  while (bi < kSahBins - 1 && x >= sp_plane(b, k, bi + 1)) bi++;
  return bi;
}
__device__ __forceinline__ float fdown(double x) { const float f = (float)x; return (double)f > x ? nextafterf(f, -INFINITY) : f; }
__device__ __forceinline__ float fup(double x) { const float f = (float)x; return (double)f < x ? nextafterf(f, INFINITY) : f; }
// bounds of triangle `t` (its record's vertices: the culling bounds) inside [a, b] on axis k, intersected
// with `within` (the reference's box); false if empty -- the host SBVH's clip (rt_host.cpp SbvhBuilder)
__device__ bool clip_tri(const TriRec64& t, int k, float a, float b, const Box6& within, Box6& out) {
  const double v[3][3] = {{t.w0x, t.w0y, t.w0z}, {t.w1x, t.w1y, t.w1z}, {t.w2x, t.w2y, t.w2z}};
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int j = 0; j < 3; j++) {
    const double* p = v[j];
    const double* q = v[(j + 1) % 3];
    if (p[k] >= a && p[k] <= b)
      for (int i = 0; i < 3; i++) { lo[i] = fmin(lo[i], p[i]); hi[i] = fmax(hi[i], p[i]); }
    const double pls[2] = {(double)a, (double)b};
    for (int s = 0; s < 2; s++) {
      const double pl = pls[s];
      if ((p[k] < pl && q[k] > pl) || (p[k] > pl && q[k] < pl)) {
        const double tt = (pl - p[k]) / (q[k] - p[k]);
        for (int i = 0; i < 3; i++) {
          const double x = i == k ? pl : p[i] + tt * (q[i] - p[i]);
          lo[i] = fmin(lo[i], x);
          hi[i] = fmax(hi[i], x);
        }
      }
    }
  }
  for (int i = 0; i < 3; i++) {
    out.lo[i] = fmaxf(fdown(lo[i]), within.lo[i]);
    out.hi[i] = fminf(fup(hi[i]), within.hi[i]);
    if (i == k) { out.lo[i] = fmaxf(out.lo[i], a); out.hi[i] = fminf(out.hi[i], b); }
    if (!(out.lo[i] <= out.hi[i])) return false;
  }
  return true;
}

__global__ void k_sah_init(const uint64_t* keys, const TriRec64* rec, int n, uint32_t* rface, Box6* rbox, int32_t* ptask) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t f = (uint32_t)keys[i];
  rface[i] = f;
  rbox[i] = tri_box(rec[f]);
  ptask[i] = 0;
}
__global__ void k_sah_stat_init(uint32_t* stat, int ntask) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntask) return;
  for (int k = 0; k < 12; k++) stat[12 * (size_t)t + k] = is_lo_word(k) ? 0xFFFFFFFFu : 0u;
}
// bins of `w` words: the first three start at all-ones (ordered minima), the rest at 0
__global__ void k_sah_bins_init(uint32_t* bins, int nbins, int w) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nbins) return;
  for (int q = 0; q < w; q++) bins[(size_t)w * b + q] = q < 3 ? 0xFFFFFFFFu : 0u;
}

// (1) box and centroid bounds of every active task (stat[t]: box lo, box hi, centroid lo, centroid hi)
__global__ __launch_bounds__(kSahBlock) void k_sah_bounds(const Box6* rbox, const int32_t* ptask, int m, uint32_t* stat) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int t = i < m ? ptask[i] : -1;
  uint32_t v[12];
  if (t >= 0) {
    const Box6 b = rbox[i];
    for (int k = 0; k < 3; k++) {
      v[k] = f2o(b.lo[k]);
      v[3 + k] = f2o(b.hi[k]);
      v[6 + k] = v[9 + k] = f2o(cen(b, k));
    }
  } else {
    for (int k = 0; k < 12; k++) v[k] = 0;
  }
  // segmented inclusive scan over equal task ids (a task's positions are contiguous)
  for (int off = 1; off < 64; off <<= 1) {
    const int tu = __shfl_up(t, off, 64);
    const bool take = lane >= off && tu == t;
    for (int k = 0; k < 12; k++) {
      const uint32_t u = __shfl_up(v[k], off, 64);
      if (take) v[k] = is_lo_word(k) ? min(v[k], u) : max(v[k], u);
    }
  }
  const int tn = __shfl_down(t, 1, 64);
  if (t >= 0 && (lane == 63 || tn != t || i == m - 1)) {
    uint32_t* s = stat + 12 * (size_t)t;
    for (int k = 0; k < 12; k++) {
      if (is_lo_word(k)) atomicMin(&s[k], v[k]); else atomicMax(&s[k], v[k]);
    }
  }
}

// (2) centroid bins of the big tasks
__global__ __launch_bounds__(kSahBlock) void k_sah_bin(const Box6* rbox, const int32_t* ptask, const SahTask* task,
                                                      const uint32_t* stat, int m, uint32_t* bins) {
  __shared__ uint32_t lb[3 * kSahBins * kObjW];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int first = blockIdx.x * blockDim.x, last = min(m - 1, first + kSahBlock - 1);
  const int t0 = ptask[first], t1 = ptask[last];
  const bool one_task = t0 == t1 && t0 >= 0 && task[t0].big >= 0;  // block-uniform
  const int t = i < m ? ptask[i] : -1;
  if (one_task) {
    for (int k = threadIdx.x; k < 3 * kSahBins * kObjW; k += kSahBlock) lb[k] = (k % kObjW) < 3 ? 0xFFFFFFFFu : 0u;
    __syncthreads();
  }
  if (t >= 0 && task[t].big >= 0) {
    const uint32_t* s = stat + 12 * (size_t)t;
    const Box6 b = rbox[i];
    const uint32_t bl[3] = {f2o(b.lo[0]), f2o(b.lo[1]), f2o(b.lo[2])}, bh[3] = {f2o(b.hi[0]), f2o(b.hi[1]), f2o(b.hi[2])};
    uint32_t* gb = bins + (size_t)task[t].big * 3 * kSahBins * kObjW;
    for (int k = 0; k < 3; k++) {
      const float clo = o2f(s[6 + k]), ext = o2f(s[9 + k]) - clo;
      if (!(ext > 0.0f)) continue;
      const int bi = sah_bin(cen(b, k), clo, kSahBins / ext);
      uint32_t* d = (one_task ? lb : gb) + (k * kSahBins + bi) * kObjW;
      for (int q = 0; q < 3; q++) { atomicMin(&d[q], bl[q]); atomicMax(&d[3 + q], bh[q]); }
      atomicAdd(&d[6], 1u);
    }
  }
  if (one_task) {
    __syncthreads();
    uint32_t* gb = bins + (size_t)task[t0].big * 3 * kSahBins * kObjW;
    for (int k = threadIdx.x; k < 3 * kSahBins; k += kSahBlock) {
      const uint32_t* d = lb + k * kObjW;
      if (d[6] == 0) continue;
      uint32_t* g = gb + k * kObjW;
      for (int q = 0; q < 3; q++) { atomicMin(&g[q], d[q]); atomicMax(&g[3 + q], d[3 + q]); }
      atomicAdd(&g[6], d[6]);
    }
  }
}

__device__ __forceinline__ void task_box(const uint32_t* s, Box6& box, float* clo, float* ext) {
  for (int k = 0; k < 3; k++) {
    box.lo[k] = o2f(s[k]);
    box.hi[k] = o2f(s[3 + k]);
    clo[k] = o2f(s[6 + k]);
    ext[k] = o2f(s[9 + k]) - clo[k];
  }
}

// (2, phase A) the best object split of every big task, and whether a spatial split is to be tried
__global__ void k_sah_split_obj(SahTask* task, int ntask, const uint32_t* stat, const uint32_t* bins, uint32_t* counters,
                                float root_area, float alpha, int spatial, int force_median) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntask) return;
  SahTask T = task[t];
  T.o_cost = INFINITY;
  T.o_axis = -1;
  T.o_bin = -1;
  T.o_nl = 0;
  T.sp = -1;
  if (T.big < 0 || force_median) { task[t] = T; return; }
  Box6 box;
  float clo[3], ext[3];
  task_box(stat + 12 * (size_t)t, box, clo, ext);
  const uint32_t* B = bins + (size_t)T.big * 3 * kSahBins * kObjW;
  Box6 lbest, rbest;
  for (int k = 0; k < 3; k++) {
    if (!(ext[k] > 0.0f)) continue;
    Box6 racc[kSahBins];
    uint32_t rcnt[kSahBins];
    Box6 acc{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
    uint32_t c = 0;
    for (int i = kSahBins - 1; i > 0; i--) {
      const uint32_t* d = B + (k * kSahBins + i) * kObjW;
      if (d[6]) for (int q = 0; q < 3; q++) { acc.lo[q] = fminf(acc.lo[q], o2f(d[q])); acc.hi[q] = fmaxf(acc.hi[q], o2f(d[3 + q])); }
      c += d[6];
      racc[i] = acc;
      rcnt[i] = c;
    }
    Box6 lacc{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
    uint32_t lc = 0;
    for (int i = 0; i < kSahBins - 1; i++) {
      const uint32_t* d = B + (k * kSahBins + i) * kObjW;
      if (d[6]) for (int q = 0; q < 3; q++) { lacc.lo[q] = fminf(lacc.lo[q], o2f(d[q])); lacc.hi[q] = fmaxf(lacc.hi[q], o2f(d[3 + q])); }
      lc += d[6];
      if (lc == 0 || rcnt[i + 1] == 0) continue;
      const float cost = sah_area(lacc.lo, lacc.hi) * lc + sah_area(racc[i + 1].lo, racc[i + 1].hi) * rcnt[i + 1];
      if (cost < T.o_cost) { T.o_cost = cost; T.o_axis = k; T.o_bin = i; T.o_nl = lc; lbest = lacc; rbest = racc[i + 1]; }
    }
  }
  if (spatial && T.budget > 0) {
    float ov = 0.0f;
    if (T.o_axis >= 0) {
      float d[3];
      for (int k = 0; k < 3; k++) d[k] = fmaxf(0.0f, fminf(lbest.hi[k], rbest.hi[k]) - fmaxf(lbest.lo[k], rbest.lo[k]));
      ov = d[0] * d[1] + d[1] * d[2] + d[2] * d[0];
    }
    if (T.o_axis < 0 || ov > alpha * root_area) T.sp = (int32_t)atomicAdd(&counters[3], 1u);
  }
  task[t] = T;
}

// (2, SBVH) spatial bins of the flagged tasks: a reference enters the bin of its low end, exits the bin of
// its high end, and adds the bounds of its clipped part to every bin it spans
__global__ __launch_bounds__(kSahBlock) void k_sah_spbin(const uint32_t* rface, const Box6* rbox, const int32_t* ptask,
                                                        const SahTask* task, const uint32_t* stat, const TriRec64* rec,
                                                        int m, uint32_t* spbins) {
  // a block whose 256 positions belong to one flagged task (the top levels: few, huge tasks) bins in LDS
  // first and flushes the non-empty bins, as k_sah_bin
  __shared__ uint32_t lb[3 * kSahBins * kSpW];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int first = blockIdx.x * blockDim.x, last = min(m - 1, first + kSahBlock - 1);
  const int t0 = ptask[first], t1 = ptask[last];
  const bool one_task = t0 == t1 && t0 >= 0 && task[t0].sp >= 0;  // block-uniform
  if (one_task) {
    for (int k = threadIdx.x; k < 3 * kSahBins * kSpW; k += kSahBlock) lb[k] = (k % kSpW) < 3 ? 0xFFFFFFFFu : 0u;
    __syncthreads();
  }
  const int t = i < m ? ptask[i] : -1;
  if (t >= 0 && task[t].sp >= 0) {
    Box6 box;
    float clo[3], ext[3];
    task_box(stat + 12 * (size_t)t, box, clo, ext);
    const Box6 r = rbox[i];
    uint32_t* S = one_task ? lb : spbins + (size_t)task[t].sp * 3 * kSahBins * kSpW;
    const TriRec64 tr = rec[rface[i]];
    for (int k = 0; k < 3; k++) {
      if (!((box.hi[k] - box.lo[k]) / kSahBins > 0.0f)) continue;
      const int b0 = sp_bin(box, k, r.lo[k]), b1 = sp_bin(box, k, r.hi[k]);
      atomicAdd(&S[(k * kSahBins + b0) * kSpW + 6], 1u);
      atomicAdd(&S[(k * kSahBins + b1) * kSpW + 7], 1u);
      for (int bi = b0; bi <= b1; bi++) {
        Box6 q;
        if (b0 == b1) q = r;
        else if (!clip_tri(tr, k, fmaxf(sp_plane(box, k, bi), r.lo[k]), fminf(sp_plane(box, k, bi + 1), r.hi[k]), r, q)) continue;
        uint32_t* d = S + (k * kSahBins + bi) * kSpW;
        for (int c = 0; c < 3; c++) { atomicMin(&d[c], f2o(q.lo[c])); atomicMax(&d[3 + c], f2o(q.hi[c])); }
      }
    }
  }
  if (one_task) {
    __syncthreads();
    uint32_t* gb = spbins + (size_t)task[t0].sp * 3 * kSahBins * kSpW;
    for (int k = threadIdx.x; k < 3 * kSahBins; k += kSahBlock) {
      const uint32_t* d = lb + k * kSpW;
      uint32_t* g = gb + k * kSpW;
      if (d[0] != 0xFFFFFFFFu)
        for (int q = 0; q < 3; q++) { atomicMin(&g[q], d[q]); atomicMax(&g[3 + q], d[3 + q]); }
      if (d[6]) atomicAdd(&g[6], d[6]);
      if (d[7]) atomicAdd(&g[7], d[7]);
    }
  }
}

// (3) the split of every task of the level
__global__ void k_sah_split(SahTask* task, int ntask, const uint32_t* stat, const uint32_t* spbins, const Box6* rbox,
                            uint8_t* side, SahTask* next, uint32_t* counters, uint32_t* nchild, Box6* ncb,
                            int leaf_size, float k_trav, int force_median) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntask) return;
  SahTask T = task[t];
  Box6 box;
  float clo[3], ext[3];
  task_box(stat + 12 * (size_t)t, box, clo, ext);
  const uint32_t n = T.count;
  const float A = fmaxf(sah_area(box.lo, box.hi), 1e-30f);
  float best = T.o_cost;
  int axis = T.o_axis, bin = T.o_bin;
  uint32_t nl = T.o_nl, est_l = T.o_nl, est_r = n - T.o_nl;
  bool exact = false;
  int ord[kSahSmall];
  if (T.sp >= 0) {  // spatial candidates: left = entries up to the plane, right = exits beyond it
    const uint32_t* S = spbins + (size_t)T.sp * 3 * kSahBins * kSpW;
    for (int k = 0; k < 3; k++) {
      if (!((box.hi[k] - box.lo[k]) / kSahBins > 0.0f)) continue;
      Box6 racc[kSahBins];
      uint32_t rcnt[kSahBins];
      Box6 acc{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
      uint32_t c = 0;
      for (int i = kSahBins - 1; i > 0; i--) {
        const uint32_t* d = S + (k * kSahBins + i) * kSpW;
        if (d[0] != 0xFFFFFFFFu) for (int q = 0; q < 3; q++) { acc.lo[q] = fminf(acc.lo[q], o2f(d[q])); acc.hi[q] = fmaxf(acc.hi[q], o2f(d[3 + q])); }
        c += d[7];
        racc[i] = acc;
        rcnt[i] = c;
      }
      Box6 lacc{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
      uint32_t lc = 0;
      for (int i = 0; i < kSahBins - 1; i++) {
        const uint32_t* d = S + (k * kSahBins + i) * kSpW;
        if (d[0] != 0xFFFFFFFFu) for (int q = 0; q < 3; q++) { lacc.lo[q] = fminf(lacc.lo[q], o2f(d[q])); lacc.hi[q] = fmaxf(lacc.hi[q], o2f(d[3 + q])); }
        lc += d[6];
        if (lc == 0 || rcnt[i + 1] == 0) continue;
        const float cost = sah_area(lacc.lo, lacc.hi) * lc + sah_area(racc[i + 1].lo, racc[i + 1].hi) * rcnt[i + 1];
        // a spatial split must duplicate within the budget (the estimate bounds the references it adds)
        if (cost < best && (int64_t)lc + rcnt[i + 1] - n <= (int64_t)T.budget) {
          best = cost; axis = 3 + k; bin = i; est_l = lc; est_r = rcnt[i + 1];
        }
      }
    }
  }
  if (!force_median && T.big < 0 && n >= 2) {
    // exact sweep over the centroids sorted along each axis (insertion sort, position order for ties)
    Box6 pb[kSahSmall];
    for (uint32_t j = 0; j < n; j++) pb[j] = rbox[T.begin + j];
    for (int k = 0; k < 3; k++) {
      if (!(ext[k] > 0.0f)) continue;
      int o[kSahSmall];
      for (uint32_t j = 0; j < n; j++) {
        int q = (int)j;
        const float c = cen(pb[j], k);
        while (q > 0 && cen(pb[o[q - 1]], k) > c) { o[q] = o[q - 1]; q--; }
        o[q] = (int)j;
      }
      float rarea[kSahSmall];
      Box6 acc{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
      for (int j = (int)n - 1; j > 0; j--) {
        for (int q = 0; q < 3; q++) { acc.lo[q] = fminf(acc.lo[q], pb[o[j]].lo[q]); acc.hi[q] = fmaxf(acc.hi[q], pb[o[j]].hi[q]); }
        rarea[j] = sah_area(acc.lo, acc.hi);
      }
      Box6 lacc{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
      for (uint32_t j = 0; j + 1 < n; j++) {
        for (int q = 0; q < 3; q++) { lacc.lo[q] = fminf(lacc.lo[q], pb[o[j]].lo[q]); lacc.hi[q] = fmaxf(lacc.hi[q], pb[o[j]].hi[q]); }
        const float cost = sah_area(lacc.lo, lacc.hi) * (float)(j + 1) + rarea[j + 1] * (float)(n - 1 - j);
        if (cost < best) {
          best = cost; axis = k; nl = j + 1; exact = true; est_l = nl; est_r = n - nl;
          for (uint32_t q = 0; q < n; q++) ord[q] = o[q];
        }
      }
    }
  }
  // the host builders' rule: a leaf when n <= leaf_size and no split is cheaper (or none exists, or the
  // depth forces medians); degenerate centroids make a leaf of <= kMaxLeaf; the root always splits
  const bool degenerate = !(ext[0] > 0.0f || ext[1] > 0.0f || ext[2] > 0.0f);
  bool leaf = n == 1;
  if (!leaf && (int)n <= leaf_size) leaf = force_median || axis < 0 || (float)n <= k_trav + best / A;
  if (!leaf && axis < 0 && degenerate && (int)n <= kMaxLeaf) leaf = true;
  if (T.parent_slot < 0) leaf = false;
  if (leaf) {
    const uint32_t id = atomicAdd(&counters[4], 1u);
    T.child = -1;
    T.bin = (int32_t)id;
    task[t] = T;
    nchild[T.parent_slot] = 0x80000000u | id;
    ncb[T.parent_slot] = box;
    return;
  }
  if (axis < 0) { axis = -1; bin = (int32_t)(n / 2); est_l = n / 2; est_r = n - n / 2; exact = false; }  // position median
  const uint32_t node = T.parent_slot < 0 ? 0u : atomicAdd(&counters[1], 1u);
  if (T.parent_slot >= 0) { nchild[T.parent_slot] = node; ncb[T.parent_slot] = box; }
  const uint32_t c = atomicAdd(&counters[0], 2u);
  // children's budgets: what is left after this split's estimated duplicates, in proportion to their sizes
  const int64_t rest = (int64_t)T.budget - ((int64_t)est_l + est_r - n);
  const int32_t bl = (int32_t)((double)rest * (double)est_l / (double)(est_l + est_r));
  for (int q = 0; q < 2; q++) {
    SahTask C{};
    C.parent_slot = (int32_t)(2 * node + q);
    C.big = -1;
    C.sp = -1;
    C.child = -1;
    C.axis = -1;
    C.bin = -1;
    C.budget = q ? (int32_t)(rest - bl) : bl;
    next[c + q] = C;  // range and bin block set by k_sah_fix
  }
  T.child = (int32_t)c;
  if (axis >= 3) T.plane = sp_plane(box, axis - 3, bin + 1);
  T.axis = exact ? -2 : axis;
  T.bin = bin;
  task[t] = T;
  if (exact)
    for (uint32_t q = 0; q < n; q++) side[T.begin + ord[q]] = q < nl ? 1 : 0;
}

// (4) sides of every position: lr = (goes left) << 32 | (goes right); fin = 1 for a finished reference
__global__ void k_sah_side(const uint32_t* rface, const Box6* rbox, const int32_t* ptask, const SahTask* task,
                           const uint32_t* stat, const TriRec64* rec, const uint8_t* side, int m, uint64_t* lr,
                           uint32_t* fin) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > m) return;
  if (i == m) { lr[i] = 0; fin[i] = 0; return; }  // the scans' end element
  const int t = ptask[i];
  uint32_t L = 0, R = 0, F = 0;
  if (t < 0) {
    F = 1;
  } else {
    const SahTask T = task[t];
    if (T.child < 0) {
      F = 1;
    } else if (T.axis >= 3) {
      const int k = T.axis - 3;
      const Box6 r = rbox[i];
      if (r.hi[k] <= T.plane) L = 1;
      else if (r.lo[k] >= T.plane) R = 1;
      else {
        Box6 q;
        const TriRec64 tr = rec[rface[i]];
        L = clip_tri(tr, k, r.lo[k], T.plane, r, q) ? 1 : 0;
        R = clip_tri(tr, k, T.plane, r.hi[k], r, q) ? 1 : 0;
        if (!L && !R) { if (cen(r, k) < T.plane) L = 1; else R = 1; }
      }
    } else if (T.axis >= 0) {
      const uint32_t* s = stat + 12 * (size_t)t;
      const float clo = o2f(s[6 + T.axis]), ext = o2f(s[9 + T.axis]) - clo;
      L = sah_bin(cen(rbox[i], T.axis), clo, kSahBins / ext) <= T.bin ? 1 : 0;
      R = 1 - L;
    } else if (T.axis == -1) {
      L = (uint32_t)(i - (int)T.begin) < (uint32_t)T.bin ? 1 : 0;
      R = 1 - L;
    } else {
      L = side[i];
      R = 1 - L;
    }
  }
  lr[i] = ((uint64_t)L << 32) | R;
  fin[i] = F;
}

__device__ __forceinline__ uint32_t out_base(const uint64_t* slr, const uint32_t* sfin, uint32_t i) {
  return sfin[i] + (uint32_t)(slr[i] >> 32) + (uint32_t)slr[i];
}

// (4) the child tasks' ranges (from the scans) and bin blocks
__global__ void k_sah_fix(const SahTask* task, int ntask, const uint64_t* slr, const uint32_t* sfin, SahTask* next,
                          uint32_t* counters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntask) return;
  const SahTask T = task[t];
  if (T.child < 0) return;
  const uint32_t b = T.begin, e = T.begin + T.count;
  const uint32_t base = out_base(slr, sfin, b);
  const uint32_t nL = (uint32_t)(slr[e] >> 32) - (uint32_t)(slr[b] >> 32), nR = (uint32_t)slr[e] - (uint32_t)slr[b];
  const uint32_t cnt[2] = {nL, nR};
  for (int q = 0; q < 2; q++) {
    SahTask& C = next[T.child + q];
    C.begin = base + (q ? nL : 0);
    C.count = cnt[q];
    C.big = cnt[q] > (uint32_t)kSahSmall ? (int32_t)atomicAdd(&counters[2], 1u) : -1;
  }
}

// (5) the next level's references: finished ones move by the scans, a splitting task's go left then right
// (a clipped straddler to both sides with its clipped boxes); a leaf of this level tags its references
__global__ void k_sah_scatter(const uint32_t* rface, const Box6* rbox, const int32_t* ptask, const SahTask* task,
                              const TriRec64* rec, const uint64_t* slr, const uint32_t* sfin, int m, uint32_t* rface_out,
                              Box6* rbox_out, int32_t* ptask_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const int t = ptask[i];
  if (t < 0 || task[t].child < 0) {
    const uint32_t o = out_base(slr, sfin, (uint32_t)i);
    rface_out[o] = rface[i];
    rbox_out[o] = rbox[i];
    ptask_out[o] = t < 0 ? t : ~task[t].bin;  // leaf id, as ~id
    return;
  }
  const SahTask T = task[t];
  const uint32_t b = T.begin, e = T.begin + T.count;
  const uint32_t base = out_base(slr, sfin, b);
  const uint32_t nL = (uint32_t)(slr[e] >> 32) - (uint32_t)(slr[b] >> 32);
  const uint32_t L = (uint32_t)(slr[i + 1] >> 32) - (uint32_t)(slr[i] >> 32), R = (uint32_t)slr[i + 1] - (uint32_t)slr[i];
  const Box6 r = rbox[i];
  Box6 bl = r, br = r;
  if (T.axis >= 3 && L && R) {
    const int k = T.axis - 3;
    const TriRec64 tr = rec[rface[i]];
    clip_tri(tr, k, r.lo[k], T.plane, r, bl);
    clip_tri(tr, k, T.plane, r.hi[k], r, br);
  }
  if (L) {
    const uint32_t o = base + (uint32_t)(slr[i] >> 32) - (uint32_t)(slr[b] >> 32);
    rface_out[o] = rface[i];
    rbox_out[o] = bl;
    ptask_out[o] = T.child;
  }
  if (R) {
    const uint32_t o = base + nL + (uint32_t)slr[i] - (uint32_t)slr[b];
    rface_out[o] = rface[i];
    rbox_out[o] = br;
    ptask_out[o] = T.child + 1;
  }
}
}  // namespace

// face_recs: one record per face (vertices = the culling bounds). Outputs: per interior node (root 0) its
// two child handles (interior node id, or make_leaf(first slot, count)) and unpadded child boxes, and the
// face of every triangle slot (leaves are contiguous slot ranges; with spatial splits a face may own
// several slots). spatial: SBVH with duplication budget `budget` x faces and overlap threshold alpha.
int gpu_build_sah(int device, const std::vector<TriRec64>& face_recs, const float lo[3], const float hi[3],
                  int leaf_size, float k_trav, bool spatial, float budget, float alpha, std::vector<uint32_t>& nchild,
                  std::vector<float>& ncb, std::vector<uint32_t>& slot_face, double* gpu_ms, int* levels) {
  const int n = (int)face_recs.size();
  if (n < 2) { set_error("gpu_build_sah: needs at least 2 triangles"); return RT_ERR_INVALID; }
  const size_t N = (size_t)n;
  const size_t cap = std::min<size_t>(spatial ? N + (size_t)(budget * (double)N) + 1 : N, (size_t)kMaxFaces);
  if (cap < N) { set_error("gpu_build_sah: too many faces"); return RT_ERR_INVALID; }
  BCHECK(hipSetDevice(device));
  PhaseTimer pt("gpu_build_sah");
  hipStream_t st;
  st = (hipStream_t)build_stream(device);
  if (!st) return RT_ERR_HIP;
  struct Guard {
    hipStream_t st;
    std::vector<void*> bufs;
    std::vector<hipEvent_t> evs;  // released on every return (the fallback paths included)
    ~Guard() {
      (void)hipStreamSynchronize(st);
      for (void* b : bufs) (void)hipFree(b);
      for (hipEvent_t e : evs) (void)hipEventDestroy(e);
    }
  } g{st, {}, {}};
  auto alloc = [&](void** p, size_t bytes) -> hipError_t {
    hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 16));
    if (e == hipSuccess) g.bufs.push_back(*p);
    return e;
  };
  const size_t maxbig = cap / kSahSmall + 2, objw = 3 * kSahBins * kObjW, spw = 3 * kSahBins * kSpW;
  TriRec64* d_rec = nullptr;
  uint64_t *d_k0 = nullptr, *d_k1 = nullptr, *d_lr = nullptr, *d_slr = nullptr;
  Box6 *d_rbox[2] = {nullptr, nullptr}, *d_ncb = nullptr;
  uint32_t *d_rface[2] = {nullptr, nullptr}, *d_stat = nullptr, *d_bins = nullptr, *d_spbins = nullptr;
  uint32_t *d_fin = nullptr, *d_sfin = nullptr, *d_cnt = nullptr, *d_nchild = nullptr;
  int32_t* d_pt[2] = {nullptr, nullptr};
  SahTask* d_task[2] = {nullptr, nullptr};
  uint8_t* d_side = nullptr;
  BCHECK(alloc((void**)&d_rec, N * sizeof(TriRec64)));
  BCHECK(alloc((void**)&d_k0, N * 8));
  BCHECK(alloc((void**)&d_k1, N * 8));
  BCHECK(alloc((void**)&d_ncb, 2 * cap * sizeof(Box6)));
  BCHECK(alloc((void**)&d_nchild, 2 * cap * 4));
  for (int q = 0; q < 2; q++) {
    BCHECK(alloc((void**)&d_rface[q], cap * 4));
    BCHECK(alloc((void**)&d_rbox[q], cap * sizeof(Box6)));
    BCHECK(alloc((void**)&d_pt[q], cap * 4));
    BCHECK(alloc((void**)&d_task[q], cap * sizeof(SahTask)));
  }
  BCHECK(alloc((void**)&d_stat, cap * 12 * 4));
  BCHECK(alloc((void**)&d_bins, maxbig * objw * 4));
  if (spatial) BCHECK(alloc((void**)&d_spbins, maxbig * spw * 4));
  BCHECK(alloc((void**)&d_lr, (cap + 1) * 8));
  BCHECK(alloc((void**)&d_slr, (cap + 1) * 8));
  BCHECK(alloc((void**)&d_fin, (cap + 1) * 4));
  BCHECK(alloc((void**)&d_sfin, (cap + 1) * 4));
  BCHECK(alloc((void**)&d_side, cap));
  BCHECK(alloc((void**)&d_cnt, 32));
  pt.mark("alloc");
  if (int rc = h2d(d_rec, face_recs.data(), N * sizeof(TriRec64))) return rc;  // pinned staging
  pt.mark("h2d_records");
  hipEvent_t e0, e1;
  BCHECK(hipEventCreate(&e0));
  g.evs.push_back(e0);
  BCHECK(hipEventCreate(&e1));
  g.evs.push_back(e1);
  BCHECK(hipEventRecord(e0, st));
  const int B = kSahBlock;
  auto grid = [&](size_t k) { return dim3((unsigned)((k + B - 1) / B)); };
  float3 flo = make_float3(lo[0], lo[1], lo[2]), fsc;
  fsc.x = hi[0] > lo[0] ? 1024.0f / (hi[0] - lo[0]) : 0.0f;
  fsc.y = hi[1] > lo[1] ? 1024.0f / (hi[1] - lo[1]) : 0.0f;
  fsc.z = hi[2] > lo[2] ? 1024.0f / (hi[2] - lo[2]) : 0.0f;
  hipLaunchKernelGGL(k_morton, grid(N), dim3(B), 0, st, (const TriRec64*)d_rec, n, flo, fsc, d_k0);
  size_t tb = 0, ts1 = 0, ts2 = 0;
  BCHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, d_k0, d_k1, n, 0, 64, st));
  BCHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, ts1, d_lr, d_slr, (int)(cap + 1), st));
  BCHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, ts2, d_fin, d_sfin, (int)(cap + 1), st));
  void* d_tmp = nullptr;
  BCHECK(alloc(&d_tmp, std::max(tb, std::max(ts1, ts2))));
  BCHECK(hipcub::DeviceRadixSort::SortKeys(d_tmp, tb, d_k0, d_k1, n, 0, 64, st));
  hipLaunchKernelGGL(k_sah_init, grid(N), dim3(B), 0, st, (const uint64_t*)d_k1, (const TriRec64*)d_rec, n, d_rface[0],
                     d_rbox[0], d_pt[0]);
  SahTask root{};
  root.begin = 0;
  root.count = (uint32_t)n;
  root.parent_slot = -1;
  root.big = n > kSahSmall ? 0 : -1;
  root.sp = -1;
  root.child = -1;
  root.axis = root.bin = -1;
  root.budget = (int32_t)(cap - N);
  BCHECK(hipMemcpyAsync(d_task[0], &root, sizeof root, hipMemcpyHostToDevice, st));
  float root_area;
  {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    root_area = std::max(dx * dy + dy * dz + dz * dx, 1e-30f);
  }
  int ntask = 1, nbig = n > kSahSmall ? 1 : 0, cur = 0, level = 0;
  uint32_t nodes = 1, leaves = 0, m = (uint32_t)n;
  const int lb = std::max(1, std::min(leaf_size, kMaxLeaf));
  while (ntask > 0) {
    if (level > 4 * kMaxDepth) { set_error("gpu_build_sah: no progress"); return RT_ERR_INVALID; }
    const int force = level >= kMaxDepth - 20 ? 1 : 0;
    uint32_t cinit[8] = {0, nodes, 0, 0, leaves, 0, 0, 0};
    BCHECK(hipMemcpyAsync(d_cnt, cinit, 32, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_sah_stat_init, grid(ntask), dim3(B), 0, st, d_stat, ntask);
    if (nbig)
      hipLaunchKernelGGL(k_sah_bins_init, grid((size_t)nbig * 3 * kSahBins), dim3(B), 0, st, d_bins, nbig * 3 * kSahBins, kObjW);
    hipLaunchKernelGGL(k_sah_bounds, grid(m), dim3(B), 0, st, (const Box6*)d_rbox[cur], (const int32_t*)d_pt[cur], (int)m, d_stat);
    if (nbig)
      hipLaunchKernelGGL(k_sah_bin, grid(m), dim3(B), 0, st, (const Box6*)d_rbox[cur], (const int32_t*)d_pt[cur],
                         (const SahTask*)d_task[cur], (const uint32_t*)d_stat, (int)m, d_bins);
    hipLaunchKernelGGL(k_sah_split_obj, grid(ntask), dim3(B), 0, st, d_task[cur], ntask, (const uint32_t*)d_stat,
                       (const uint32_t*)d_bins, d_cnt, root_area, alpha, spatial ? 1 : 0, force);
    if (spatial && nbig) {
      uint32_t nsp = 0;
      BCHECK(hipMemcpyAsync(&nsp, d_cnt + 3, 4, hipMemcpyDeviceToHost, st));
      BCHECK(hipStreamSynchronize(st));
      if (nsp > maxbig) { set_error("gpu_build_sah: spatial task bound exceeded"); return RT_ERR_INVALID; }
      if (nsp) {
        hipLaunchKernelGGL(k_sah_bins_init, grid((size_t)nsp * 3 * kSahBins), dim3(B), 0, st, d_spbins, (int)nsp * 3 * kSahBins, kSpW);
        hipLaunchKernelGGL(k_sah_spbin, grid(m), dim3(B), 0, st, (const uint32_t*)d_rface[cur], (const Box6*)d_rbox[cur],
                           (const int32_t*)d_pt[cur], (const SahTask*)d_task[cur], (const uint32_t*)d_stat,
                           (const TriRec64*)d_rec, (int)m, d_spbins);
      }
    }
    hipLaunchKernelGGL(k_sah_split, grid(ntask), dim3(B), 0, st, d_task[cur], ntask, (const uint32_t*)d_stat,
                       (const uint32_t*)d_spbins, (const Box6*)d_rbox[cur], d_side, d_task[1 - cur], d_cnt, d_nchild,
                       d_ncb, lb, k_trav, force);
    hipLaunchKernelGGL(k_sah_side, grid(m + 1), dim3(B), 0, st, (const uint32_t*)d_rface[cur], (const Box6*)d_rbox[cur],
                       (const int32_t*)d_pt[cur], (const SahTask*)d_task[cur], (const uint32_t*)d_stat,
                       (const TriRec64*)d_rec, (const uint8_t*)d_side, (int)m, d_lr, d_fin);
    BCHECK(hipcub::DeviceScan::ExclusiveSum(d_tmp, ts1, d_lr, d_slr, (int)(m + 1), st));
    BCHECK(hipcub::DeviceScan::ExclusiveSum(d_tmp, ts2, d_fin, d_sfin, (int)(m + 1), st));
    hipLaunchKernelGGL(k_sah_fix, grid(ntask), dim3(B), 0, st, (const SahTask*)d_task[cur], ntask, (const uint64_t*)d_slr,
                       (const uint32_t*)d_sfin, d_task[1 - cur], d_cnt);
    uint64_t slr_m = 0;
    uint32_t sfin_m = 0;
    BCHECK(hipMemcpyAsync(&slr_m, d_slr + m, 8, hipMemcpyDeviceToHost, st));
    BCHECK(hipMemcpyAsync(&sfin_m, d_sfin + m, 4, hipMemcpyDeviceToHost, st));
    BCHECK(hipStreamSynchronize(st));
    const uint32_t m_next = sfin_m + (uint32_t)(slr_m >> 32) + (uint32_t)slr_m;
    if (m_next > cap || m_next < m) { set_error("gpu_build_sah: reference bound exceeded"); return RT_ERR_INVALID; }
    hipLaunchKernelGGL(k_sah_scatter, grid(m), dim3(B), 0, st, (const uint32_t*)d_rface[cur], (const Box6*)d_rbox[cur],
                       (const int32_t*)d_pt[cur], (const SahTask*)d_task[cur], (const TriRec64*)d_rec,
                       (const uint64_t*)d_slr, (const uint32_t*)d_sfin, (int)m, d_rface[1 - cur], d_rbox[1 - cur],
                       d_pt[1 - cur]);
    BCHECK(hipGetLastError());
    uint32_t cnt[8];
    BCHECK(hipMemcpyAsync(cnt, d_cnt, 32, hipMemcpyDeviceToHost, st));
    BCHECK(hipStreamSynchronize(st));
    ntask = (int)cnt[0];
    nodes = cnt[1];
    nbig = (int)cnt[2];
    leaves = cnt[4];
    m = m_next;
    if ((size_t)nbig > maxbig || nodes > cap || (size_t)ntask > cap) { set_error("gpu_build_sah: task bound exceeded"); return RT_ERR_INVALID; }
    cur = 1 - cur;
    level++;
  }
  BCHECK(hipEventRecord(e1, st));
  std::vector<int32_t> ptag(m);
  nchild.resize(2 * (size_t)nodes);
  ncb.resize(12 * (size_t)nodes);
  slot_face.resize(m);
  BCHECK(hipStreamSynchronize(st));
  pt.mark("levels");
  if (int rc = d2h(nchild.data(), d_nchild, 2 * (size_t)nodes * 4)) return rc;  // pinned staging
  if (int rc = d2h(ncb.data(), d_ncb, 2 * (size_t)nodes * sizeof(Box6))) return rc;
  if (int rc = d2h(slot_face.data(), d_rface[cur], (size_t)m * 4)) return rc;
  if (int rc = d2h(ptag.data(), d_pt[cur], (size_t)m * 4)) return rc;
  pt.mark("d2h");
  float ms = 0.0f;
  BCHECK(hipEventElapsedTime(&ms, e0, e1));
  if (gpu_ms) *gpu_ms = ms;
  if (levels) *levels = level;
  // leaves: each leaf id's references are one contiguous run of the final order
  std::vector<uint32_t> first(leaves, UINT32_MAX), count(leaves, 0);
  for (uint32_t i = 0; i < m; i++) {
    const int32_t tg = ptag[i];
    const uint32_t id = (uint32_t)~tg;
    if (tg >= 0 || id >= leaves) { set_error("gpu_build_sah: unfinished reference"); return RT_ERR_INVALID; }
    if (first[id] == UINT32_MAX) first[id] = i;
    else if (first[id] + count[id] != i) { set_error("gpu_build_sah: leaf %u not contiguous", id); return RT_ERR_INVALID; }
    count[id]++;
  }
  for (uint32_t& h : nchild) {
    if (!(h & 0x80000000u)) continue;
    const uint32_t id = h & 0x7FFFFFFFu;
    if (id >= leaves || count[id] == 0 || count[id] > (uint32_t)kMaxLeaf) { set_error("gpu_build_sah: bad leaf %u", id); return RT_ERR_INVALID; }
    h = make_leaf(first[id], count[id]);
  }
  return RT_OK;
}

}  // namespace rt
