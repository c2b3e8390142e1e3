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
  BCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct Guard {
    hipStream_t st;
    std::vector<void*> bufs;
    ~Guard() {
      (void)hipStreamSynchronize(st);
      for (void* b : bufs) (void)hipFree(b);
      (void)hipStreamDestroy(st);
    }
  } g{st, {}};
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
  BCHECK(hipMemcpyAsync(d_rec, face_recs.data(), (size_t)n * sizeof(TriRec64), hipMemcpyHostToDevice, st));
  BCHECK(hipMemsetAsync(d_flags, 0, (size_t)n * 4, st));
  hipEvent_t e0, e1;
  BCHECK(hipEventCreate(&e0));
  BCHECK(hipEventCreate(&e1));
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
  BCHECK(hipMemcpyAsync(nodes.data(), d_nodes, (size_t)(n - 1) * sizeof(Node64), hipMemcpyDeviceToHost, st));
  BCHECK(hipMemcpyAsync(tris.data(), d_tris, (size_t)n * sizeof(TriRec64), hipMemcpyDeviceToHost, st));
  BCHECK(hipStreamSynchronize(st));
  float ms = 0.0f;
  BCHECK(hipEventElapsedTime(&ms, e0, e1));
  if (gpu_ms) *gpu_ms = ms;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
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
  BCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct Guard {
    hipStream_t st;
    std::vector<void*> bufs;
    ~Guard() {
      (void)hipStreamSynchronize(st);
      for (void* b : bufs) (void)hipFree(b);
      (void)hipStreamDestroy(st);
    }
  } g{st, {}};
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
  BCHECK(hipMemcpyAsync(d_rec, face_recs.data(), (size_t)n * sizeof(TriRec64), hipMemcpyHostToDevice, st));
  BCHECK(hipMemsetAsync(d_pint, 0xFF, (size_t)n * 4, st));  // the root's parent: -1
  BCHECK(hipMemsetAsync(d_cflags, 0, (size_t)n * 4, st));
  hipEvent_t e0, e1;
  BCHECK(hipEventCreate(&e0));
  BCHECK(hipEventCreate(&e1));
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
  BCHECK(hipMemcpyAsync(child2.data(), d_child, (size_t)(n - 1) * sizeof(int2), hipMemcpyDeviceToHost, st));
  BCHECK(hipMemcpyAsync(box6.data(), d_nbox, (size_t)(n - 1) * sizeof(Box6), hipMemcpyDeviceToHost, st));
  BCHECK(hipMemcpyAsync(leaf.data(), d_leaf, (size_t)(n - 1), hipMemcpyDeviceToHost, st));
  BCHECK(hipStreamSynchronize(st));
  float ms = 0.0f;
  BCHECK(hipEventElapsedTime(&ms, e0, e1));
  if (gpu_ms) *gpu_ms = ms;
  if (iterations) *iterations = iters;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return RT_OK;
}


// ---------------------------------------------------------------------------------------------------
// Top-down binned SAH on the GPU (RT_BUILDER_SAH_GPU): the host SAH builder's algorithm -- 32 centroid
// bins per axis, cost k_trav * A + sum(n_side * A_side), leaf when <= leaf_size triangles and no costlier
// -- run breadth first, one level of the tree per round of launches. Triangles keep their Morton order
// inside every node's contiguous range (stable partition by one scan), so small tasks stay coherent.
//   per level: (1) every active task's box and centroid bounds: a segmented wave reduction over its
//   contiguous positions, one atomic per segment and wave; (2) tasks above kSahSmall triangles: centroid
//   bins (ordered-uint atomics; a block whose 256 positions belong to one task bins in LDS first);
//   (3) one thread per task picks the split: the bins' sweep for big tasks, an exact sweep over the sorted
//   centroids (<= kSahSmall) for small ones, the object median when the centroids are degenerate or the
//   depth is near the stack bound; a leaf writes its handle into its parent, a split allocates its node
//   and two child tasks; (4) the side of every position; (5) one exclusive scan and a scatter.
// ---------------------------------------------------------------------------------------------------
namespace {
constexpr int kSahBins = 32, kSahSmall = 16, kSahBlock = 256;

struct SahTask {
  uint32_t begin, count;
  int32_t parent_slot;  // 2 * parent node + side, -1 for the root
  int32_t big;          // bin block index (count > kSahSmall) or -1
  int32_t child;        // first child task of the next level, -1 for a leaf
  int32_t axis, bin;    // split: axis and last left bin (bin -1: position median / exact sweep sides)
  uint32_t nleft;
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
__device__ __forceinline__ int sah_bin(float c, float lo, float sc) {
  return min(kSahBins - 1, (int)((c - lo) * sc));
}

__global__ void k_sah_init(const uint64_t* keys, const TriRec64* rec, int n, Box6* pbox, uint32_t* idx, int32_t* ptask) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t f = (uint32_t)keys[i];
  pbox[f] = tri_box(rec[f]);
  idx[i] = f;
  ptask[i] = 0;
}

__global__ void k_sah_stat_init(uint32_t* stat, int ntask) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntask) return;
  uint32_t* s = stat + 12 * (size_t)t;
  for (int k = 0; k < 12; k++) s[k] = (k < 3 || (k >= 6 && k < 9)) ? 0xFFFFFFFFu : 0u;
}
__global__ void k_sah_bins_init(uint32_t* bins, int nbig) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nbig * 3 * kSahBins) return;
  uint32_t* d = bins + 7 * (size_t)b;
  for (int q = 0; q < 7; q++) d[q] = q < 3 ? 0xFFFFFFFFu : 0u;
}

// (1) box and centroid bounds of every active task (stat[t]: 12 ordered uints: box lo, box hi, cen lo, cen hi)
__global__ __launch_bounds__(kSahBlock) void k_sah_bounds(const Box6* pbox, const uint32_t* idx, const int32_t* ptask,
                                                         int n, uint32_t* stat) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int t = i < n ? ptask[i] : -1;
  uint32_t v[12];
  if (t >= 0) {
    const Box6 b = pbox[idx[i]];
    for (int k = 0; k < 3; k++) {
      v[k] = f2o(b.lo[k]);
      v[3 + k] = f2o(b.hi[k]);
      v[6 + k] = v[9 + k] = f2o(cen(b, k));
    }
  } else {
    for (int k = 0; k < 12; k++) v[k] = 0;
  }
  // segmented inclusive scan (min for the lo halves, max for the hi halves) over equal task ids
  for (int off = 1; off < 64; off <<= 1) {
    const int tu = __shfl_up(t, off, 64);
    const bool take = lane >= off && tu == t;
    for (int k = 0; k < 12; k++) {
      const uint32_t u = __shfl_up(v[k], off, 64);
      const bool lo = (k < 3) || (k >= 6 && k < 9);
      if (take) v[k] = lo ? min(v[k], u) : max(v[k], u);
    }
  }
  const int tn = __shfl_down(t, 1, 64);
  if (t >= 0 && (lane == 63 || tn != t || i == n - 1)) {
    uint32_t* s = stat + 12 * (size_t)t;
    for (int k = 0; k < 12; k++) {
      const bool lo = (k < 3) || (k >= 6 && k < 9);
      if (lo) atomicMin(&s[k], v[k]); else atomicMax(&s[k], v[k]);
    }
  }
}

// (2) centroid bins of the big tasks: bins[big][axis][bin] = 7 uints (box lo, box hi ordered; count)
__global__ __launch_bounds__(kSahBlock) void k_sah_bin(const Box6* pbox, const uint32_t* idx, const int32_t* ptask,
                                                      const SahTask* task, const uint32_t* stat, int n, uint32_t* bins) {
  __shared__ uint32_t lb[3 * kSahBins * 7];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int first = blockIdx.x * blockDim.x, last = min(n - 1, first + kSahBlock - 1);
  const int t0 = ptask[first], t1 = ptask[last];
  const bool uniform_task = t0 == t1 && t0 >= 0 && task[t0].big >= 0;  // block-uniform
  const int t = i < n ? ptask[i] : -1;
  if (uniform_task) {
    for (int k = threadIdx.x; k < 3 * kSahBins * 7; k += kSahBlock) lb[k] = (k % 7) < 3 ? 0xFFFFFFFFu : 0u;
    __syncthreads();
  }
  if (t >= 0 && task[t].big >= 0) {
    const uint32_t* s = stat + 12 * (size_t)t;
    const Box6 b = pbox[idx[i]];
    const uint32_t bl[3] = {f2o(b.lo[0]), f2o(b.lo[1]), f2o(b.lo[2])}, bh[3] = {f2o(b.hi[0]), f2o(b.hi[1]), f2o(b.hi[2])};
    uint32_t* gb = bins + (size_t)task[t].big * 3 * kSahBins * 7;
    for (int k = 0; k < 3; k++) {
      const float clo = o2f(s[6 + k]), ext = o2f(s[9 + k]) - clo;
      if (!(ext > 0.0f)) continue;
      const int bi = sah_bin(cen(b, k), clo, kSahBins / ext);
      uint32_t* d = (uniform_task ? lb : gb) + (k * kSahBins + bi) * 7;
      for (int q = 0; q < 3; q++) { atomicMin(&d[q], bl[q]); atomicMax(&d[3 + q], bh[q]); }
      atomicAdd(&d[6], 1u);
    }
  }
  if (uniform_task) {
    __syncthreads();
    uint32_t* gb = bins + (size_t)task[t0].big * 3 * kSahBins * 7;
    for (int k = threadIdx.x; k < 3 * kSahBins; k += kSahBlock) {
      const uint32_t* d = lb + k * 7;
      if (d[6] == 0) continue;
      uint32_t* g = gb + k * 7;
      for (int q = 0; q < 3; q++) { atomicMin(&g[q], d[q]); atomicMax(&g[3 + q], d[3 + q]); }
      atomicAdd(&g[6], d[6]);
    }
  }
}

// (3) the split of every task of the level
__global__ void k_sah_split(SahTask* task, int ntask, const uint32_t* stat, const uint32_t* bins, const Box6* pbox,
                            const uint32_t* idx, uint8_t* side, SahTask* next, uint32_t* counters, uint32_t* nchild,
                            Box6* ncb, int leaf_size, float k_trav, int force_median) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntask) return;
  SahTask T = task[t];
  const uint32_t* s = stat + 12 * (size_t)t;
  Box6 box;
  float clo[3], ext[3];
  for (int k = 0; k < 3; k++) {
    box.lo[k] = o2f(s[k]);
    box.hi[k] = o2f(s[3 + k]);
    clo[k] = o2f(s[6 + k]);
    ext[k] = o2f(s[9 + k]) - clo[k];
  }
  const uint32_t n = T.count;
  const float A = fmaxf(sah_area(box.lo, box.hi), 1e-30f);
  float best = INFINITY;
  int axis = -1, bin = -1;
  uint32_t nl = 0;
  bool exact = false;  // small task: sides written here from the sorted order
  int ord[kSahSmall];
  if (!force_median && T.big >= 0) {
    const uint32_t* B = bins + (size_t)T.big * 3 * kSahBins * 7;
    for (int k = 0; k < 3; k++) {
      if (!(ext[k] > 0.0f)) continue;
      float rarea[kSahBins];
      uint32_t rcnt[kSahBins];
      float alo[3] = {INFINITY, INFINITY, INFINITY}, ahi[3] = {-INFINITY, -INFINITY, -INFINITY};
      uint32_t c = 0;
      for (int i = kSahBins - 1; i > 0; i--) {
        const uint32_t* d = B + (k * kSahBins + i) * 7;
        if (d[6]) for (int q = 0; q < 3; q++) { alo[q] = fminf(alo[q], o2f(d[q])); ahi[q] = fmaxf(ahi[q], o2f(d[3 + q])); }
        c += d[6];
        rarea[i] = c ? sah_area(alo, ahi) : 0.0f;
        rcnt[i] = c;
      }
      float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
      uint32_t lc = 0;
      for (int i = 0; i < kSahBins - 1; i++) {
        const uint32_t* d = B + (k * kSahBins + i) * 7;
        if (d[6]) for (int q = 0; q < 3; q++) { llo[q] = fminf(llo[q], o2f(d[q])); lhi[q] = fmaxf(lhi[q], o2f(d[3 + q])); }
        lc += d[6];
        if (lc == 0 || rcnt[i + 1] == 0) continue;
        const float cost = sah_area(llo, lhi) * lc + rarea[i + 1] * rcnt[i + 1];
        if (cost < best) { best = cost; axis = k; bin = i; nl = lc; }
      }
    }
  } else if (!force_median && n >= 2) {
    // exact sweep over the centroids sorted along each axis (insertion sort by centroid, position order for ties)
    Box6 pb[kSahSmall];
    for (uint32_t j = 0; j < n; j++) pb[j] = pbox[idx[T.begin + j]];
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
      float alo[3] = {INFINITY, INFINITY, INFINITY}, ahi[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (int j = (int)n - 1; j > 0; j--) {
        for (int q = 0; q < 3; q++) { alo[q] = fminf(alo[q], pb[o[j]].lo[q]); ahi[q] = fmaxf(ahi[q], pb[o[j]].hi[q]); }
        rarea[j] = sah_area(alo, ahi);
      }
      float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (uint32_t j = 0; j + 1 < n; j++) {
        for (int q = 0; q < 3; q++) { llo[q] = fminf(llo[q], pb[o[j]].lo[q]); lhi[q] = fmaxf(lhi[q], pb[o[j]].hi[q]); }
        const float cost = sah_area(llo, lhi) * (float)(j + 1) + rarea[j + 1] * (float)(n - 1 - j);
        if (cost < best) {
          best = cost; axis = k; nl = j + 1; exact = true;
          for (uint32_t q = 0; q < n; q++) ord[q] = o[q];
        }
      }
    }
  }
  // the host builders' rule (rt_host.cpp BvhBuilder::build): a leaf when n <= leaf_size and no split is
  // cheaper (or none exists, or the depth forces medians); degenerate centroids make a leaf of <= kMaxLeaf
  // triangles; the root always splits (its handle has no parent slot)
  const bool degenerate = !(ext[0] > 0.0f || ext[1] > 0.0f || ext[2] > 0.0f);
  bool leaf = n == 1;
  if (!leaf && (int)n <= leaf_size) leaf = force_median || axis < 0 || (float)n <= k_trav + best / A;
  if (!leaf && axis < 0 && degenerate && (int)n <= kMaxLeaf) leaf = true;
  if (T.parent_slot < 0) leaf = false;
  if (leaf) {
    T.child = -1;
    task[t] = T;
    const uint32_t h = make_leaf(T.begin, n);
    if (T.parent_slot >= 0) { nchild[T.parent_slot] = h; ncb[T.parent_slot] = box; }
    return;
  }
  if (axis < 0) { bin = -1; nl = n / 2; exact = false; }  // object median by position (Morton order)
  const uint32_t node = T.parent_slot < 0 ? 0u : atomicAdd(&counters[1], 1u);
  if (T.parent_slot >= 0) { nchild[T.parent_slot] = node; ncb[T.parent_slot] = box; }
  const uint32_t c = atomicAdd(&counters[0], 2u);
  const uint32_t cnt[2] = {nl, n - nl};
  for (int q = 0; q < 2; q++) {
    SahTask C;
    C.begin = T.begin + (q ? nl : 0);
    C.count = cnt[q];
    C.parent_slot = (int32_t)(2 * node + q);
    C.big = C.count > (uint32_t)kSahSmall ? (int32_t)atomicAdd(&counters[2], 1u) : -1;
    C.child = -1;
    C.axis = -1;
    C.bin = -1;
    C.nleft = 0;
    next[c + q] = C;
  }
  T.child = (int32_t)c;
  T.axis = exact ? -2 : axis;  // -2: sides written here
  T.bin = bin;
  T.nleft = nl;
  task[t] = T;
  if (exact) {
    for (uint32_t q = 0; q < n; q++) side[T.begin + ord[q]] = q < nl ? 1 : 0;
  }
}

// (4) sides of the bin / median splits, and the scan flags (1: left side of a splitting task)
__global__ void k_sah_side(const Box6* pbox, const uint32_t* idx, const int32_t* ptask, const SahTask* task,
                           const uint32_t* stat, int n, uint8_t* side, uint32_t* flag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = ptask[i];
  uint32_t f = 0;
  if (t >= 0) {
    const SahTask T = task[t];
    if (T.child >= 0) {
      if (T.axis >= 0) {
        const uint32_t* s = stat + 12 * (size_t)t;
        const float clo = o2f(s[6 + T.axis]), ext = o2f(s[9 + T.axis]) - clo;
        f = sah_bin(cen(pbox[idx[i]], T.axis), clo, kSahBins / ext) <= T.bin ? 1u : 0u;
      } else if (T.axis == -1) {
        f = (uint32_t)(i - (int)T.begin) < T.nleft ? 1u : 0u;
      } else {
        f = side[i];
      }
    }
  }
  flag[i] = f;
}

// (5) stable partition of every splitting task's range; positions of leaves keep their place
__global__ void k_sah_scatter(const uint32_t* idx, const int32_t* ptask, const SahTask* task, const uint32_t* flag,
                              const uint32_t* scan, int n, uint32_t* idx_out, int32_t* ptask_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = ptask[i];
  if (t < 0 || task[t].child < 0) {
    idx_out[i] = idx[i];
    ptask_out[i] = -1;
    return;
  }
  const SahTask T = task[t];
  const uint32_t r = scan[i] - scan[T.begin];  // left positions of this task before i
  const uint32_t np = flag[i] ? T.begin + r : T.begin + T.nleft + ((uint32_t)i - T.begin - r);
  idx_out[np] = idx[i];
  ptask_out[np] = T.child + (flag[i] ? 0 : 1);
}
}  // namespace

// face_recs: one record per face (vertices = the culling bounds). Outputs: per interior node (root 0) its
// two child handles (interior node id, or make_leaf(first slot, count)) and unpadded child boxes, and the
// face of every triangle slot (leaves are contiguous slot ranges).
int gpu_build_sah(int device, const std::vector<TriRec64>& face_recs, const float lo[3], const float hi[3],
                  int leaf_size, float k_trav, std::vector<uint32_t>& nchild, std::vector<float>& ncb,
                  std::vector<uint32_t>& slot_face, double* gpu_ms, int* levels) {
  const int n = (int)face_recs.size();
  if (n < 2) { set_error("gpu_build_sah: needs at least 2 triangles"); return RT_ERR_INVALID; }
  BCHECK(hipSetDevice(device));
  hipStream_t st;
  BCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct Guard {
    hipStream_t st;
    std::vector<void*> bufs;
    ~Guard() {
      (void)hipStreamSynchronize(st);
      for (void* b : bufs) (void)hipFree(b);
      (void)hipStreamDestroy(st);
    }
  } g{st, {}};
  auto alloc = [&](void** p, size_t bytes) -> hipError_t {
    hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 16));
    if (e == hipSuccess) g.bufs.push_back(*p);
    return e;
  };
  const size_t N = (size_t)n, maxbig = N / kSahSmall + 2, binw = 3 * kSahBins * 7;
  TriRec64* d_rec = nullptr;
  uint64_t *d_k0 = nullptr, *d_k1 = nullptr;
  Box6 *d_pbox = nullptr, *d_ncb = nullptr;
  uint32_t *d_idx[2] = {nullptr, nullptr}, *d_stat = nullptr, *d_bins = nullptr, *d_flag = nullptr, *d_scan = nullptr;
  uint32_t *d_cnt = nullptr, *d_nchild = nullptr;
  int32_t* d_pt[2] = {nullptr, nullptr};
  SahTask* d_task[2] = {nullptr, nullptr};
  uint8_t* d_side = nullptr;
  BCHECK(alloc((void**)&d_rec, N * sizeof(TriRec64)));
  BCHECK(alloc((void**)&d_k0, N * 8));
  BCHECK(alloc((void**)&d_k1, N * 8));
  BCHECK(alloc((void**)&d_pbox, N * sizeof(Box6)));
  BCHECK(alloc((void**)&d_ncb, 2 * N * sizeof(Box6)));
  BCHECK(alloc((void**)&d_nchild, 2 * N * 4));
  for (int q = 0; q < 2; q++) {
    BCHECK(alloc((void**)&d_idx[q], N * 4));
    BCHECK(alloc((void**)&d_pt[q], N * 4));
    BCHECK(alloc((void**)&d_task[q], N * sizeof(SahTask)));
  }
  BCHECK(alloc((void**)&d_stat, N * 12 * 4));
  BCHECK(alloc((void**)&d_bins, maxbig * binw * 4));
  BCHECK(alloc((void**)&d_flag, N * 4));
  BCHECK(alloc((void**)&d_scan, N * 4));
  BCHECK(alloc((void**)&d_side, N));
  BCHECK(alloc((void**)&d_cnt, 16));
  BCHECK(hipMemcpyAsync(d_rec, face_recs.data(), N * sizeof(TriRec64), hipMemcpyHostToDevice, st));
  hipEvent_t e0, e1;
  BCHECK(hipEventCreate(&e0));
  BCHECK(hipEventCreate(&e1));
  BCHECK(hipEventRecord(e0, st));
  const int B = kSahBlock, G = (n + B - 1) / B;
  float3 flo = make_float3(lo[0], lo[1], lo[2]), fsc;
  fsc.x = hi[0] > lo[0] ? 1024.0f / (hi[0] - lo[0]) : 0.0f;
  fsc.y = hi[1] > lo[1] ? 1024.0f / (hi[1] - lo[1]) : 0.0f;
  fsc.z = hi[2] > lo[2] ? 1024.0f / (hi[2] - lo[2]) : 0.0f;
  hipLaunchKernelGGL(k_morton, dim3(G), dim3(B), 0, st, (const TriRec64*)d_rec, n, flo, fsc, d_k0);
  size_t tb = 0, tscan = 0;
  BCHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, d_k0, d_k1, n, 0, 64, st));
  BCHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tscan, d_flag, d_scan, n, st));
  void* d_tmp = nullptr;
  BCHECK(alloc(&d_tmp, std::max(tb, tscan)));
  BCHECK(hipcub::DeviceRadixSort::SortKeys(d_tmp, tb, d_k0, d_k1, n, 0, 64, st));
  hipLaunchKernelGGL(k_sah_init, dim3(G), dim3(B), 0, st, (const uint64_t*)d_k1, (const TriRec64*)d_rec, n, d_pbox,
                     d_idx[0], d_pt[0]);
  SahTask root{0u, (uint32_t)n, -1, n > kSahSmall ? 0 : -1, -1, -1, -1, 0u};
  BCHECK(hipMemcpyAsync(d_task[0], &root, sizeof root, hipMemcpyHostToDevice, st));
  int ntask = 1, nbig = n > kSahSmall ? 1 : 0, cur = 0, level = 0;
  uint32_t nodes = 1;
  const int lb = std::max(1, std::min(leaf_size, kMaxLeaf));
  while (ntask > 0) {
    if (level > 4 * kMaxDepth) { set_error("gpu_build_sah: no progress"); return RT_ERR_INVALID; }
    // stats: lo halves start at all-ones, hi halves at 0 (ordered uints)
    hipLaunchKernelGGL(k_sah_stat_init, dim3((ntask + 255) / 256), dim3(256), 0, st, d_stat, ntask);
    if (nbig) hipLaunchKernelGGL(k_sah_bins_init, dim3((nbig * 3 * kSahBins + 255) / 256), dim3(256), 0, st, d_bins, nbig);
    hipLaunchKernelGGL(k_sah_bounds, dim3(G), dim3(B), 0, st, (const Box6*)d_pbox, (const uint32_t*)d_idx[cur],
                       (const int32_t*)d_pt[cur], n, d_stat);
    if (nbig)
      hipLaunchKernelGGL(k_sah_bin, dim3(G), dim3(B), 0, st, (const Box6*)d_pbox, (const uint32_t*)d_idx[cur],
                         (const int32_t*)d_pt[cur], (const SahTask*)d_task[cur], (const uint32_t*)d_stat, n, d_bins);
    BCHECK(hipMemsetAsync(d_cnt, 0, 16, st));
    const uint32_t init_nodes[1] = {nodes};
    BCHECK(hipMemcpyAsync(d_cnt + 1, init_nodes, 4, hipMemcpyHostToDevice, st));
    const int force = level >= kMaxDepth - 20 ? 1 : 0;
    hipLaunchKernelGGL(k_sah_split, dim3((ntask + 127) / 128), dim3(128), 0, st, d_task[cur], ntask,
                       (const uint32_t*)d_stat, (const uint32_t*)d_bins, (const Box6*)d_pbox, (const uint32_t*)d_idx[cur],
                       d_side, d_task[1 - cur], d_cnt, d_nchild, d_ncb, lb, k_trav, force);
    hipLaunchKernelGGL(k_sah_side, dim3(G), dim3(B), 0, st, (const Box6*)d_pbox, (const uint32_t*)d_idx[cur],
                       (const int32_t*)d_pt[cur], (const SahTask*)d_task[cur], (const uint32_t*)d_stat, n, d_side, d_flag);
    BCHECK(hipcub::DeviceScan::ExclusiveSum(d_tmp, tscan, d_flag, d_scan, n, st));
    hipLaunchKernelGGL(k_sah_scatter, dim3(G), dim3(B), 0, st, (const uint32_t*)d_idx[cur], (const int32_t*)d_pt[cur],
                       (const SahTask*)d_task[cur], (const uint32_t*)d_flag, (const uint32_t*)d_scan, n, d_idx[1 - cur],
                       d_pt[1 - cur]);
    BCHECK(hipGetLastError());
    uint32_t cnt[4];
    BCHECK(hipMemcpyAsync(cnt, d_cnt, 16, hipMemcpyDeviceToHost, st));
    BCHECK(hipStreamSynchronize(st));
    ntask = (int)cnt[0];
    nodes = cnt[1];
    nbig = (int)cnt[2];
    if ((size_t)nbig > maxbig || nodes > N) { set_error("gpu_build_sah: task bound exceeded"); return RT_ERR_INVALID; }
    cur = 1 - cur;
    level++;
  }
  BCHECK(hipEventRecord(e1, st));
  nchild.resize(2 * (size_t)nodes);
  ncb.resize(12 * (size_t)nodes);
  slot_face.resize(N);
  BCHECK(hipMemcpyAsync(nchild.data(), d_nchild, 2 * (size_t)nodes * 4, hipMemcpyDeviceToHost, st));
  BCHECK(hipMemcpyAsync(ncb.data(), d_ncb, 2 * (size_t)nodes * sizeof(Box6), hipMemcpyDeviceToHost, st));
  BCHECK(hipMemcpyAsync(slot_face.data(), d_idx[cur], N * 4, hipMemcpyDeviceToHost, st));
  BCHECK(hipStreamSynchronize(st));
  float ms = 0.0f;
  BCHECK(hipEventElapsedTime(&ms, e0, e1));
  if (gpu_ms) *gpu_ms = ms;
  if (levels) *levels = level;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return RT_OK;
}

}  // namespace rt
