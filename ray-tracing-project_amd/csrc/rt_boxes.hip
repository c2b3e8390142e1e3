// rt_boxes.hip -- the reference's flat box partition on the GPU (second half):
// generateBoundingBoxes (flyscene.cpp:399-428) with BoundingBox::splitBox / averageVertexCoord /
// outsideFaces / fitFaces (BoundingBox.cpp:41-161), bit-exact.
//
// Layout: every box owns a contiguous segment of two permuted arrays, the faces' nine object-space
// vertex coordinates (36-B records, so every sweep over a box streams) and the face ids. Splitting a
// box is a stable partition of its segment: the faces that stay keep the front, the faces that move
// become the new box's segment right behind them. Box *indices* follow the reference's creation order
// (appended in box order within a pass), segments need not.
//
// One pass of the reference loop = one launch, one workgroup per box that still qualifies; the block
// runs splitBox's axis retries itself (no host round trip per attempt):
//   * averageVertexCoord is a sequential float sum (its rounding depends on the order), so one lane
//     adds every coordinate in face order while the other 15 waves stage the next chunk in LDS;
//   * hasFace / outsideFaces: block-wide count, then a stable scatter (ballot ranks + wave offsets);
//   * fitFaces: min / max over (value, position) pairs -- among equal values the first in face order
//     wins, as the reference's `if (x < min)` keeps it (only visible for -0.0 / +0.0).
// Vertices with non-finite coordinates are reported and the caller uses the host builder.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rt_scene.h"

#define XCHECK(expr)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) {                                                                   \
      rt::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
      return RT_ERR_HIP;                                                                      \
    }                                                                                         \
  } while (0)

namespace rt {
namespace {

constexpr int kBS = 1024;      // threads per box
constexpr int kWaves = kBS / 64;
constexpr int kChunk = 2048;   // faces per staged chunk of the sequential sum (2 x 24 KB LDS)

// one box of the partition (BoundingBox low / high / failed + its segment)
struct DBox {
  float low[3], high[3];
  int32_t start, count;
  int32_t failed[3];
  int32_t result;  // splitBox outcome: 1 = split (child written), -1 = every axis failed
};
static_assert(sizeof(DBox) == 48, "DBox layout");

struct Pair {
  float v;
  int32_t pos;
};
__device__ __forceinline__ Pair pmin(Pair a, Pair b) {
  if (b.v < a.v) return b;
  if (a.v < b.v) return a;
  return b.pos < a.pos ? b : a;
}
__device__ __forceinline__ Pair pmax(Pair a, Pair b) {
  if (b.v > a.v) return b;
  if (a.v > b.v) return a;
  return b.pos < a.pos ? b : a;
}
__device__ __forceinline__ Pair shfl_pair(Pair p, int m) {
  return Pair{__shfl_xor(p.v, m), __shfl_xor(p.pos, m)};
}

// fv[9 f + 3 k + a] = coordinate a of vertex k of face f (x, y, z as Tucano reads them); ids[f] = f
__global__ void k_gather(const float* v4, const uint32_t* fidx, int nf, float* fv, int32_t* ids, int32_t* nonfinite) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nf) return;
  bool bad = false;
  for (int k = 0; k < 3; k++) {
    const float* v = v4 + 4 * (size_t)fidx[3 * (size_t)f + k];
    for (int a = 0; a < 3; a++) {
      fv[9 * (size_t)f + 3 * k + a] = v[a];
      bad |= !isfinite(v[a]);
    }
  }
  ids[f] = f;
  if (bad) atomicOr(nonfinite, 1);
}

// block-wide reduction of 6 (value, position) pairs: min x,y,z then max x,y,z; result in `out` (all threads)
__device__ void block_fit(Pair (&p)[6], Pair (*red)[6], Pair (&out)[6]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int m = 32; m >= 1; m >>= 1)
    for (int j = 0; j < 6; j++) {
      const Pair q = shfl_pair(p[j], m);
      p[j] = j < 3 ? pmin(p[j], q) : pmax(p[j], q);
    }
  if (lane == 0)
    for (int j = 0; j < 6; j++) red[w][j] = p[j];
  __syncthreads();
  for (int j = 0; j < 6; j++) {
    Pair r = red[0][j];
    for (int q = 1; q < kWaves; q++) r = j < 3 ? pmin(r, red[q][j]) : pmax(r, red[q][j]);
    out[j] = r;
  }
  __syncthreads();
}

__device__ __forceinline__ void fit_acc(Pair (&p)[6], const float* r, int pos0) {
  for (int k = 0; k < 3; k++)
    for (int a = 0; a < 3; a++) {
      const Pair q{r[3 * k + a], pos0 + k};
      p[a] = pmin(p[a], q);
      p[3 + a] = pmax(p[3 + a], q);
    }
}
__device__ __forceinline__ void fit_init(Pair (&p)[6]) {
  for (int a = 0; a < 3; a++) {
    p[a] = Pair{INFINITY, INT32_MAX};
    p[3 + a] = Pair{-INFINITY, INT32_MAX};
  }
}

// fitMesh / fitFaces over the whole face list (the first box)
__global__ __launch_bounds__(kBS) void k_fit_all(const float* fv, int nf, DBox* box) {
  __shared__ Pair red[kWaves][6];
  Pair p[6];
  fit_init(p);
  for (int f = threadIdx.x; f < nf; f += kBS) {
    float r[9];
    for (int j = 0; j < 9; j++) r[j] = fv[9 * (size_t)f + j];
    fit_acc(p, r, 3 * f);
  }
  Pair out[6];
  block_fit(p, red, out);
  if (threadIdx.x == 0) {
    for (int a = 0; a < 3; a++) { box->low[a] = out[a].v; box->high[a] = out[3 + a].v; }
    box->start = 0;
    box->count = nf;
    box->failed[0] = box->failed[1] = box->failed[2] = 0;
    box->result = 0;
  }
}

__device__ __forceinline__ bool has_face(const float* r, const float lo[3], const float hi[3]) {
  bool in = true;
  for (int k = 0; k < 3; k++)
    in = in && r[3 * k] >= lo[0] && r[3 * k] <= hi[0] && r[3 * k + 1] >= lo[1] && r[3 * k + 1] <= hi[1] &&
         r[3 * k + 2] >= lo[2] && r[3 * k + 2] <= hi[2];
  return in;
}

// one pass of generateBoundingBoxes: block b runs `while (box == newBox) newBox = box->splitBox()` for
// todo box b. boxes[b] is updated in place; child[b] receives the new box when result == 1.
__global__ __launch_bounds__(kBS) void k_split_pass(DBox* boxes, DBox* child, float* fv, int32_t* ids, float* fv_tmp,
                                                    int32_t* ids_tmp) {
  __shared__ __align__(16) float stage[2][3 * kChunk];
  __shared__ Pair red[kWaves][6];
  __shared__ int32_t wcnt[kWaves];
  __shared__ float s_avg;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  DBox b = boxes[blockIdx.x];
  const int start = b.start, count = b.count;
  const float* seg = fv + 9 * (size_t)start;
  for (;;) {
    // splitBox's axis choice (BoundingBox.cpp:114-127); shape = high - low as reshape() stores it
    const float wd = b.high[0] - b.low[0], ht = b.high[1] - b.low[1], dp = b.high[2] - b.low[2];
    int choice;
    if ((wd >= ht || b.failed[1]) && (wd >= dp || b.failed[2]) && !b.failed[0]) choice = 0;
    else if ((ht >= wd || b.failed[0]) && (ht >= dp || b.failed[2]) && !b.failed[1]) choice = 1;
    else if (!(b.failed[0] && b.failed[1] && b.failed[2])) choice = 2;
    else {
      if (tid == 0) { b.result = -1; boxes[blockIdx.x] = b; }
      return;
    }
    // averageVertexCoord (BoundingBox.cpp:151-160): one lane, face order, v0 v1 v2 of each face
    {
      const int nchunks = (count + kChunk - 1) / kChunk;
      for (int q = tid; q < min(count, kChunk); q += kBS)
        for (int k = 0; k < 3; k++) stage[0][3 * q + k] = seg[9 * (size_t)q + 3 * k + choice];
      __syncthreads();
      float acc = 0.0f;
      for (int c = 0; c < nchunks; c++) {
        if (w != 0) {
          const int c1 = c + 1, base = c1 * kChunk, n1 = min(count - base, kChunk);
          float* dst = stage[c1 & 1];
          for (int q = tid - 64; q < n1; q += kBS - 64)
            for (int k = 0; k < 3; k++) dst[3 * q + k] = seg[9 * (size_t)(base + q) + 3 * k + choice];
        } else {
          // the whole wave adds the same sequence (broadcast LDS reads, uniform loop): 16 float4 reads in
          // flight, then 64 dependent adds in face order
          const int n = 3 * min(count - c * kChunk, kChunk);
          const float* src = stage[c & 1];
          int i = 0;
          for (; i + 64 <= n; i += 64) {
            float4 v[16];
#pragma unroll
            for (int u = 0; u < 16; u++) v[u] = *reinterpret_cast<const float4*>(src + i + 4 * u);
#pragma unroll
            for (int u = 0; u < 16; u++) {
              acc += v[u].x;
              acc += v[u].y;
              acc += v[u].z;
              acc += v[u].w;
            }
          }
          for (; i < n; i++) acc += src[i];
        }
        __syncthreads();
      }
      if (tid == 0) s_avg = acc / (float)(3ull * (unsigned long long)count);
      __syncthreads();
    }
    float hi2[3] = {b.high[0], b.high[1], b.high[2]};
    hi2[choice] = s_avg;
    // outsideFaces (BoundingBox.cpp:88-105) in one sweep: the faces that stay are written to the
    // scratch segment front to back, the faces that move back to front (both in face order), and both
    // halves are fitted on the way. An impossible split leaves the segment as it was.
    Pair pin[6], pout[6];
    fit_init(pin);
    fit_init(pout);
    int base_in = 0, base_out = 0;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int c0 = 0; c0 < count; c0 += kBS) {
      const int p = c0 + tid;
      const bool valid = p < count;
      float r[9];
      bool in = false;
      if (valid) {
        for (int j = 0; j < 9; j++) r[j] = seg[9 * (size_t)p + j];
        in = has_face(r, b.low, hi2);
      }
      const uint64_t bin = __ballot(valid && in), bout = __ballot(valid && !in);
      if (lane == 0) wcnt[w] = __popcll(bin);
      __syncthreads();
      int off_in = 0, tot_in = 0;
      for (int q = 0; q < kWaves; q++) {
        off_in += q < w ? wcnt[q] : 0;
        tot_in += wcnt[q];
      }
      const int n_valid = min(count - c0, kBS);
      // every earlier wave of the chunk is full, so its outside count is 64 minus its inside count
      const int off_out = w * 64 - off_in;
      if (valid) {
        int dst;
        if (in) {
          dst = base_in + off_in + __popcll(bin & lt);
          fit_acc(pin, r, 3 * p);
        } else {
          dst = count - 1 - (base_out + off_out + __popcll(bout & lt));
          fit_acc(pout, r, 3 * p);
        }
        for (int j = 0; j < 9; j++) fv_tmp[9 * ((size_t)start + dst) + j] = r[j];
        ids_tmp[start + dst] = ids[start + p];
      }
      base_in += tot_in;
      base_out += n_valid - tot_in;
      __syncthreads();
    }
    const int n_in = base_in;
    if (n_in == 0 || n_in == count) {
      // impossible split: the face list keeps its order, the bounds are restored, the axis is marked
      b.failed[choice] = 1;
      continue;
    }
    // copy back: stayers in order, then the movers (stored reversed) in order
    for (int p = tid; p < count; p += kBS) {
      const int q = p < n_in ? p : count - 1 - (p - n_in);
      for (int j = 0; j < 9; j++) fv[9 * ((size_t)start + p) + j] = fv_tmp[9 * ((size_t)start + q) + j];
      ids[start + p] = ids_tmp[start + q];
    }
    Pair fin[6], fout[6];
    block_fit(pin, red, fin);
    block_fit(pout, red, fout);
    if (tid == 0) {
      DBox nb;
      for (int a = 0; a < 3; a++) {
        b.low[a] = fin[a].v; b.high[a] = fin[3 + a].v;
        nb.low[a] = fout[a].v; nb.high[a] = fout[3 + a].v;
        b.failed[a] = 0; nb.failed[a] = 0;
      }
      nb.start = start + n_in;
      nb.count = count - n_in;
      nb.result = 0;
      b.count = n_in;
      b.result = 1;
      boxes[blockIdx.x] = b;
      child[blockIdx.x] = nb;
    }
    return;
  }
}

}  // namespace

int gpu_build_ref_boxes(int device, HostScene& hs, const float* v4, int32_t min_faces, int32_t max_boxes,
                        double* gpu_ms, bool* nonfinite_out) {
  const int nf = hs.nf;
  *nonfinite_out = false;
  XCHECK(hipSetDevice(device));
  PhaseTimer pt("boxes-gpu");
  hipStream_t st;
  st = (hipStream_t)build_stream(device);
  if (!st) return RT_ERR_HIP;
  struct Guard {
    hipStream_t st;
    std::vector<void*> bufs;
    std::vector<hipEvent_t> evs;
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
  float *d_v4 = nullptr, *d_fv = nullptr, *d_fvt = nullptr;
  uint32_t* d_fidx = nullptr;
  int32_t *d_ids = nullptr, *d_idt = nullptr, *d_flag = nullptr;
  DBox *d_boxes = nullptr, *d_child = nullptr;
  XCHECK(alloc((void**)&d_v4, 16 * (size_t)hs.nv));
  XCHECK(alloc((void**)&d_fidx, 12 * (size_t)nf));
  XCHECK(alloc((void**)&d_fv, 36 * (size_t)nf));
  XCHECK(alloc((void**)&d_fvt, 36 * (size_t)nf));
  XCHECK(alloc((void**)&d_ids, 4 * (size_t)nf));
  XCHECK(alloc((void**)&d_idt, 4 * (size_t)nf));
  XCHECK(alloc((void**)&d_flag, 4));
  // todo / child records of one pass: at most every box splits, and a pass can hold all boxes
  size_t cap = 1024;
  XCHECK(alloc((void**)&d_boxes, cap * sizeof(DBox)));
  XCHECK(alloc((void**)&d_child, cap * sizeof(DBox)));
  hipEvent_t e0, e1;
  XCHECK(hipEventCreate(&e0));
  g.evs.push_back(e0);
  XCHECK(hipEventCreate(&e1));
  g.evs.push_back(e1);
  pt.mark("alloc");
  // pageable sources through the pinned staging copies (h2d; a plain async copy from pageable memory runs
  // at ~1 GB/s)
  if (int rc = h2d(d_v4, v4, 16 * (size_t)hs.nv)) return rc;
  if (int rc = h2d(d_fidx, hs.fidx.data(), 12 * (size_t)nf)) return rc;
  pt.mark("h2d");
  XCHECK(hipMemsetAsync(d_flag, 0, 4, st));
  XCHECK(hipEventRecord(e0, st));
  hipLaunchKernelGGL(k_gather, dim3((nf + 255) / 256), dim3(256), 0, st, (const float*)d_v4, (const uint32_t*)d_fidx, nf,
                     d_fv, d_ids, d_flag);
  hipLaunchKernelGGL(k_fit_all, dim3(1), dim3(kBS), 0, st, (const float*)d_fv, nf, d_boxes);
  XCHECK(hipGetLastError());
  int32_t flag = 0;
  std::vector<DBox> boxes(1);
  XCHECK(hipMemcpyAsync(&flag, d_flag, 4, hipMemcpyDeviceToHost, st));
  XCHECK(hipMemcpyAsync(boxes.data(), d_boxes, sizeof(DBox), hipMemcpyDeviceToHost, st));
  XCHECK(hipStreamSynchronize(st));
  if (flag) { *nonfinite_out = true; return RT_OK; }
  // the passes of generateBoundingBoxes (flyscene.cpp:404-417)
  std::vector<DBox> todo, kids;
  std::vector<size_t> todo_idx;
  const bool timing = debug_env("RT_TIMING") != nullptr;
  auto tp = std::chrono::steady_clock::now();
  int pass = 0;
  bool notDone = true;
  while (notDone && (int64_t)boxes.size() < (int64_t)max_boxes) {
    notDone = false;
    todo.clear();
    todo_idx.clear();
    for (size_t i = 0; i < boxes.size(); i++) {
      const DBox& b = boxes[i];
      if (b.count > min_faces && (!b.failed[0] || !b.failed[1] || !b.failed[2])) {
        todo.push_back(b);
        todo_idx.push_back(i);
      }
    }
    if (todo.empty()) break;
    notDone = true;
    if (todo.size() > cap) {
      while (cap < todo.size()) cap *= 2;
      void *nb = nullptr, *nc = nullptr;
      XCHECK(alloc(&nb, cap * sizeof(DBox)));
      XCHECK(alloc(&nc, cap * sizeof(DBox)));
      d_boxes = (DBox*)nb;
      d_child = (DBox*)nc;
    }
    kids.resize(todo.size());
    XCHECK(hipMemcpyAsync(d_boxes, todo.data(), todo.size() * sizeof(DBox), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_split_pass, dim3((unsigned)todo.size()), dim3(kBS), 0, st, d_boxes, d_child, d_fv, d_ids, d_fvt,
                       d_idt);
    XCHECK(hipGetLastError());
    XCHECK(hipMemcpyAsync(todo.data(), d_boxes, todo.size() * sizeof(DBox), hipMemcpyDeviceToHost, st));
    XCHECK(hipMemcpyAsync(kids.data(), d_child, todo.size() * sizeof(DBox), hipMemcpyDeviceToHost, st));
    XCHECK(hipStreamSynchronize(st));
    if (timing) {
      const double now = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp).count();
      int maxc = 0;
      for (const DBox& b : todo) maxc = std::max(maxc, b.count);
      fprintf(stderr, "[rt] box pass %d: %zu boxes (largest %d faces before) %.2f ms\n", pass, todo.size(), maxc, now);
      tp = std::chrono::steady_clock::now();
    }
    pass++;
    for (size_t i = 0; i < todo.size(); i++) boxes[todo_idx[i]] = todo[i];
    // the reference appends each new box right after its split: box order within the pass
    for (size_t i = 0; i < todo.size(); i++)
      if (todo[i].result == 1) boxes.push_back(kids[i]);
  }
  XCHECK(hipEventRecord(e1, st));
  pt.mark("passes");
  std::vector<int32_t> ids(nf);
  XCHECK(hipMemcpyAsync(ids.data(), d_ids, 4 * (size_t)nf, hipMemcpyDeviceToHost, st));
  XCHECK(hipStreamSynchronize(st));
  pt.mark("d2h_ids");
  float ms = 0.0f;
  XCHECK(hipEventElapsedTime(&ms, e0, e1));
  if (gpu_ms) *gpu_ms = ms;
  hs.boxes.assign(boxes.size(), RefBox());
  for (size_t i = 0; i < boxes.size(); i++) {
    const DBox& d = boxes[i];
    RefBox& b = hs.boxes[i];
    for (int a = 0; a < 3; a++) {
      b.low[a] = d.low[a];
      b.high[a] = d.high[a];
      b.shape[a] = d.high[a] - d.low[a];
      b.failed[a] = d.failed[a] != 0;
    }
    b.faces.assign(ids.begin() + d.start, ids.begin() + d.start + d.count);
  }
  pt.mark("host_boxes");
  return RT_OK;
}

}  // namespace rt
