// rt_device.hip -- the product library's gfx950 kernels and device-side C ABI of the MI355X ray-traversal
// library. The device code of the hot path is rt_kernels.h (shared with the A/B variants of
// rt_variants.hip); this file instantiates the product kernels, holds the non-template kernels (dispatch
// order, box colours, output path, known-answer tests) and the host glue (scene upload, frame dispatch,
// ray-list queries).
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/file.h>
#include <unistd.h>

#include <atomic>
#include <cctype>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rt_kernels.h"

namespace rt {

// Longest-first dispatch order for the next frame of the same shape (after the frame, one workgroup per
// XCD class). The default order hands XCD x the dispatch positions p = 8r + x and fills them with the
// logical waves of class x (below `full`: runs of C consecutive waves, j = (k / C) 8C + x C + k % C for
// k = p / 8, so an XCD's L2 serves neighbouring tiles; the trailing partial group identity-mapped).
// This keeps every wave in its class and stably reorders each class by the wave's measured cost,
// longest first: LPT scheduling -- the waves that finish a frame late become the cheap ones (the
// measured one-frame tail was 40% of the frame) -- while waves of equal cost keep their spatial order.
// Counting sort over kLptBuckets log-spaced cost buckets (4 per octave, from the float exponent and two
// mantissa bits): per-thread counts in LDS, one wave-parallel exclusive scan per bucket, then every
// thread places its contiguous run of waves. Any order is a permutation: every frame renders identical
// bits.
constexpr int kLptBuckets = 32, kLptThreads = 512, kLptRefresh = 8;
constexpr bool kLptMoved = true;  // re-sort after every lone frame whose camera moved since the map's frame
constexpr int kLptDilate = 2;     // a moving camera's map: each wave's cost = the max over (2r+1)^2 waves around it
// ... or around the waves where its content is expected next frame (FrameParams::pred), then over a ring of 1
// (profiles/ab/r06_moving_prediction_ab.txt: C5 moving lone frames 0.295 -> 0.26 ms)
constexpr bool kLptPred = true;
constexpr int kLptDilatePred = 1;

// The camera's last step as a view-space transform, D = V_n V_(n-1)^-1 (both world -> view, column-major 4 x 4
// affine, tucano Camera::view_matrix); its translation (FrameParams::pred_step). Flycamera::translate (the
// reference's WASD keys, flycamera.hpp:196-202) moves translation_vector under a fixed rotation, so D is a pure
// translation there; a rotated step keeps only its translation (the prediction is a dispatch-order hint).
static void camera_step(const float* vp_prev, const float* v_cur, float* step3) {
  double R[3][3], t[3], Ri[3][3];
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) R[i][j] = vp_prev[4 * j + i];
    t[i] = vp_prev[12 + i];
  }
  const double det = R[0][0] * (R[1][1] * R[2][2] - R[1][2] * R[2][1]) - R[0][1] * (R[1][0] * R[2][2] - R[1][2] * R[2][0]) +
                     R[0][2] * (R[1][0] * R[2][1] - R[1][1] * R[2][0]);
  step3[0] = step3[1] = step3[2] = 0.0f;
  if (!(std::fabs(det) > 1e-30)) return;  // degenerate previous view: no step
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      const int a = (j + 1) % 3, b = (j + 2) % 3, c = (i + 1) % 3, d = (i + 2) % 3;
      Ri[i][j] = (R[a][c] * R[b][d] - R[a][d] * R[b][c]) / det;  // inverse = adjugate / det
    }
  for (int i = 0; i < 3; i++) {  // D's translation: t_n - R_n R_(n-1)^-1 t_(n-1)
    double m = v_cur[12 + i];
    for (int j = 0; j < 3; j++) {
      double rr = 0.0;
      for (int k = 0; k < 3; k++) rr += (double)v_cur[4 * k + i] * Ri[k][j];
      m -= rr * t[j];
    }
    step3[i] = (float)m;
  }
}
constexpr int kSplitK = 1536;  // FULL lone frames: waves split into 16-lane sub-waves (FrameParams::split_k); round 5
                               // re-sweep without the spill: 1536 +2.5..6% over 2048 (profiles/ab/r05_c5_split_ab.txt)
constexpr int kSplitKPrimary = 256;   // the same for k_primary_fused (small scenes); round 6 re-sweep after the
                                      // scene-level map: 256 against 1024 -2.5% static, -7% moving, -8% at a stopped
                                      // pose (C2 lone frames, profiles/ab/r06_split_size_ab.txt)
__device__ __forceinline__ uint32_t lpt_bucket(uint32_t c, int shift) {
  // 4 buckets per octave: exponent and 2 mantissa bits of (float)c; costs of 2^10 .. 2^18 shader cycles
  // (0.5 .. 120 us at 2.1 GHz) spread over the buckets, longest first (bucket 0)
  const int q = (int)(__float_as_uint((float)(c | 1u)) >> 21) - ((127 + 10) << 2);
  const int b = (q < 0 ? 0 : (q > 4 * 8 - 1 ? 4 * 8 - 1 : q)) >> shift;
  return (uint32_t)((kLptBuckets >> shift) - 1 - b);
}
// The sort reads `cost` (the recording frame's per-wave costs, or with a moving camera their dilation: the
// render kernel's waves raised cost_dil over their neighbourhoods, wave_clock_end) and clears what it read in
// both arrays, so the next recording frame starts from zeros -- the atomic maxima of split sub-waves and of the
// dilation need them -- without a fill on the frame's own critical path. Counts live in LDS, one column per
// thread (a register array indexed by the bucket compiled to a waterfall loop per access: 15 us per sort).
__global__ __launch_bounds__(kLptThreads) void k_order_lpt(uint32_t* cost, uint32_t* clear2, uint32_t* order, int n, int C,
                                                           int shift) {
  __shared__ uint32_t cnt[kLptBuckets][kLptThreads];
  __shared__ uint32_t base[kLptBuckets];
  const int x = (int)blockIdx.x, t = (int)threadIdx.x, lane = t & 63, wv = t >> 6;
  const int full = (n / (8 * C)) * 8 * C;
  const int m = (n - x + 7) / 8;  // positions 8r + x < n of this class
  const int chunk = (m + kLptThreads - 1) / kLptThreads, r0 = t * chunk, r1 = min(m, r0 + chunk);
  const int nb = kLptBuckets >> shift;
  auto item = [&](int r) {  // the logical wave the default order puts at position 8r + x
    const int p = 8 * r + x;
    if (p >= full) return p;
    const int k = p >> 3;
    return (k / C) * 8 * C + x * C + (k % C);
  };
  for (int b = 0; b < nb; b++) cnt[b][t] = 0;
  for (int r = r0; r < r1; r++) cnt[lpt_bucket(cost[item(r)], shift)][t]++;
  __syncthreads();
  // exclusive scan of each bucket's per-thread counts: wave w scans buckets w, w + 8, ..; lane i owns
  // threads 8i .. 8i + 7
  for (int b = wv; b < nb; b += kLptThreads / 64) {
    uint32_t v[8], s = 0;
    for (int k = 0; k < 8; k++) { v[k] = cnt[b][8 * lane + k]; s += v[k]; }
    uint32_t incl = s;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = __shfl_up(incl, off, 64);
      if (lane >= off) incl += o;
    }
    uint32_t run = incl - s;
    for (int k = 0; k < 8; k++) { cnt[b][8 * lane + k] = run; run += v[k]; }
    if (lane == 63) base[b] = incl;  // bucket total
  }
  __syncthreads();
  if (wv == 0) {  // bucket totals -> start ranks, longest bucket first (one lane per bucket)
    const uint32_t v = lane < nb ? base[lane] : 0u;
    uint32_t incl = v;
    for (int off = 1; off < 32; off <<= 1) {
      const uint32_t o = __shfl_up(incl, off, 64);
      if (lane >= off) incl += o;
    }
    if (lane < nb) base[lane] = incl - v;
  }
  __syncthreads();
  for (int r = r0; r < r1; r++) {
    const int j = item(r);
    const uint32_t b = lpt_bucket(cost[j], shift);
    const uint32_t rr = base[b] + cnt[b][t]++;
    order[8 * rr + x] = (uint32_t)j;
    cost[j] = 0u;
    if (clear2) clear2[j] = 0u;
  }
}

// RT_MODE_BOX_COLORS, once per colour set: for every face id, color += box->color over the reference
// boxes in creation order whose [low, high] holds all three object-space vertices (BoundingBox::hasFace,
// BoundingBox.cpp:26-39; flyscene.cpp:337-341), summed in that order in fp32 as the reference does. One
// thread per face; the boxes (bounds from the refbox array, colours) are staged through LDS in chunks and
// read as wave-wide broadcasts.
constexpr int kBoxColorChunk = 1024;
__global__ __launch_bounds__(256) void k_face_box_colors(const float* fv9, const float* refbox, const float* col3,
                                                         int nb, int nf, float* out4) {
  __shared__ float sb[9][kBoxColorChunk];  // low xyz, high xyz, colour rgb
  const int f = (int)(blockIdx.x * 256u + threadIdx.x);
  const bool act = f < nf;
  float v[9];
  for (int k = 0; k < 9; k++) v[k] = act ? fv9[9 * (size_t)f + k] : 0.0f;
  float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f;
  for (int b0 = 0; b0 < nb; b0 += kBoxColorChunk) {
    const int n = min(kBoxColorChunk, nb - b0);
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += 256) {
      const float* rb = refbox + 8 * (size_t)(b0 + i);
      sb[0][i] = rb[0]; sb[1][i] = rb[1]; sb[2][i] = rb[2];
      sb[3][i] = rb[4]; sb[4][i] = rb[5]; sb[5][i] = rb[6];
      const float* c = col3 + 3 * (size_t)(b0 + i);
      sb[6][i] = c[0]; sb[7][i] = c[1]; sb[8][i] = c[2];
    }
    __syncthreads();
    if (act)
      for (int i = 0; i < n; i++) {
        bool in = true;
        for (int k = 0; k < 3; k++) {
          const float x = v[3 * k], y = v[3 * k + 1], z = v[3 * k + 2];
          in = in && x >= sb[0][i] && x <= sb[3][i] && y >= sb[1][i] && y <= sb[4][i] && z >= sb[2][i] && z <= sb[5][i];
        }
        if (in) { c0 += sb[6][i]; c1 += sb[7][i]; c2 += sb[8][i]; }
      }
  }
  if (act) reinterpret_cast<float4*>(out4)[f] = make_float4(c0, c1, c2, 0.0f);
}

// Output path: the float frame -> the PPM's 8-bit values on the device, so the host
// reads 3 B/px instead of 12. Value = min(255, (int)(255*c)) as writePPMImage computes it
// (tucano/utils/ppmIO.hpp:135-156; x86 cvttss2si: NaN / out of range -> INT_MIN); values outside
// 0..255 (NaN or negative colours) are clamped and flagged, so the caller knows when the 8-bit frame is
// not exactly the PPM's numbers.
__global__ __launch_bounds__(256) void k_frame_rgb8(const float* rgb, uint8_t* out, uint32_t n, uint32_t* anomaly) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  bool bad = false;
  if (i < n) {
    const float x = 255.0f * rgb[i];
    int v = (x >= -2147483648.0f && x < 2147483648.0f) ? (int)x : INT_MIN;
    v = min(255, v);
    bad = v < 0;
    out[i] = (uint8_t)max(v, 0);
  }
  if (ballot(bad) && lane_id() == 0) atomicOr(anomaly, 1u);
}

// Multi-GPU frame assembly (f3): a rank packs the 8-bit values of its own 16x16 tiles contiguously
// (tile order of its shard, 768 B per tile, pixels outside the frame zero) so that one gather of equal
// slices (RCCL over xGMI) brings every shard to one GPU, which unpacks them into the frame.
__device__ __forceinline__ uint8_t ppm_u8(float c) {
  const float x = 255.0f * c;
  const int v = (x >= -2147483648.0f && x < 2147483648.0f) ? (int)x : INT_MIN;
  return (uint8_t)max(min(255, v), 0);
}
// anomaly (may be null): set when some value is NaN or negative (as k_frame_rgb8 flags it)
__global__ __launch_bounds__(256) void k_pack_shard(const float* rgb, uint8_t* out, int W, int H, int tiles_x,
                                                    int si, int sc, int n_tiles, int S, uint32_t* anomaly) {
  const int L = blockIdx.x;  // one block per tile slot of the shard, one thread per pixel
  if (L >= n_tiles) return;
  int tx, ty;
  shard_tile_xy(tiles_x, S, si, sc, L, tx, ty);
  const int x = tx * 16 + (threadIdx.x & 15), y = ty * 16 + (threadIdx.x >> 4);
  uint8_t* o = out + ((size_t)L * 256 + threadIdx.x) * 3;
  bool bad = false;
  if (x < W && y < H) {
    const float* c = rgb + 3 * ((size_t)y * W + x);
    for (int k = 0; k < 3; k++) {
      o[k] = ppm_u8(c[k]);
      const float x = 255.0f * c[k];  // k_frame_rgb8's test: the PPM's number (int)x below 0, or NaN
      bad = bad || ((x >= -2147483648.0f && x < 2147483648.0f) ? (int)x : INT_MIN) < 0;
    }
  } else {
    o[0] = o[1] = o[2] = 0;
  }
  if (anomaly && ballot(bad) && lane_id() == 0) atomicOr(anomaly, 1u);
}
// Multi-device frame assembly: a replica packs its tiles' 32-bit values (ch per pixel: colour 3, face id or
// t 1) contiguously in its shard's slot order (256 * ch words per tile, pixels outside the frame zero), so
// one copy per device brings them to the host, which places the tiles into the caller's frame.
__global__ __launch_bounds__(256) void k_pack_tiles32(const uint32_t* src, uint32_t* out, int W, int H, int tiles_x,
                                                      int si, int sc, int n_tiles, int S, int ch) {
  const int L = blockIdx.x;
  if (L >= n_tiles) return;
  int tx, ty;
  shard_tile_xy(tiles_x, S, si, sc, L, tx, ty);
  const int x = tx * 16 + (threadIdx.x & 15), y = ty * 16 + (threadIdx.x >> 4);
  const bool in = x < W && y < H;
  uint32_t* o = out + ((size_t)L * 256 + threadIdx.x) * ch;
  const uint32_t* c = src + (size_t)ch * (in ? (size_t)y * W + x : 0);
  for (int k = 0; k < ch; k++) o[k] = in ? c[k] : 0u;
}
__global__ __launch_bounds__(256) void k_unpack_shards(const uint8_t* packed, uint8_t* frame, int W, int H, int tiles_x,
                                                       int n, size_t slice_bytes, int S) {
  const size_t p = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= (size_t)W * H) return;
  const int x = (int)(p % W), y = (int)(p / W);
  // the inverse of shard_tile_xy: tile -> super-tile s -> (owner s % n, slot (s / n) * S^2 + in-super index)
  const int tx = x >> 4, ty = y >> 4, sxn = (tiles_x + S - 1) / S;
  const int s = (ty / S) * sxn + tx / S, slot = (s / n) * S * S + (ty % S) * S + tx % S;
  const uint8_t* src = packed + (size_t)(s % n) * slice_bytes + ((size_t)slot * 256 + (y & 15) * 16 + (x & 15)) * 3;
  frame[3 * p + 0] = src[0];
  frame[3 * p + 1] = src[1];
  frame[3 * p + 2] = src[2];
}

// Device-side assembly of a multi-device scene's frame (assemble_device): block (L, k) places tile slot L of replica
// k's packed slice (k_pack_tiles32 / k_pack_shard layout: 256 pixels of E bytes per tile) into the frame on device 0
struct UnpackArgs {
  int32_t n_rep, W, H, tiles_x, E;
  int32_t si[RT_MAX_DEVICES], sc[RT_MAX_DEVICES], S[RT_MAX_DEVICES], n_tiles[RT_MAX_DEVICES];
  uint64_t off[RT_MAX_DEVICES], flag_off[RT_MAX_DEVICES];  // byte offsets of slice k and of its exactness flag
};
__global__ __launch_bounds__(256) void k_unpack_tiles(const uint8_t* gather, uint8_t* frame, UnpackArgs a) {
  const int k = (int)blockIdx.y, L = (int)blockIdx.x;
  if (k >= a.n_rep || L >= a.n_tiles[k]) return;
  int tx, ty;
  shard_tile_xy(a.tiles_x, a.S[k], a.si[k], a.sc[k], L, tx, ty);
  const int x = tx * 16 + (int)(threadIdx.x & 15), y = ty * 16 + (int)(threadIdx.x >> 4);
  if (x >= a.W || y >= a.H) return;
  const size_t src = a.off[k] + ((size_t)L * 256 + threadIdx.x) * (size_t)a.E, dst = ((size_t)y * a.W + x) * (size_t)a.E;
  if (a.E == 3) {
    frame[dst] = gather[src];
    frame[dst + 1] = gather[src + 1];
    frame[dst + 2] = gather[src + 2];
  } else {  // 4 or 12 bytes, 4-byte aligned (slices start on 16 B)
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(gather + src);
    uint32_t* d4 = reinterpret_cast<uint32_t*>(frame + dst);
    for (int w = 0; w < a.E / 4; w++) d4[w] = s4[w];
  }
}
// the 8-bit frame's exactness flags of every replica, OR-ed into the word after the frame
__global__ void k_or_flags(const uint8_t* gather, UnpackArgs a, uint32_t* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t f = 0;
  for (int k = 0; k < a.n_rep; k++) f |= *reinterpret_cast<const uint32_t*>(gather + a.flag_off[k]);
  *out = f;
}

__global__ void k_debug_math(int op, int n, int in_len, int out_len, const float* in, float* out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) debug_math_case(op, in + (size_t)k * in_len, out + (size_t)k * out_len);
}

// ------------------------------------------------------------------------------------------------
// Host glue
// ------------------------------------------------------------------------------------------------
// Host -> device copy of scene data. Large copies from pageable host memory go through two pinned 8-MiB
// staging buffers on their own stream (host memcpy of one chunk overlaps the DMA of the other): a plain
// hipMemcpy from pageable memory measured ~1 GB/s for the scene upload (263 ms for the 1M soup's ~250 MB,
// BENCH_r03 build_ms.upload).
// One stream per device for scene construction (the builders' kernels, the staged copies): created on
// first use and kept for the process, so building scenes creates no HIP streams beyond it. Each stream a
// process creates is bound to one of the device's few hardware queues; transient build streams created
// before a scene's frame-slot streams changed which queues those landed on.
void* build_stream(int device) {
  static std::mutex mu;
  static hipStream_t st[64] = {};
  if (device < 0 || device >= 64) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (!st[device]) {
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&st[device], hipStreamNonBlocking) != hipSuccess)
      st[device] = nullptr;
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  return (void*)st[device];
}

// First use of the device in a process (its construction stream, a first allocation), run on a helper thread
// while rt_scene_create prepares the host arrays: measured ~0.14 s before the first builder's allocations
// on a fresh process (C3, RT_TIMING), which otherwise adds to the scene setup after the host preparation.
void device_warmup(int device) {
  PhaseTimer pt("warmup");
  if (device < 0 || hipSetDevice(device) != hipSuccess) return;
  pt.mark("set_device");
  (void)build_stream(device);
  pt.mark("stream");
  void* p = nullptr;
  if (hipMalloc(&p, 1u << 20) == hipSuccess) (void)hipFree(p);
  pt.mark("malloc");
}

// One pair of pinned 8-MiB staging buffers (+ their events) per device for the staged copies below, created
// at the device's first large copy and kept for the process beside its build stream (allocating
// and freeing pinned memory per copy can synchronise the device, stalling frames other scenes have in
// flight, and added to the setup time). Copies to one device serialise on its staging mutex.
struct Staging {
  std::mutex mu;
  void* buf[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
};
constexpr size_t kStageChunk = 8u << 20;
static int staging(int device, Staging** out) {
  static Staging st[64];
  if (device < 0 || device >= 64) { set_error("device %d out of range for staging", device); return RT_ERR_INVALID; }
  *out = &st[device];
  return RT_OK;
}
// (caller holds g.mu and has made `device` current)
static int staging_ready(Staging& g) {
  for (int k = 0; k < 2; k++) {
    if (!g.buf[k]) HIPCHECK(hipHostMalloc(&g.buf[k], kStageChunk, hipHostMallocDefault));
    if (!g.ev[k]) HIPCHECK(hipEventCreateWithFlags(&g.ev[k], hipEventDisableTiming));
  }
  return RT_OK;
}

int h2d(void* dst, const void* src, size_t bytes) {
  if (bytes < 2 * kStageChunk) {
    HIPCHECK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return RT_OK;
  }
  int dev = 0;
  HIPCHECK(hipGetDevice(&dev));
  Staging* gp = nullptr;
  int rc = staging(dev, &gp);
  if (rc) return rc;
  Staging& g = *gp;
  std::lock_guard<std::mutex> lock(g.mu);
  if ((rc = staging_ready(g))) return rc;
  hipStream_t st = (hipStream_t)build_stream(dev);
  if (!st) { set_error("no build stream on device %d", dev); return RT_ERR_HIP; }
  // on any return the stream drains first: the staging buffers are reused by the next copy
  struct Drain { hipStream_t st; ~Drain() { (void)hipStreamSynchronize(st); } } drain{st};
  bool used[2] = {false, false};
  int k = 0;
  for (size_t off = 0; off < bytes; off += kStageChunk, k ^= 1) {
    const size_t n = std::min(kStageChunk, bytes - off);
    if (used[k]) HIPCHECK(hipEventSynchronize(g.ev[k]));  // this staging buffer's previous DMA is done
    memcpy(g.buf[k], static_cast<const char*>(src) + off, n);
    HIPCHECK(hipMemcpyAsync(static_cast<char*>(dst) + off, g.buf[k], n, hipMemcpyHostToDevice, st));
    HIPCHECK(hipEventRecord(g.ev[k], st));
    used[k] = true;
  }
  HIPCHECK(hipStreamSynchronize(st));
  return RT_OK;
}

// Device -> host copy into pageable memory, the same way round: DMA into one pinned 8-MiB staging buffer
// while the host copies the other out (the device builders' read-backs).
int d2h(void* dst, const void* src, size_t bytes) {
  if (bytes < 2 * kStageChunk) {
    HIPCHECK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return RT_OK;
  }
  int dev = 0;
  HIPCHECK(hipGetDevice(&dev));
  Staging* gp = nullptr;
  int rc = staging(dev, &gp);
  if (rc) return rc;
  Staging& g = *gp;
  std::lock_guard<std::mutex> lock(g.mu);
  if ((rc = staging_ready(g))) return rc;
  hipStream_t st = (hipStream_t)build_stream(dev);
  if (!st) { set_error("no build stream on device %d", dev); return RT_ERR_HIP; }
  struct Drain { hipStream_t st; ~Drain() { (void)hipStreamSynchronize(st); } } drain{st};
  const size_t nchunks = (bytes + kStageChunk - 1) / kStageChunk;
  auto issue = [&](size_t c) -> int {
    const size_t off = c * kStageChunk, n = std::min(kStageChunk, bytes - off);
    HIPCHECK(hipMemcpyAsync(g.buf[c & 1], static_cast<const char*>(src) + off, n, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipEventRecord(g.ev[c & 1], st));
    return RT_OK;
  };
  if ((rc = issue(0))) return rc;
  for (size_t c = 0; c < nchunks; c++) {
    if (c + 1 < nchunks && (rc = issue(c + 1))) return rc;  // the next chunk's DMA overlaps this copy-out
    HIPCHECK(hipEventSynchronize(g.ev[c & 1]));
    const size_t off = c * kStageChunk, n = std::min(kStageChunk, bytes - off);
    memcpy(static_cast<char*>(dst) + off, g.buf[c & 1], n);
  }
  return RT_OK;
}

template <typename T>
static int dalloc_copy(T** dst, const void* src, size_t bytes, int64_t& total) {
  *dst = nullptr;
  if (bytes == 0) bytes = 16;
  HIPCHECK(hipMalloc((void**)dst, bytes));
  total += (int64_t)bytes;
  if (src) return h2d(*dst, src, bytes);
  return RT_OK;
}

static size_t alloc_bytes(size_t bytes) { return bytes == 0 ? 16 : bytes; }  // what dalloc_copy allocates

// The scene's device and its frame-slot streams (one per frame in flight). Each slot stream gets a hardware
// queue of its own: an ordinary HIP stream is bound to one of a small per-process pool of queues
// (GPU_MAX_HW_QUEUES, 4 on the boxes), shared with every other stream of the process in creation order, and two
// slots on one queue run their frames one after the other -- measured in a fresh process: C5 with 4 frames in
// flight 8.3 Grays/s with the slots on the pool (kernel ms per frame 0.49, two frames overlapping) against 12.3
// when the pool had been used by two other streams first, or with 8 queues per process
// (profiles/ab/r05_queue_probe.txt). A stream created with a CU mask is given a dedicated queue outside that
// pool, so the slots are created with the full mask (every CU: no restriction), whatever streams the process
// made before; a runtime that refuses falls back to an ordinary stream.
// At most kDedicatedSlotQueues such queues per device and process (two scenes' worth of slots): beyond that the
// device's queues are oversubscribed and the hardware time-slices them -- eight replicas of one scene on one GPU
// (32 dedicated queues) ran 2.3x slower than two (profiles/ab/r05_queue_probe.txt) -- so further slots take the
// pool. dedicated_slots counts the live dedicated queues per device (released by release_slot_stream).
// A deliberate exception to the per-process GPU_MAX_HW_QUEUES pool: it is what lets one process's
// frames in flight overlap (C5 with 4 frames in flight 11.9 against 8.6 Grays/s on the pool); RT_SLOT_POOL (A/B
// knob) puts every slot on the pool.
constexpr int kDedicatedSlotQueues = 8;
// Across the processes that share a GPU (the cap was counted per process only; four renderer processes
// on one GPU held 32 dedicated queues and ran 4.1x slower than with every slot on the pool, and a shared cap of 8
// queues still halved them -- profiles/ab/r06_slot_queues_ab.txt), only one process per GPU holds dedicated slot
// queues. A lock file per physical GPU (/tmp/rtamd_hwq_<PCI bus id>) lists "pid count" of the processes holding
// them; entries of processes that no longer exist are dropped, and the file is removed when no holder is left.
// Without the file (no /tmp, another user's file) a process keeps its own cap only.
static bool hwq_registry(int dev, int delta) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, (int)sizeof bus - 1, dev) != hipSuccess) { (void)hipGetLastError(); return delta < 0; }
  std::string path = "/tmp/rtamd_hwq_";
  for (const char* c = bus; *c; c++) path += (isalnum((unsigned char)*c) ? *c : '_');
  const int fd = open(path.c_str(), O_RDWR | O_CREAT, 0666);
  if (fd < 0) return delta < 0;
  struct Close { int fd; ~Close() { flock(fd, LOCK_UN); close(fd); } } close_{fd};
  if (flock(fd, LOCK_EX) != 0) return delta < 0;
  std::string text;
  char buf[4096];
  ssize_t n;
  while ((n = read(fd, buf, sizeof buf)) > 0) text.append(buf, (size_t)n);
  const long me = (long)getpid();
  long mine = 0, others = 0;
  std::string out;
  size_t pos = 0;
  while (pos < text.size()) {
    const size_t e = std::min(text.find('\n', pos), text.size());
    long pid = 0, cnt = 0;
    if (sscanf(text.c_str() + pos, "%ld %ld", &pid, &cnt) == 2 && pid > 0 && cnt > 0) {
      if (pid == me) mine = cnt;
      else if (kill((pid_t)pid, 0) == 0 || errno == EPERM) { others += cnt; out += std::to_string(pid) + " " + std::to_string(cnt) + "\n"; }
    }
    pos = e + 1;
  }
  bool ok = true;
  // one process per GPU holds dedicated queues (the first to ask): every other renderer process on that GPU takes
  // the pool. (RT_HWQ_GPU_CAP=N, A/B knob: instead grant while all processes together hold at most N.)
  const char* cap_env = debug_env("RT_HWQ_GPU_CAP");
  if (delta > 0 && (cap_env ? others + mine + delta > atol(cap_env) : others > 0)) ok = false;
  else mine = std::max(0L, mine + delta);
  if (mine > 0) out += std::to_string(me) + " " + std::to_string(mine) + "\n";
  if (out.empty()) {  // no holder left: leave nothing behind (a process waiting on the old file re-counts alone)
    (void)unlink(path.c_str());
    return ok;
  }
  if (ftruncate(fd, 0) == 0 && lseek(fd, 0, SEEK_SET) == 0) {
    const ssize_t w = write(fd, out.data(), out.size());
    (void)w;
  }
  return ok;
}
static std::mutex g_slot_mu;
static int g_dedicated_slots[64] = {};
static hipStream_t slot_stream(int dev, bool* dedicated) {
  *dedicated = false;
  hipDeviceProp_t prop;
  hipStream_t st = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_slot_mu);
    // (RT_SLOT_POOL, A/B knob: every slot on the runtime's pooled queues, as an ordinary stream)
    const char* pool_env = debug_env("RT_SLOT_POOL");
    if (!(pool_env && atoi(pool_env)) && dev >= 0 && dev < 64 && g_dedicated_slots[dev] < kDedicatedSlotQueues &&
        hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0 && hwq_registry(dev, 1)) {
      std::vector<uint32_t> mask((size_t)(prop.multiProcessorCount + 31) / 32, 0xFFFFFFFFu);
      if (hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()) == hipSuccess) {
        g_dedicated_slots[dev]++;
        *dedicated = true;
        return st;
      }
      (void)hipGetLastError();
      (void)hwq_registry(dev, -1);
      st = nullptr;
    }
  }
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return nullptr;
  return st;
}
static void release_slot_stream(int dev, void* st, bool dedicated) {
  if (st) (void)hipStreamDestroy((hipStream_t)st);
  if (dedicated && dev >= 0 && dev < 64) {
    std::lock_guard<std::mutex> lk(g_slot_mu);
    g_dedicated_slots[dev]--;
    (void)hwq_registry(dev, -1);
  }
}
constexpr int kEventFrames = 128;
static int init_slots(rt_scene* s, int dev) {
  HIPCHECK(hipSetDevice(dev));
  s->device = dev;
  s->n_slots = std::max(1, std::min((int)s->opts.frames_in_flight, (int)rt_scene::kMaxSlots));
  for (int k = 0; k < s->n_slots; k++) {
    bool dedicated = false;
    hipStream_t st = slot_stream(dev, &dedicated);
    if (!st) { set_error("device %d: no stream for frame slot %d", dev, k); return RT_ERR_HIP; }
    s->slots[k].stream = st;
    s->slots[k].dedicated_queue = dedicated;
  }
  s->stream = s->slots[0].stream;
  // the timing events of the first kEventFrames frames between two rt_synchronize calls, made here rather than
  // one frame at a time inside a caller's frame loop
  for (int k = (int)s->ev_pool.size(); k < 3 * kEventFrames; k++) {
    hipEvent_t e;
    HIPCHECK(hipEventCreate(&e));
    s->ev_pool.push_back(e);
  }
  return RT_OK;
}

int current_device() {
  int ndev = 0, dev = -1;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return -1;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  return dev;
}

int device_upload(rt_scene* s) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("no HIP device available (the library has no CPU fallback)");
    return RT_ERR_NO_DEVICE;
  }
  int dev = s->opts.device;
  if (dev < 0) HIPCHECK(hipGetDevice(&dev));
  if (dev >= ndev) { set_error("device %d out of range (%d devices)", dev, ndev); return RT_ERR_INVALID; }
  int rc = init_slots(s, dev);
  if (rc) return rc;
  PhaseTimer pt("upload");
  HostScene& hs = s->hs;
  int64_t& tot = s->device_bytes;
  tot = 0;
  s->static_pad = scene_static_pad(hs);
  s->cert_origin_max = cert_origin_max(hs);
  pt.mark("pads");
  {
    // BVH nodes and triangle records share one allocation (triangles right after the nodes), so one
    // base plus a 32-bit byte offset reaches either: each uploaded node's pad0 / pad1
    // hold the offsets of its children's records (a leaf child: its first triangle)
    const size_t nn = hs.nodes.size(), nt = hs.tris.size();
    // the fp32 4-wide tree's eight octant copies follow, 128-B aligned (one L2 line per record), when
    // every wide record offset stays below kLeafBit; else the binary tree serves alone (record_layout)
    const size_t nw = hs.wide.size();
    uint64_t wide_base = 0;
    const size_t bytes = (size_t)record_layout(nn, nt, nw, &wide_base);
    if (bytes == 0 && nn + nt > 0) {  // cannot happen below kMaxFaces (rt_scene_create checks it)
      set_error("scene records exceed 4 GiB (%zu nodes, %zu triangles)", nn, nt);
      return RT_ERR_INVALID;
    }
    static_assert(sizeof(Node128) == 128, "wide record size (record_layout)");
    const size_t wide_bytes = 8 * nw * sizeof(Node128);
    s->wide_base = (uint32_t)wide_base;
    s->wide_copy_bytes = wide_base ? (uint32_t)(nw * sizeof(Node128)) : 0;
    if ((rc = dalloc_copy(&s->d_nodes, nullptr, bytes, tot))) return rc;
    s->nodes_bytes = alloc_bytes(bytes);
    pt.mark("alloc");
    // the device form of the binary records, filled on the host threads (no value-initialisation pass):
    // pad0 / pad1 = the children's record offsets (prefetch targets) with the octant order bits in their
    // low bits, interior children as byte offsets of their records (node_offset)
    std::unique_ptr<Node64[]> nodes(new Node64[std::max<size_t>(nn, 1)]);
    {
      auto pf = [&](uint32_t c) -> uint32_t {
        return (uint32_t)(64 * (is_leaf(c) ? nn + leaf_first(c) : (size_t)c));
      };
      parallel_for(nn, [&](size_t b, size_t e) {
        for (size_t i = b; i < e; i++) {
          Node64 nd = hs.nodes[i];
          const uint32_t order = nd.pad0;  // octant_order() (rt_host.cpp), moved into the low offset bits
          nd.pad0 = pf(nd.child0) | (order & 0x3Fu);
          nd.pad1 = pf(nd.child1) | ((order >> 6) & 0x3u);
          if (!is_leaf(nd.child0)) nd.child0 *= 64u;
          if (!is_leaf(nd.child1)) nd.child1 *= 64u;
          nodes[i] = nd;
        }
      });
    }
    pt.mark("node_prep");
    if (nn && (rc = h2d(s->d_nodes, nodes.get(), nn * 64))) return rc;
    pt.mark("h2d_nodes");
    s->d_tris = reinterpret_cast<TriRec64*>(s->d_nodes + nn);
    if (nt && (rc = h2d(s->d_tris, hs.tris.data(), nt * 64))) return rc;
    pt.mark("h2d_tris");
    if (s->wide_copy_bytes) {
      std::vector<Node128> wide(8 * nw);
      for (uint32_t o = 0; o < 8; o++) {
        const size_t copy = (size_t)o * nw;
        auto rec_off = [&](size_t i) { return (uint32_t)(wide_base + (copy + i) * sizeof(Node128)); };
        for (size_t i = 0; i < nw; i++) {
          const Wide4& w = hs.wide[i];
          Node128& r = wide[copy + i];
          for (int k = 0; k < 4; k++) {
            const int c = w.order[o][k];
            memcpy(r.box[k], w.box[c], sizeof r.box[k]);
            const uint32_t h = w.child[c];
            if (c >= w.n) {
              r.child[k] = kWideEmpty;
              r.pf[k] = rec_off(i);
            } else if (is_leaf(h)) {
              r.child[k] = h;
              r.pf[k] = (uint32_t)(64 * (nn + leaf_first(h)));
            } else {
              r.child[k] = rec_off(h);
              r.pf[k] = rec_off(h);
            }
          }
        }
      }
      if ((rc = h2d(reinterpret_cast<char*>(s->d_nodes) + wide_base, wide.data(), wide_bytes))) return rc;
    }
  }
  if ((rc = dalloc_copy(&s->d_nodes4, hs.nodes4.data(), hs.nodes4.size() * sizeof(Node4Q), tot))) return rc;
  s->nodes4_bytes = alloc_bytes(hs.nodes4.size() * sizeof(Node4Q));
  {
    // per-slot shading record (float4 x 3), in the triangle records' (BVH leaf) order: the unit normals of
    // the slot's face's three vertices (Mesh normals as interpolateNormal normalises them,
    // flyscene.cpp:599) and the material id in the first .w. Indexed by slot, not face id, so a hit's two
    // gathers (triangle record, shading record) are independent and issue together.
    const size_t nsl = hs.tris.size();
    std::unique_ptr<float[]> fsh(new float[std::max<size_t>(12 * nsl, 4)]);  // >= the 16 B an empty copy moves
    if (nsl == 0) std::fill(fsh.get(), fsh.get() + 4, 0.0f);
    parallel_for(nsl, [&](size_t b, size_t e) {
      for (size_t sl = b; sl < e; sl++) {
        const uint32_t f = hs.tris[sl].face;
        float* r = fsh.get() + 12 * sl;
        for (int k = 0; k < 3; k++) {
          const f3 n = hs.vnn[hs.fidx[3 * f + k]];
          r[4 * k] = n.x; r[4 * k + 1] = n.y; r[4 * k + 2] = n.z; r[4 * k + 3] = 0.0f;
        }
        const int32_t m = hs.fmat[f];
        memcpy(&r[3], &m, 4);
      }
    });
    pt.mark("fshade_prep");
    if ((rc = dalloc_copy(&s->d_fshade, fsh.get(), 12 * nsl * 4, tot))) return rc;
    s->fshade_bytes = alloc_bytes(12 * nsl * 4);
    pt.mark("h2d_fshade");
  }
  std::vector<float> rb(8 * hs.boxes.size());
  for (size_t b = 0; b < hs.boxes.size(); b++) {
    for (int k = 0; k < 3; k++) { rb[8 * b + k] = hs.boxes[b].low[k]; rb[8 * b + 4 + k] = hs.boxes[b].high[k]; }
  }
  if ((rc = dalloc_copy(&s->d_refbox, rb.data(), rb.size() * 4, tot))) return rc;
  s->refbox_bytes = alloc_bytes(rb.size() * 4);
  std::vector<DevMat> dm(hs.mats.size());
  for (size_t m = 0; m < hs.mats.size(); m++) {
    DevMat& d = dm[m];
    memset(&d, 0, sizeof d);
    for (int k = 0; k < 3; k++) { d.ka[k] = hs.mats[m].ka[k]; d.kd[k] = hs.mats[m].kd[k]; d.ks[k] = hs.mats[m].ks[k]; }
    d.ns = hs.mats[m].shininess;
  }
  if ((rc = dalloc_copy(&s->d_mats, dm.data(), dm.size() * sizeof(DevMat), tot))) return rc;
  s->mats_bytes = alloc_bytes(dm.size() * sizeof(DevMat));
  if ((rc = dalloc_copy(&s->d_stats, nullptr, kStatSlots * sizeof(unsigned long long), tot))) return rc;
  if ((rc = dalloc_copy(&s->d_pf_check, nullptr, 16, tot))) return rc;
  HIPCHECK(hipMemset(s->d_pf_check, 0, 16));
  pt.mark("rest");
  return RT_OK;
}

void stop_workers(rt_scene* s);  // (below)

void device_release(rt_scene* s) {
  stop_workers(s);      // no worker touches a replica from here on
  s->replicas.clear();  // each replica releases its own device state (~rt_scene)
  if (s->device == RT_DEVICE_NONE) return;
  (void)hipSetDevice(s->device);
  for (int k = 0; k < s->n_slots; k++)
    if (s->slots[k].stream) (void)hipStreamSynchronize((hipStream_t)s->slots[k].stream);
  void* bufs[] = {s->d_nodes, s->d_nodes4, s->d_fshade, s->d_refbox, s->d_mats, s->d_stats,
                  s->d_face_boxcolor, s->asm_buf.d_pack, s->d_pf_check};  // d_tris: inside d_nodes
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (s->asm_buf.h_pack) (void)hipHostFree(s->asm_buf.h_pack);
  s->asm_buf = rt_scene::Assembly{};
  if (s->dasm.d_gather) (void)hipFree(s->dasm.d_gather);
  if (s->dasm.d_frame) (void)hipFree(s->dasm.d_frame);
  if (s->dasm.h_frame) (void)hipHostFree(s->dasm.h_frame);
  for (void* e : s->dasm.ev_chunk)
    if (e) (void)hipEventDestroy((hipEvent_t)e);
  s->dasm = rt_scene::DevAssembly{};
  if (s->asm_ev) (void)hipEventDestroy((hipEvent_t)s->asm_ev);
  s->asm_ev = nullptr;
  s->d_nodes = nullptr; s->d_nodes4 = nullptr; s->d_tris = nullptr; s->d_fshade = nullptr;
  s->d_refbox = nullptr; s->d_mats = nullptr; s->d_stats = nullptr; s->d_pf_check = nullptr;
  for (int k = 0; k < s->n_slots; k++) {
    rt_scene::FrameSlot& f = s->slots[k];
    void* fb[] = {f.d_rgb, f.d_face, f.d_t, f.d_hits, f.d_rgb8, f.d_full, f.d_queue, f.d_timeline, f.d_wave_stats};
    for (void* b : fb)
      if (b) (void)hipFree(b);
    release_slot_stream(s->device, f.stream, f.dedicated_queue);
    f = rt_scene::FrameSlot{};
  }
  if (s->lpt.d_cost) (void)hipFree(s->lpt.d_cost);
  if (s->lpt.d_cost_dil) (void)hipFree(s->lpt.d_cost_dil);
  if (s->lpt.d_order) (void)hipFree(s->lpt.d_order);
  s->lpt = rt_scene::LptMap{};
  for (void* e : s->ev_pool) (void)hipEventDestroy((hipEvent_t)e);
  s->ev_pool.clear();
  s->ev_used = 0;
  s->stream = nullptr;
  s->d_face_boxcolor = nullptr;
  s->face_boxcolor_valid = false;
  s->device = RT_DEVICE_NONE;  // released: a second release is a no-op
}

int resolve_devices(rt_scene_opts& o) {
  if (o.n_devices == 0) return RT_OK;
  if (o.n_devices < RT_DEVICES_ALL || o.n_devices > RT_MAX_DEVICES) {
    set_error("rt_scene_opts.n_devices %d outside -1..%d", o.n_devices, RT_MAX_DEVICES);
    return RT_ERR_INVALID;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("no HIP device available (the library has no CPU fallback)");
    return RT_ERR_NO_DEVICE;
  }
  if (o.n_devices == RT_DEVICES_ALL) {
    o.n_devices = std::min(ndev, (int)RT_MAX_DEVICES);
    for (int k = 0; k < o.n_devices; k++) o.devices[k] = k;
  }
  for (int k = 0; k < o.n_devices; k++)
    if (o.devices[k] < 0 || o.devices[k] >= ndev) {
      set_error("rt_scene_opts.devices[%d] = %d: %d devices visible", k, o.devices[k], ndev);
      return RT_ERR_INVALID;
    }
  o.device = o.devices[0];
  return RT_OK;
}

// One replica: device `dst->opts.device` gets its own frame slots and a copy of src's device buffers,
// device to device (over xGMI between GPUs with peer access; a plain device copy when both replicas share
// a GPU). The host scene is shared (hsp), so nothing is rebuilt and nothing crosses PCIe.
static int replicate_one(const rt_scene* src, rt_scene* dst) {
  const int dev = dst->opts.device;
  int rc = init_slots(dst, dev);
  if (rc) return rc;
  if (dev != src->device) {
    int can = 0;
    HIPCHECK(hipDeviceCanAccessPeer(&can, dev, src->device));
    if (can) {
      const hipError_t e = hipDeviceEnablePeerAccess(src->device, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHECK(e);
      (void)hipGetLastError();  // clear an "already enabled" status
    }
  }
  dst->static_pad = src->static_pad;
  dst->cert_origin_max = src->cert_origin_max;
  dst->wide_base = src->wide_base;
  dst->wide_copy_bytes = src->wide_copy_bytes;
  dst->box_colors = src->box_colors;
  hipStream_t st = (hipStream_t)build_stream(dev);
  if (!st) { set_error("no build stream on device %d", dev); return RT_ERR_HIP; }
  struct Drain { hipStream_t st; ~Drain() { (void)hipStreamSynchronize(st); } } drain{st};
  int64_t& tot = dst->device_bytes;
  tot = 0;
  auto copy = [&](auto** d, const void* sp, size_t bytes) -> int {
    HIPCHECK(hipMalloc((void**)d, bytes));
    tot += (int64_t)bytes;
    if (dev == src->device) HIPCHECK(hipMemcpyAsync(*d, sp, bytes, hipMemcpyDeviceToDevice, st));
    else HIPCHECK(hipMemcpyPeerAsync(*d, dev, sp, src->device, bytes, st));
    return RT_OK;
  };
  if ((rc = copy(&dst->d_nodes, src->d_nodes, src->nodes_bytes))) return rc;
  dst->d_tris = reinterpret_cast<TriRec64*>(reinterpret_cast<char*>(dst->d_nodes) +
                                            (reinterpret_cast<const char*>(src->d_tris) - reinterpret_cast<const char*>(src->d_nodes)));
  if ((rc = copy(&dst->d_nodes4, src->d_nodes4, src->nodes4_bytes))) return rc;
  if ((rc = copy(&dst->d_fshade, src->d_fshade, src->fshade_bytes))) return rc;
  if ((rc = copy(&dst->d_refbox, src->d_refbox, src->refbox_bytes))) return rc;
  if ((rc = copy(&dst->d_mats, src->d_mats, src->mats_bytes))) return rc;
  dst->nodes_bytes = src->nodes_bytes;
  dst->nodes4_bytes = src->nodes4_bytes;
  dst->fshade_bytes = src->fshade_bytes;
  dst->refbox_bytes = src->refbox_bytes;
  dst->mats_bytes = src->mats_bytes;
  HIPCHECK(hipMalloc((void**)&dst->d_stats, kStatSlots * sizeof(unsigned long long)));
  tot += (int64_t)(kStatSlots * sizeof(unsigned long long));
  HIPCHECK(hipMalloc((void**)&dst->d_pf_check, 16));
  HIPCHECK(hipMemsetAsync(dst->d_pf_check, 0, 16, st));
  tot += 16;
  HIPCHECK(hipStreamSynchronize(st));
  return RT_OK;
}

int device_replicate(rt_scene* s) {
  const auto t0 = std::chrono::steady_clock::now();
  s->replicas.clear();
  const int D = s->opts.n_devices;
  for (int k = 1; k < D; k++) {
    std::unique_ptr<rt_scene> r(new rt_scene(s->hsp));
    r->opts = s->opts;
    r->opts.n_devices = 0;
    r->opts.device = s->opts.devices[k];
    r->is_replica = true;
    r->builder_used = s->builder_used;
    r->box_builder_used = s->box_builder_used;
    s->replicas.push_back(std::move(r));
  }
  // one host thread per replica (each makes its device current and copies from device 0's buffers)
  std::vector<int> rcs(s->replicas.size(), RT_OK);
  std::vector<std::string> errs(s->replicas.size());
  std::vector<std::thread> workers;
  for (size_t k = 0; k < s->replicas.size(); k++) {
    auto job = [&, k] {
      rcs[k] = replicate_one(s, s->replicas[k].get());
      if (rcs[k]) errs[k] = rt_last_error();
    };
    try {
      workers.emplace_back(job);
    } catch (const std::exception&) {
      job();  // no helper thread: copy on this one
    }
  }
  for (auto& w : workers) w.join();
  (void)hipSetDevice(s->device);
  for (size_t k = 0; k < rcs.size(); k++)
    if (rcs[k]) {
      set_error("replicating the scene to device %d: %s", s->opts.devices[k + 1], errs[k].c_str());
      s->replicas.clear();
      return rcs[k];
    }
  s->replicate_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return RT_OK;
}

}  // namespace rt

rt_scene::~rt_scene() { rt::device_release(this); }

namespace rt {

// RT_MODE_BOX_COLORS: (re)computes the per-face box-colour sums when the colours changed. The scene's
// streams are drained first (earlier box-colour frames in flight read the table). A replica never sets
// colours itself: render_multi gives the scene its default colours, and with them every replica, before any
// enqueue worker runs (a replica's worker calling rt_scene_set_box_colors wrote every replica's
// colour vector while the other workers read theirs).
static int ensure_face_boxcolor(rt_scene* s) {
  if (s->face_boxcolor_valid) return RT_OK;
  HostScene& hs = s->hs;
  if (s->box_colors.size() != 3 * hs.boxes.size()) {
    if (s->is_replica) { set_error("device %d: replica without box colours", s->device); return RT_ERR_INVALID; }
    const int rc = rt_scene_set_box_colors(s, nullptr);
    if (rc) return rc;
  }
  if (hs.ov3.size() != 3 * (size_t)hs.nv) { set_error("scene has no object-space vertices"); return RT_ERR_INVALID; }
  for (int k = 0; k < s->n_slots; k++) HIPCHECK(hipStreamSynchronize((hipStream_t)s->slots[k].stream));
  const size_t nf = (size_t)hs.nf, nb = hs.boxes.size();
  if (!s->d_face_boxcolor) {
    HIPCHECK(hipMalloc((void**)&s->d_face_boxcolor, 16 * std::max<size_t>(nf, 1)));
    s->device_bytes += (int64_t)(16 * std::max<size_t>(nf, 1));
  }
  if (nf > 0) {
    std::vector<float> fv(9 * nf);
    for (size_t f = 0; f < nf; f++)
      for (int k = 0; k < 3; k++) memcpy(&fv[9 * f + 3 * k], &hs.ov3[3 * (size_t)hs.fidx[3 * f + k]], 12);
    float *d_fv = nullptr, *d_col = nullptr;
    struct Free { float** a; float** b; ~Free() { if (*a) (void)hipFree(*a); if (*b) (void)hipFree(*b); } } free_{&d_fv, &d_col};
    HIPCHECK(hipMalloc((void**)&d_fv, fv.size() * 4));
    HIPCHECK(hipMalloc((void**)&d_col, std::max<size_t>(nb, 1) * 12));
    HIPCHECK(hipMemcpy(d_fv, fv.data(), fv.size() * 4, hipMemcpyHostToDevice));
    if (nb) HIPCHECK(hipMemcpy(d_col, s->box_colors.data(), nb * 12, hipMemcpyHostToDevice));
    hipStream_t st = (hipStream_t)s->stream;
    hipLaunchKernelGGL(k_face_box_colors, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, st, d_fv, s->d_refbox, d_col,
                       (int)nb, (int)nf, s->d_face_boxcolor);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(st));
  }
  s->face_boxcolor_valid = true;
  return RT_OK;
}

static void fill_scene_params(const rt_scene* s, FrameParams& P) {
  memset(&P, 0, sizeof P);
  const HostScene& hs = s->hs;
  P.sc.nodes = s->d_nodes;
  P.sc.tris = s->d_tris;
  P.sc.fshade = s->d_fshade;
  P.sc.refbox = s->d_refbox;
  P.sc.mats = s->d_mats;
  P.sc.root = !is_leaf(hs.root) ? hs.root * 64u : hs.root;
  P.sc.n_nodes = (int32_t)hs.nodes.size();
  P.sc.nodes4 = s->d_nodes4;
  P.sc.root4 = 0;
  P.sc.n_nodes4 = (int32_t)hs.nodes4.size();
  P.sc.static_pad = s->static_pad;
  P.sc.cert_origin_max = s->cert_origin_max;
  P.sc.wide_base = s->wide_base;
  P.sc.wide_copy_bytes = s->wide_copy_bytes;
  P.sc.rec_bytes = (uint32_t)((hs.nodes.size() + hs.tris.size()) * 64);
  P.sc.tri_bytes = (uint32_t)(hs.tris.size() * 64);
  P.sc.all_bytes = (uint32_t)std::min<size_t>(s->nodes_bytes, 0xFFFFFFFFu);
  P.sc.pf_check = s->d_pf_check;
  memcpy(P.sc.Minv, hs.Minv, 64);
  memcpy(P.Minv, hs.Minv, 64);
  memcpy(P.MS, hs.MS, 36);
  const rt_material& dm = s->opts.default_material;
  for (int k = 0; k < 3; k++) { P.defmat.ka[k] = dm.ka[k]; P.defmat.kd[k] = dm.kd[k]; P.defmat.ks[k] = dm.ks[k]; }
  P.defmat.ns = dm.shininess;
  memcpy(P.bg, s->opts.background, 12);
}

// FULL pipeline hand-off buffers: state0, state1 (32 B), refl (32 B), hits1 (8 B), blk0, blk1, list0,
// list1 (4 B) per pixel; then per list wave wcount0/1, woff0/1; then the counters
constexpr size_t kFullBytesPerPixel = 32 + 32 + 32 + 8 + 4 + 4 + 4 + 4;
static size_t full_waves(size_t npix) { return (npix + 63) / 64 + 8; }
static int ensure_full(rt_scene::FrameSlot& f, size_t npix) {
  if (npix <= f.full_pixels) return RT_OK;
  HIPCHECK(hipStreamSynchronize((hipStream_t)f.stream));  // the slot's previous frames may still read it
  if (f.d_full) (void)hipFree(f.d_full);
  f.d_full = nullptr;
  f.full_pixels = 0;
  HIPCHECK(hipMalloc(&f.d_full, npix * kFullBytesPerPixel + 16 * full_waves(npix) + 64));
  f.full_pixels = npix;
  return RT_OK;
}
static void bind_full(const rt_scene::FrameSlot& f, FrameParams& P) {
  char* b = (char*)f.d_full;
  const size_t n = f.full_pixels;
  P.state0 = (HitState*)b;
  P.state1 = (HitState*)(b + 32 * n);
  P.refl = (RayRec*)(b + 64 * n);
  P.hits1 = (uint2*)(b + 96 * n);
  P.blk0 = (uint32_t*)(b + 104 * n);
  P.blk1 = (uint32_t*)(b + 108 * n);
  P.list0 = (uint32_t*)(b + 112 * n);
  P.list1 = (uint32_t*)(b + 116 * n);
  const size_t q = full_waves(n);
  char* w = b + 120 * n;
  P.wcount0 = (uint32_t*)w;
  P.wcount1 = (uint32_t*)(w + 4 * q);
  P.woff0 = (uint32_t*)(w + 8 * q);
  P.woff1 = (uint32_t*)(w + 12 * q);
  P.counters = (uint32_t*)(w + 16 * q);
  P.n_waves_max = (int32_t)q;
}

static int ensure_fb(rt_scene::FrameSlot& f, size_t npix) {
  if (npix <= f.fb_pixels) return RT_OK;
  HIPCHECK(hipStreamSynchronize((hipStream_t)f.stream));  // the slot's previous frames may still use them
  if (f.d_rgb) (void)hipFree(f.d_rgb);
  if (f.d_face) (void)hipFree(f.d_face);
  if (f.d_t) (void)hipFree(f.d_t);
  if (f.d_hits) (void)hipFree(f.d_hits);
  f.d_rgb = nullptr; f.d_face = nullptr; f.d_t = nullptr; f.d_hits = nullptr;
  f.fb_pixels = 0;
  HIPCHECK(hipMalloc((void**)&f.d_rgb, npix * 12));
  HIPCHECK(hipMalloc((void**)&f.d_face, npix * 4));
  HIPCHECK(hipMalloc((void**)&f.d_t, npix * 4));
  HIPCHECK(hipMalloc((void**)&f.d_hits, npix * 8));
  f.fb_pixels = npix;
  return RT_OK;
}

// variant bits (debug knob RT_KERNEL_VARIANT, for A/B measurements; 0 = the measured-best default):
// 1 = binary nodes + lane-register (VGPR) stack, 2 = 4-wide quantised nodes (when the scene has
// them), 4 = XCD-contiguous tile order, 512 / 1024 / 1536 = block runs of 4 / 16 / plain dispatch order
// instead of the default 64-block runs per XCD, 16 = FULL as the stage pipeline (k_full_*) instead of one
// kernel; with 16: 32 / 64 / 128 = per-lane traversal for the reflection rays / the shadow rays of
// reflection hits / the shadow rays of primary hits; 256 = two rays per lane (PRIMARY), 2048 =
// persistent-threads PRIMARY traversal with per-XCD work counters (4096: without stealing); 32768 =
// PRIMARY as trace + shade kernels instead of the fused k_primary_fused; 8192 /
// 16384 = the FULL megakernel's 8-wave / small-scene (6-wave) build regardless of the scene size;
// 65536 = the generic traceRay kernel (k_render_depth) also at the modes' own depths; 131072 = the
// default chunked-XCD dispatch order instead of longest-first (k_order_lpt); 262144 = longest-first
// with half as many cost buckets (2 per octave: coarser, more spatial order kept); 524288 = longest-first
// also while other frames are in flight; 2097152 = PRIMARY packets on the binary tree instead of the fp32
// 4-wide tree (traverse_wide_fast).
// Default: binary nodes + LDS stack, FULL as one kernel (k_render_full) at the occupancy its scene
// size selects.
static int pick_trav(const FrameParams& P, int variant) {
  if (variant & 1) return TRAV_B2_VGPR;
  if ((variant & 2) && P.sc.n_nodes4 > 0) return TRAV_W4;
  return TRAV_B2_LDS;
}
// The product's traversal flavour is the binary tree with the LDS wave stack (TRAV_B2_LDS); the other
// flavours are A/B variants built only into the variants library (variant_launch).
template <bool STATS>
static void launch_trace(const FrameParams& P, int grid, hipStream_t st, int trav) {
  if (trav != TRAV_B2_LDS) {
    VariantCall c;
    c.P = P, c.grid = grid, c.st = st, c.trav = trav, c.stats = STATS;
    variant_launch(VOP_TRACE_PRIMARY, c);
    return;
  }
  hipLaunchKernelGGL((k_trace_primary<STATS, TRAV_B2_LDS>), dim3(grid * (4 / kTraceWPB)), dim3(64 * kTraceWPB), 0, st, P);
}
template <bool STATS, bool HITS>
static void launch_full(const FrameParams& P, int grid, hipStream_t st, int trav, bool small) {
  if (trav != TRAV_B2_LDS) {
    VariantCall c;
    c.P = P, c.grid = grid, c.st = st, c.trav = trav, c.stats = STATS, c.hits = HITS, c.small = small;
    variant_launch(VOP_RENDER_FULL, c);
    return;
  }
  const dim3 g(grid * (4 / kFullWPB) + 3 * P.split_k), b(64 * kFullWPB);
  if (!STATS && small) hipLaunchKernelGGL((k_render_full<STATS, HITS, TRAV_B2_LDS, kFullWavesPerEuSmall>), g, b, 0, st, P);
  else hipLaunchKernelGGL((k_render_full<STATS, HITS, TRAV_B2_LDS>), g, b, 0, st, P);
}

// The variants library defines the strong variant_launch / variants_linked (rt_variants.hip); in the
// product library these weak defaults stand, and rt_render_async refuses a variant-only frame up front.
__attribute__((weak)) bool variants_linked() { return false; }
__attribute__((weak)) int variant_launch(int, const VariantCall&) { return RT_ERR_UNSUPPORTED; }

static std::atomic<int> g_variant{0};  // rt_debug_set_variant(), or RT_KERNEL_VARIANT once rt_debug_env_knobs(1)
static int kernel_variant() { return g_variant.load(std::memory_order_relaxed); }

}  // namespace rt

using namespace rt;

static int check_device_scene(rt_scene* s) {
  if (!s) { set_error("null scene"); return RT_ERR_INVALID; }
  if (s->device == RT_DEVICE_NONE) { set_error("scene was created host-only (RT_DEVICE_NONE)"); return RT_ERR_NO_DEVICE; }
  HIPCHECK(hipSetDevice(s->device));
  return RT_OK;
}

extern "C" int rt_debug_timeline(rt_scene* s, int64_t capacity_waves, uint32_t* out8, int64_t* n_waves) {
  int rc = check_device_scene(s);
  if (rc) return rc;
  const rt_scene::FrameSlot& f = s->slots[s->last_slot];
  if (!(s->last_flags & RT_FRAME_TIMELINE) || !f.d_timeline) { set_error("rt_debug_timeline: last frame had no RT_FRAME_TIMELINE"); return RT_ERR_INVALID; }
  if (n_waves) *n_waves = s->last_timeline_waves;
  if (!out8) return RT_OK;
  if (capacity_waves < s->last_timeline_waves) { set_error("rt_debug_timeline: buffer too small"); return RT_ERR_INVALID; }
  HIPCHECK(hipStreamSynchronize((hipStream_t)f.stream));
  HIPCHECK(hipMemcpy(out8, f.d_timeline, (size_t)s->last_timeline_waves * 32, hipMemcpyDeviceToHost));
  return RT_OK;
}

extern "C" int rt_debug_wave_stats(rt_scene* s, int64_t capacity_waves, uint32_t* out8, int64_t* n_waves) {
  int rc = check_device_scene(s);
  if (rc) return rc;
  const rt_scene::FrameSlot& f = s->slots[s->last_slot];
  if (!(s->last_flags & RT_FRAME_WAVE_STATS) || !(s->last_flags & RT_FRAME_STATS) || !f.d_wave_stats) {
    set_error("rt_debug_wave_stats: last frame had no RT_FRAME_STATS | RT_FRAME_WAVE_STATS");
    return RT_ERR_INVALID;
  }
  if (n_waves) *n_waves = s->last_wave_stats_waves;
  if (!out8) return RT_OK;
  if (capacity_waves < s->last_wave_stats_waves) { set_error("rt_debug_wave_stats: buffer too small"); return RT_ERR_INVALID; }
  HIPCHECK(hipStreamSynchronize((hipStream_t)f.stream));
  HIPCHECK(hipMemcpy(out8, f.d_wave_stats, (size_t)s->last_wave_stats_waves * 32, hipMemcpyDeviceToHost));
  return RT_OK;
}

extern "C" int rt_debug_counters(rt_scene* s, int64_t n, int64_t* out) {
  int rc = check_device_scene(s);
  if (rc) return rc;
  if (!out || n < 0) { set_error("rt_debug_counters: no output"); return RT_ERR_INVALID; }
  if (!(s->last_flags & RT_FRAME_STATS)) { set_error("rt_debug_counters: last frame had no RT_FRAME_STATS"); return RT_ERR_INVALID; }
  HIPCHECK(hipSetDevice(s->device));
  HIPCHECK(hipDeviceSynchronize());
  unsigned long long c[kStatSlots];
  HIPCHECK(hipMemcpy(c, s->d_stats, sizeof c, hipMemcpyDeviceToHost));
  for (int64_t i = 0; i < n; i++) out[i] = i < ST_COUNT ? (int64_t)c[i] : 0;
  return RT_OK;
}

extern "C" int rt_debug_lpt_stats(const rt_scene* s, int64_t* out3) {
  if (!s || !out3) { set_error("rt_debug_lpt_stats: null argument"); return RT_ERR_INVALID; }
  out3[0] = s->lpt.frames;
  out3[1] = s->lpt.sorts;
  out3[2] = s->lpt.valid ? 1 : 0;
  return RT_OK;
}

extern "C" int rt_debug_env_knobs(int32_t on) {
  set_debug_env(on != 0);
  if (on) {  // RT_KERNEL_VARIANT: the A/B kernel variant of this process (rt_debug_set_variant overrides it)
    const char* e = debug_env("RT_KERNEL_VARIANT");
    const int v = e ? atoi(e) : 0;
    g_variant.store(v < 0 ? 0 : v);
  }
  return RT_OK;
}

extern "C" int rt_debug_set_variant(int32_t v) {
  const int prev = kernel_variant();
  g_variant.store(v < 0 ? 0 : v);
  return prev;
}

extern "C" int rt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// Super-tile width of a shard_count-way split (shard_tile_xy, rt_api.h rt_frame): 4x4 tiles (64x64
// pixels) per super-tile when the frame is split, so that the waves an XCD runs together trace
// neighbouring pixels (the rank's L2 working set stays compact): C4 over 8 / 4 GPUs +10% / +7% per GPU
// against single tiles interleaved (profiles/ab/r02_super_tiles_ab.txt); an unsplit frame keeps its tile
// order (super-tiles there: C3 +-1%, C4 -3%). A pure function of the shard count: the render,
// rt_frame_shard_tiles, the pack on every rank and the unpack on rank 0 derive the same layout, whatever
// the process environment or the kernel variant.
static int frame_super_tile(int shard_count) { return shard_count > 1 ? kShardSuperTile : 1; }

// one device's share of a frame (the whole frame on a single-device scene; a replica's shard otherwise)
static int render_one(rt_scene* s, const rt_camera* cam, const rt_light* lights, int32_t n_lights, const rt_frame* fr) {
  int rc = check_device_scene(s);
  if (rc) return rc;
  if (!cam || !fr || fr->width <= 0 || fr->height <= 0 || n_lights < 0 || n_lights > RT_MAX_LIGHTS ||
      (n_lights && !lights)) {
    set_error("rt_render: invalid arguments");
    return RT_ERR_INVALID;
  }
  if (fr->mode != RT_MODE_PRIMARY && fr->mode != RT_MODE_FULL && fr->mode != RT_MODE_BOX_COLORS) {
    set_error("rt_render: bad mode %d", fr->mode);
    return RT_ERR_INVALID;
  }
  if (fr->max_depth < 0 || fr->max_depth > RT_MAX_TRACE_DEPTH) {
    set_error("rt_render: max_depth %d outside 0..%d", fr->max_depth, RT_MAX_TRACE_DEPTH);
    return RT_ERR_INVALID;
  }
  const int sc = fr->shard_count > 0 ? fr->shard_count : 1;
  const int si = fr->shard_index;
  if (si < 0 || si >= sc) { set_error("rt_render: shard %d of %d", si, sc); return RT_ERR_INVALID; }
  const size_t npix = (size_t)fr->width * fr->height;
  const bool boxcol = fr->mode == RT_MODE_BOX_COLORS;
  if (boxcol && (rc = ensure_face_boxcolor(s))) return rc;
  // frames in flight: round-robin over the slots; a slot's stream orders its own frames, frames on
  // different slots overlap (tail of one frame with the start of the next)
  const int slot_id = s->next_slot;
  rt_scene::FrameSlot& slot = s->slots[slot_id];
  if ((rc = ensure_fb(slot, npix))) return rc;
  FrameParams P;
  fill_scene_params(s, P);
  // camera (camera.hpp:115-118,155-173,263-266)
  affinv(cam->view_matrix, P.vinv);
  {
    float L[9], Li[9];
    linear_of(cam->view_matrix, L);
    m3inv(L, Li);
    const f3 e = m3v3(Li, f3{-cam->view_matrix[12], -cam->view_matrix[13], -cam->view_matrix[14]});
    P.eye[0] = e.x; P.eye[1] = e.y; P.eye[2] = e.z;
    const f3 eo = affv3(s->hs.Minv, e);
    P.eye_obj[0] = eo.x; P.eye_obj[1] = eo.y; P.eye_obj[2] = eo.z;
  }
  memcpy(P.vp, cam->viewport, 16);
  const float persp = (float)((double)1.0f / tan((double)(cam->fovy / 2.0f) * (M_PI / 180.0)));
  const float scale = (float)(1.0 / (double)persp);
  P.xscale = cam->aspect_ratio * scale;
  P.yscale = scale;
  P.n_lights = n_lights;
  {  // calculateColor's order: point lights first, then directional lights (each in array order)
    int k = 0;
    for (int pass = 0; pass < 2; pass++)
      for (int l = 0; l < n_lights; l++) {
        const int kind = lights[l].kind == RT_LIGHT_DIRECTIONAL ? RT_LIGHT_DIRECTIONAL : RT_LIGHT_POINT;
        if (kind != (pass ? RT_LIGHT_DIRECTIONAL : RT_LIGHT_POINT)) continue;
        memcpy(P.lights[k].p, lights[l].position, 12);
        memcpy(P.lights[k].c, lights[l].color, 12);
        P.lights[k].kind = kind;
        k++;
      }
  }
  P.W = fr->width;
  P.H = fr->height;
  P.tiles_x = (fr->width + 15) / 16;
  P.tiles_y = (fr->height + 15) / 16;
  const int ntiles = P.tiles_x * P.tiles_y;
  P.shard_index = si;
  P.shard_count = sc;
  P.super_tile = frame_super_tile(sc);
  P.n_tiles_shard = shard_tile_slots(P.tiles_x, P.tiles_y, P.super_tile, si, sc);
  (void)ntiles;
  P.mode = fr->mode;
  P.flags = fr->flags;
  P.rgb = slot.d_rgb;
  P.face_out = slot.d_face;
  P.t_out = slot.d_t;
  P.stats = s->d_stats;
  P.hits = slot.d_hits;
  P.face_boxcolor = s->d_face_boxcolor;
  hipStream_t st = (hipStream_t)slot.stream;
  const bool stats = (fr->flags & RT_FRAME_STATS) != 0;
  const bool hits = (fr->flags & RT_FRAME_WRITE_HITS) != 0;
  if (stats) {
    // the counters are shared: a counting frame waits for every frame in flight on the other slots
    for (int k = 0; k < s->n_slots; k++)
      if (k != slot_id && s->slots[k].last_done) HIPCHECK(hipStreamWaitEvent(st, (hipEvent_t)s->slots[k].last_done, 0));
    HIPCHECK(hipMemsetAsync(s->d_stats, 0, kStatSlots * sizeof(unsigned long long), st));
  }
  const int grid = P.n_tiles_shard;
  const int variant = kernel_variant();
  if (variant & 2097152) P.sc.wide_copy_bytes = 0;  // PRIMARY octant packets on the binary tree (A/B)
  // PRIMARY with two packets per wave (k_primary_dual): variant bit 1048576
  const bool dual = (fr->mode == RT_MODE_PRIMARY || fr->mode == RT_MODE_BOX_COLORS) && !stats &&
                    (fr->max_depth <= 1 || fr->mode == RT_MODE_BOX_COLORS) && !(variant & (1 | 2 | 4 | 32768 | 256 | 2048 | 65536)) &&
                    (variant & 1048576);
  const size_t units = (size_t)grid * (dual ? 2 : 4);  // one-wave blocks of the render kernel
  // (RT_TIMELINE_SPLIT, diagnostics only: a timeline frame keeps the lone-frame split of its costliest
  // waves; one record per block, so room for the 3 K extra blocks)
  const bool timeline_split = (fr->flags & RT_FRAME_TIMELINE) && debug_env("RT_TIMELINE_SPLIT");
  if (fr->flags & RT_FRAME_TIMELINE) {  // one record per one-wave block of the render kernel
    const size_t waves = timeline_split ? 2 * units : units;
    if (waves > slot.timeline_waves) {
      HIPCHECK(hipStreamSynchronize(st));
      if (slot.d_timeline) (void)hipFree(slot.d_timeline);
      slot.d_timeline = nullptr;
      slot.timeline_waves = 0;
      HIPCHECK(hipMalloc((void**)&slot.d_timeline, waves * 32));
      slot.timeline_waves = waves;
    }
    HIPCHECK(hipMemsetAsync(slot.d_timeline, 0, waves * 32, st));
    P.timeline = slot.d_timeline;
    s->last_timeline_waves = (int64_t)waves;
  }
  if (stats && (fr->flags & RT_FRAME_WAVE_STATS)) {  // per logical wave (tile * 4 + quarter)
    const size_t lw = (size_t)grid * 4;
    if (lw > slot.wave_stats_waves) {
      HIPCHECK(hipStreamSynchronize(st));
      if (slot.d_wave_stats) (void)hipFree(slot.d_wave_stats);
      slot.d_wave_stats = nullptr;
      slot.wave_stats_waves = 0;
      HIPCHECK(hipMalloc((void**)&slot.d_wave_stats, lw * 32));
      slot.wave_stats_waves = lw;
    }
    HIPCHECK(hipMemsetAsync(slot.d_wave_stats, 0, lw * 32, st));
    P.wave_stats = slot.d_wave_stats;
    s->last_wave_stats_waves = (int64_t)lw;
  }
  if (fr->mode == RT_MODE_FULL && (variant & 16)) {
    if (sc > 1) { set_error("rt_render: the FULL stage-pipeline variant renders whole frames only"); return RT_ERR_UNSUPPORTED; }
    // sized by the 16x16-padded frame: every wave of the tile grid has a count slot
    const size_t npad = (size_t)P.tiles_x * 16 * (size_t)P.tiles_y * 16;
    if ((rc = ensure_full(slot, npad))) return rc;
    bind_full(slot, P);
  }
  // a frame alone on the GPU: no other frame of this scene in flight (the dispatch order below and the
  // longest-first order depend on it)
  bool alone = true;
  for (int k = 0; k < s->n_slots; k++)
    if (k != slot_id && s->slots[k].last_done && hipEventQuery((hipEvent_t)s->slots[k].last_done) == hipErrorNotReady)
      alone = false;
  // block order: chunked XCD order -- block b runs on XCD b % 8, and the XCD's k-th block takes the k-th
  // position of its runs of C consecutive blocks. Scenes whose records exceed the chip's 32 MiB of L2 take
  // one contiguous band of the frame per XCD (C = units / 8), so that each XCD's 4 MiB L2 holds the part
  // of the scene its band sees (L2 hit 0.90 -> 0.94 on C3): a frame alone on the GPU +4.3% on C3, +8.7%
  // on C4. With frames in flight the XCDs' bands rotate frame by frame (xcd_rot), so that no XCD keeps
  // the costliest band of every frame: +1.5% on C3 at 100 frames (fixed bands lost 1-3% there); all in
  // profiles/ab/r05_xcd_bands_ab.txt. L2-resident scenes keep runs of C = 64 (bunny one frame alone with
  // bands: PRIMARY -9%, FULL -6..-12% -- no locality to gain, and the bands differ in cost; runs of
  // 32 .. 256 within noise, profiles/ab/r05_xcd_run_ab.txt; 64 against the plain order -4% trace time on
  // C3 before the bands). Variant bits 512 / 1024 select runs of 4 / 16 blocks, 1536 the plain dispatch
  // order, 4 one contiguous tile range per XCD (256-thread blocks)
  {
    const int sel = (variant >> 9) & 3;
    const bool l2_resident = (s->hs.nodes.size() + s->hs.tris.size()) * 64 <= kFullSmallSceneBytes;
    const int run = l2_resident ? 64 : std::max<int>(2, (int)(units / 8));
    P.xcd_remap = (variant & 4) ? 1 : (sel == 0 ? run : sel == 1 ? 4 : sel == 2 ? 16 : 0);
    const char* run_env = debug_env("RT_XCD_RUN");  // (A/B only: another run length of the chunked order)
    if (run_env && atoi(run_env) >= 2) P.xcd_remap = atoi(run_env);
    if (!alone && !l2_resident && P.xcd_remap >= 2) P.xcd_rot = (int32_t)(s->band_rot++ & 7u);
  }
  const int trav = pick_trav(P, variant);
  {
    const bool prim_mode = fr->mode == RT_MODE_PRIMARY || boxcol;
    const bool need = trav != TRAV_B2_LDS || dual || (fr->mode == RT_MODE_FULL && (variant & 16)) ||
                      (prim_mode && !stats && (variant & (256 | 2048)));
    if (need && !variants_linked()) {
      set_error("rt_render: kernel variant %d is an A/B build option, not in this library (make variants)", variant);
      return RT_ERR_UNSUPPORTED;
    }
  }
  // longest-first dispatch (k_order_lpt) for the one-wave render kernels of the default build: this
  // slot's previous frame of the same shape left its per-wave costs and the order computed from them
  // box-colour frames return before any reflection: one depth, the PRIMARY kernels' dispatch
  const bool prim = fr->mode == RT_MODE_PRIMARY || boxcol;
  const int mode_depth0 = fr->mode == RT_MODE_FULL ? 2 : 1;
  const int depth0 = (fr->max_depth > 0 && !boxcol) ? fr->max_depth : mode_depth0;
  const bool one_wave_kernel = !stats && trav == TRAV_B2_LDS &&
                               ((prim && depth0 == 1 && !(variant & (32768 | 256 | 2048 | 65536))) ||
                                (fr->mode == RT_MODE_FULL && depth0 == 2 && !(variant & (16 | 65536))) ||
                                (!boxcol && (depth0 != mode_depth0 || (variant & 65536))));
  // Only for a frame that has the GPU to itself (no other frame of this scene in flight): then the
  // tail of the frame would leave the GPU idle and longest-first fills it (one frame at a time: C3
  // +18%, C5 +28%); with frames in flight the next frame fills the tail and the default order's tile
  // locality is worth more (LPT measured -3..-7% there). Variant 524288 forces it, 131072 disables it.
  // (variant 524288, A/B only: also with frames in flight -- then the map is shared by frames that overlap,
  // a race on the order's values only: any order is a permutation)
  const bool lpt = one_wave_kernel && !(variant & 131072) && P.xcd_remap >= 2 && grid > 0 && (alone || (variant & 524288));
  bool lpt_sort = false;
  int lpt_dilate = 0;
  rt_scene::LptMap& lm = s->lpt;
  if (lpt) {
    const size_t waves = units;
    if (waves > lm.waves) {
      for (int k = 0; k < s->n_slots; k++) HIPCHECK(hipStreamSynchronize((hipStream_t)s->slots[k].stream));
      if (lm.d_cost) (void)hipFree(lm.d_cost);
      if (lm.d_cost_dil) (void)hipFree(lm.d_cost_dil);
      if (lm.d_order) (void)hipFree(lm.d_order);
      lm.d_cost = lm.d_cost_dil = lm.d_order = nullptr;
      lm.waves = 0;
      lm.valid = false;
      HIPCHECK(hipMalloc((void**)&lm.d_cost, waves * 4));
      HIPCHECK(hipMalloc((void**)&lm.d_cost_dil, waves * 4));
      HIPCHECK(hipMalloc((void**)&lm.d_order, waves * 4));
      HIPCHECK(hipMemsetAsync(lm.d_cost, 0, waves * 4, st));  // (each sort clears what it read after this)
      HIPCHECK(hipMemsetAsync(lm.d_cost_dil, 0, waves * 4, st));
      lm.waves = waves;
    }

    const int64_t key[8] = {fr->width, fr->height, si, sc, fr->mode, depth0, P.xcd_remap, (int64_t)waves};
    const bool same = lm.valid && memcmp(key, lm.key, sizeof key) == 0;
    if (same) P.order = lm.d_order;
    // The order is recomputed from this frame's costs after the frame when it is missing, has served
    // kLptRefresh frames, or -- kLptMoved -- the camera has moved since the frame that recorded it (the
    // reference's Flycamera moves every frame while a key is held, flyscene.cpp:116-127): a moving camera then
    // dispatches every lone frame by the previous frame's costs. The sort costs a few microseconds on the frame's
    // stream. (RT_LPT_REFRESH / RT_LPT_MOVED: A/B knobs, debug environment only.)
    const char* refresh_env = debug_env("RT_LPT_REFRESH");
    const char* moved_env = debug_env("RT_LPT_MOVED");
    const int refresh = refresh_env ? std::max(1, atoi(refresh_env)) : kLptRefresh;
    const bool key_moved = moved_env ? atoi(moved_env) != 0 : kLptMoved;
    const bool moved = memcmp(cam->view_matrix, lm.view, sizeof lm.view) != 0;
    // moving: this frame's camera differs from the previous lone frame's -> its costs are placed where each wave's
    // content is expected in the next frame (the camera repeating its step, FrameParams::pred) and dilated before the
    // sort (whole frames only: the wave grid of a shard is not contiguous). RT_LPT_DILATE / RT_LPT_PRED: A/B knobs
    const bool moving = memcmp(cam->view_matrix, lm.prev_view, sizeof lm.prev_view) != 0;
    float prev_view[16];
    memcpy(prev_view, lm.prev_view, sizeof prev_view);
    memcpy(lm.prev_view, cam->view_matrix, sizeof lm.prev_view);
    // Measured under the reference's moving camera (profiles/ab/r06_moving_camera_ab.txt, one frame at a time):
    // an L2-resident scene whose lone frames split their costliest waves (C5: the bunny's silhouette tiles) loses
    // the split's gain with a map even one frame old (0.38 ms against 0.227 with an exact map) and regains most
    // of it with a fresh, dilated map (0.31 ms), more with the costs moved to their predicted waves (0.26 ms,
    // profiles/ab/r06_moving_prediction_ab.txt); the soup's per-wave costs decorrelate within a frame of motion
    // (fresh or 8 frames old, dilated or not: 0.233-0.237 ms, no map 0.245; predicted: 0.226 ms, but the sort on
    // every frame's path takes it back), so large scenes keep the 8-frame refresh and spend no sort per frame.
    // (RT_LPT_MOVED forces either rule.)
    const bool l2_small = (s->hs.nodes.size() + s->hs.tris.size()) * 64 <= kFullSmallSceneBytes;
    const bool resort_on_motion = moved_env ? key_moved : (key_moved && l2_small);
    // (a dilated map is replaced by the first frame after the camera stopped: dilated, the map spends the split on
    // the costly waves' neighbours -- 0.30 ms instead of 0.22 on C5 at an exact pose)
    lpt_sort = !same || ++lm.age >= refresh || (resort_on_motion && moved) || (lm.dilated_map && !moving);
    lm.frames++;
    if (lpt_sort) {
      memcpy(lm.key, key, sizeof key);
      memcpy(lm.view, cam->view_matrix, sizeof lm.view);
      lm.valid = false;  // until this frame's k_order_lpt has been queued
      P.cost = lm.d_cost;
      lm.sorts++;
      // RT_LPT_PRED (A/B knob): each wave's cost lands where its content is expected next frame (FrameParams::pred)
      const char* pred_env = debug_env("RT_LPT_PRED");
      const bool pred = pred_env ? atoi(pred_env) != 0 : kLptPred;
      const char* dil_env = debug_env("RT_LPT_DILATE");  // (2 + 2 r)^2 <= 64 lanes
      const int r = dil_env ? std::max(0, std::min(3, atoi(dil_env))) : (pred ? kLptDilatePred : kLptDilate);
      const char* dilw_env = debug_env("RT_LPT_DILW");  // A/B knob: the ring's weight 1 - 2^-w (default 3/4)
      const int dil_w = dilw_env ? std::max(1, std::min(8, atoi(dilw_env))) : 2;
      const bool moving_map = moving && resort_on_motion && sc == 1 && !dual && (r > 0 || pred);
      lpt_dilate = moving_map;
      lm.dilated_map = moving_map;
      if (moving_map) {
        lm.dilated++;
        P.cost_dil = lm.d_cost_dil;
        P.dil_r = r;
        P.dil_w = dil_w;
        if (pred) {  // a pixel's view-space direction (nx xscale, ny yscale, -1) as (a px + b, c py + e, -1)
          P.pred = 1;
          P.pred_proj[0] = 2.0f * P.xscale / P.vp[2];
          P.pred_proj[1] = -(2.0f * P.vp[0] / P.vp[2] + 1.0f) * P.xscale;
          P.pred_proj[2] = -2.0f * P.yscale / P.vp[3];
          P.pred_proj[3] = (1.0f + 2.0f * P.vp[1] / P.vp[3]) * P.yscale;
          camera_step(prev_view, cam->view_matrix, P.pred_step);
        }
      }
    }
  }
  if (s->ev_used + 3 > s->ev_pool.size()) {  // (init_slots creates kEventFrames frames' worth up front)
    if (s->ev_pool.size() >= 3 * 2048) { set_error("more than 2048 renders without rt_synchronize"); return RT_ERR_INVALID; }
    for (int k = 0; k < 3; k++) {
      hipEvent_t e;
      HIPCHECK(hipEventCreate(&e));
      s->ev_pool.push_back(e);
    }
  }
  // three events per frame: start | after the traversal kernel | after the frame
  hipEvent_t ev_a = (hipEvent_t)s->ev_pool[s->ev_used], ev_m = (hipEvent_t)s->ev_pool[s->ev_used + 1],
             ev_b = (hipEvent_t)s->ev_pool[s->ev_used + 2];
  s->ev_used += 3;
  HIPCHECK(hipEventRecord(ev_a, st));
  const int mode_depth = fr->mode == RT_MODE_FULL ? 2 : 1;
  const int depth = depth0;
  P.max_depth = depth;
  P.shadows = fr->mode == RT_MODE_FULL ? 1 : 0;
  if (grid > 0 && !boxcol && (depth != mode_depth || (variant & 65536))) {
    // any other recursion limit: the generic traceRay kernel (one 8x8 wave per block)
    const dim3 g(grid * 4), b(64);
    if (stats) { if (hits) hipLaunchKernelGGL((k_render_depth<true, true>), g, b, 0, st, P); else hipLaunchKernelGGL((k_render_depth<true, false>), g, b, 0, st, P); }
    else { if (hits) hipLaunchKernelGGL((k_render_depth<false, true>), g, b, 0, st, P); else hipLaunchKernelGGL((k_render_depth<false, false>), g, b, 0, st, P); }
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipEventRecord(ev_m, st));
  } else if (grid > 0) {
    if (dual && grid > 0) {
      VariantCall vc;
      vc.P = P, vc.units = units, vc.st = st, vc.hits = hits, vc.boxcol = boxcol;
      variant_launch(VOP_PRIMARY_DUAL, vc);
      HIPCHECK(hipGetLastError());
      HIPCHECK(hipEventRecord(ev_m, st));
    } else if (prim && !stats && !(variant & (32768 | 256 | 2048)) && trav == TRAV_B2_LDS) {
      // lone frames of small scenes: the costliest waves as 16-lane sub-waves, as k_render_full does
      // (RT_SPLIT_KP waves)
      const char* split_p_env = debug_env("RT_SPLIT_KP");
      const int split_p = split_p_env ? atoi(split_p_env) : kSplitKPrimary;
      // (RT_SPLIT_KP_ANY, A/B only: split lone frames of any scene size)
      const bool small_p = (s->hs.nodes.size() + s->hs.tris.size()) * 64 <= kFullSmallSceneBytes || debug_env("RT_SPLIT_KP_ANY");
      P.split_k = (P.order && small_p && (!P.timeline || timeline_split) && kTraceWPB == 1)
                      ? std::max(0, std::min<int>(split_p, (int)(units / 4))) & ~7 : 0;
      // (sub-waves take the max into the cost map, which the previous sort left at zero)
      const dim3 g(grid * (4 / kTraceWPB) + 3 * P.split_k), b(64 * kTraceWPB);
      // RT_LDS_PAD (diagnostics): extra dynamic LDS per block, to cap the resident waves per CU in
      // occupancy experiments (160 KiB / (pad + 1 KiB) blocks per CU)
      const char* lds_pad_env = debug_env("RT_LDS_PAD");
      const unsigned lds_pad = lds_pad_env ? (unsigned)atoi(lds_pad_env) : 0u;
      if (boxcol) {
        if (hits) hipLaunchKernelGGL((k_primary_fused<true, true>), g, b, lds_pad, st, P);
        else hipLaunchKernelGGL((k_primary_fused<false, true>), g, b, lds_pad, st, P);
      } else {
        if (hits) hipLaunchKernelGGL(k_primary_fused<true>, g, b, lds_pad, st, P);
        else hipLaunchKernelGGL(k_primary_fused<false>, g, b, lds_pad, st, P);
      }
      HIPCHECK(hipGetLastError());
      HIPCHECK(hipEventRecord(ev_m, st));
    } else if (prim) {
      if (stats) launch_trace<true>(P, grid, st, trav);
      else if ((variant & 256) && trav == TRAV_B2_LDS) {
        VariantCall vc;
        vc.P = P, vc.grid = grid, vc.st = st;
        variant_launch(VOP_PRIMARY_X2, vc);
      } else if ((variant & 2048) && trav == TRAV_B2_LDS && !P.wcount0) {
        if (!slot.d_queue) HIPCHECK(hipMalloc((void**)&slot.d_queue, 8 * sizeof(uint32_t)));
        HIPCHECK(hipMemsetAsync(slot.d_queue, 0, 8 * sizeof(uint32_t), st));
        VariantCall vc;
        vc.P = P, vc.grid = grid, vc.st = st, vc.variant = variant, vc.device = s->device, vc.queue = slot.d_queue;
        variant_launch(VOP_PRIMARY_PERSISTENT, vc);
      }
      else launch_trace<false>(P, grid, st, trav);
      HIPCHECK(hipGetLastError());
      HIPCHECK(hipEventRecord(ev_m, st));
      if (boxcol) {
        if (hits) hipLaunchKernelGGL((k_shade_primary<true, true>), dim3(grid), dim3(256), 0, st, P);
        else hipLaunchKernelGGL((k_shade_primary<false, true>), dim3(grid), dim3(256), 0, st, P);
      } else {
        if (hits) hipLaunchKernelGGL((k_shade_primary<true, false>), dim3(grid), dim3(256), 0, st, P);
        else hipLaunchKernelGGL((k_shade_primary<false, false>), dim3(grid), dim3(256), 0, st, P);
      }
    } else if (!(variant & 16)) {  // FULL as one kernel (default); 16 = the stage pipeline
      // occupancy by scene size (k_render_full); variant bits 8192 / 16384 force the 8-wave / small build
      const size_t rec_bytes = (s->hs.nodes.size() + s->hs.tris.size()) * 64;
      const bool small = (variant & 16384) || (!(variant & 8192) && rec_bytes <= kFullSmallSceneBytes);
      // a lone frame of a small (L2-resident) scene, dispatched longest-first, splits its costliest waves
      // into 16-lane sub-waves (FrameParams::split_k; RT_SPLIT_K waves, rounded down to a multiple of 8
      // and at most a quarter of the frame's waves): such a frame's span is its slowest waves' (C5 one
      // frame alone: 2.2 resident waves per SIMD on average), and a 16-ray packet of their incoherent
      // secondary rays finishes sooner. A large scene's FULL frame is not tail bound (5.7 resident waves
      // per SIMD on the soup) and the extra waves only cost (-6%), so it keeps whole waves. Results do not
      // depend on the grouping (exact per-lane culling, (t, rank) argmin).
      const char* split_k_env = debug_env("RT_SPLIT_K");
      const int split_env = split_k_env ? atoi(split_k_env) : kSplitK;
      if (P.order && small && (!P.timeline || timeline_split) && !stats && kFullWPB == 1 && trav == TRAV_B2_LDS)
        P.split_k = std::max(0, std::min<int>(split_env, (int)(units / 4))) & ~7;
      else
        P.split_k = 0;
      // (sub-waves take the max into the cost map, which the previous sort left at zero)
      if (stats) { if (hits) launch_full<true, true>(P, grid, st, trav, small); else launch_full<true, false>(P, grid, st, trav, small); }
      else { if (hits) launch_full<false, true>(P, grid, st, trav, small); else launch_full<false, false>(P, grid, st, trav, small); }
      HIPCHECK(hipEventRecord(ev_m, st));
    } else {
      VariantCall vc;
      vc.P = P, vc.grid = grid, vc.st = st, vc.trav = trav, vc.variant = variant, vc.stats = stats, vc.hits = hits,
      vc.ev_m = ev_m;
      variant_launch(VOP_FULL_PIPELINE, vc);
    }
    HIPCHECK(hipGetLastError());
  } else {
    HIPCHECK(hipEventRecord(ev_m, st));
  }
  // the sort for the scene's next lone frame of this shape, on this frame's stream before its done event: the next
  // lone frame is queued only once every other slot's done event has passed (`alone`), so it finds the order
  // complete whichever slot it takes
  if (lpt_sort) {
    uint32_t* in = lpt_dilate ? lm.d_cost_dil : lm.d_cost;
    hipLaunchKernelGGL(k_order_lpt, dim3(8), dim3(kLptThreads), 0, st, in, lpt_dilate ? lm.d_cost : (uint32_t*)nullptr,
                       lm.d_order, (int)units, P.xcd_remap, (variant & 262144) ? 1 : 0);
    HIPCHECK(hipGetLastError());
    lm.valid = true;
    lm.age = 0;
  }
  HIPCHECK(hipEventRecord(ev_b, st));
  slot.last_done = ev_b;
  s->last_slot = slot_id;
  s->next_slot = (slot_id + 1) % s->n_slots;
  s->last_W = fr->width;
  s->last_H = fr->height;
  s->last_shard_index = si;
  s->last_shard_count = sc;
  s->last_flags = fr->flags;
  // primary rays of this shard: pixels inside the frame of the shard's tiles (a walk over the shard's tiles,
  // done once per frame shape: it is host time on every frame's enqueue path otherwise)
  const int64_t rkey[4] = {fr->width, fr->height, si, sc};
  if (memcmp(rkey, s->rays_key, sizeof rkey) != 0) {
    int64_t rays = 0;
    for (int L = 0; L < P.n_tiles_shard; L++) {
      int tx, ty;
      shard_tile_xy(P.tiles_x, P.super_tile, si, sc, L, tx, ty);
      if (tx < P.tiles_x && ty < P.tiles_y)
        rays += (int64_t)std::min(16, fr->width - tx * 16) * std::min(16, fr->height - ty * 16);
    }
    memcpy(s->rays_key, rkey, sizeof rkey);
    s->rays_of_key = rays;
  }
  s->last_rays = s->rays_of_key;
  s->pending = true;
  return RT_OK;
}

// RT_CHECK_PREFETCH debug build: an out-of-range scalar prefetch offset recorded by the kernels fails the call
static int check_prefetch_word(rt_scene* s) {
#ifdef RT_CHECK_PREFETCH
  uint32_t w = 0;
  HIPCHECK(hipMemcpy(&w, s->d_pf_check, 4, hipMemcpyDeviceToHost));
  if (w) {
    set_error("RT_CHECK_PREFETCH: out-of-range scalar load offset (sites 0x%x: 0 node, 1/2 child prefetch, 3 leaf "
              "prefetch, 4 wide prefetch, 5 wide node)", w);
    return RT_ERR_HIP;
  }
#endif
  (void)s;
  return RT_OK;
}

static int sync_one(rt_scene* s, rt_stats* out) {
  int rc = check_device_scene(s);
  if (rc) return rc;
  // every slot's stream drained. (Round 6 tried waiting for each slot's frame-done event only, so that a lone
  // frame's trailing sort could overlap the caller's turn: the same frames with 4 in flight then ran 4-25% slower
  // from one process to the next -- C2 29.8-35.0 against 37.6-38.5 Grays/s, profiles/ab/r06_sync_ab.txt.)
  for (int k = 0; k < s->n_slots; k++) HIPCHECK(hipStreamSynchronize((hipStream_t)s->slots[k].stream));
  if ((rc = check_prefetch_word(s))) return rc;
  struct Reset {
    rt_scene* s;
    ~Reset() {
      s->ev_used = 0;
      s->pending = false;
      for (int k = 0; k < s->n_slots; k++) s->slots[k].last_done = nullptr;
    }
  } reset_{s};
  if (out) {
    memset(out, 0, sizeof *out);
    double tot = 0.0, trav = 0.0;
    for (size_t k = 0; k + 3 <= s->ev_used; k += 3) {
      float ms = 0.0f, ms1 = 0.0f;
      HIPCHECK(hipEventElapsedTime(&ms, (hipEvent_t)s->ev_pool[k], (hipEvent_t)s->ev_pool[k + 2]));
      HIPCHECK(hipEventElapsedTime(&ms1, (hipEvent_t)s->ev_pool[k], (hipEvent_t)s->ev_pool[k + 1]));
      tot += ms;
      trav += ms1;
    }
    out->kernel_ms = tot;
    out->trace_kernel_ms = trav;
    out->launches = (int64_t)(s->ev_used / 3);
    out->primary_rays = s->last_rays;
    out->total_rays = s->last_rays;
    if (s->last_flags & RT_FRAME_STATS) {
      unsigned long long c[kStatSlots];
      HIPCHECK(hipMemcpy(c, s->d_stats, sizeof c, hipMemcpyDeviceToHost));
      out->node_visits = (int64_t)c[ST_NODE];
      out->tri_tests = (int64_t)c[ST_TRI];
      out->wave_node_fetches = (int64_t)(c[ST_WNODE] + c[ST_WWIDE]);
      out->wave_node_bytes = (int64_t)(64 * c[ST_WNODE] + sizeof(Node128) * c[ST_WWIDE]);
      out->wave_tri_fetches = (int64_t)c[ST_WTRI];
      out->hits = (int64_t)c[ST_HITS];
      out->total_rays = (int64_t)c[ST_TOTAL];
    }
  }
  return RT_OK;
}

// ------------------------------------------------------------------------------------------------
// Multi-device scenes (rt_scene_opts.n_devices > 1): one frame over the scene's replicas
// ------------------------------------------------------------------------------------------------
static rt_scene* replica(rt_scene* s, int k) { return k == 0 ? s : s->replicas[(size_t)k - 1].get(); }
static int n_replicas(const rt_scene* s) { return 1 + (int)s->replicas.size(); }

// Enqueue workers of a multi-device scene. Queueing one device's share of a frame costs ~20 us of host time
// (frame parameters, three events, the launch); done for D devices one after the other on the caller's
// thread that is D x 20 us per frame, which at 8 devices exceeds a device's share of the frame. So each
// further replica has a host thread of its own: the caller posts the frame to every worker, queues replica 0
// itself, and returns once every worker has queued its share (so errors are reported by this call and the
// frames stay in call order on every device). A worker waits for work spinning for a while, then blocks.
namespace rt {
struct EnqueueWorker {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<uint32_t> posted{0}, done{0};  // job sequence numbers
  bool quit = false;
  rt_scene* r = nullptr;
  rt_camera cam;
  rt_light lights[RT_MAX_LIGHTS];
  int32_t n_lights = 0;
  rt_frame fr;
  int rc = RT_OK;
  std::string err;
};

static void worker_loop(EnqueueWorker* w) {
  uint32_t seen = 0;
  for (;;) {
    // spin ~50 us for the next frame (frames come at sub-millisecond cadence), then block
    for (int i = 0; i < 20000 && w->posted.load(std::memory_order_acquire) == seen; i++) __builtin_ia32_pause();
    if (w->posted.load(std::memory_order_acquire) == seen) {
      std::unique_lock<std::mutex> lk(w->mu);
      w->cv.wait(lk, [&] { return w->quit || w->posted.load(std::memory_order_acquire) != seen; });
    }
    {
      std::lock_guard<std::mutex> lk(w->mu);
      if (w->quit && w->posted.load(std::memory_order_acquire) == seen) return;
    }
    seen = w->posted.load(std::memory_order_acquire);
    w->rc = render_one(w->r, &w->cam, w->n_lights ? w->lights : nullptr, w->n_lights, &w->fr);
    if (w->rc) w->err = rt_last_error();
    w->done.store(seen, std::memory_order_release);
    { std::lock_guard<std::mutex> lk(w->mu); }
    w->cv.notify_all();
  }
}

void stop_workers(rt_scene* s) {
  for (auto& w : s->workers) {
    {
      std::lock_guard<std::mutex> lk(w->mu);
      w->quit = true;
    }
    w->cv.notify_all();
    if (w->th.joinable()) w->th.join();
  }
  s->workers.clear();
}

static int start_workers(rt_scene* s) {
  if (s->workers.size() == s->replicas.size()) return RT_OK;
  stop_workers(s);
  for (auto& r : s->replicas) {
    auto w = std::make_shared<EnqueueWorker>();
    w->r = r.get();
    try {
      w->th = std::thread(worker_loop, w.get());
    } catch (const std::exception&) {
      stop_workers(s);  // no threads: the caller queues every device itself
      return RT_ERR_UNSUPPORTED;
    }
    s->workers.push_back(std::move(w));
  }
  return RT_OK;
}

}  // namespace rt

// The caller's frame (shard si of sc, normally the whole frame) goes to the D replicas as shards of an
// sc*D-way split: replica k renders shard si + sc*k, so the D shards together are exactly the caller's
// shard (super-tile t: t % (sc*D) = si + sc*k  <=>  t % sc = si). Each replica renders on its own slot
// streams, its launches queued by its own worker thread (replica 0's by the caller); nothing is exchanged
// between devices.
static int render_multi(rt_scene* s, const rt_camera* cam, const rt_light* lights, int32_t n_lights, const rt_frame* fr) {
  if (!fr || !cam || n_lights < 0 || n_lights > RT_MAX_LIGHTS || (n_lights && !lights)) {
    set_error("rt_render: invalid arguments");
    return RT_ERR_INVALID;
  }
  const int D = n_replicas(s);
  const int sc = fr->shard_count > 0 ? fr->shard_count : 1, si = fr->shard_index;
  if (si < 0 || si >= sc) { set_error("rt_render: shard %d of %d", si, sc); return RT_ERR_INVALID; }
  if ((int64_t)sc * D > (1 << 24)) { set_error("rt_render: %d shards x %d devices", sc, D); return RT_ERR_INVALID; }
  auto shard_of = [&](int k) {
    rt_frame f = *fr;
    f.shard_count = sc * D;
    f.shard_index = si + sc * k;
    return f;
  };
  // the reference's default box colours (setRandomColor draws) reach every replica here, on the caller's
  // thread, before any worker reads its replica's colours
  if (fr->mode == RT_MODE_BOX_COLORS && s->box_colors.size() != 3 * s->hs.boxes.size()) {
    const int rc = rt_scene_set_box_colors(s, nullptr);
    if (rc) return rc;
  }
  if (start_workers(s) != RT_OK) {  // (no helper threads: queue every device from this thread)
    for (int k = 0; k < D; k++) {
      const rt_frame f = shard_of(k);
      const int rc = render_one(replica(s, k), cam, lights, n_lights, &f);
      if (rc) return rc;
    }
    HIPCHECK(hipSetDevice(s->device));
    return RT_OK;
  }
  std::vector<uint32_t> seq(s->workers.size());
  for (size_t k = 0; k < s->workers.size(); k++) {
    EnqueueWorker& w = *s->workers[k];
    {
      std::lock_guard<std::mutex> lk(w.mu);
      w.cam = *cam;
      w.n_lights = n_lights;
      if (n_lights) memcpy(w.lights, lights, sizeof(rt_light) * (size_t)n_lights);
      w.fr = shard_of((int)k + 1);
      seq[k] = w.posted.load(std::memory_order_relaxed) + 1;
      w.posted.store(seq[k], std::memory_order_release);
    }
    w.cv.notify_all();
  }
  const rt_frame f0 = shard_of(0);
  int rc = render_one(s, cam, lights, n_lights, &f0);
  std::string err0 = rc ? rt_last_error() : "";
  for (size_t k = 0; k < s->workers.size(); k++) {  // every worker has queued its share before this returns
    EnqueueWorker& w = *s->workers[k];
    for (int i = 0; i < 200000 && w.done.load(std::memory_order_acquire) != seq[k]; i++) __builtin_ia32_pause();
    if (w.done.load(std::memory_order_acquire) != seq[k]) {
      std::unique_lock<std::mutex> lk(w.mu);
      w.cv.wait(lk, [&] { return w.done.load(std::memory_order_acquire) == seq[k]; });
    }
    if (w.rc && rc == RT_OK) {
      rc = w.rc;
      err0 = "device " + std::to_string(w.r->device) + ": " + w.err;
    }
  }
  if (rc) {
    set_error("%s", err0.c_str());
    return rc;
  }
  HIPCHECK(hipSetDevice(s->device));
  return RT_OK;
}

extern "C" int rt_render_async(rt_scene* s, const rt_camera* cam, const rt_light* lights, int32_t n_lights,
                               const rt_frame* fr) {
  if (s && !s->replicas.empty()) return render_multi(s, cam, lights, n_lights, fr);
  return render_one(s, cam, lights, n_lights, fr);
}

extern "C" int rt_synchronize_devices(rt_scene* s, rt_stats* out, int32_t capacity, rt_stats* per_device) {
  if (!s) { set_error("null scene"); return RT_ERR_INVALID; }
  const int D = n_replicas(s);
  rt_stats tot;
  memset(&tot, 0, sizeof tot);
  int first_rc = RT_OK;
  for (int k = 0; k < D; k++) {  // every device is drained, even after a failure on one of them
    rt_stats st;
    const int rc = sync_one(replica(s, k), &st);
    if (rc) {
      if (first_rc == RT_OK) first_rc = rc;
      continue;
    }
    if (per_device && k < capacity) per_device[k] = st;
    tot.kernel_ms = std::max(tot.kernel_ms, st.kernel_ms);
    tot.trace_kernel_ms = std::max(tot.trace_kernel_ms, st.trace_kernel_ms);
    tot.launches = std::max(tot.launches, st.launches);
    tot.primary_rays += st.primary_rays;
    tot.total_rays += st.total_rays;
    tot.hits += st.hits;
    tot.node_visits += st.node_visits;
    tot.tri_tests += st.tri_tests;
    tot.wave_node_fetches += st.wave_node_fetches;
    tot.wave_tri_fetches += st.wave_tri_fetches;
    tot.wave_node_bytes += st.wave_node_bytes;
  }
  if (D > 1 && s->device != RT_DEVICE_NONE) (void)hipSetDevice(s->device);
  if (first_rc) return first_rc;
  if (out) *out = tot;
  return D;
}

extern "C" int rt_synchronize(rt_scene* s, rt_stats* out) {
  const int rc = rt_synchronize_devices(s, out, 0, nullptr);
  return rc < 0 ? rc : RT_OK;
}

// Frame assembly of a multi-device scene: every replica packs its tiles of its last frame (contiguous, its
// shard's slot order: k_pack_tiles32 / k_pack_shard) and copies them into its pinned host buffer, all
// devices queued first; then one host worker per device waits for its copy and places the tiles into the
// caller's frame (rows of 16 pixels). Only the tiles of the replicas' shards are written.
enum AsmKind { ASM_RGB = 0, ASM_FACE = 1, ASM_T = 2, ASM_RGB8 = 3 };

// Device-side assembly (SURVEY e1 "peer-writes to GPU0"; A/B knob RT_ASM_DEVICE, see assemble):
// when the replicas rendered the whole frame between them, each packs its tiles on its own stream and copies
// them into device 0's gather buffer (hipMemcpyPeerAsync over xGMI; a device copy when replicas share a GPU),
// device 0 waits for every slice (one event per replica), places all tiles with one kernel (k_unpack_tiles)
// and copies the frame to pinned host memory in kChunks pieces, which host threads move into the caller's
// buffer as each lands.
static int assemble_device(rt_scene* s, AsmKind kind, void* out, int32_t* exact, const char* what) {
  const int D = n_replicas(s);
  const int W = s->last_W, H = s->last_H, tiles_x = (W + 15) / 16, tiles_y = (H + 15) / 16;
  const size_t E = kind == ASM_RGB ? 12 : kind == ASM_RGB8 ? 3 : 4;
  UnpackArgs ua;
  memset(&ua, 0, sizeof ua);
  ua.n_rep = D, ua.W = W, ua.H = H, ua.tiles_x = tiles_x, ua.E = (int32_t)E;
  size_t total = 0;
  int max_tiles = 0;
  for (int k = 0; k < D; k++) {
    rt_scene* r = replica(s, k);
    ua.si[k] = r->last_shard_index;
    ua.sc[k] = r->last_shard_count;
    ua.S[k] = frame_super_tile(ua.sc[k]);
    ua.n_tiles[k] = shard_tile_slots(tiles_x, tiles_y, ua.S[k], ua.si[k], ua.sc[k]);
    max_tiles = std::max(max_tiles, ua.n_tiles[k]);
    const size_t bytes = (size_t)ua.n_tiles[k] * 256 * E, flag_at = (bytes + 15) & ~(size_t)15;
    ua.off[k] = total;
    ua.flag_off[k] = total + flag_at;
    total += flag_at + 16;
  }
  const size_t frame_bytes = (size_t)W * H * E;
  rt_scene::DevAssembly& g = s->dasm;
  HIPCHECK(hipSetDevice(s->device));
  if (total > g.gather_bytes || frame_bytes + 16 > g.frame_bytes || frame_bytes + 16 > g.h_bytes) {
    for (int k = 0; k < D; k++) {  // no replica's copy into the old buffers may be in flight
      rt_scene* r = replica(s, k);
      HIPCHECK(hipSetDevice(r->device));
      for (int q = 0; q < r->n_slots; q++) HIPCHECK(hipStreamSynchronize((hipStream_t)r->slots[q].stream));
    }
    HIPCHECK(hipSetDevice(s->device));
    if (total > g.gather_bytes) {
      if (g.d_gather) (void)hipFree(g.d_gather);
      g.d_gather = nullptr, g.gather_bytes = 0;
      HIPCHECK(hipMalloc(&g.d_gather, total));
      g.gather_bytes = total;
    }
    if (frame_bytes + 16 > g.frame_bytes) {
      if (g.d_frame) (void)hipFree(g.d_frame);
      g.d_frame = nullptr, g.frame_bytes = 0;
      HIPCHECK(hipMalloc(&g.d_frame, frame_bytes + 16));
      g.frame_bytes = frame_bytes + 16;
    }
    if (frame_bytes + 16 > g.h_bytes) {
      if (g.h_frame) (void)hipHostFree(g.h_frame);
      g.h_frame = nullptr, g.h_bytes = 0;
      HIPCHECK(hipHostMalloc(&g.h_frame, frame_bytes + 16, hipHostMallocDefault));
      g.h_bytes = frame_bytes + 16;
    }
  }
  for (int c = 0; c < rt_scene::DevAssembly::kChunks; c++)
    if (!g.ev_chunk[c]) {
      hipEvent_t e;
      HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      g.ev_chunk[c] = e;
    }
  uint8_t* gather = (uint8_t*)g.d_gather;
  // every replica: pack behind its share of the frame; replicas 1.. copy their slice to device 0
  for (int k = 0; k < D; k++) {
    rt_scene* r = replica(s, k);
    HIPCHECK(hipSetDevice(r->device));
    rt_scene::FrameSlot& f = r->slots[r->last_slot];
    hipStream_t st = (hipStream_t)f.stream;
    const size_t need = ua.flag_off[k] - ua.off[k] + 16;
    uint8_t* dst;
    if (k == 0) {
      dst = gather + ua.off[0];
    } else {
      rt_scene::Assembly& a = r->asm_buf;
      if (need > a.bytes) {
        HIPCHECK(hipStreamSynchronize(st));
        if (a.d_pack) (void)hipFree(a.d_pack);
        if (a.h_pack) (void)hipHostFree(a.h_pack);
        a = rt_scene::Assembly{};
        HIPCHECK(hipMalloc(&a.d_pack, need));
        HIPCHECK(hipHostMalloc(&a.h_pack, need, hipHostMallocDefault));
        a.bytes = need;
      }
      dst = (uint8_t*)a.d_pack;
      if (!r->asm_ev) {
        hipEvent_t e;
        HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        r->asm_ev = e;
      }
    }
    if (ua.n_tiles[k] > 0) {
      if (kind == ASM_RGB8) {
        uint32_t* flag = (uint32_t*)(dst + (ua.flag_off[k] - ua.off[k]));
        HIPCHECK(hipMemsetAsync(flag, 0, 4, st));
        hipLaunchKernelGGL(k_pack_shard, dim3(ua.n_tiles[k]), dim3(256), 0, st, (const float*)f.d_rgb, dst, W, H, tiles_x,
                           ua.si[k], ua.sc[k], ua.n_tiles[k], ua.S[k], flag);
      } else {
        const uint32_t* src = kind == ASM_RGB ? (const uint32_t*)f.d_rgb
                              : kind == ASM_FACE ? (const uint32_t*)f.d_face : (const uint32_t*)f.d_t;
        hipLaunchKernelGGL(k_pack_tiles32, dim3(ua.n_tiles[k]), dim3(256), 0, st, src, (uint32_t*)dst, W, H, tiles_x,
                           ua.si[k], ua.sc[k], ua.n_tiles[k], ua.S[k], kind == ASM_RGB ? 3 : 1);
      }
      HIPCHECK(hipGetLastError());
    } else if (kind == ASM_RGB8) {
      HIPCHECK(hipMemsetAsync(dst + (ua.flag_off[k] - ua.off[k]), 0, 4, st));
    }
    if (k > 0) {
      if (r->device == s->device) HIPCHECK(hipMemcpyAsync(gather + ua.off[k], dst, need, hipMemcpyDeviceToDevice, st));
      else HIPCHECK(hipMemcpyPeerAsync(gather + ua.off[k], s->device, dst, r->device, need, st));
      HIPCHECK(hipEventRecord((hipEvent_t)r->asm_ev, st));
    }
  }
  // device 0: every slice in, tiles placed, the frame to the host in chunks
  HIPCHECK(hipSetDevice(s->device));
  hipStream_t st0 = (hipStream_t)s->slots[s->last_slot].stream;
  for (int k = 1; k < D; k++) HIPCHECK(hipStreamWaitEvent(st0, (hipEvent_t)replica(s, k)->asm_ev, 0));
  uint8_t* frame = (uint8_t*)g.d_frame;
  if (max_tiles > 0) {
    hipLaunchKernelGGL(k_unpack_tiles, dim3((unsigned)max_tiles, (unsigned)D), dim3(256), 0, st0, (const uint8_t*)gather, frame, ua);
    HIPCHECK(hipGetLastError());
  }
  if (kind == ASM_RGB8) {
    hipLaunchKernelGGL(k_or_flags, dim3(1), dim3(64), 0, st0, (const uint8_t*)gather, ua, (uint32_t*)(frame + frame_bytes));
    HIPCHECK(hipGetLastError());
  }
  const int C = (int)std::max<size_t>(1, std::min<size_t>(rt_scene::DevAssembly::kChunks, frame_bytes >> 21));
  const size_t cb = ((frame_bytes + C - 1) / C + 63) & ~(size_t)63;
  auto span = [&](int c, size_t& o, size_t& n) {
    o = std::min(frame_bytes, (size_t)c * cb);
    n = std::min(frame_bytes, o + cb) - o;
  };
  for (int c = 0; c < C; c++) {
    size_t o, n;
    span(c, o, n);
    const size_t extra = (c == C - 1 && kind == ASM_RGB8) ? 4 : 0;  // the OR-ed flag follows the frame
    if (n + extra) HIPCHECK(hipMemcpyAsync((uint8_t*)g.h_frame + o, frame + o, n + extra, hipMemcpyDeviceToHost, st0));
    HIPCHECK(hipEventRecord((hipEvent_t)g.ev_chunk[c], st0));
  }
  std::vector<int> ok((size_t)C, 1);
  auto take = [&](int c) {
    if (hipEventSynchronize((hipEvent_t)g.ev_chunk[c]) != hipSuccess) { ok[c] = 0; return; }
    size_t o, n;
    span(c, o, n);
    if (n) memcpy((uint8_t*)out + o, (const uint8_t*)g.h_frame + o, n);
  };
  std::vector<std::thread> th;
  for (int c = 1; c < C; c++) {
    try {
      th.emplace_back(take, c);
    } catch (const std::exception&) {
      take(c);
    }
  }
  take(0);
  for (auto& t : th) t.join();
  for (int c = 0; c < C; c++)
    if (!ok[c]) { set_error("%s: frame copy to the host failed", what); return RT_ERR_HIP; }
  if (exact) {
    uint32_t fl = 0;
    memcpy(&fl, (const uint8_t*)g.h_frame + frame_bytes, 4);
    *exact = fl ? 0 : 1;
  }
  return RT_OK;
}

static int assemble(rt_scene* s, AsmKind kind, int64_t capacity_pixels, void* out, int32_t* exact, const char* what) {
  const int D = n_replicas(s);
  const int W = s->last_W, H = s->last_H, tiles_x = (W + 15) / 16, tiles_y = (H + 15) / 16;
  const size_t E = kind == ASM_RGB ? 12 : kind == ASM_RGB8 ? 3 : 4;  // bytes per pixel
  if (W <= 0 || H <= 0) { set_error("%s: no frame rendered", what); return RT_ERR_INVALID; }
  if (capacity_pixels < (int64_t)W * H) {
    set_error("%s: buffers hold %lld pixels, the last frame has %lld (%d x %d)", what, (long long)capacity_pixels,
              (long long)W * H, W, H);
    return RT_ERR_INVALID;
  }
  {  // the replicas' frames must be of the scene's last size (and carry hit records for face / t)
    for (int k = 0; k < D; k++) {
      rt_scene* r = replica(s, k);
      int rc = check_device_scene(r);
      if (rc) return rc;
      const rt_scene::FrameSlot& f = r->slots[r->last_slot];
      if (!f.d_rgb || r->last_W != W || r->last_H != H || (size_t)W * H > f.fb_pixels) {
        set_error("%s: device %d has no frame of the scene's last size", what, r->device);
        return RT_ERR_INVALID;
      }
      if ((kind == ASM_FACE || kind == ASM_T) && !(r->last_flags & RT_FRAME_WRITE_HITS)) {
        set_error("last frame was rendered without RT_FRAME_WRITE_HITS");
        return RT_ERR_INVALID;
      }
    }
    // The host path below is the default: with the replicas on distinct GPUs every device copies its own tiles
    // over its own PCIe link at once, where the device-side assembly funnels the whole frame through device 0's
    // link. With replicas sharing one GPU (the only measurable case here: one link either way) the two measured
    // level -- 8 replicas, 4K 8-bit frame: 1.10-1.36 vs 1.21-1.27 ms (profiles/ab/r06_assembly_ab.txt). The
    // device-side path (the whole frame split over the replicas) is kept behind the A/B knob RT_ASM_DEVICE.
    const bool whole = s->last_shard_count == D && s->last_shard_index == 0;
    const char* dev_env = debug_env("RT_ASM_DEVICE");
    if (whole && dev_env && atoi(dev_env)) {
      const int rc = assemble_device(s, kind, out, exact, what);
      HIPCHECK(hipSetDevice(s->device));
      return rc;
    }
  }
  struct Job {
    rt_scene* r;
    int si, sc, S, n_tiles;
    size_t bytes, flag_off;
  };
  std::vector<Job> jobs((size_t)D);
  for (int k = 0; k < D; k++) {
    rt_scene* r = replica(s, k);
    int rc = check_device_scene(r);
    if (rc) return rc;
    rt_scene::FrameSlot& f = r->slots[r->last_slot];
    if (!f.d_rgb || r->last_W != W || r->last_H != H || (size_t)W * H > f.fb_pixels) {
      set_error("%s: device %d has no frame of the scene's last size", what, r->device);
      return RT_ERR_INVALID;
    }
    if ((kind == ASM_FACE || kind == ASM_T) && !(r->last_flags & RT_FRAME_WRITE_HITS)) {
      set_error("last frame was rendered without RT_FRAME_WRITE_HITS");
      return RT_ERR_INVALID;
    }
    Job& j = jobs[k];
    j.r = r;
    j.si = r->last_shard_index;
    j.sc = r->last_shard_count;
    j.S = frame_super_tile(j.sc);
    j.n_tiles = shard_tile_slots(tiles_x, tiles_y, j.S, j.si, j.sc);
    j.bytes = (size_t)j.n_tiles * 256 * E;
    j.flag_off = (j.bytes + 15) & ~(size_t)15;
    const size_t need = j.flag_off + 16;
    hipStream_t st = (hipStream_t)f.stream;
    rt_scene::Assembly& a = r->asm_buf;
    if (need > a.bytes) {
      HIPCHECK(hipStreamSynchronize(st));
      if (a.d_pack) (void)hipFree(a.d_pack);
      if (a.h_pack) (void)hipHostFree(a.h_pack);
      a = rt_scene::Assembly{};
      HIPCHECK(hipMalloc(&a.d_pack, need));
      HIPCHECK(hipHostMalloc(&a.h_pack, need, hipHostMallocDefault));
      a.bytes = need;
    }
    uint32_t* flag = (uint32_t*)((char*)a.d_pack + j.flag_off);
    if (j.n_tiles > 0) {
      if (kind == ASM_RGB8) {
        HIPCHECK(hipMemsetAsync(flag, 0, 4, st));
        hipLaunchKernelGGL(k_pack_shard, dim3(j.n_tiles), dim3(256), 0, st, (const float*)f.d_rgb, (uint8_t*)a.d_pack, W,
                           H, tiles_x, j.si, j.sc, j.n_tiles, j.S, flag);
      } else {
        const uint32_t* src = kind == ASM_RGB ? (const uint32_t*)f.d_rgb
                              : kind == ASM_FACE ? (const uint32_t*)f.d_face : (const uint32_t*)f.d_t;
        hipLaunchKernelGGL(k_pack_tiles32, dim3(j.n_tiles), dim3(256), 0, st, src, (uint32_t*)a.d_pack, W, H, tiles_x,
                           j.si, j.sc, j.n_tiles, j.S, kind == ASM_RGB ? 3 : 1);
      }
      HIPCHECK(hipGetLastError());
      HIPCHECK(hipMemcpyAsync(a.h_pack, a.d_pack, kind == ASM_RGB8 ? need : j.bytes, hipMemcpyDeviceToHost, st));
    }
  }
  // host workers: device k's tiles into the caller's frame once its copy has landed
  std::vector<int> rcs((size_t)D, RT_OK);
  std::vector<std::string> errs((size_t)D);
  std::vector<uint32_t> flags((size_t)D, 0);
  auto place = [&](int k) {
    const Job& j = jobs[k];
    if (hipSetDevice(j.r->device) != hipSuccess ||
        hipStreamSynchronize((hipStream_t)j.r->slots[j.r->last_slot].stream) != hipSuccess) {
      rcs[k] = RT_ERR_HIP;
      errs[k] = "frame copy to the host failed";
      return;
    }
    const char* src = (const char*)j.r->asm_buf.h_pack;
    char* dst = (char*)out;
    for (int L = 0; L < j.n_tiles; L++) {
      int tx, ty;
      shard_tile_xy(tiles_x, j.S, j.si, j.sc, L, tx, ty);
      if (tx >= tiles_x || ty >= tiles_y) continue;
      const size_t w = (size_t)std::min(16, W - tx * 16) * E;
      const int h = std::min(16, H - ty * 16);
      for (int yy = 0; yy < h; yy++)
        memcpy(dst + ((size_t)(ty * 16 + yy) * W + (size_t)tx * 16) * E, src + ((size_t)L * 256 + (size_t)yy * 16) * E, w);
    }
    if (kind == ASM_RGB8 && j.n_tiles > 0) memcpy(&flags[k], src + j.flag_off, 4);
  };
  std::vector<std::thread> workers;
  for (int k = 1; k < D; k++) {
    try {
      workers.emplace_back(place, k);
    } catch (const std::exception&) {
      place(k);
    }
  }
  place(0);
  for (auto& w : workers) w.join();
  HIPCHECK(hipSetDevice(s->device));
  for (int k = 0; k < D; k++)
    if (rcs[k]) { set_error("%s: device %d: %s", what, jobs[k].r->device, errs[k].c_str()); return rcs[k]; }
  if (exact) {
    *exact = 1;
    for (uint32_t fl : flags)
      if (fl) *exact = 0;
  }
  return RT_OK;
}

extern "C" int rt_frame_download(rt_scene* s, int64_t capacity_pixels, float* rgb, int32_t* face, float* t) {
  int rc = check_device_scene(s);
  if (rc) return rc;
  if (!s->replicas.empty()) {  // the devices' tiles assembled in the caller's buffers
    if (rgb && (rc = assemble(s, ASM_RGB, capacity_pixels, rgb, nullptr, "rt_frame_download"))) return rc;
    if (face && (rc = assemble(s, ASM_FACE, capacity_pixels, face, nullptr, "rt_frame_download"))) return rc;
    if (t && (rc = assemble(s, ASM_T, capacity_pixels, t, nullptr, "rt_frame_download"))) return rc;
    return RT_OK;
  }
  const rt_scene::FrameSlot& f = s->slots[s->last_slot];
  HIPCHECK(hipStreamSynchronize((hipStream_t)f.stream));
  const size_t npix = (size_t)s->last_W * s->last_H;
  if (!f.d_rgb || npix > f.fb_pixels) { set_error("rt_frame_download: no frame rendered"); return RT_ERR_INVALID; }
  if (capacity_pixels < (int64_t)npix) {
    set_error("rt_frame_download: buffers hold %lld pixels, the last frame has %zu (%d x %d)", (long long)capacity_pixels,
              npix, s->last_W, s->last_H);
    return RT_ERR_INVALID;
  }
  if (rgb) HIPCHECK(hipMemcpy(rgb, f.d_rgb, npix * 12, hipMemcpyDeviceToHost));
  if ((face || t) && !(s->last_flags & RT_FRAME_WRITE_HITS)) { set_error("last frame was rendered without RT_FRAME_WRITE_HITS"); return RT_ERR_INVALID; }
  if (face) HIPCHECK(hipMemcpy(face, f.d_face, npix * 4, hipMemcpyDeviceToHost));
  if (t) HIPCHECK(hipMemcpy(t, f.d_t, npix * 4, hipMemcpyDeviceToHost));
  return RT_OK;
}

extern "C" int rt_frame_download_rgb8(rt_scene* s, int64_t capacity_pixels, uint8_t* rgb8, int32_t* exact) {
  int rc = check_device_scene(s);
  if (rc) return rc;
  if (!rgb8) { set_error("rt_frame_download_rgb8: null output"); return RT_ERR_INVALID; }
  if (!s->replicas.empty()) return assemble(s, ASM_RGB8, capacity_pixels, rgb8, exact, "rt_frame_download_rgb8");
  rt_scene::FrameSlot& f = s->slots[s->last_slot];
  const size_t npix = (size_t)s->last_W * s->last_H;
  if (!f.d_rgb || npix == 0 || npix > f.fb_pixels) { set_error("rt_frame_download_rgb8: no frame rendered"); return RT_ERR_INVALID; }
  if (capacity_pixels < (int64_t)npix) {
    set_error("rt_frame_download_rgb8: buffer holds %lld pixels, the last frame has %zu (%d x %d)",
              (long long)capacity_pixels, npix, s->last_W, s->last_H);
    return RT_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)f.stream;
  if (npix > f.rgb8_pixels) {
    HIPCHECK(hipStreamSynchronize(st));
    if (f.d_rgb8) (void)hipFree(f.d_rgb8);
    f.d_rgb8 = nullptr;
    f.rgb8_pixels = 0;
    HIPCHECK(hipMalloc((void**)&f.d_rgb8, npix * 3 + 64));
    f.rgb8_pixels = npix;
  }
  uint32_t* flag = (uint32_t*)(f.d_rgb8 + ((npix * 3 + 15) / 16) * 16);
  HIPCHECK(hipMemsetAsync(flag, 0, 4, st));
  const uint32_t n = (uint32_t)(npix * 3);
  hipLaunchKernelGGL(k_frame_rgb8, dim3((n + 255) / 256), dim3(256), 0, st, (const float*)f.d_rgb, f.d_rgb8, n, flag);
  HIPCHECK(hipGetLastError());
  uint32_t h_flag = 0;
  HIPCHECK(hipMemcpyAsync(rgb8, f.d_rgb8, npix * 3, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipMemcpyAsync(&h_flag, flag, 4, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  if (exact) *exact = h_flag ? 0 : 1;
  return RT_OK;
}

extern "C" int64_t rt_frame_shard_bytes(int32_t W, int32_t H, int32_t shard_count) {
  if (W <= 0 || H <= 0 || shard_count <= 0) return 0;
  // shard 0 has the most tile slots
  return (int64_t)shard_tile_slots((W + 15) / 16, (H + 15) / 16, frame_super_tile(shard_count), 0, shard_count) * 768;
}

extern "C" int32_t rt_frame_shard_tiles(int32_t W, int32_t H, int32_t shard_index, int32_t shard_count, int32_t* tiles_xy,
                                        int32_t capacity) {
  if (W <= 0 || H <= 0 || shard_count <= 0 || shard_index < 0 || shard_index >= shard_count) return 0;
  const int tiles_x = (W + 15) / 16, tiles_y = (H + 15) / 16, S = frame_super_tile(shard_count);
  const int slots = shard_tile_slots(tiles_x, tiles_y, S, shard_index, shard_count);
  int32_t n = 0;
  for (int L = 0; L < slots; L++) {
    int tx, ty;
    shard_tile_xy(tiles_x, S, shard_index, shard_count, L, tx, ty);
    if (tx >= tiles_x || ty >= tiles_y) continue;
    if (tiles_xy && n < capacity) { tiles_xy[2 * n] = tx; tiles_xy[2 * n + 1] = ty; }
    n++;
  }
  return n;
}

extern "C" int rt_frame_pack_shard_rgb8(rt_scene* s, void* dst_device) {
  int rc = check_device_scene(s);
  if (rc) return rc;
  if (!dst_device) { set_error("rt_frame_pack_shard_rgb8: null destination"); return RT_ERR_INVALID; }
  if (!s->replicas.empty()) {
    set_error("rt_frame_pack_shard_rgb8: a multi-device scene assembles its frame itself (rt_frame_download_rgb8)");
    return RT_ERR_UNSUPPORTED;
  }
  rt_scene::FrameSlot& f = s->slots[s->last_slot];
  if (!f.d_rgb || (size_t)s->last_W * s->last_H > f.fb_pixels) { set_error("rt_frame_pack_shard_rgb8: no frame rendered"); return RT_ERR_INVALID; }
  const int W = s->last_W, H = s->last_H, tiles_x = (W + 15) / 16, tiles_y = (H + 15) / 16;
  const int si = s->last_shard_index, sc = s->last_shard_count, S = frame_super_tile(sc);
  const int n_tiles = shard_tile_slots(tiles_x, tiles_y, S, si, sc);
  hipStream_t st = (hipStream_t)f.stream;
  const int64_t slice = rt_frame_shard_bytes(W, H, sc);
  if ((int64_t)n_tiles * 768 < slice) HIPCHECK(hipMemsetAsync((uint8_t*)dst_device + (size_t)n_tiles * 768, 0, (size_t)(slice - (int64_t)n_tiles * 768), st));
  if (n_tiles > 0)
    hipLaunchKernelGGL(k_pack_shard, dim3(n_tiles), dim3(256), 0, st, (const float*)f.d_rgb, (uint8_t*)dst_device, W, H,
                       tiles_x, si, sc, n_tiles, S, (uint32_t*)nullptr);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipStreamSynchronize(st));
  return RT_OK;
}

extern "C" int rt_frame_unpack_shards_rgb8(const void* packed_device, int32_t shard_count, int32_t W, int32_t H,
                                           void* frame_device, int32_t device) {
  if (!packed_device || !frame_device || shard_count <= 0 || W <= 0 || H <= 0) {
    set_error("rt_frame_unpack_shards_rgb8: invalid arguments");
    return RT_ERR_INVALID;
  }
  int dev = device;
  if (dev < 0) HIPCHECK(hipGetDevice(&dev));
  HIPCHECK(hipSetDevice(dev));
  const size_t npix = (size_t)W * H;
  hipLaunchKernelGGL(k_unpack_shards, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, 0, (const uint8_t*)packed_device,
                     (uint8_t*)frame_device, W, H, (W + 15) / 16, shard_count, (size_t)rt_frame_shard_bytes(W, H, shard_count),
                     frame_super_tile(shard_count));
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipDeviceSynchronize());
  return RT_OK;
}

extern "C" int rt_render(rt_scene* s, const rt_camera* cam, const rt_light* lights, int32_t n_lights, const rt_frame* fr,
                         float* out_rgb, rt_stats* stats) {
  int rc = rt_render_async(s, cam, lights, n_lights, fr);
  if (rc) return rc;
  const int W = fr->width, H = fr->height;
  if (!s->replicas.empty() && out_rgb) {
    // multi-device: each device's tile packing and copy are queued right behind its share of the frame, and
    // its host worker writes its tiles into the caller's frame as soon as that device is done (the rest of
    // the frame untouched); the stats are collected after
    if ((rc = assemble(s, ASM_RGB, (int64_t)W * H, out_rgb, nullptr, "rt_render"))) {
      (void)rt_synchronize(s, nullptr);
      return rc;
    }
    return rt_synchronize(s, stats);
  }
  if ((rc = rt_synchronize(s, stats))) return rc;
  if (!out_rgb) return RT_OK;
  const int sc = fr->shard_count > 0 ? fr->shard_count : 1;
  if (sc == 1) return rt_frame_download(s, (int64_t)W * H, out_rgb, nullptr, nullptr);
  std::vector<float> full((size_t)W * H * 3);
  if ((rc = rt_frame_download(s, (int64_t)W * H, full.data(), nullptr, nullptr))) return rc;
  const int tiles_x = (W + 15) / 16, tiles_y = (H + 15) / 16, S = frame_super_tile(sc);
  const int slots = shard_tile_slots(tiles_x, tiles_y, S, fr->shard_index, sc);
  for (int L = 0; L < slots; L++) {
    int tx, ty;
    shard_tile_xy(tiles_x, S, fr->shard_index, sc, L, tx, ty);
    if (tx >= tiles_x || ty >= tiles_y) continue;
    for (int y = ty * 16; y < std::min(H, ty * 16 + 16); y++) {
      const size_t o = ((size_t)y * W + tx * 16) * 3;
      memcpy(out_rgb + o, full.data() + o, sizeof(float) * 3 * (size_t)(std::min(W, tx * 16 + 16) - tx * 16));
    }
  }
  return RT_OK;
}

// ray-list queries: closest (face, t, P, optional interpolated normal), any-hit (blocked) or colour
static int trace_rays(rt_scene* s, int query, int32_t n, const float* o, const float* d, int32_t* face, float* t,
                      float* P3, float* N3, int32_t* blocked, float* rgb, const rt_light* lights, int32_t n_lights) {
  int rc = check_device_scene(s);
  if (rc) return rc;
  if (n < 0 || (n && (!o || !d)) || n_lights < 0 || n_lights > RT_MAX_LIGHTS || (n_lights && !lights)) {
    set_error("trace: invalid arguments");
    return RT_ERR_INVALID;
  }
  if (n == 0) return RT_OK;
  FrameParams P;
  fill_scene_params(s, P);
  if (query == Q_COLOR) {  // calculateColor's order: point lights, then directional lights
    int k = 0;
    for (int pass = 0; pass < 2; pass++)
      for (int l = 0; l < n_lights; l++) {
        const int kind = lights[l].kind == RT_LIGHT_DIRECTIONAL ? RT_LIGHT_DIRECTIONAL : RT_LIGHT_POINT;
        if (kind != (pass ? RT_LIGHT_DIRECTIONAL : RT_LIGHT_POINT)) continue;
        memcpy(P.lights[k].p, lights[l].position, 12);
        memcpy(P.lights[k].c, lights[l].color, 12);
        P.lights[k].kind = kind;
        k++;
      }
    P.n_lights = n_lights;
  }
  const size_t n3 = (size_t)n * 12;
  hipStream_t st = (hipStream_t)s->stream;
  std::vector<void*> bufs;
  struct Free {
    std::vector<void*>& b;
    ~Free() { for (void* p : b) (void)hipFree(p); }
  } free_{bufs};
  auto dalloc = [&](size_t bytes) -> void* {
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    bufs.push_back(p);
    return p;
  };
  RayParams R{};
  R.n = n;
  float* d_o = (float*)dalloc(n3);
  float* d_d = (float*)dalloc(n3);
  if (!d_o || !d_d) { set_error("trace: device allocation failed"); return RT_ERR_NOMEM; }
  HIPCHECK(hipMemcpy(d_o, o, n3, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(d_d, d, n3, hipMemcpyHostToDevice));
  R.o = d_o;
  R.d = d_d;
  if (query == Q_SHADOW) {
    if (!(R.blocked = (int32_t*)dalloc((size_t)n * 4))) { set_error("trace: device allocation failed"); return RT_ERR_NOMEM; }
  } else {
    R.face = (int32_t*)dalloc((size_t)n * 4);
    R.t = (float*)dalloc((size_t)n * 4);
    if (!R.face || !R.t) { set_error("trace: device allocation failed"); return RT_ERR_NOMEM; }
    if (query == Q_CLOSEST && P3 && !(R.P = (float*)dalloc(n3))) { set_error("trace: device allocation failed"); return RT_ERR_NOMEM; }
    if (query == Q_CLOSEST && N3 && !(R.N = (float*)dalloc(n3))) { set_error("trace: device allocation failed"); return RT_ERR_NOMEM; }
    if (query == Q_COLOR && !(R.rgb = (float*)dalloc(n3))) { set_error("trace: device allocation failed"); return RT_ERR_NOMEM; }
  }
  const int grid = (n + 255) / 256;
  const bool w4 = pick_trav(P, kernel_variant()) == TRAV_W4;
  if (w4 && !variants_linked()) {
    set_error("trace: kernel variant %d is an A/B build option, not in this library (make variants)", kernel_variant());
    return RT_ERR_UNSUPPORTED;
  }
  if (w4) {
    VariantCall vc;
    vc.P = P, vc.R = R, vc.grid = grid, vc.st = st, vc.query = query;
    variant_launch(VOP_RAYS, vc);
  } else if (query == Q_COLOR) {
    hipLaunchKernelGGL((k_rays_color<TRAV_B2_LDS>), dim3(grid), dim3(256), 0, st, P, R);
  } else {
    if (query == Q_SHADOW) hipLaunchKernelGGL((k_rays<true, TRAV_B2_LDS>), dim3(grid), dim3(256), 0, st, P, R);
    else hipLaunchKernelGGL((k_rays<false, TRAV_B2_LDS>), dim3(grid), dim3(256), 0, st, P, R);
  }
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipStreamSynchronize(st));
  if ((rc = check_prefetch_word(s))) return rc;
  if (query == Q_SHADOW) {
    HIPCHECK(hipMemcpy(blocked, R.blocked, (size_t)n * 4, hipMemcpyDeviceToHost));
  } else {
    if (face) HIPCHECK(hipMemcpy(face, R.face, (size_t)n * 4, hipMemcpyDeviceToHost));
    if (t) HIPCHECK(hipMemcpy(t, R.t, (size_t)n * 4, hipMemcpyDeviceToHost));
    if (R.P) HIPCHECK(hipMemcpy(P3, R.P, n3, hipMemcpyDeviceToHost));
    if (R.N) HIPCHECK(hipMemcpy(N3, R.N, n3, hipMemcpyDeviceToHost));
    if (R.rgb) HIPCHECK(hipMemcpy(rgb, R.rgb, n3, hipMemcpyDeviceToHost));
  }
  return RT_OK;
}

extern "C" int rt_trace_closest(rt_scene* s, int32_t n, const float* o, const float* d, int32_t* face, float* t,
                                float* P3) {
  return trace_rays(s, Q_CLOSEST, n, o, d, face, t, P3, nullptr, nullptr, nullptr, nullptr, 0);
}

extern "C" int rt_trace_closest_normal(rt_scene* s, int32_t n, const float* o, const float* d, int32_t* face, float* t,
                                       float* P3, float* N3) {
  return trace_rays(s, Q_CLOSEST, n, o, d, face, t, P3, N3, nullptr, nullptr, nullptr, 0);
}

extern "C" int rt_trace_shadow(rt_scene* s, int32_t n, const float* P3, const float* L3, int32_t* blocked) {
  if (!blocked && n > 0) { set_error("rt_trace_shadow: null output"); return RT_ERR_INVALID; }
  return trace_rays(s, Q_SHADOW, n, P3, L3, nullptr, nullptr, nullptr, nullptr, blocked, nullptr, nullptr, 0);
}

extern "C" int rt_trace_color(rt_scene* s, int32_t n, const float* o, const float* d, const rt_light* lights,
                              int32_t n_lights, float* rgb, int32_t* face, float* t) {
  if (!rgb && n > 0) { set_error("rt_trace_color: null output"); return RT_ERR_INVALID; }
  return trace_rays(s, Q_COLOR, n, o, d, face, t, nullptr, nullptr, nullptr, rgb, lights, n_lights);
}

extern "C" int rt_debug_math_device(int32_t op, int32_t n, const float* in, float* out) {
  static const int in_len[] = {6, 3, 6, 12, 19, 20, 9, 16, 4, 6, 6, 6, 6, 13, 3, 16, 24, 2};
  static const int out_len[] = {1, 3, 3, 3, 3, 4, 9, 16, 16, 3, 3, 3, 3, 3, 1, 3, 3, 1};
  if (op < 0 || op > 17 || n <= 0 || !in || !out) { set_error("rt_debug_math_device: bad arguments"); return RT_ERR_INVALID; }
  if (rt_device_count() == 0) { set_error("no HIP device"); return RT_ERR_NO_DEVICE; }
  float *di = nullptr, *dout = nullptr;
  const size_t ib = (size_t)n * in_len[op] * 4, ob = (size_t)n * out_len[op] * 4;
  HIPCHECK(hipMalloc((void**)&di, ib));
  HIPCHECK(hipMalloc((void**)&dout, ob));
  HIPCHECK(hipMemcpy(di, in, ib, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_debug_math, dim3((n + 255) / 256), dim3(256), 0, 0, (int)op, (int)n, in_len[op], out_len[op], di, dout);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipDeviceSynchronize());
  HIPCHECK(hipMemcpy(out, dout, ob, hipMemcpyDeviceToHost));
  (void)hipFree(di);
  (void)hipFree(dout);
  return RT_OK;
}
