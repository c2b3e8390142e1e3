// rt_device.hip -- gfx950 kernels and device-side C ABI of the MI355X ray-traversal library.
//
// Hot path (reference: src/flyscene.cpp:299-614):
//   one wave = one 8x8 pixel tile, one ray per lane; rays generated in registers (traceRayThread +
//   Camera::screenToWorld, fp64 NDC as camera.hpp:159-162);
//   wave-packet BVH traversal: every node record is fetched once per wave with a scalar load
//   (s_load_dwordx16 of the 64-B node), each lane slab-tests both children, the wave descends by
//   ballot (near child first by lane majority) and keeps ONE traversal stack for the wave (held in
//   LDS or in the lanes of a VGPR -- template switch); lanes that cannot improve their
//   hit simply vote "no", so the wave stays converged and only visits nodes some lane still needs;
//   triangle test = the reference's calculateDistance/interpolateNormal arithmetic bit for bit
//   (flyscene.cpp:444-478,572-600), tie-break by reference iteration rank (calculateMinimumFace
//   keeps the first minimum, flyscene.cpp:381-391), plus the reference's own object-space box test
//   (intersectBox, flyscene.cpp:484-507) for the candidate's reference box;
//   shading = calculateColor/calcSingleColor (flyscene.cpp:542-614); FULL mode adds the shadow any-hit
//   per light (flyscene.cpp:510-526) and the one reflection bounce of traceRay (flyscene.cpp:317-371).
// No MFMA: there is no dense contraction in this path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <vector>

#include "rt_kat.h"
#include "rt_scene.h"

using rt::f3;

#define HIPCHECK(expr)                                                                   \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) {                                                              \
      rt::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
      return RT_ERR_HIP;                                                                 \
    }                                                                                    \
  } while (0)

namespace rt {

// ------------------------------------------------------------------------------------------------
// uniform (scalar) loads: a generic pointer re-typed into the constant address space makes hipcc
// emit s_load_dwordx16 for wave-uniform indices (one fetch per wave, data in SGPRs)
// ------------------------------------------------------------------------------------------------
typedef int i16v __attribute__((ext_vector_type(16)));

// One s_load_dwordx16 per 64-B record (hipcc otherwise splits the record into x4/x8 pieces, one
// scalar-cache request each, and sinks parts below the first use). The wait is inside the asm
// because the compiler does not track the counter of an inline-asm load.
template <typename T>
__device__ __forceinline__ T sload64(const T* base, uint32_t i) {
  static_assert(sizeof(T) == 64, "64-byte records");
  const uint32_t off = __builtin_amdgcn_readfirstlane(i) * 64u;  // byte offset in an SGPR (< 4 GiB)
  // the base is uniform, but inside divergent regions (FULL mode's secondary packets) the compiler
  // may keep it in VGPRs; readfirstlane folds away when it is already scalar
  const uint64_t b = (uint64_t)base;
  const uint64_t bs = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  i16v v;
  asm volatile("s_load_dwordx16 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(bs), "s"(off) : "memory");
  T r;
  __builtin_memcpy(&r, &v, 64);
  return r;
}
// Interior node handles on the device are byte offsets of the node record (RT_BYTE_HANDLES, set by
// device_upload: index * 64, < 2^31 below kMaxFaces), so a node fetch needs no shift per step; leaf
// handles keep the (first triangle, count) form. 0 = record indices (A/B).
#ifndef RT_BYTE_HANDLES
#define RT_BYTE_HANDLES 1
#endif
__device__ __forceinline__ uint32_t node_index(uint32_t h) { return RT_BYTE_HANDLES ? h >> 6 : h; }
__device__ __forceinline__ uint32_t node_offset(uint32_t h) { return RT_BYTE_HANDLES ? h : h * 64u; }
__device__ __forceinline__ Node64 sload_node(const Node64* base, uint32_t h) { return sload64(base, node_index(h)); }
// The same node fetch, then a prefetch of both children's records into the scalar cache, issued the
// moment the node has arrived so that it overlaps this node's box tests: one dword each pulls in the
// 64-B line. pad0 / pad1 (loaded alongside, same line) are the byte offsets from the nodes base of
// child 0 / 1's node record or, for a leaf child, of its first triangle record (device_upload).
// pf0 / pf1 receive the prefetched dwords: the caller keeps them live until an s_waitcnt
// lgkmcnt(0) has retired the loads (the hardware writes them whenever the data returns).
__device__ __forceinline__ Node64 sload_node_pf(const Node64* base, uint32_t h, uint32_t& pf0, uint32_t& pf1) {
  const uint32_t off = node_offset(__builtin_amdgcn_readfirstlane(h));
  const uint64_t b = (uint64_t)base;
  const uint64_t bs = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  i16v v;
  asm volatile(
      "s_load_dwordx16 %0, %3, %4\n\t"
      "s_load_dword %1, %3, %4 offset:0x38\n\t"
      "s_load_dword %2, %3, %4 offset:0x3c\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_load_dword %1, %3, %1\n\t"
      "s_load_dword %2, %3, %2"
      : "=&s"(v), "=&s"(pf0), "=&s"(pf1)
      : "s"(bs), "s"(off)
      : "memory");
  Node64 r;
  __builtin_memcpy(&r, &v, 64);
  return r;
}
// The same with the prefetch sinks carried from the previous node step ("+s"): this load's own
// s_waitcnt retires the previous step's prefetches too, so a node step needs no wait of its own (the
// sinks stay allocated for the whole traversal; traverse_fast waits once at its end). The child
// offsets land in registers of their own (o0, o1): a previous prefetch may still be in flight into the
// sinks when they are loaded (scalar loads return out of order).
__device__ __forceinline__ Node64 sload_node_pf_carry(const Node64* base, uint32_t h, uint32_t& pf0, uint32_t& pf1) {
  const uint32_t off = node_offset(__builtin_amdgcn_readfirstlane(h));
  const uint64_t b = (uint64_t)base;
  const uint64_t bs = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  i16v v;
  uint32_t o0, o1;
  asm volatile(
      "s_load_dwordx16 %0, %5, %6\n\t"
      "s_load_dword %3, %5, %6 offset:0x38\n\t"
      "s_load_dword %4, %5, %6 offset:0x3c\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_load_dword %1, %5, %3\n\t"
      "s_load_dword %2, %5, %4"
      : "=&s"(v), "+&s"(pf0), "+&s"(pf1), "=&s"(o0), "=&s"(o1)
      : "s"(bs), "s"(off)
      : "memory");
  Node64 r;
  __builtin_memcpy(&r, &v, 64);
  return r;
}
// RT_PF_INREG: the same carried prefetch, with the child offsets read from the node record's own
// registers (Node64::pad0 / pad1, words 14 / 15 of the x16 load) instead of two extra one-dword loads:
// two scalar-memory instructions fewer per node step. The prefetch is a second asm right after the
// load's wait; the ray's reciprocal direction, passed through it as a read-write operand (a loop-carried
// copy, no move), keeps the box tests below it.
#ifndef RT_PF_INREG
#define RT_PF_INREG 1
#endif
__device__ __forceinline__ Node64 sload_node_pf_inreg(const Node64* base, uint32_t h, uint32_t& pf0, uint32_t& pf1,
                                                      f3& id) {
  const uint32_t off = node_offset(__builtin_amdgcn_readfirstlane(h));
  const uint64_t b = (uint64_t)base;
  const uint64_t bs = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  i16v v;
  asm volatile("s_load_dwordx16 %0, %3, %4\n\ts_waitcnt lgkmcnt(0)" : "=&s"(v), "+s"(pf0), "+s"(pf1) : "s"(bs), "s"(off) : "memory");
  Node64 r;
  __builtin_memcpy(&r, &v, 64);
  asm volatile("s_load_dword %0, %5, %6\n\ts_load_dword %1, %5, %7"
               : "+s"(pf0), "+s"(pf1), "+v"(id.x), "+v"(id.y), "+v"(id.z)
               : "s"(bs), "s"(r.pad0), "s"(r.pad1)
               : "memory");
  return r;
}
__device__ __forceinline__ TriRec64 sload_tri(const TriRec64* base, uint32_t i) { return sload64(base, i); }
// node fetch by byte offset with one carried prefetch sink (RT_PF_MODE 1 / 2: the step's own s_waitcnt
// retires the previous step's far-child prefetch)
__device__ __forceinline__ Node64 sload_node_sink(const Node64* base, uint32_t h, uint32_t& sink) {
  const uint32_t off = node_offset(__builtin_amdgcn_readfirstlane(h));
  const uint64_t b = (uint64_t)base;
  const uint64_t bs = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  i16v v;
  asm volatile("s_load_dwordx16 %0, %2, %3\n\ts_waitcnt lgkmcnt(0)" : "=&s"(v), "+&s"(sink) : "s"(bs), "s"(off) : "memory");
  Node64 r;
  __builtin_memcpy(&r, &v, 64);
  return r;
}

__device__ __forceinline__ uint32_t uniform(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

// counters of the RT_FRAME_STATS counting run
// ST_WPOP / ST_WCULL (counting run, closest hit): stack pops per wave, and those pops at which no lane
// that wanted the entry still could (every such lane's entry distance into it, recorded at the push,
// now beyond its closest hit) -- what culling at the pop would save (rt_debug_counters)
// ST_WWIDE: 128-B fp32 4-wide node records fetched per wave (ST_WNODE: 64-B binary / quantised records)
// ST_WCAND / ST_WPRE / ST_WINS (counting run, per wave-level triangle test): some lane passed the plane-
// distance stage; some candidate lane's hit point lies inside the triangle's bounding box grown by 1e-3 of
// its extent (what a box prefilter would keep); some lane passed the reference's edge tests. ST_WE1 / ST_WE2:
// the staged edge tests (RT_TRI_STAGED) left no candidate after the first / the second edge
enum { ST_NODE = 0, ST_TRI, ST_WNODE, ST_WTRI, ST_RAYS, ST_HITS, ST_TOTAL, ST_WPOP, ST_WCULL, ST_WWIDE,
       ST_WCAND, ST_WPRE, ST_WINS, ST_WE1, ST_WE2,
       // round 4: the same triangle-stage counts with the candidates restricted to the lanes whose ray entered
       // the leaf's box (ST_WCANDM .. ST_WINSM), the triangle tests of leaves reached by descent (ST_WTRID) and
       // their entry-masked candidate count (ST_WCANDD: popped leaves unmasked), and wave-level tests where a
       // lane that never entered the leaf accepted (ST_WACCX: 0 if leaf-entry masking is exact)
       ST_WCANDM, ST_WE1M, ST_WE2M, ST_WINSM, ST_WTRID, ST_WCANDD, ST_WACCX,
       // RT_STATS_FRUSTUM experiment: child tests where some lane's own slab test enters but the packet's
       // interval test does not (must stay 0: the interval test is conservative)
       ST_WFVIOL, ST_COUNT };
constexpr int kStatSlots = 24;

struct Hit {
  float t;
  uint32_t rank;
  uint32_t slot;
};

struct Ray {
  f3 o, d;      // world space (triangle tests)
  f3 id;        // culling: 1/d (zeros nudged)
  f3 oa, ob;    // culling: -(o + p)/d and -(o - p)/d, the lo / hi plane offsets of boxes grown by p
  f3 o2, d2;    // object space (reference intersectBox): Minv*o_box, normalized(MS*d)
};

__device__ __forceinline__ float nudge(float x) { return fabsf(x) < 1e-20f ? copysignf(1e-20f, x) : x; }

// Culling set-up of a ray, once per ray.
// The BVH boxes carry a static pad for the scene-scale rounding of the reference's arithmetic (bvh_pad,
// rt_host.cpp). The rounding of the reference's hit point P = o + t d, and of this slab test, also grows
// with the ray origin's magnitude: both are a few ulp of |o| + |t d| <= 2|o| + R per axis (R: the scene's
// magnitude). So every ray grows the boxes it tests by its own pad p = kCullPadRel * |o|_inf, folded into
// two per-axis offsets: with box [lo - p, hi + p] the plane distances are fma(lo, 1/d, -(o + p)/d) and
// fma(hi, 1/d, -(o - p)/d). That costs no instruction per node (the octant loops pick the offset of each
// plane at compile time). kCullPadRel = 4e-5 is ~100x the worst-case rounding (<= 6 ulp of |o|, each
// 2^-24 |o|), so for every origin the culling never drops a face the reference accepts.
// Outside the range where these products stay finite (|o|_inf > 1e18, |d|_inf outside [1e-12, 1e18], or
// non-finite input) the ray's boxes grow without bound instead: p = inf, every box is entered, and the
// packet tests every triangle with the exact test -- still the reference's result, by brute force.
#ifndef RT_DYN_PAD  // 0: static pad only (round-2 behaviour, kept to demonstrate the far-origin tests failing)
#define RT_DYN_PAD 1
#endif
constexpr float kCullPadRel = 4e-5f, kCullOriginMax = 1e18f, kCullDirMin = 1e-12f, kCullDirMax = 1e18f;
// The ray's own pad is needed only once it exceeds the static one (every box already carries
// static_pad >= the ray's pad, so the same ~100x margin holds): for origins near the scene -- every
// secondary ray, and primary rays of an eye near it -- the boxes keep exactly their static size.
__device__ __forceinline__ void setup_cull(Ray& r, float static_pad) {
  const float om = fmaxf(fmaxf(fabsf(r.o.x), fabsf(r.o.y)), fabsf(r.o.z));
  const float dm = fmaxf(fmaxf(fabsf(r.d.x), fabsf(r.d.y)), fabsf(r.d.z));
  const bool certified = !RT_DYN_PAD || (om <= kCullOriginMax && dm >= kCullDirMin && dm <= kCullDirMax);  // false for NaN
  if (certified) {
    r.id = f3{__builtin_amdgcn_rcpf(nudge(r.d.x)), __builtin_amdgcn_rcpf(nudge(r.d.y)),
              __builtin_amdgcn_rcpf(nudge(r.d.z))};
    const float pr = kCullPadRel * om;
    const float p = RT_DYN_PAD && pr > static_pad ? pr : 0.0f;
    r.oa = f3{-(r.o.x + p) * r.id.x, -(r.o.y + p) * r.id.y, -(r.o.z + p) * r.id.z};
    r.ob = f3{-(r.o.x - p) * r.id.x, -(r.o.y - p) * r.id.y, -(r.o.z - p) * r.id.z};
  } else {
    // unbounded boxes: lo planes at -inf, hi planes at +inf along the (kept) direction signs
    r.id = f3{copysignf(1.0f, nudge(r.d.x)), copysignf(1.0f, nudge(r.d.y)), copysignf(1.0f, nudge(r.d.z))};
    r.oa = f3{-r.id.x * INFINITY, -r.id.y * INFINITY, -r.id.z * INFINITY};
    r.ob = f3{r.id.x * INFINITY, r.id.y * INFINITY, r.id.z * INFINITY};
  }
}

#ifndef RT_TRI_VREG  // edge differences from VGPR copies of w0 / w1 (fewer moves)
#define RT_TRI_VREG 1
#endif
#ifndef RT_EYE_VREG  // k_primary_fused keeps the eye in VGPRs
#define RT_EYE_VREG 1
#endif
// Conservative slab test for one padded child box (culling only; exactness comes from padding):
// returns the entry distance tmin and the exit distance clipped to [0, tmax_ray] (hit iff tmin <= tmax)
struct Span {
  float tmin, tmax;
};
__device__ __forceinline__ Span slab(float lx, float hx, float ly, float hy, float lz, float hz, const Ray& r,
                                     float tmax_ray) {
  const float tx0 = __builtin_fmaf(lx, r.id.x, r.oa.x), tx1 = __builtin_fmaf(hx, r.id.x, r.ob.x);
  const float ty0 = __builtin_fmaf(ly, r.id.y, r.oa.y), ty1 = __builtin_fmaf(hy, r.id.y, r.ob.y);
  const float tz0 = __builtin_fmaf(lz, r.id.z, r.oa.z), tz1 = __builtin_fmaf(hz, r.id.z, r.ob.z);
  Span s;
  s.tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
  s.tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax_ray));
  return s;
}
// The same span when the wave's active rays share one direction octant (OCT bit k: axis k negative,
// by the sign of the nudged reciprocal): fma(., id, offset) is monotone in the box coordinate, so the
// near / far plane of each axis is known and min(t0, t1) / max(t0, t1) are exactly the near / far
// values -- identical results with 8 fewer min/max per child. OCT < 0: the generic test.
#ifndef RT_CLIP_ASM
#define RT_CLIP_ASM 1
#endif
// CLIP = false (octant loops of packets whose rays all start in front of the scene, trace_oct): the entry
// distance is not clipped at 0. That admits a superset of boxes (max(tmin, 0) >= tmin), so culling stays
// conservative, and for such a packet it admits no extra box: every box lies inside the root's, which
// each ray enters at t >= 0 or misses, and the rounded plane distances are monotone in the coordinates.
template <int OCT, bool CLIP = true>
__device__ __forceinline__ Span slab_o(float lx, float hx, float ly, float hy, float lz, float hz, const Ray& r,
                                       float tmax_ray) {
  if (OCT < 0) return slab(lx, hx, ly, hy, lz, hz, r, tmax_ray);
  // near plane of a positive axis: lo (offset oa); of a negative axis: hi (offset ob); far the other
  const float nx = (OCT & 1) ? hx : lx, fx = (OCT & 1) ? lx : hx;
  const float ny = (OCT & 2) ? hy : ly, fy = (OCT & 2) ? ly : hy;
  const float nz = (OCT & 4) ? hz : lz, fz = (OCT & 4) ? lz : hz;
  const float nox = (OCT & 1) ? r.ob.x : r.oa.x, fox = (OCT & 1) ? r.oa.x : r.ob.x;
  const float noy = (OCT & 2) ? r.ob.y : r.oa.y, foy = (OCT & 2) ? r.oa.y : r.ob.y;
  const float noz = (OCT & 4) ? r.ob.z : r.oa.z, foz = (OCT & 4) ? r.oa.z : r.ob.z;
  Span s;
  if (CLIP)
    s.tmin = fmaxf(fmaxf(__builtin_fmaf(nx, r.id.x, nox), __builtin_fmaf(ny, r.id.y, noy)),
                   fmaxf(__builtin_fmaf(nz, r.id.z, noz), 0.0f));
  else
    s.tmin = fmaxf(fmaxf(__builtin_fmaf(nx, r.id.x, nox), __builtin_fmaf(ny, r.id.y, noy)),
                   __builtin_fmaf(nz, r.id.z, noz));
#if RT_CLIP_ASM
  // min of the three far planes and tmax_ray in two instructions (the compiler's fminf would first
  // canonicalise tmax_ray, a loop-carried value, with an extra v_max per node)
  asm("v_min3_f32 %0, %1, %2, %3\n\tv_min_f32 %0, %0, %4"
      : "=&v"(s.tmax)
      : "v"(__builtin_fmaf(fx, r.id.x, fox)), "v"(__builtin_fmaf(fy, r.id.y, foy)),
        "v"(__builtin_fmaf(fz, r.id.z, foz)), "v"(tmax_ray));
#else
  s.tmax = fminf(fminf(__builtin_fmaf(fx, r.id.x, fox), __builtin_fmaf(fy, r.id.y, foy)),
                 fminf(__builtin_fmaf(fz, r.id.z, foz), tmax_ray));
#endif
  return s;
}
// lane masks straight from v_cmp (no bool materialisation): llvm.amdgcn.fcmp predicates
constexpr int kFcmpOLE = 5;
__device__ __forceinline__ uint64_t mask_le(float a, float b) { return __builtin_amdgcn_fcmpf(a, b, kFcmpOLE); }

// The reference's object-space box test, exact (flyscene.cpp:484-507)
__device__ __forceinline__ bool ref_box_test(const Ray& r, const float* bx) {
  const float lo[3] = {bx[0], bx[1], bx[2]}, hi[3] = {bx[4], bx[5], bx[6]};
  const float o2[3] = {r.o2.x, r.o2.y, r.o2.z}, d2[3] = {r.d2.x, r.d2.y, r.d2.z};
  float tin3[3], tout3[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float a = (lo[k] - o2[k]) / d2[k];
    const float b = (hi[k] - o2[k]) / d2[k];
    tin3[k] = smin(a, b);
    tout3[k] = smax(a, b);
  }
  const float tin = smax(tin3[0], smax(tin3[1], tin3[2]));
  const float tout = smin(tout3[0], smin(tout3[1], tout3[2]));
  return !(tin > tout || tout < 0);
}

__device__ __forceinline__ f3 ld3(const float* p) { return f3{p[0], p[1], p[2]}; }

// Lane masks straight from the compares (llvm.amdgcn.fcmp / icmp predicates): candidate sets stay in
// SGPR pairs and wave-level decisions are one s_cmp, with no bool materialisation in VGPRs
constexpr int kFcmpOEQ = 1, kFcmpOGE = 3, kFcmpOLT = 4, kFcmpUNE = 14, kIcmpULT = 36;
template <int PRED>
__device__ __forceinline__ uint64_t fmask(float a, float b) { return __builtin_amdgcn_fcmpf(a, b, PRED); }
__device__ __forceinline__ bool lane_in(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }

#ifndef RT_BOX_CERT  // 1: certified faces (kBoxCertBit) skip the reference box predicate
#define RT_BOX_CERT 1
#endif
// Rare path of a candidate (uniform triangle): interpolated normal non-zero (calculateDistance's
// norm()==0 check, flyscene.cpp:467) and the reference box predicate. All loads wave-uniform.
__device__ __forceinline__ uint64_t accept_candidate(const DevScene& P, const TriRec64& tr, uint32_t slot, f3 e0, f3 e2,
                                                    f3 a0, f3 a1, f3 a2, f3 p, const Ray& r, uint64_t cand) {
  if (!(tr.box & kSafeNormalBit)) {  // uniform branch: only faces the host could not certify
    const float area0 = norm(a0) / 2, area1 = norm(a1) / 2, area2 = norm(a2) / 2;
    const float area = norm(cross(e0, neg(e2))) / 2;
    const float* fs = P.fshade + 12 * (size_t)slot;
    const f3 n0 = ld3(fs), n1 = ld3(fs + 4), n2 = ld3(fs + 8);
    const f3 nn = blend_normal(n0, n1, n2, area0, area1, area2, area);
    cand &= fmask<kFcmpUNE>(norm(nn), 0.0f);
  }
#if defined(RT_EXP_NO_BOXPRED)  // timing experiment only: the reference box predicate skipped (wrong results)
  return cand;
#endif
  if (RT_BOX_CERT && (tr.box & kBoxCertBit)) {
    // certified face (kBoxCertBit): the predicate holds for every candidate lane whose object-space
    // origin is within the certified range (NaN fails the compare and takes the path below)
    const float om = fmaxf(fmaxf(fabsf(r.o2.x), fabsf(r.o2.y)), fabsf(r.o2.z));
    if ((cand & ~ballot(om <= P.cert_origin_max)) == 0) return cand;
  }
  // reference box predicate. Fast path: the object-space hit point lies inside the reference box
  // with a margin (1e-5 relative) far above the reference slab test's rounding, so the exact ray
  // crosses the box interior at t >= 0 and intersectBox accepts. Otherwise run the exact test.
  const float* bx = P.refbox + 8 * (size_t)(tr.box & kBoxIndexMask);
  const f3 X = affv3(P.Minv, p);
  const float lo[3] = {bx[0], bx[1], bx[2]}, hi[3] = {bx[4], bx[5], bx[6]};
  const float xs[3] = {X.x, X.y, X.z}, os[3] = {r.o2.x, r.o2.y, r.o2.z};
  bool inside = true;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float m = 1e-5f * ((hi[k] - lo[k]) + fabsf(lo[k]) + fabsf(hi[k]) + fabsf(os[k])) + 1e-30f;
    inside = inside & (xs[k] > lo[k] + m) & (xs[k] < hi[k] - m);
  }
  const uint64_t ins = ballot(inside);
  if ((cand & ~ins) == 0) return cand;
  return cand & (ins | ballot(ref_box_test(r, bx)));
}

// calculateDistance (flyscene.cpp:444-478) against a wave-uniform triangle record, for the lanes of
// `act`. CLOSEST: update (t, rank, slot) if 0 <= t < best (rank breaks ties as the reference's order
// does). ANY: any valid t >= 0 (shadow(), flyscene.cpp:519).
#ifndef RT_TRI_STAGED  // 1: the three edge tests one at a time, the wave leaving once no candidate is left
#define RT_TRI_STAGED 1
#endif
#ifndef RT_TRI_CLASS  // 1: the closest-hit candidate range test as one v_cmp_class (same set)
#define RT_TRI_CLASS 1
#endif
template <bool ANY, bool STATS = false>
__device__ __forceinline__ void test_tri(const DevScene& P, const TriRec64& tr, uint32_t slot, const Ray& r,
                                         uint64_t act, Hit& h, bool& found, uint32_t* cnt = nullptr,
                                         uint64_t entry = ~0ull, bool desc = false) {
  const f3 n{tr.nx, tr.ny, tr.nz};
  const float dn = dot(n, r.d);                 // facenormal.dot(dir)
  const float orth = tr.dist - dot(r.o, n);     // distancePlane - origin.dot(facenormal)
  const float t = orth / dn;                    // / dir.dot(facenormal)  (same bits as dn)
  uint64_t cand;
  if (!ANY && RT_TRI_CLASS) {
    // dn != 0 && 0 <= t < inf in one class test: t is -0, +0, +denormal or +normal (dn == 0 makes t
    // +-inf or NaN, which the class excludes as the separate tests did)
    uint64_t cls;
    asm("v_cmp_class_f32_e64 %0, %1, %2" : "=s"(cls) : "v"(t), "v"(0x1E0u));
    cand = act & cls &
           (fmask<kFcmpOLT>(t, h.t) | (fmask<kFcmpOEQ>(t, h.t) & __builtin_amdgcn_uicmp(tr.rank, h.rank, kIcmpULT)));
  } else {
    cand = act & fmask<kFcmpUNE>(dn, 0.0f) & fmask<kFcmpOGE>(t, 0.0f);
    if (!ANY)
      cand &= fmask<kFcmpOLT>(t, INFINITY) &
              (fmask<kFcmpOLT>(t, h.t) | (fmask<kFcmpOEQ>(t, h.t) & __builtin_amdgcn_uicmp(tr.rank, h.rank, kIcmpULT)));
  }
  if (STATS) cnt[ST_WCAND] += cand != 0;
  const f3 p{r.o.x + t * r.d.x, r.o.y + t * r.d.y, r.o.z + t * r.d.z};
  const f3 w0{tr.w0x, tr.w0y, tr.w0z}, w1{tr.w1x, tr.w1y, tr.w1z}, w2{tr.w2x, tr.w2y, tr.w2z};
  if (STATS) {
    // entry-masked stage counts: all three edge masks evaluated for every lane, the stages derived
    const uint64_t cm = cand & entry;
    const uint64_t b0 = ballot(dot(n, cross(sub(w1, w0), sub(p, w0))) < 0);
    const uint64_t b1 = ballot(dot(n, cross(sub(w2, w1), sub(p, w1))) < 0);
    const uint64_t b2 = ballot(dot(n, cross(sub(w0, w2), sub(p, w2))) < 0);
    cnt[ST_WCANDM] += cm != 0;
    cnt[ST_WE1M] += cm != 0 && (cm & ~b0) == 0;
    cnt[ST_WE2M] += (cm & ~b0) != 0 && (cm & ~b0 & ~b1) == 0;
    cnt[ST_WINSM] += (cm & ~b0 & ~b1 & ~b2) != 0;
    if (desc) cnt[ST_WTRID]++;
    cnt[ST_WCANDD] += (cand & (desc ? entry : ~0ull)) != 0;
  }
  if (cand == 0) return;
  if (STATS) {
    const f3 lo{fminf(fminf(w0.x, w1.x), w2.x), fminf(fminf(w0.y, w1.y), w2.y), fminf(fminf(w0.z, w1.z), w2.z)};
    const f3 hi{fmaxf(fmaxf(w0.x, w1.x), w2.x), fmaxf(fmaxf(w0.y, w1.y), w2.y), fmaxf(fmaxf(w0.z, w1.z), w2.z)};
    const float m = 1e-3f * fmaxf(fmaxf(hi.x - lo.x, hi.y - lo.y), hi.z - lo.z);
    const bool in = p.x >= lo.x - m && p.x <= hi.x + m && p.y >= lo.y - m && p.y <= hi.y + m &&
                    p.z >= lo.z - m && p.z <= hi.z + m;
    cnt[ST_WPRE] += (cand & ballot(in)) != 0;
  }
#if RT_TRI_VREG
  // the record is wave-uniform (SGPRs) and a VALU op reads at most one SGPR: w0 and w1 copied into
  // VGPRs once serve all three edge differences (6 moves instead of 9; same float operations)
  f3 v0 = w0, v1 = w1;
  asm("" : "+v"(v0.x), "+v"(v0.y), "+v"(v0.z), "+v"(v1.x), "+v"(v1.y), "+v"(v1.z));
  const f3 e0 = sub(w1, v0), e1 = sub(w2, v1), e2 = sub(v0, w2);
#else
  const f3 e0 = sub(w1, w0), e1 = sub(w2, w1), e2 = sub(w0, w2);
#endif
  f3 a0, a1, a2;
  if (RT_TRI_STAGED || STATS) {
    // the reference's three edge tests are independent (interpolateNormal, flyscene.cpp:591: rejected if any is
    // negative), so they run one at a time and the wave stops as soon as no candidate lane is left --
    // the same values, the same set; a packet wholly beyond one edge line skips the other edges' work
    a0 = cross(e0, sub(p, w0));
    cand &= ~ballot(dot(n, a0) < 0);
    if (STATS) cnt[ST_WE1] += cand == 0;
    if (cand == 0) return;
    a1 = cross(e1, sub(p, w1));
    cand &= ~ballot(dot(n, a1) < 0);
    if (STATS) cnt[ST_WE2] += cand == 0;
    if (cand == 0) return;
    a2 = cross(e2, sub(p, w2));
    cand &= ~ballot(dot(n, a2) < 0);
  } else {
    a0 = cross(e0, sub(p, w0)), a1 = cross(e1, sub(p, w1)), a2 = cross(e2, sub(p, w2));
    cand &= ~ballot((int)(dot(n, a0) < 0) | (int)(dot(n, a1) < 0) | (int)(dot(n, a2) < 0));
  }
  if (STATS) cnt[ST_WINS] += cand != 0;
  if (cand == 0) return;
  const bool acc = lane_in(accept_candidate(P, tr, slot, e0, e2, a0, a1, a2, p, r, cand));
  if (STATS) cnt[ST_WACCX] += (ballot(acc) & ~entry) != 0;
  if (ANY) {
    found = found | acc;
  } else {
    h.t = acc ? t : h.t;
    h.rank = acc ? tr.rank : h.rank;
    h.slot = acc ? slot : h.slot;
  }
}

// ------------------------------------------------------------------------------------------------
// Wave-packet traversal. STACK_LDS selects the wave stack home: LDS (one uint32 row per wave) or the
// 64 lanes of one VGPR (v_writelane / v_readlane with an SGPR lane index).
// ------------------------------------------------------------------------------------------------
struct WaveStack {
  uint32_t v = 0;
  int sp = 0;
};

// Wave-packet loop with every option: VGPR or LDS stack and the counting run (RT_FRAME_STATS). The
// production closest-hit / any-hit path is traverse_fast() below (same visit order, leaner per-node
// code); this loop serves the counting run and the VGPR-stack A/B variant.
// Knobs (A/B builds; results are identical either way):
//   RT_ORDER_BITS       octant-specialised loops take the near child from the node's precomputed order
//                       bit for the wave's octant (split-axis rule, octant_order() in rt_host.cpp)
//                       instead of a lane-majority vote: 3 fewer SALU and one fewer v_cmp per node step
//                       (default 1; C3 +3.7% at 4 frames in flight, bunny +2.6%; 0 = the vote)
//   RT_EXPERIMENT_SALU  timing experiment: N extra independent SALU per node step
//   RT_EXPERIMENT_VALU  timing experiment: N extra independent VALU per node step
#ifndef RT_ORDER_BITS
#define RT_ORDER_BITS 1
#endif
#ifndef RT_FAST_LOOP
#define RT_FAST_LOOP 1
#endif
#ifndef RT_VADDR_PUSH  // 1: the wave stack's push address is scaled by a VALU op instead of an SALU op
#define RT_VADDR_PUSH 0
#endif
#ifndef RT_EXPERIMENT_SALU
#define RT_EXPERIMENT_SALU 0
#endif
#ifndef RT_EXPERIMENT_VALU
#define RT_EXPERIMENT_VALU 0
#endif
// RT_PREFETCH: the fast loop prefetches both children's records into the scalar cache (Node64::pad0/1
// then hold prefetch offsets, with the order bits in their low bits)
#ifndef RT_PREFETCH
#define RT_PREFETCH 1
#endif
#ifndef RT_PREFETCH_PADLOAD  // 1: offsets re-loaded inside the node-load asm (0: tie-ordered separate asm, measured ±0.5%)
#define RT_PREFETCH_PADLOAD 1
#endif
#ifndef RT_PF_MODE  // 0: both children prefetched at node arrival (RT_PREFETCH); 1: far child after the decision; 2: none;
                    // 3: the near child (octant order bit) at node arrival; 4: 3 + the far child's line
                    // into L2 by a vector load; 5: both children by vector loads
#define RT_PF_MODE 0
#endif
#ifndef RT_PF_CARRY  // 1: prefetch sinks carried to the next node step (no wait at the end of a step)
#define RT_PF_CARRY 1
#endif
#ifndef RT_TOS  // 1: the stack top mirrored in a register, refilled from LDS right after a pop (A/B)
#define RT_TOS 0
#endif
// With RT_PREFETCH, Node64::pad0 / pad1 hold the children's record offsets (multiples of 64), so the
// eight octant order bits travel in their low bits: octants 0-5 in pad0 bits 0-5, octants 6-7 in pad1
// bits 0-1. A scalar load ignores the two low offset bits and the rest stays inside the 64-B record,
// so the prefetch still touches the child's cache line.
template <int OCT>
__device__ __forceinline__ uint32_t order_word(const Node64& nd) {
  return RT_PREFETCH ? (OCT < 6 ? nd.pad0 : nd.pad1) : nd.pad0;
}
template <int OCT>
constexpr int order_bit() {
  return RT_PREFETCH ? (OCT < 6 ? OCT : OCT - 6) : (OCT & 7);
}
#define RT_STR2(x) #x
#define RT_STR(x) RT_STR2(x)
// RT_STATS_FRUSTUM (counting-run experiment, ablib builds only): the closest-hit octant loops of the
// counting run descend by a conservative wave-uniform interval test of the packet (common origin, the
// interval of each reciprocal direction component over the wave, the wave's largest t_best) instead of
// the union of the per-lane slab tests; triangle tests stay per lane, so the frame is unchanged and the
// counters say how many node steps / triangle records that test visits.
#ifndef RT_STATS_FRUSTUM
#define RT_STATS_FRUSTUM 0
#endif
__device__ __forceinline__ float wave_minf(float v) {
  for (int off = 32; off > 0; off >>= 1) v = fminf(v, __shfl_xor(v, off, 64));
  return v;
}
__device__ __forceinline__ float wave_maxf(float v) {
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}
struct Frustum {
  f3 o, idmin, idmax;
};
// min / max over id in [a, b] of c * id
__device__ __forceinline__ float imul_min(float c, float a, float b) { return c >= 0.0f ? c * a : c * b; }
__device__ __forceinline__ float imul_max(float c, float a, float b) { return c >= 0.0f ? c * b : c * a; }
template <int OCT>
__device__ __forceinline__ bool frustum_enter(const Frustum& F, float lx, float hx, float ly, float hy, float lz, float hz,
                                              float T) {
  const float nx = (OCT & 1) ? hx : lx, fx = (OCT & 1) ? lx : hx;
  const float ny = (OCT & 2) ? hy : ly, fy = (OCT & 2) ? ly : hy;
  const float nz = (OCT & 4) ? hz : lz, fz = (OCT & 4) ? lz : hz;
  const float tn = fmaxf(fmaxf(imul_min(nx - F.o.x, F.idmin.x, F.idmax.x), imul_min(ny - F.o.y, F.idmin.y, F.idmax.y)),
                         fmaxf(imul_min(nz - F.o.z, F.idmin.z, F.idmax.z), 0.0f));
  const float tf = fminf(fminf(imul_max(fx - F.o.x, F.idmin.x, F.idmax.x), imul_max(fy - F.o.y, F.idmin.y, F.idmax.y)),
                         fminf(imul_max(fz - F.o.z, F.idmin.z, F.idmax.z), T));
  return tn <= tf;
}

template <bool ANY, bool STATS, bool STACK_LDS, int OCT = -1>
__device__ __forceinline__ void traverse(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                         uint32_t* lds_stack, uint32_t* cnt) {
  if (P.n_nodes == 0) return;
  constexpr bool FRU = RT_STATS_FRUSTUM && STATS && !ANY && OCT >= 0;
  Frustum F{};
  bool fru = false;  // the packet has one common origin (primary rays): the interval test drives descent
  if (FRU) {
    const float ox = __shfl(r.o.x, (int)__builtin_ctzll(ballot(active) | (1ull << 63)), 64);
    const float oy = __shfl(r.o.y, (int)__builtin_ctzll(ballot(active) | (1ull << 63)), 64);
    const float oz = __shfl(r.o.z, (int)__builtin_ctzll(ballot(active) | (1ull << 63)), 64);
    fru = ballot(active && (r.o.x != ox || r.o.y != oy || r.o.z != oz)) == 0 && ballot(active) != 0;
    F.o = f3{ox, oy, oz};
    F.idmin = f3{wave_minf(active ? r.id.x : INFINITY), wave_minf(active ? r.id.y : INFINITY), wave_minf(active ? r.id.z : INFINITY)};
    F.idmax = f3{wave_maxf(active ? r.id.x : -INFINITY), wave_maxf(active ? r.id.y : -INFINITY), wave_maxf(active ? r.id.z : -INFINITY)};
  }
  uint32_t stackv = 0;     // lane k holds stack entry k (VGPR stack)
  int sp = 0;              // wave-uniform stack depth (SGPR)
  uint64_t flagstack = 0;  // STATS: per-lane "my ray wanted this entry" bit per stack level
  float tstack[STATS ? 64 : 1];  // STATS: per-lane entry distance into each stack entry
  bool want = active;      // STATS: this lane's ray intersects the current node
  bool desc = false;       // STATS: the current node was reached by descent (not popped)
  uint32_t node = P.root;
  const float tmax_any = INFINITY;
  uint64_t act = ballot(active);  // lanes still tracing (wave-uniform mask)
  uint32_t exp_s = 0, exp_v = 0;  // RT_EXPERIMENT_SALU / _VALU sinks
  // one pop site and branch-free pushes keep the per-node control flow to the two uniform branches
  // (interior vs leaf, pop vs descend)
  for (;;) {
    bool pop = true;
    if (!is_leaf(node)) {
      const Node64 nd = sload_node(P.nodes, node);  // one scalar 64-B fetch per wave
      if (STATS) {
        if (want) cnt[ST_NODE]++;
        cnt[ST_WNODE]++;
      }
      const float tcut = ANY ? tmax_any : h.t;
      const Span s0 = slab_o<OCT>(nd.c0lx, nd.c0hx, nd.c0ly, nd.c0hy, nd.c0lz, nd.c0hz, r, tcut);
      const Span s1 = slab_o<OCT>(nd.c1lx, nd.c1hx, nd.c1ly, nd.c1hy, nd.c1lz, nd.c1hz, r, tcut);
#ifdef RT_EXPERIMENT_NODES_TWICE  // timing experiment only: the box tests once more on opaque copies
      {
        Ray r2 = r;
        float tc2 = tcut;
        asm volatile("" : "+v"(r2.id.x), "+v"(r2.id.y), "+v"(r2.id.z), "+v"(r2.oa.x), "+v"(r2.oa.y), "+v"(r2.oa.z), "+v"(tc2));
        const Span q0 = slab(nd.c0lx, nd.c0hx, nd.c0ly, nd.c0hy, nd.c0lz, nd.c0hz, r2, tc2);
        const Span q1 = slab(nd.c1lx, nd.c1hx, nd.c1ly, nd.c1hy, nd.c1lz, nd.c1hz, r2, tc2);
        uint64_t mm = mask_le(q0.tmin, q0.tmax) | mask_le(q1.tmin, q1.tmax);
        asm volatile("" ::"s"(mm));
      }
#endif
      uint64_t m0 = mask_le(s0.tmin, s0.tmax) & act, m1 = mask_le(s1.tmin, s1.tmax) & act;
      const uint64_t lm0 = m0, lm1 = m1;  // the lanes' own verdicts (want flags)
      if (FRU && fru) {
        const float T = wave_maxf(active ? h.t : -INFINITY);
        const bool f0 = frustum_enter<OCT>(F, nd.c0lx, nd.c0hx, nd.c0ly, nd.c0hy, nd.c0lz, nd.c0hz, T);
        const bool f1 = frustum_enter<OCT>(F, nd.c1lx, nd.c1hx, nd.c1ly, nd.c1hy, nd.c1lz, nd.c1hz, T);
        cnt[ST_WFVIOL] += (m0 != 0 && !f0) + (m1 != 0 && !f1);
        m0 = f0 ? ~0ull : 0ull;
        m1 = f1 ? ~0ull : 0ull;
      }
#if RT_EXPERIMENT_SALU > 0  // timing experiment only: N extra independent SALU per node step
      exp_s = uniform(exp_s);
      asm volatile(".rept " RT_STR(RT_EXPERIMENT_SALU) "\n\ts_add_u32 %0, %0, 1\n\t.endr" : "+s"(exp_s));
#endif
#if RT_EXPERIMENT_VALU > 0  // timing experiment only: N extra independent VALU per node step
      asm volatile(".rept " RT_STR(RT_EXPERIMENT_VALU) "\n\tv_add_u32 %0, %0, 1\n\t.endr" : "+v"(exp_v));
#endif
      bool first0;
      if (RT_ORDER_BITS && OCT >= 0) {
        // the node's order bit for this octant, overridden when only one child is needed
        const bool pref1 = (order_word<OCT>(nd) >> order_bit<OCT>()) & 1u;
        first0 = m1 == 0 || (m0 != 0 && !pref1);
      } else {
        // near child first by lane majority: each lane that needs a child votes for the one it enters
        // first (covers m0 == 0 -> child 1 and m1 == 0 -> child 0)
        const uint64_t v0 = m0 & (~m1 | mask_le(s0.tmin, s1.tmin));
        first0 = 2 * __popcll(v0) >= __popcll(m0 | m1);
      }
      const uint32_t far = first0 ? nd.child1 : nd.child0;
      // the far child is written above the top unconditionally and kept only when both are needed
      if (STACK_LDS) lds_stack[sp] = far;
      else asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0"
                        : "+v"(stackv)
                        : "s"(uniform(far)), "s"(uniform((uint32_t)sp))
                        : "m0");
      if (STATS) {
        const bool h0 = (lm0 >> lane_id()) & 1, h1 = (lm1 >> lane_id()) & 1;
        const bool wf = first0 ? h1 : h0;
        flagstack = (flagstack & ~(1ull << sp)) | ((uint64_t)wf << sp);
        want = first0 ? h0 : h1;
        desc = true;
        tstack[sp] = first0 ? s1.tmin : s0.tmin;
      }
      sp += ((m0 != 0) & (m1 != 0)) ? 1 : 0;
      node = first0 ? nd.child0 : nd.child1;
      pop = (m0 | m1) == 0;
    } else {
      // leaf: its triangles are fetched once per wave and tested by every lane
      const uint32_t first = leaf_first(node), count = leaf_count(node);
      if (STATS) {
        if (want) cnt[ST_TRI] += count;
        cnt[ST_WTRI] += count;
      }
      for (uint32_t k = 0; k < count; k++) {
        const TriRec64 tr = sload_tri(P.tris, first + k);
        test_tri<ANY, STATS>(P, tr, first + k, r, act, h, found, cnt, STATS ? ballot(want) : ~0ull, desc);
      }
#ifdef RT_EXPERIMENT_TRIS_TWICE  // timing experiment only: the same leaf tested again (no effect)
      for (uint32_t k = 0; k < count; k++) {
        const TriRec64 tr = sload_tri(P.tris, first + k);
        test_tri<ANY>(P, tr, first + k, r, act, h, found);
      }
#endif
      if (ANY) {
        active = active & !found;
        act = ballot(active);
        if (!act) break;
      }
    }
    if (pop) {
      if (sp == 0) break;
      sp--;
      node = STACK_LDS ? uniform(lds_stack[sp]) : (uint32_t)__builtin_amdgcn_readlane(stackv, sp);
      if (STATS) {
        want = (flagstack >> sp) & 1;
        desc = false;
        cnt[ST_WPOP]++;
        if (!ANY && ballot(want && tstack[sp] <= h.t) == 0) cnt[ST_WCULL]++;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// The production packet loop (LDS wave stack, no counting): the same visit order as traverse(), with
// the per-node work arranged for the scalar unit, which is this kernel's tightest resource (measured:
// one extra SALU per node step costs ~0.9% of the trace time, one extra VALU ~0.2%):
//  * the descend / push / pop decision is one straight-line SALU block; a pop is signalled by the
//    marker handle kPopMarker (leaf bit set, never a real leaf), so the interior loop needs one
//    compare-and-branch per step and there is a single pop site;
//  * lanes without a ray (closest hit) carry t_best = -1 and lanes whose shadow ray is blocked (any
//    hit) carry a box-test limit of -1, so every box test fails for them and the masks need no
//    "& active lanes" step.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kPopMarker = 0xFFFFFFFFu;

#ifndef RT_DECIDE8  // 1: the octant loops' post-mask decision in 8 SALU instead of 9 (same result)
#define RT_DECIDE8 1
#endif
#ifndef RT_EARLY_PUSH
#define RT_EARLY_PUSH 1
#endif
// the fast loop's wave-stack push as inline asm: a ds_write issued where it stands (the compiler would
// otherwise schedule the store with the decision block at the end of the step)
__device__ __forceinline__ void lds_push(uint32_t* slot, uint32_t v) {
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)slot;
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
// RT_STACK_ASM (A/B, off: the compiler pads the inline asm with s_nop wait states, a net loss): the push / pop address base + 4 sp in one VALU op (v_lshl_add_u32 with the depth as its
// scalar operand) instead of a scalar shift plus a move into a VGPR
#ifndef RT_STACK_ASM
#define RT_STACK_ASM 0
#endif
__device__ __forceinline__ uint32_t lds_base(const uint32_t* stack) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const uint32_t*)stack;
}
__device__ __forceinline__ void lds_push_at(const uint32_t* stack, uint32_t sp, uint32_t v) {
  // one asm: the address op separates the scalar write of v (the caller's s_cselect) from its move
  // into a VGPR, so no wait state is needed between them
  uint32_t a, d;
  asm volatile("v_lshl_add_u32 %0, %2, 2, %3\n\tv_mov_b32 %1, %4\n\tds_write_b32 %0, %1"
               : "=&v"(a), "=&v"(d)
               : "s"(sp), "v"(lds_base(stack)), "s"(v)
               : "memory");
}
__device__ __forceinline__ uint32_t lds_pop_at(const uint32_t* stack, uint32_t sp) {
  uint32_t a, v;
  asm("v_lshl_add_u32 %0, %1, 2, %2" : "=v"(a) : "s"(sp), "v"(lds_base(stack)));
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return __builtin_amdgcn_readfirstlane(v);
}

// traverse_fast from a given state (node handle, stack depth): the whole traversal starts at the root
// with an empty stack; the dual-chain loop (traverse_dual) hands over a half-finished one
// VST: the wave stack lives in the 64 lanes of one VGPR (v_writelane push, v_readlane pop: one VALU op
// each, no LDS address moves and no LDS read latency on the pop) -- only for a caller whose exec mask is
// full throughout (k_primary_fused): a VGPR copy under a partial exec mask would drop stack entries
#ifndef RT_VSTACK
#define RT_VSTACK 0
#endif
template <bool ANY, int OCT, bool CLIP = true, bool VST = false>
__device__ __forceinline__ void traverse_fast_from(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                                   uint32_t* lds_stack, uint32_t node, int sp) {
  int vstk = 0;  // VST: lane k holds stack entry k
  // lanes still tracing: used by the any-hit triangle tests only (a closest-hit lane without a ray
  // carries t_best = -1, which no candidate t >= -0 passes, so its triangle tests need no mask)
  uint64_t act = ANY ? ballot(active) : ~0ull;
  float tlim = active ? INFINITY : -1.0f;  // ANY: box-test limit (-1 once the lane is blocked)
  if (!ANY && !active) h.t = -1.0f;
#if RT_PREFETCH && RT_PF_CARRY
  uint32_t cpf0 = 0, cpf1 = 0;  // prefetch sinks, live across the traversal
#endif
  uint32_t fsink = 0;  // RT_PF_MODE 1 / 3 / 4: the scalar prefetch's sink
  uint32_t vsink0 = 0, vsink1 = 0;  // RT_PF_MODE 4 / 5: the vector prefetches' sinks
  uint32_t tos = 0;  // RT_TOS: lds_stack[sp - 1] while sp > 0
  f3 rid = r.id;  // RT_PF_INREG: loop-carried copy threaded through the prefetch asm
  for (;;) {
    while (!is_leaf(node)) {
      const int sp_before = sp;
      const uint32_t cur_off = node_offset(uniform(node));  // RT_PF_MODE 1
#if RT_PF_MODE != 0
      // 1: the far child is prefetched after the decision, only when it is pushed; 2: no prefetch
      const Node64 nd = sload_node_sink(P.nodes, node, fsink);
#elif RT_PREFETCH && RT_PF_CARRY && RT_PF_INREG
      const Node64 nd = sload_node_pf_inreg(P.nodes, node, cpf0, cpf1, rid);
#elif RT_PREFETCH && RT_PF_CARRY
      const Node64 nd = sload_node_pf_carry(P.nodes, node, cpf0, cpf1);
#elif RT_PREFETCH
      uint32_t pf0, pf1;
#if RT_PREFETCH_PADLOAD
      const Node64 nd = sload_node_pf(P.nodes, node, pf0, pf1);
#else
      Node64 nd = sload_node(P.nodes, node);
      // both children's records into the scalar cache, issued the moment the node has arrived: the
      // box coordinates are declared read-write operands so the box tests cannot be scheduled above it
      asm volatile("s_load_dword %0, %4, %5\n\ts_load_dword %1, %4, %6"
                   : "=&s"(pf0), "=&s"(pf1), "+s"(nd.c0lx), "+s"(nd.c1lx)
                   : "s"(P.nodes), "s"(nd.pad0), "s"(nd.pad1)
                   : "memory");
#endif
#else
      const Node64 nd = sload_node(P.nodes, node);  // one scalar 64-B fetch per wave
#endif
      // RT_EARLY_PUSH (octant loops): when both children are needed the far one is fixed by the node's
      // order bit for this octant alone, so it is chosen and pushed the moment the node has arrived --
      // the LDS write completes under the box tests instead of delaying the next node fetch (the loop
      // head's s_waitcnt lgkmcnt(0) drains it), and the post-mask decision chain is 9 SALU, not 12
      uint32_t nearb = 0, farb = 0;
      if (RT_EARLY_PUSH && RT_ORDER_BITS && OCT >= 0) {
        sp = (int)uniform((uint32_t)sp);
        asm("s_bitcmp1_b32 %[bits], %[oct]\n\t"
            "s_cselect_b32 %[nb], %[c1], %[c0]\n\t"
            "s_cselect_b32 %[fb], %[c0], %[c1]"
            : [nb] "=&s"(nearb), [fb] "=&s"(farb)
            : [bits] "s"(uniform(order_word<OCT>(nd))), [oct] "i"(order_bit<OCT>()), [c0] "s"(uniform(nd.child0)),
              [c1] "s"(uniform(nd.child1))
            : "scc");
        if (VST) asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(vstk) : "s"(farb), "s"(sp));
        else if (RT_STACK_ASM) lds_push_at(lds_stack, (uint32_t)sp, farb);
        else lds_push(lds_stack + sp, farb);
      }
      if ((RT_PF_MODE == 4 || RT_PF_MODE == 5) && RT_EARLY_PUSH && RT_ORDER_BITS && OCT >= 0) {
        // 4: the far child's line into L2 by one vector load (its own counter: no scalar wait is tied to
        // it; the pop reads it from L2), the near child by a scalar prefetch as in 3; 5: both by vector loads
        const uint32_t o0 = uniform(nd.pad0), o1 = uniform(nd.pad1);
        uint32_t fa, na;
        asm("s_bitcmp1_b32 %[bits], %[oct]\n\t"
            "s_cselect_b32 %[fa], %[p0], %[p1]\n\t"
            "s_cselect_b32 %[na], %[p1], %[p0]"
            : [fa] "=&s"(fa), [na] "=&s"(na)
            : [bits] "s"(uniform(order_word<OCT>(nd))), [oct] "i"(order_bit<OCT>()), [p0] "s"(o0), [p1] "s"(o1)
            : "scc");
        const uint64_t bb = (uint64_t)P.nodes;
        const uint64_t bs = ((uint64_t)uniform((uint32_t)(bb >> 32)) << 32) | (uint32_t)uniform((uint32_t)bb);
        asm volatile("global_load_dword %0, %1, %2" : "+&v"(vsink0) : "v"(fa & ~3u), "s"(bs) : "memory");
        if (RT_PF_MODE == 5)
          asm volatile("global_load_dword %0, %1, %2" : "+&v"(vsink1) : "v"(na & ~3u), "s"(bs) : "memory");
        else
          asm volatile("s_load_dword %0, %1, %2" : "+&s"(fsink) : "s"(bs), "s"(na) : "memory");
      }
      if (RT_PF_MODE == 3 && RT_EARLY_PUSH && RT_ORDER_BITS && OCT >= 0) {
        // the near child (the next node whenever it is needed) into the scalar cache, now: the next
        // step's wait then covers this one line, not the far child's too
        const uint64_t bb = (uint64_t)P.nodes;
        const uint64_t bs = ((uint64_t)uniform((uint32_t)(bb >> 32)) << 32) | (uint32_t)uniform((uint32_t)bb);
        uint32_t a;
        asm volatile("s_bitcmp1_b32 %[bits], %[oct]\n\t"
                     "s_cselect_b32 %[a], %[p1], %[p0]\n\t"
                     "s_load_dword %[sink], %[base], %[a]"
                     : [sink] "+&s"(fsink), [a] "=&s"(a)
                     : [bits] "s"(uniform(order_word<OCT>(nd))), [oct] "i"(order_bit<OCT>()), [p0] "s"(uniform(nd.pad0)),
                       [p1] "s"(uniform(nd.pad1)), [base] "s"(bs)
                     : "scc", "memory");
      }
      uint32_t pf_far = 0;
      if (RT_PF_MODE == 1 && RT_EARLY_PUSH && RT_ORDER_BITS && OCT >= 0) {
        asm("s_bitcmp1_b32 %[bits], %[oct]\n\t"
            "s_cselect_b32 %[pf], %[p0], %[p1]"
            : [pf] "=&s"(pf_far)
            : [bits] "s"(uniform(order_word<OCT>(nd))), [oct] "i"(order_bit<OCT>()), [p0] "s"(uniform(nd.pad0)),
              [p1] "s"(uniform(nd.pad1))
            : "scc");
      }
      const float tcut = ANY ? tlim : h.t;
#if RT_PREFETCH && RT_PF_CARRY && RT_PF_INREG && RT_PF_MODE == 0
      Ray rb = r;
      rb.id = rid;
#else
      const Ray& rb = r;
#endif
      const Span s0 = slab_o<OCT, CLIP>(nd.c0lx, nd.c0hx, nd.c0ly, nd.c0hy, nd.c0lz, nd.c0hz, rb, tcut);
      const Span s1 = slab_o<OCT, CLIP>(nd.c1lx, nd.c1hx, nd.c1ly, nd.c1hy, nd.c1lz, nd.c1hz, rb, tcut);
      const uint64_t m0 = mask_le(s0.tmin, s0.tmax), m1 = mask_le(s1.tmin, s1.tmax);
      uint32_t nxt, far, ta, tb;
      uint64_t tt;
      // the far child is written above the top unconditionally and kept only when both are needed
      // (the store takes the stack depth before the decision block updates it)
      // (uniform(): inside FULL mode's divergent regions the compiler may otherwise hand the scalar
      // decision block values it keeps in VGPRs; readfirstlane folds away on SGPR values)
      sp = (int)uniform((uint32_t)sp);
      const uint32_t c0 = uniform(nd.child0), c1 = uniform(nd.child1);
#if defined(RT_EXP_NODE_VALU)  // timing experiment only: N extra VALU per node step
      { uint32_t xv = c0; asm volatile(".rept " RT_STR(RT_EXP_NODE_VALU) "\n\tv_add_u32 %0, %0, 1\n\t.endr" : "+v"(xv)); }
#endif
#if defined(RT_EXP_NODE_SALU)  // timing experiment only: N extra SALU per node step
      { uint32_t xs = c0; asm volatile(".rept " RT_STR(RT_EXP_NODE_SALU) "\n\ts_add_u32 %0, %0, 1\n\t.endr" : "+s"(xs) :: "scc"); }
#endif
#if RT_VADDR_PUSH
      // the push address scaled in a VALU op (the scalar unit is the loop's tighter resource)
      uint32_t vsp = (uint32_t)sp;
      asm("" : "+v"(vsp));  // the depth as a VGPR operand: the shift below becomes a VALU op
      uint32_t* const slot = lds_stack + vsp;
#else
      uint32_t* const slot = lds_stack + sp;
#endif
      if (RT_EARLY_PUSH && RT_ORDER_BITS && OCT >= 0) {
        // both needed: the near child chosen above; one needed: that one; none: the pop marker
#if RT_DECIDE8
        // 8 SALU: any1 picks (c1 | pop) and (near | c0), any0 then chooses between them; both -> push
        asm("s_cmp_lg_u64 %[m1], 0\n\t"
            "s_cselect_b32 %[nxt], %[c1], -1\n\t"
            "s_cselect_b32 %[ta], %[nb], %[c0]\n\t"
            "s_cselect_b64 %[tt], %[m0], 0\n\t"
            "s_cmp_lg_u64 %[m0], 0\n\t"
            "s_cselect_b32 %[nxt], %[ta], %[nxt]\n\t"
            "s_cmp_lg_u64 %[tt], 0\n\t"
            "s_addc_u32 %[sp], %[sp], 0"
            : [nxt] "=&s"(nxt), [sp] "+s"(sp), [tt] "=&s"(tt), [ta] "=&s"(ta)
            : [m0] "s"(m0), [m1] "s"(m1), [c0] "s"(c0), [c1] "s"(c1), [nb] "s"(nearb)
            : "scc");
#else
        asm("s_cmp_lg_u64 %[m1], 0\n\t"
            "s_cselect_b32 %[nxt], %[nb], %[c0]\n\t"
            "s_cmp_eq_u64 %[m0], 0\n\t"
            "s_cselect_b32 %[nxt], %[c1], %[nxt]\n\t"
            "s_cselect_b64 %[tt], 0, %[m1]\n\t"
            "s_cmp_lg_u64 %[tt], 0\n\t"
            "s_addc_u32 %[sp], %[sp], 0\n\t"
            "s_or_b64 %[tt], %[m0], %[m1]\n\t"
            "s_cselect_b32 %[nxt], %[nxt], -1"
            : [nxt] "=&s"(nxt), [sp] "+s"(sp), [tt] "=&s"(tt)
            : [m0] "s"(m0), [m1] "s"(m1), [c0] "s"(c0), [c1] "s"(c1), [nb] "s"(nearb)
            : "scc");
#endif
        far = farb;
        (void)ta;
        (void)tb;
        if (RT_PF_MODE == 1) {
          // the pushed far child's record into the scalar cache for its pop (the current node's own line,
          // a hit, when nothing was pushed)
          const uint64_t bb = (uint64_t)P.nodes;
          const uint64_t bs = ((uint64_t)uniform((uint32_t)(bb >> 32)) << 32) | (uint32_t)uniform((uint32_t)bb);
          uint32_t a;
          asm volatile("s_cmp_lg_u32 %[sp], %[sp0]\n\t"
                       "s_cselect_b32 %[a], %[pf], %[cur]\n\t"
                       "s_load_dword %[sink], %[base], %[a]"
                       : [sink] "+&s"(fsink), [a] "=&s"(a)
                       : [sp] "s"(sp), [sp0] "s"((uint32_t)sp_before), [pf] "s"(pf_far), [cur] "s"(cur_off), [base] "s"(bs)
                       : "scc", "memory");
        }
      } else if (RT_ORDER_BITS && OCT >= 0) {
        // near child from the node's order bit for this octant (Node64::pad0), overridden when only
        // one child is needed
        asm("s_cmp_lg_u64 %[m1], 0\n\t"
            "s_cselect_b32 %[ta], %[bits], 0\n\t"
            "s_bitcmp1_b32 %[ta], %[oct]\n\t"
            "s_cselect_b32 %[nxt], %[c1], %[c0]\n\t"
            "s_cselect_b32 %[far], %[c0], %[c1]\n\t"
            "s_cmp_eq_u64 %[m0], 0\n\t"
            "s_cselect_b32 %[nxt], %[c1], %[nxt]\n\t"
            "s_cselect_b64 %[tt], 0, %[m1]\n\t"
            "s_cmp_lg_u64 %[tt], 0\n\t"
            "s_addc_u32 %[sp], %[sp], 0\n\t"
            "s_or_b64 %[tt], %[m0], %[m1]\n\t"
            "s_cselect_b32 %[nxt], %[nxt], -1"
            : [nxt] "=&s"(nxt), [far] "=&s"(far), [sp] "+s"(sp), [ta] "=&s"(ta), [tt] "=&s"(tt)
            : [m0] "s"(m0), [m1] "s"(m1), [c0] "s"(c0), [c1] "s"(c1), [bits] "s"(uniform(order_word<OCT>(nd))),
              [oct] "i"(order_bit<OCT>())
            : "scc");
        (void)tb;
        *slot = far;
      } else {
        // near child by lane majority: each lane that needs a child votes for the one it enters first
        // (v0: lanes voting child 0; 2 * |v0| >= |m0 | m1| picks child 0, which also covers m1 == 0)
        const uint64_t le = mask_le(s0.tmin, s1.tmin);
        asm("s_orn2_b64 %[tt], %[le], %[m1]\n\t"
            "s_and_b64 %[tt], %[tt], %[m0]\n\t"
            "s_bcnt1_i32_b64 %[ta], %[tt]\n\t"
            "s_or_b64 %[tt], %[m0], %[m1]\n\t"
            "s_bcnt1_i32_b64 %[tb], %[tt]\n\t"
            "s_lshl_b32 %[ta], %[ta], 1\n\t"
            "s_cmp_ge_u32 %[ta], %[tb]\n\t"
            "s_cselect_b32 %[nxt], %[c0], %[c1]\n\t"
            "s_cselect_b32 %[far], %[c1], %[c0]\n\t"
            "s_cmp_lg_u64 %[m0], 0\n\t"
            "s_cselect_b64 %[tt], %[m1], 0\n\t"
            "s_cmp_lg_u64 %[tt], 0\n\t"
            "s_addc_u32 %[sp], %[sp], 0\n\t"
            "s_cmp_eq_u32 %[tb], 0\n\t"
            "s_cselect_b32 %[nxt], -1, %[nxt]"
            : [nxt] "=&s"(nxt), [far] "=&s"(far), [sp] "+s"(sp), [ta] "=&s"(ta), [tb] "=&s"(tb),
              [tt] "=&s"(tt)
            : [m0] "s"(m0), [m1] "s"(m1), [le] "s"(le), [c0] "s"(c0), [c1] "s"(c1)
            : "scc");
        *slot = far;
      }
      if (RT_TOS) tos = sp != sp_before ? far : tos;
      node = nxt;
#if RT_PREFETCH && !RT_PF_CARRY
      // the prefetch registers stay allocated until their data has landed (the hardware writes them
      // whenever the load returns); the next record load then hits the scalar cache
      asm volatile("s_waitcnt lgkmcnt(0)" ::"s"(pf0), "s"(pf1) : "memory");
#endif
    }
    if (node != kPopMarker) {
      // leaf: its triangles are fetched once per wave and tested by every lane
      const uint32_t first = leaf_first(node), count = leaf_count(node);
#if RT_PREFETCH >= 2
      // triangles 1..3 of the leaf requested together with triangle 0 (the parent prefetched
      // triangle 0), so the per-triangle fetches of the loop below hit the scalar cache
      uint32_t q1, q2, q3;
      {
        const uint32_t last = first + count - 1;
        asm volatile("s_load_dword %0, %3, %4\n\ts_load_dword %1, %3, %5\n\ts_load_dword %2, %3, %6"
                     : "=&s"(q1), "=&s"(q2), "=&s"(q3)
                     : "s"(P.tris), "s"(uniform(min(first + 1, last) * 64u)), "s"(uniform(min(first + 2, last) * 64u)),
                       "s"(uniform(min(first + 3, last) * 64u))
                     : "memory");
      }
#endif
#if RT_PREFETCH >= 3
      // the record the pop after this leaf will fetch (the stack top), requested while the
      // triangles are tested (its handle from the LDS stack; a leaf's first triangle for a leaf)
      uint32_t q4;
      {
        const uint32_t top = uniform(lds_stack[sp > 0 ? sp - 1 : 0]);
        uint32_t off = is_leaf(top) ? 64u * ((uint32_t)P.n_nodes + leaf_first(top)) : node_offset(top);
        off = sp > 0 ? off : 0u;
        asm volatile("s_load_dword %0, %1, %2" : "=&s"(q4) : "s"(P.nodes), "s"(uniform(off)) : "memory");
      }
#endif
      for (uint32_t k = 0; k < count; k++) {
        const TriRec64 tr = sload_tri(P.tris, first + k);
        test_tri<ANY>(P, tr, first + k, r, act, h, found);
#if defined(RT_EXP_TRI_TWICE)  // timing experiment only: each triangle tested again (no effect on results)
        TriRec64 t2 = tr;
        asm volatile("" : "+s"(t2.nx), "+s"(t2.ny), "+s"(t2.nz), "+s"(t2.dist));
        test_tri<ANY>(P, t2, first + k, r, act, h, found);
#endif
      }
#if RT_PREFETCH >= 3
      asm volatile("s_waitcnt lgkmcnt(0)" ::"s"(q1), "s"(q2), "s"(q3), "s"(q4) : "memory");
#elif RT_PREFETCH >= 2
      asm volatile("s_waitcnt lgkmcnt(0)" ::"s"(q1), "s"(q2), "s"(q3) : "memory");
#endif
      if (ANY) {
        active = active & !found;
        act = ballot(active);
        if (!act) break;
        tlim = active ? INFINITY : -1.0f;
      }
    }
    if (sp == 0) break;
    sp--;
    if (RT_TOS) {
      // the popped handle is already in a register; the new top is read now and is needed only at
      // the next pop, by when a node or triangle load's wait has retired the read
      node = uniform(tos);
      tos = lds_stack[sp > 0 ? sp - 1 : 0];
    } else {
      node = VST ? (uint32_t)__builtin_amdgcn_readlane(vstk, sp)
                 : RT_STACK_ASM ? lds_pop_at(lds_stack, (uint32_t)sp) : uniform(lds_stack[sp]);
    }
  }
#if RT_PREFETCH && RT_PF_CARRY
  asm volatile("s_waitcnt lgkmcnt(0)" ::"s"(cpf0), "s"(cpf1) : "memory");  // the last prefetches landed
#endif
  asm volatile("s_waitcnt lgkmcnt(0)" ::"s"(fsink) : "memory");
  if (RT_PF_MODE == 4 || RT_PF_MODE == 5) asm volatile("s_waitcnt vmcnt(0)" ::"v"(vsink0), "v"(vsink1) : "memory");
  if (!ANY && !active) h.t = INFINITY;
}

template <bool ANY, int OCT, bool CLIP = true, bool VST = false>
__device__ __forceinline__ void traverse_fast(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                              uint32_t* lds_stack) {
  if (P.n_nodes == 0) return;
  traverse_fast_from<ANY, OCT, CLIP, VST>(P, r, active, h, found, lds_stack, P.root, 0);
}

// ------------------------------------------------------------------------------------------------
// fp32 4-wide packet traversal (Node128, the default PRIMARY tree). A node step fetches the 128-B record
// with two s_load_dwordx16 under one wait, slab-tests the four children per lane (exact fp32 boxes, no
// dequantisation), and -- the children being stored in this octant's near-to-far order -- writes every
// hit child to the wave stack farthest first with a conditional increment, takes the nearest hit child
// as the next node and drops it from the top again: no sort, no lane vote, 14 SALU. Same exact triangle
// tests and (t, rank) argmin as the binary loops, so every result is identical; only the visit order
// differs. Half the dependent node fetches of the binary tree per wave (SBVH soup: 52 vs 100 per wave).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ Node128 sload128(const void* base, uint32_t off) {
  const uint64_t b = (uint64_t)base;
  const uint64_t bs = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t o = __builtin_amdgcn_readfirstlane(off);
  i16v lo, hi;
  asm volatile("s_load_dwordx16 %0, %2, %3\n\ts_load_dwordx16 %1, %2, %3 offset:0x40\n\ts_waitcnt lgkmcnt(0)"
               : "=&s"(lo), "=&s"(hi)
               : "s"(bs), "s"(o)
               : "memory");
  Node128 r;
  __builtin_memcpy(&r, &lo, 64);
  __builtin_memcpy(reinterpret_cast<char*>(&r) + 64, &hi, 64);
  return r;
}

// Reference form with the counting run's statistics (RT_FRAME_STATS): the same visit order as
// traverse_wide_fast. OCT < 0 (mixed-octant packets): the generic slab test, copy 0's child order.
template <bool ANY, bool STATS, int OCT>
__device__ __forceinline__ void traverse_wide(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                              uint32_t* lds_stack, uint64_t* lds_mask, uint32_t* cnt) {
  uint64_t act = ballot(active);
  float tlim = active ? INFINITY : -1.0f;
  if (!ANY && !active) h.t = -1.0f;
  bool want = active;
  int sp = 0;
  uint32_t node = P.wide_base + (uint32_t)(OCT < 0 ? 0 : OCT) * P.wide_copy_bytes;
  for (;;) {
    while (!is_leaf(node)) {
      const Node128 nd = sload128(P.nodes, node);
      if (STATS) {
        if (want) cnt[ST_NODE]++;
        cnt[ST_WWIDE]++;
      }
      const float tcut = ANY ? tlim : h.t;
      uint64_t m[4];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const float* b = nd.box[c];
        const Span s = slab_o<OCT>(b[0], b[1], b[2], b[3], b[4], b[5], r, tcut);
        m[c] = mask_le(s.tmin, s.tmax);
      }
      uint32_t nxt = kPopMarker;
      uint64_t wm = 0;
#pragma unroll
      for (int c = 3; c >= 0; c--) {  // farthest first; the nearest hit ends on top and is taken next
        lds_stack[sp] = nd.child[c];
        if (STATS) lds_mask[sp] = m[c];
        if (m[c] != 0) {
          nxt = nd.child[c];
          wm = m[c];
          sp++;
        }
      }
      sp = (int)uniform((uint32_t)sp);
      if (nxt != kPopMarker) sp--;
      if (STATS) want = (wm >> lane_id()) & 1;
      node = uniform(nxt);
    }
    if (node != kPopMarker) {
      const uint32_t first = leaf_first(node), count = leaf_count(node);
      if (STATS) {
        if (want) cnt[ST_TRI] += count;
        cnt[ST_WTRI] += count;
      }
      for (uint32_t k = 0; k < count; k++) {
        const TriRec64 tr = sload_tri(P.tris, first + k);
        test_tri<ANY>(P, tr, first + k, r, act, h, found);
      }
      if (ANY) {
        active = active & !found;
        act = ballot(active);
        if (!act) break;
        tlim = active ? INFINITY : -1.0f;
      }
    }
    if (sp == 0) break;
    sp--;
    node = uniform(lds_stack[sp]);
    if (STATS) {
      want = (lds_mask[sp] >> lane_id()) & 1;
      cnt[ST_WPOP]++;
    }
  }
  if (!ANY && !active) h.t = INFINITY;
}

// RT_WIDE_PF: scalar-cache prefetch per wide node step (default 4, measured best: profiles/ab/r03_wide_tree_ab.txt) -- 2: both 64-B halves of every child's record
// (8 one-dword loads), 1: the first half of every child's, 3: both halves of the two nearest children,
// 4: both halves of the nearest child, 0: none
#ifndef RT_WIDE_PF
#define RT_WIDE_PF 4
#endif
// The production form (octant loops, no counting): node fetch + child prefetches, the four slab tests,
// and the decision as one SALU block interleaved with the four stack writes.
template <bool ANY, int OCT>
__device__ __forceinline__ void traverse_wide_fast(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                                   uint32_t* lds_stack) {
  uint64_t act = ballot(active);
  float tlim = active ? INFINITY : -1.0f;
  if (!ANY && !active) h.t = -1.0f;
  int sp = 0;
  const uint32_t vbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)lds_stack;
  const uint64_t bb = (uint64_t)P.nodes;
  const uint64_t bs = ((uint64_t)uniform((uint32_t)(bb >> 32)) << 32) | (uint32_t)uniform((uint32_t)bb);
  uint32_t sink = 0;  // the prefetches' destination (values unused): retired by the next node load's wait
  // RT_WIDE_PF 5 / 6: vector prefetches into L2 (their own counter, vmcnt: no scalar wait is tied to
  // them; retired once at the end). Lane l loads half l & 1 of child `first + min(l >> 1, 3 - first)`.
  uint32_t vsink = 0;
  const int vlane = (int)(threadIdx.x & 63);
  const int vfirst = RT_WIDE_PF == 5 ? 1 : 0;
  const int vsel = min(vfirst + (vlane >> 1), 3);
  const uint32_t vhalf = (uint32_t)(vlane & 1) * 64u;
  uint32_t node = uniform(P.wide_base + (uint32_t)OCT * P.wide_copy_bytes);
  Ray rr = r;
  // the node loop is rotated: the record load that follows a descent sits at the end of the loop body
  // and a separate copy serves the entry after a pop, so a wait the compiler needs after the leaf path
  // (its kernel-argument reloads) stays on that path instead of heading every node step
  auto load = [&](uint32_t off, i16v& lo, i16v& hi) {
    asm volatile("s_load_dwordx16 %0, %3, %4\n\ts_load_dwordx16 %1, %3, %4 offset:0x40\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(lo), "=&s"(hi), "+&s"(sink)
                 : "s"(bs), "s"(off)
                 : "memory");
  };
  for (;;) {
    if (!is_leaf(node)) {
      i16v lo, hi;
      load(node, lo, hi);
      for (;;) {
      Node128 nd;
      __builtin_memcpy(&nd, &lo, 64);
      __builtin_memcpy(reinterpret_cast<char*>(&nd) + 64, &hi, 64);
      // the ray's reciprocal direction passes through the prefetch asm ("+v", carried across steps: no
      // copies), so the slab tests that read it cannot be scheduled above the prefetches: those are issued
      // the moment the node has arrived
      if (RT_WIDE_PF == 2) {
        asm volatile("s_load_dword %[k], %[b], %[p0]\n\ts_load_dword %[k], %[b], %[p0] offset:0x40\n\t"
                     "s_load_dword %[k], %[b], %[p1]\n\ts_load_dword %[k], %[b], %[p1] offset:0x40\n\t"
                     "s_load_dword %[k], %[b], %[p2]\n\ts_load_dword %[k], %[b], %[p2] offset:0x40\n\t"
                     "s_load_dword %[k], %[b], %[p3]\n\ts_load_dword %[k], %[b], %[p3] offset:0x40"
                     : [k] "+&s"(sink), "+v"(rr.id.x), "+v"(rr.id.y), "+v"(rr.id.z)
                     : [b] "s"(bs), [p0] "s"(uniform(nd.pf[0])), [p1] "s"(uniform(nd.pf[1])), [p2] "s"(uniform(nd.pf[2])),
                       [p3] "s"(uniform(nd.pf[3]))
                     : "memory");
      } else if (RT_WIDE_PF == 3) {  // both halves of the two nearest children only
        asm volatile("s_load_dword %[k], %[b], %[p0]\n\ts_load_dword %[k], %[b], %[p0] offset:0x40\n\t"
                     "s_load_dword %[k], %[b], %[p1]\n\ts_load_dword %[k], %[b], %[p1] offset:0x40"
                     : [k] "+&s"(sink), "+v"(rr.id.x), "+v"(rr.id.y), "+v"(rr.id.z)
                     : [b] "s"(bs), [p0] "s"(uniform(nd.pf[0])), [p1] "s"(uniform(nd.pf[1]))
                     : "memory");
      } else if (RT_WIDE_PF == 4) {  // both halves of the nearest child only
        asm volatile("s_load_dword %[k], %[b], %[p0]\n\ts_load_dword %[k], %[b], %[p0] offset:0x40"
                     : [k] "+&s"(sink), "+v"(rr.id.x), "+v"(rr.id.y), "+v"(rr.id.z)
                     : [b] "s"(bs), [p0] "s"(uniform(nd.pf[0]))
                     : "memory");
      } else if (RT_WIDE_PF == 1) {
        asm volatile("s_load_dword %[k], %[b], %[p0]\n\ts_load_dword %[k], %[b], %[p1]\n\t"
                     "s_load_dword %[k], %[b], %[p2]\n\ts_load_dword %[k], %[b], %[p3]"
                     : [k] "+&s"(sink), "+v"(rr.id.x), "+v"(rr.id.y), "+v"(rr.id.z)
                     : [b] "s"(bs), [p0] "s"(uniform(nd.pf[0])), [p1] "s"(uniform(nd.pf[1])), [p2] "s"(uniform(nd.pf[2])),
                       [p3] "s"(uniform(nd.pf[3]))
                     : "memory");
      } else if (RT_WIDE_PF == 5 || RT_WIDE_PF == 6) {
        // 5: the nearest child into the scalar cache (both halves), the other three into L2 by one vector
        // load; 6: all four into L2 by one vector load
        if (RT_WIDE_PF == 5)
          asm volatile("s_load_dword %[k], %[b], %[p0]\n\ts_load_dword %[k], %[b], %[p0] offset:0x40"
                       : [k] "+&s"(sink), "+v"(rr.id.x), "+v"(rr.id.y), "+v"(rr.id.z)
                       : [b] "s"(bs), [p0] "s"(uniform(nd.pf[0]))
                       : "memory");
        const uint32_t p1 = uniform(nd.pf[1]), p2 = uniform(nd.pf[2]), p3 = uniform(nd.pf[3]);
        const uint32_t po = (vsel == 0 ? uniform(nd.pf[0]) : vsel == 1 ? p1 : vsel == 2 ? p2 : p3) + vhalf;
        asm volatile("global_load_dword %[k], %[o], %[b]"
                     : [k] "+&v"(vsink), "+v"(rr.id.x), "+v"(rr.id.y), "+v"(rr.id.z)
                     : [o] "v"(po), [b] "s"(bs)
                     : "memory");
      }
      // the handles into VGPRs for the stack writes (off the masks' critical path)
      uint32_t v0 = nd.child[0], v1 = nd.child[1], v2 = nd.child[2], v3 = nd.child[3];
      asm("" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
      const float tcut = ANY ? tlim : h.t;
      uint64_t m[4];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const float* b = nd.box[c];
        const Span s = slab_o<OCT>(b[0], b[1], b[2], b[3], b[4], b[5], rr, tcut);
        m[c] = mask_le(s.tmin, s.tmax);
      }
      sp = (int)uniform((uint32_t)sp);
      uint32_t nxt, a0, a1, a2, a3;
      asm volatile(
          "v_lshl_add_u32 %[a3], %[sp], 2, %[vb]\n\t"
          "s_cmp_lg_u64 %[m3], 0\n\t"
          "s_cselect_b32 %[nxt], %[h3], -1\n\t"
          "s_addc_u32 %[sp], %[sp], 0\n\t"
          "ds_write_b32 %[a3], %[v3]\n\t"
          "v_lshl_add_u32 %[a2], %[sp], 2, %[vb]\n\t"
          "s_cmp_lg_u64 %[m2], 0\n\t"
          "s_cselect_b32 %[nxt], %[h2], %[nxt]\n\t"
          "s_addc_u32 %[sp], %[sp], 0\n\t"
          "ds_write_b32 %[a2], %[v2]\n\t"
          "v_lshl_add_u32 %[a1], %[sp], 2, %[vb]\n\t"
          "s_cmp_lg_u64 %[m1], 0\n\t"
          "s_cselect_b32 %[nxt], %[h1], %[nxt]\n\t"
          "s_addc_u32 %[sp], %[sp], 0\n\t"
          "ds_write_b32 %[a1], %[v1]\n\t"
          "v_lshl_add_u32 %[a0], %[sp], 2, %[vb]\n\t"
          "s_cmp_lg_u64 %[m0], 0\n\t"
          "s_cselect_b32 %[nxt], %[h0], %[nxt]\n\t"
          "s_addc_u32 %[sp], %[sp], 0\n\t"
          "ds_write_b32 %[a0], %[v0]\n\t"
          "s_cmp_lg_u32 %[nxt], -1\n\t"
          "s_subb_u32 %[sp], %[sp], 0"
          : [nxt] "=&s"(nxt), [sp] "+&s"(sp), [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3)
          : [m0] "s"(m[0]), [m1] "s"(m[1]), [m2] "s"(m[2]), [m3] "s"(m[3]), [h0] "s"(uniform(nd.child[0])),
            [h1] "s"(uniform(nd.child[1])), [h2] "s"(uniform(nd.child[2])), [h3] "s"(uniform(nd.child[3])),
            [v0] "v"(v0), [v1] "v"(v1), [v2] "v"(v2), [v3] "v"(v3), [vb] "v"(vbase)
          : "scc", "memory");
      node = nxt;
      if (is_leaf(node)) break;
      load(node, lo, hi);
      }
    }
    if (node != kPopMarker) {
      const uint32_t first = leaf_first(node), count = leaf_count(node);
      for (uint32_t k = 0; k < count; k++) {
        const TriRec64 tr = sload_tri(P.tris, first + k);
        test_tri<ANY>(P, tr, first + k, r, act, h, found);
      }
      if (ANY) {
        active = active & !found;
        act = ballot(active);
        if (!act) break;
        tlim = active ? INFINITY : -1.0f;
      }
    }
    if (sp == 0) break;
    sp--;
    node = uniform(lds_stack[sp]);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::"s"(sink) : "memory");  // the last prefetches have landed
  if (RT_WIDE_PF == 5 || RT_WIDE_PF == 6) asm volatile("s_waitcnt vmcnt(0)" ::"v"(vsink) : "memory");
  if (!ANY && !active) h.t = INFINITY;
}

// ------------------------------------------------------------------------------------------------
// Dual-chain traversal (PRIMARY, closest hit): one wave walks the BVH for TWO independent 8x8 packets
// at once -- two node handles, two LDS stacks, two rays per lane. Each node step fetches both packets'
// records with one wait and then runs both box tests and decisions, so the two dependent fetch ->
// test -> decide chains overlap inside the wave: the kernel is latency bound (throughput still grows
// with every extra resident wave at 8 per SIMD), and this doubles the chains in flight per wave slot.
// Leaves are tested per packet; once one packet's walk ends the other finishes alone (traverse_fast_from).
// Each packet visits exactly the nodes and triangles of its single-chain walk, in the same order, so
// the hits are identical bit for bit.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kChainDone = 0xFFFFFFFEu;  // leaf-flagged: ends the dual node loop for that chain

__device__ __forceinline__ void sload_node2(const Node64* base, uint32_t ha, uint32_t hb, Node64& a, Node64& b) {
  const uint32_t offa = node_offset(__builtin_amdgcn_readfirstlane(ha));
  const uint32_t offb = node_offset(__builtin_amdgcn_readfirstlane(hb));
  const uint64_t bp = (uint64_t)base;
  const uint64_t bs = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(bp >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)bp);
  i16v va, vb;
  asm volatile("s_load_dwordx16 %0, %2, %3\n\ts_load_dwordx16 %1, %2, %4\n\ts_waitcnt lgkmcnt(0)"
               : "=&s"(va), "=&s"(vb)
               : "s"(bs), "s"(offa), "s"(offb)
               : "memory");
  __builtin_memcpy(&a, &va, 64);
  __builtin_memcpy(&b, &vb, 64);
}

// one octant-loop node step of a chain whose record has arrived: early push of the far child, both
// slab tests, the 9-SALU decision (as traverse_fast); returns the next handle (kPopMarker: pop)
template <int OCT>
__device__ __forceinline__ uint32_t chain_step(const Node64& nd, const Ray& r, float tcut, int& sp, uint32_t* stack) {
  sp = (int)uniform((uint32_t)sp);
  const uint32_t c0 = uniform(nd.child0), c1 = uniform(nd.child1);
  uint32_t nearb, farb, nxt;
  uint64_t tt;
  asm("s_bitcmp1_b32 %[bits], %[oct]\n\t"
      "s_cselect_b32 %[nb], %[c1], %[c0]\n\t"
      "s_cselect_b32 %[fb], %[c0], %[c1]"
      : [nb] "=&s"(nearb), [fb] "=&s"(farb)
      : [bits] "s"(uniform(order_word<OCT>(nd))), [oct] "i"(order_bit<OCT>()), [c0] "s"(c0), [c1] "s"(c1)
      : "scc");
  lds_push(stack + sp, farb);
  const Span s0 = slab_o<OCT>(nd.c0lx, nd.c0hx, nd.c0ly, nd.c0hy, nd.c0lz, nd.c0hz, r, tcut);
  const Span s1 = slab_o<OCT>(nd.c1lx, nd.c1hx, nd.c1ly, nd.c1hy, nd.c1lz, nd.c1hz, r, tcut);
  const uint64_t m0 = mask_le(s0.tmin, s0.tmax), m1 = mask_le(s1.tmin, s1.tmax);
  asm("s_cmp_lg_u64 %[m1], 0\n\t"
      "s_cselect_b32 %[nxt], %[nb], %[c0]\n\t"
      "s_cmp_eq_u64 %[m0], 0\n\t"
      "s_cselect_b32 %[nxt], %[c1], %[nxt]\n\t"
      "s_cselect_b64 %[tt], 0, %[m1]\n\t"
      "s_cmp_lg_u64 %[tt], 0\n\t"
      "s_addc_u32 %[sp], %[sp], 0\n\t"
      "s_or_b64 %[tt], %[m0], %[m1]\n\t"
      "s_cselect_b32 %[nxt], %[nxt], -1"
      : [nxt] "=&s"(nxt), [sp] "+s"(sp), [tt] "=&s"(tt)
      : [m0] "s"(m0), [m1] "s"(m1), [c0] "s"(c0), [c1] "s"(c1), [nb] "s"(nearb)
      : "scc");
  return nxt;
}

// a chain that left the dual node loop at a leaf or the pop marker: its triangles, then its pop
__device__ __forceinline__ void chain_leaf(const DevScene& P, const Ray& r, uint64_t act, Hit& h, uint32_t& node,
                                           int& sp, const uint32_t* stack) {
  if (node == kChainDone || !is_leaf(node)) return;
  bool dummy = false;
  if (node != kPopMarker) {
    const uint32_t first = leaf_first(node), count = leaf_count(node);
    for (uint32_t k = 0; k < count; k++) {
      const TriRec64 tr = sload_tri(P.tris, first + k);
      test_tri<false>(P, tr, first + k, r, act, h, dummy);
    }
  }
  if (sp == 0) {
    node = kChainDone;
  } else {
    sp--;
    node = uniform(stack[sp]);
  }
}

template <int OCT>
__device__ __forceinline__ void traverse_dual(const DevScene& P, const Ray& ra, const Ray& rb, bool acta, bool actb,
                                              Hit& ha, Hit& hb, uint32_t* sta, uint32_t* stb) {
  if (P.n_nodes == 0) return;
  const uint64_t ma = ballot(acta), mb = ballot(actb);
  if (!acta) ha.t = -1.0f;  // lanes without a ray: neutral (no box passes tmin <= -1)
  if (!actb) hb.t = -1.0f;
  uint32_t na = ma ? P.root : kChainDone, nb = mb ? P.root : kChainDone;
  int spa = 0, spb = 0;
  for (;;) {
    while (!is_leaf(na) && !is_leaf(nb)) {
      Node64 a, b;
      sload_node2(P.nodes, na, nb, a, b);
      na = chain_step<OCT>(a, ra, ha.t, spa, sta);
      nb = chain_step<OCT>(b, rb, hb.t, spb, stb);
    }
    chain_leaf(P, ra, ma, ha, na, spa, sta);
    chain_leaf(P, rb, mb, hb, nb, spb, stb);
    if (na == kChainDone || nb == kChainDone) break;
  }
  bool dummy = false;
  if (na != kChainDone) traverse_fast_from<false, OCT>(P, ra, acta, ha, dummy, sta, na, spa);
  else if (nb != kChainDone) traverse_fast_from<false, OCT>(P, rb, actb, hb, dummy, stb, nb, spb);
  if (!acta) ha.t = INFINITY;
  if (!actb) hb.t = INFINITY;
}

// both packets' closest hits: the dual loop when all their rays share one direction octant, else the
// two single-chain walks one after the other (generic loop)
__device__ __forceinline__ void trace_dual(const DevScene& P, const Ray& ra, const Ray& rb, bool acta, bool actb,
                                           Hit& ha, Hit& hb, uint32_t* sta, uint32_t* stb) {
  const uint64_t act = ballot(acta) | ballot(actb);
  const uint64_t sx = (ballot(acta && (__float_as_uint(ra.id.x) >> 31)) | ballot(actb && (__float_as_uint(rb.id.x) >> 31))),
                 sy = (ballot(acta && (__float_as_uint(ra.id.y) >> 31)) | ballot(actb && (__float_as_uint(rb.id.y) >> 31))),
                 sz = (ballot(acta && (__float_as_uint(ra.id.z) >> 31)) | ballot(actb && (__float_as_uint(rb.id.z) >> 31)));
  const uint64_t ax = ballot(acta && !(__float_as_uint(ra.id.x) >> 31)) | ballot(actb && !(__float_as_uint(rb.id.x) >> 31)),
                 ay = ballot(acta && !(__float_as_uint(ra.id.y) >> 31)) | ballot(actb && !(__float_as_uint(rb.id.y) >> 31)),
                 az = ballot(acta && !(__float_as_uint(ra.id.z) >> 31)) | ballot(actb && !(__float_as_uint(rb.id.z) >> 31));
  if (act && (sx == 0 || ax == 0) && (sy == 0 || ay == 0) && (sz == 0 || az == 0)) {
    const int oct = (sx ? 1 : 0) | (sy ? 2 : 0) | (sz ? 4 : 0);
    switch (oct) {
      case 0: traverse_dual<0>(P, ra, rb, acta, actb, ha, hb, sta, stb); return;
      case 1: traverse_dual<1>(P, ra, rb, acta, actb, ha, hb, sta, stb); return;
      case 2: traverse_dual<2>(P, ra, rb, acta, actb, ha, hb, sta, stb); return;
      case 3: traverse_dual<3>(P, ra, rb, acta, actb, ha, hb, sta, stb); return;
      case 4: traverse_dual<4>(P, ra, rb, acta, actb, ha, hb, sta, stb); return;
      case 5: traverse_dual<5>(P, ra, rb, acta, actb, ha, hb, sta, stb); return;
      case 6: traverse_dual<6>(P, ra, rb, acta, actb, ha, hb, sta, stb); return;
      default: traverse_dual<7>(P, ra, rb, acta, actb, ha, hb, sta, stb); return;
    }
  }
  bool dummy = false;
  traverse_fast<false, -1>(P, ra, acta, ha, dummy, sta);
  traverse_fast<false, -1>(P, rb, actb, hb, dummy, stb);
}

// ------------------------------------------------------------------------------------------------
// 4-wide traversal over the quantised nodes (Node4Q). Per node one scalar 64-B fetch; every lane
// slab-tests the four children against the dequantised boxes (origin + q * 2^e, rounded outward on
// the host, so culling stays conservative). The nearest hit child (entry distance seen by the first
// interested lane) is visited next; the other hit children go onto the LDS wave stack, farthest
// deepest.
// ------------------------------------------------------------------------------------------------
// SALU select of child i (0..3) without control flow
__device__ __forceinline__ uint32_t pick4(uint32_t i, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
  uint32_t a, b;
  asm("s_bitcmp1_b32 %2, 0\n\t"
      "s_cselect_b32 %0, %4, %3\n\t"
      "s_cselect_b32 %1, %6, %5\n\t"
      "s_bitcmp1_b32 %2, 1\n\t"
      "s_cselect_b32 %0, %1, %0"
      : "=&s"(a), "=&s"(b)
      : "s"(i), "s"(c0), "s"(c1), "s"(c2), "s"(c3)
      : "scc");
  return a;
}
__device__ __forceinline__ uint32_t rdlane(float v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(v), lane);
}
// all-ones / zero 64-bit lane mask from bit c of a uniform byte
__device__ __forceinline__ uint64_t bitmask64(uint32_t bits, int c) {
  const uint32_t m = (uint32_t)((int32_t)(bits << (31 - c)) >> 31);
  return ((uint64_t)m << 32) | m;
}

template <bool ANY, bool STATS>
__device__ __forceinline__ void traverse4(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                          uint32_t* lds_stack, uint64_t* lds_mask, uint32_t* cnt) {
  if (P.n_nodes == 0) return;
  int sp = 0;
  bool want = active;
  uint32_t node = P.root4;
  uint64_t act = ballot(active);
  // lanes 0..3 stand for children 0..3 when the far children are pushed (lanes >= 3 duplicate 3)
  const int lc = lane_id() < 3 ? lane_id() : 3;
  for (;;) {
    if (!is_leaf(node)) {
      const Node4Q nd = sload64(P.nodes4, node);
      if (STATS) {
        if (want) cnt[ST_NODE]++;
        cnt[ST_WNODE]++;
      }
      const float tcut = ANY ? INFINITY : h.t;
      const float sx = __uint_as_float((uint32_t)nd.ex << 23) * r.id.x;
      const float sy = __uint_as_float((uint32_t)nd.ey << 23) * r.id.y;
      const float sz = __uint_as_float((uint32_t)nd.ez << 23) * r.id.z;
      const float bx = __builtin_fmaf(nd.ox, r.id.x, r.oa.x), bxh = __builtin_fmaf(nd.ox, r.id.x, r.ob.x);
      const float by = __builtin_fmaf(nd.oy, r.id.y, r.oa.y), byh = __builtin_fmaf(nd.oy, r.id.y, r.ob.y);
      const float bz = __builtin_fmaf(nd.oz, r.id.z, r.oa.z), bzh = __builtin_fmaf(nd.oz, r.id.z, r.ob.z);
      uint64_t m[4];
      float tm[4];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const float tx0 = __builtin_fmaf((float)((nd.qlx >> (8 * c)) & 255u), sx, bx);
        const float tx1 = __builtin_fmaf((float)((nd.qhx >> (8 * c)) & 255u), sx, bxh);
        const float ty0 = __builtin_fmaf((float)((nd.qly >> (8 * c)) & 255u), sy, by);
        const float ty1 = __builtin_fmaf((float)((nd.qhy >> (8 * c)) & 255u), sy, byh);
        const float tz0 = __builtin_fmaf((float)((nd.qlz >> (8 * c)) & 255u), sz, bz);
        const float tz1 = __builtin_fmaf((float)((nd.qhz >> (8 * c)) & 255u), sz, bzh);
        const float tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
        const float tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tcut));
        m[c] = mask_le(tmin, tmax) & act & bitmask64(nd.valid, c);
        tm[c] = tmin;
      }
      const uint64_t any = m[0] | m[1] | m[2] | m[3];
      if (any == 0) {
        if (sp == 0) break;
        sp--;
        node = uniform(lds_stack[sp]);
        if (STATS) want = (lds_mask[sp] >> lane_id()) & 1;
        continue;
      }
      // keys: entry distance seen by the first interested lane (tmin >= 0, so its bits order as
      // uint32), child index in the low two bits; children nobody needs sort last
      const int rep = (int)__builtin_ctzll(any);
      uint32_t k[4];
#pragma unroll
      for (int c = 0; c < 4; c++) k[c] = m[c] ? ((rdlane(tm[c], rep) & ~3u) | (uint32_t)c) : 0xFFFFFFFFu;
      const uint32_t kmin = uniform(min(min(k[0], k[1]), min(k[2], k[3])));
      const int nhit = (int)__builtin_popcount(((m[0] != 0) ? 1u : 0u) | ((m[1] != 0) ? 2u : 0u) |
                                               ((m[2] != 0) ? 4u : 0u) | ((m[3] != 0) ? 8u : 0u));
      if (nhit > 1) {
        // lane c (c < 4) writes child c at sp + ((nhit - 1 - rank_c) & 3): the far children land
        // farthest-deepest below the new top, the near child and the unused ones above it
        const uint32_t myk = lc == 0 ? k[0] : (lc == 1 ? k[1] : (lc == 2 ? k[2] : k[3]));
        const int rank = (k[0] < myk) + (k[1] < myk) + (k[2] < myk) + (k[3] < myk);
        const int pos = sp + ((nhit - 1 - rank) & 3);
        lds_stack[pos] = lc == 0 ? nd.child[0] : (lc == 1 ? nd.child[1] : (lc == 2 ? nd.child[2] : nd.child[3]));
        if (STATS) lds_mask[pos] = lc == 0 ? m[0] : (lc == 1 ? m[1] : (lc == 2 ? m[2] : m[3]));
        sp += nhit - 1;
      }
      node = pick4(kmin & 3, nd.child[0], nd.child[1], nd.child[2], nd.child[3]);
      if (STATS) {
        const uint32_t ci = kmin & 3;
        want = (((ci == 0) ? m[0] : (ci == 1) ? m[1] : (ci == 2) ? m[2] : m[3]) >> lane_id()) & 1;
      }
      continue;
    }
    const uint32_t first = leaf_first(node), count = leaf_count(node);
    if (STATS) {
      if (want) cnt[ST_TRI] += count;
      cnt[ST_WTRI] += count;
    }
    for (uint32_t q = 0; q < count; q++) {
      const TriRec64 tr = sload_tri(P.tris, first + q);
      test_tri<ANY>(P, tr, first + q, r, act, h, found);
    }
    if (ANY) {
      active = active & !found;
      act = ballot(active);
      if (!act) break;
    }
    if (sp == 0) break;
    sp--;
    node = uniform(lds_stack[sp]);
    if (STATS) want = (lds_mask[sp] >> lane_id()) & 1;
  }
}

// ------------------------------------------------------------------------------------------------
// Per-lane traversal for incoherent rays (reflection and secondary shadow rays): every lane walks its
// own path with its own stack ("while-while": descend interior nodes until every lane holds a leaf or
// is done, then test leaves). Node and triangle records are per-lane vector loads. The triangle test
// is the same arithmetic as test_tri, per lane, so results are identical.
// ------------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T vload64(const T* base, uint32_t i) {
  static_assert(sizeof(T) == 64, "64-byte records");
  const float4* p = reinterpret_cast<const float4*>(base + i);
  T r;
  float4* q = reinterpret_cast<float4*>(&r);
  q[0] = p[0]; q[1] = p[1]; q[2] = p[2]; q[3] = p[3];
  return r;
}

// the rare accept path of one lane (accept_candidate, per lane)
__device__ __forceinline__ bool accept_lane(const DevScene& P, const TriRec64& tr, uint32_t slot, f3 e0, f3 e2, f3 a0,
                                            f3 a1, f3 a2, f3 p, const Ray& r) {
  if (!(tr.box & kSafeNormalBit)) {
    const float area0 = norm(a0) / 2, area1 = norm(a1) / 2, area2 = norm(a2) / 2;
    const float area = norm(cross(e0, neg(e2))) / 2;
    const float* fs = P.fshade + 12 * (size_t)slot;
    const f3 n0 = ld3(fs), n1 = ld3(fs + 4), n2 = ld3(fs + 8);
    const f3 nn = blend_normal(n0, n1, n2, area0, area1, area2, area);
    if (!(norm(nn) != 0)) return false;
  }
  if (RT_BOX_CERT && (tr.box & kBoxCertBit) &&
      fmaxf(fmaxf(fabsf(r.o2.x), fabsf(r.o2.y)), fabsf(r.o2.z)) <= P.cert_origin_max)
    return true;
  const float* bx = P.refbox + 8 * (size_t)(tr.box & kBoxIndexMask);
  const f3 X = affv3(P.Minv, p);
  const float lo[3] = {bx[0], bx[1], bx[2]}, hi[3] = {bx[4], bx[5], bx[6]};
  const float xs[3] = {X.x, X.y, X.z}, os[3] = {r.o2.x, r.o2.y, r.o2.z};
  bool inside = true;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float m = 1e-5f * ((hi[k] - lo[k]) + fabsf(lo[k]) + fabsf(hi[k]) + fabsf(os[k])) + 1e-30f;
    inside = inside & (xs[k] > lo[k] + m) & (xs[k] < hi[k] - m);
  }
  return inside || ref_box_test(r, bx);
}

// calculateDistance (flyscene.cpp:444-478) of one lane against its own triangle record
template <bool ANY>
__device__ __forceinline__ void test_tri_lane(const DevScene& P, const TriRec64& tr, uint32_t slot, const Ray& r,
                                              Hit& h, bool& found) {
  const f3 n{tr.nx, tr.ny, tr.nz};
  const float dn = dot(n, r.d);
  const float orth = tr.dist - dot(r.o, n);
  const float t = orth / dn;
  bool cand = (dn != 0.0f) & (t >= 0.0f);
  if (!ANY) cand = cand & (t < INFINITY) & ((t < h.t) | ((t == h.t) & (tr.rank < h.rank)));
  if (!cand) return;
  const f3 p{r.o.x + t * r.d.x, r.o.y + t * r.d.y, r.o.z + t * r.d.z};
  const f3 w0{tr.w0x, tr.w0y, tr.w0z}, w1{tr.w1x, tr.w1y, tr.w1z}, w2{tr.w2x, tr.w2y, tr.w2z};
  const f3 e0 = sub(w1, w0), e1 = sub(w2, w1), e2 = sub(w0, w2);
  const f3 a0 = cross(e0, sub(p, w0)), a1 = cross(e1, sub(p, w1)), a2 = cross(e2, sub(p, w2));
  if ((int)(dot(n, a0) < 0) | (int)(dot(n, a1) < 0) | (int)(dot(n, a2) < 0)) return;
  if (!accept_lane(P, tr, slot, e0, e2, a0, a1, a2, p, r)) return;
  if (ANY) {
    found = true;
  } else {
    h.t = t;
    h.rank = tr.rank;
    h.slot = slot;
  }
}

constexpr int kLaneStack = kMaxDepth + 4;

template <bool ANY, bool STATS>
__device__ __forceinline__ void traverse_lane(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                              uint32_t* cnt) {
  if (P.n_nodes == 0) return;
  uint32_t stack[kLaneStack];  // per-lane stack (private memory)
  int sp = 0;
  uint32_t node = P.root;
  bool done = !active;
  for (;;) {
    // descend interior nodes until this lane holds a leaf or has nothing left
    while (!done && !is_leaf(node)) {
      const Node64 nd = vload64(P.nodes, node_index(node));
      if (STATS) cnt[ST_NODE]++;
      const float tcut = ANY ? INFINITY : h.t;
      const Span s0 = slab(nd.c0lx, nd.c0hx, nd.c0ly, nd.c0hy, nd.c0lz, nd.c0hz, r, tcut);
      const Span s1 = slab(nd.c1lx, nd.c1hx, nd.c1ly, nd.c1hy, nd.c1lz, nd.c1hz, r, tcut);
      const bool h0 = s0.tmin <= s0.tmax, h1 = s1.tmin <= s1.tmax;
      if (h0 && h1) {
        const bool first0 = s0.tmin <= s1.tmin;
        stack[sp++] = first0 ? nd.child1 : nd.child0;
        node = first0 ? nd.child0 : nd.child1;
      } else if (h0 | h1) {
        node = h0 ? nd.child0 : nd.child1;
      } else if (sp > 0) {
        node = stack[--sp];
      } else {
        done = true;
      }
    }
    if (!done) {
      const uint32_t first = leaf_first(node), count = leaf_count(node);
      if (STATS) cnt[ST_TRI] += count;
      for (uint32_t k = 0; k < count; k++) {
        const TriRec64 tr = vload64(P.tris, first + k);
        test_tri_lane<ANY>(P, tr, first + k, r, h, found);
        if (ANY && found) break;
      }
      if (ANY && found) done = true;
      else if (sp > 0) node = stack[--sp];
      else done = true;
    }
    if (ballot(!done) == 0) break;
  }
}

// Traversal flavours (A/B knob RT_KERNEL_VARIANT): binary nodes with the VGPR or the LDS stack, or
// the 4-wide quantised nodes
enum { TRAV_B2_VGPR = 0, TRAV_B2_LDS = 1, TRAV_W4 = 2, TRAV_LANE = 3 };

template <int TRAV, bool STATS>
struct WaveLds {
  // binary LDS-stack kernels also run the fp32 4-wide loops (traverse_wide*): kStackW entries
  static constexpr int kEntries = TRAV == TRAV_W4 ? kStack4 : (TRAV == TRAV_LANE ? 1 : (TRAV == TRAV_B2_LDS ? kStackW : 64));
  uint32_t stack[4][kEntries];
  uint64_t mask[4][(STATS && (TRAV == TRAV_W4 || TRAV == TRAV_B2_LDS)) ? kEntries : 1];
  uint32_t clk[4];  // one-wave kernels: the wave's start clocks (wave_clock_start), kept out of registers
};

template <bool ANY, bool STATS, int TRAV>
__device__ __forceinline__ void trace(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                      WaveLds<TRAV, STATS>& L, int wv, uint32_t* cnt) {
  if (TRAV == TRAV_W4) traverse4<ANY, STATS>(P, r, active, h, found, L.stack[wv], L.mask[STATS ? wv : 0], cnt);
  else if (TRAV == TRAV_LANE) traverse_lane<ANY, STATS>(P, r, active, h, found, cnt);
  else if (RT_FAST_LOOP && !STATS && TRAV == TRAV_B2_LDS) traverse_fast<ANY, -1>(P, r, active, h, found, L.stack[wv]);
  else traverse<ANY, STATS, TRAV == TRAV_B2_LDS>(P, r, active, h, found, L.stack[wv], cnt);
}

// Closest-hit packet traversal specialised by the wave's direction octant when every active ray shares
// it (coherent camera / reflection packets); mixed-octant waves take the generic loop.
#ifndef RT_OCT_SPECIALIZE
#define RT_OCT_SPECIALIZE 1
#endif
// WIDE: packets whose rays share an octant walk the fp32 4-wide tree when the scene has one
// (traverse_wide_fast; the counting run traverse_wide); mixed-octant packets keep the binary loop.
// SPLIT (FULL mode's secondary packets, RT_FULL_SPLIT_OCT): a packet whose rays span several direction
// octants is walked once per octant present, each walk with that octant's lanes only (ballot masks) and
// the octant loop's cheaper slab test, instead of one generic walk of the union; a one-octant packet is
// the loop's single iteration. Each lane is traced by exactly one walk, so results are unchanged.
// Whether every active ray of the wave enters the root's box at t >= 0 or misses it (its origin is not
// inside the scene's bounds and the scene is not behind it): then the octant loops may skip the entry
// distance's clip at 0 (slab_o CLIP), two VALU per node step. Uniform.
#ifndef RT_NOCLIP
#define RT_NOCLIP 0
#endif
template <int OCT>
__device__ __forceinline__ bool packet_in_front(const DevScene& P, const Ray& r, bool active) {
  if (is_leaf(P.root)) return false;
  const Node64 rn = sload_node(P.nodes, P.root);
  const float lx = fminf(rn.c0lx, rn.c1lx), ly = fminf(rn.c0ly, rn.c1ly), lz = fminf(rn.c0lz, rn.c1lz);
  const float hx = fmaxf(rn.c0hx, rn.c1hx), hy = fmaxf(rn.c0hy, rn.c1hy), hz = fmaxf(rn.c0hz, rn.c1hz);
  const Span s = slab_o<OCT, false>(lx, hx, ly, hy, lz, hz, r, INFINITY);
  return ballot(active && !(s.tmin >= 0.0f || s.tmin > s.tmax)) == 0;
}
template <bool ANY, bool STATS, int TRAV, bool LANE_MIXED = false, bool WIDE = false, bool SPLIT = false,
          bool NOCLIP = false>
__device__ __forceinline__ void trace_oct(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                          WaveLds<TRAV, STATS>& L, int wv, uint32_t* cnt) {
  if (SPLIT && RT_OCT_SPECIALIZE && RT_FAST_LOOP && !STATS && TRAV == TRAV_B2_LDS) {
    const uint32_t loct = (__float_as_uint(r.id.x) >> 31) | ((__float_as_uint(r.id.y) >> 31) << 1) |
                          ((__float_as_uint(r.id.z) >> 31) << 2);
    uint64_t rem = ballot(active);
    Hit hres = h;
    bool fres = found;
    while (rem != 0) {
      const uint32_t oct = uniform((uint32_t)__builtin_amdgcn_readlane((int)loct, (int)__builtin_ctzll(rem)));
      const uint64_t sub = ballot(loct == oct) & rem;
      rem &= ~sub;
      const bool a = lane_in(sub);
      Hit hs = h;
      bool fs = false;
      switch (oct) {
        case 0: traverse_fast<ANY, 0>(P, r, a, hs, fs, L.stack[wv]); break;
        case 1: traverse_fast<ANY, 1>(P, r, a, hs, fs, L.stack[wv]); break;
        case 2: traverse_fast<ANY, 2>(P, r, a, hs, fs, L.stack[wv]); break;
        case 3: traverse_fast<ANY, 3>(P, r, a, hs, fs, L.stack[wv]); break;
        case 4: traverse_fast<ANY, 4>(P, r, a, hs, fs, L.stack[wv]); break;
        case 5: traverse_fast<ANY, 5>(P, r, a, hs, fs, L.stack[wv]); break;
        case 6: traverse_fast<ANY, 6>(P, r, a, hs, fs, L.stack[wv]); break;
        default: traverse_fast<ANY, 7>(P, r, a, hs, fs, L.stack[wv]); break;
      }
      hres.t = a ? hs.t : hres.t;
      hres.rank = a ? hs.rank : hres.rank;
      hres.slot = a ? hs.slot : hres.slot;
      fres = fres | (a & fs);
    }
    h = hres;
    found = fres;
    return;
  }
  if (RT_OCT_SPECIALIZE && (TRAV == TRAV_B2_LDS || TRAV == TRAV_B2_VGPR)) {
    constexpr bool SL = TRAV == TRAV_B2_LDS;
    const uint64_t act = ballot(active);
    const uint64_t sx = ballot(__float_as_uint(r.id.x) >> 31) & act, sy = ballot(__float_as_uint(r.id.y) >> 31) & act,
                   sz = ballot(__float_as_uint(r.id.z) >> 31) & act;
    if ((sx == 0 || sx == act) && (sy == 0 || sy == act) && (sz == 0 || sz == act)) {
      const int oct = (sx ? 1 : 0) | (sy ? 2 : 0) | (sz ? 4 : 0);
      if (WIDE && SL && P.wide_copy_bytes != 0) {
        uint32_t* st = L.stack[wv];
        uint64_t* mk = L.mask[STATS ? wv : 0];
#define RT_WIDE_CASE(o)                                                              \
  case o:                                                                           \
    if (STATS) traverse_wide<ANY, STATS, o>(P, r, active, h, found, st, mk, cnt);   \
    else traverse_wide_fast<ANY, o>(P, r, active, h, found, st);                    \
    return;
        switch (oct) {
          RT_WIDE_CASE(0) RT_WIDE_CASE(1) RT_WIDE_CASE(2) RT_WIDE_CASE(3)
          RT_WIDE_CASE(4) RT_WIDE_CASE(5) RT_WIDE_CASE(6) default: RT_WIDE_CASE(7)
        }
#undef RT_WIDE_CASE
      }
      if (NOCLIP && RT_NOCLIP && RT_FAST_LOOP && !STATS && SL) {
#define RT_NOCLIP_CASE(o)                                                                      \
  case o:                                                                                     \
    if (packet_in_front<o>(P, r, active)) traverse_fast<ANY, o, false, RT_VSTACK>(P, r, active, h, found, L.stack[wv]); \
    else traverse_fast<ANY, o, true, RT_VSTACK>(P, r, active, h, found, L.stack[wv]);                  \
    return;
        switch (oct) {
          RT_NOCLIP_CASE(0) RT_NOCLIP_CASE(1) RT_NOCLIP_CASE(2) RT_NOCLIP_CASE(3)
          RT_NOCLIP_CASE(4) RT_NOCLIP_CASE(5) RT_NOCLIP_CASE(6) default: RT_NOCLIP_CASE(7)
        }
#undef RT_NOCLIP_CASE
      }
      if (RT_FAST_LOOP && !STATS && SL) {
        switch (oct) {
          case 0: traverse_fast<ANY, 0>(P, r, active, h, found, L.stack[wv]); return;
          case 1: traverse_fast<ANY, 1>(P, r, active, h, found, L.stack[wv]); return;
          case 2: traverse_fast<ANY, 2>(P, r, active, h, found, L.stack[wv]); return;
          case 3: traverse_fast<ANY, 3>(P, r, active, h, found, L.stack[wv]); return;
          case 4: traverse_fast<ANY, 4>(P, r, active, h, found, L.stack[wv]); return;
          case 5: traverse_fast<ANY, 5>(P, r, active, h, found, L.stack[wv]); return;
          case 6: traverse_fast<ANY, 6>(P, r, active, h, found, L.stack[wv]); return;
          default: traverse_fast<ANY, 7>(P, r, active, h, found, L.stack[wv]); return;
        }
      }
      switch (oct) {
        case 0: traverse<ANY, STATS, SL, 0>(P, r, active, h, found, L.stack[wv], cnt); return;
        case 1: traverse<ANY, STATS, SL, 1>(P, r, active, h, found, L.stack[wv], cnt); return;
        case 2: traverse<ANY, STATS, SL, 2>(P, r, active, h, found, L.stack[wv], cnt); return;
        case 3: traverse<ANY, STATS, SL, 3>(P, r, active, h, found, L.stack[wv], cnt); return;
        case 4: traverse<ANY, STATS, SL, 4>(P, r, active, h, found, L.stack[wv], cnt); return;
        case 5: traverse<ANY, STATS, SL, 5>(P, r, active, h, found, L.stack[wv], cnt); return;
        case 6: traverse<ANY, STATS, SL, 6>(P, r, active, h, found, L.stack[wv], cnt); return;
        default: traverse<ANY, STATS, SL, 7>(P, r, active, h, found, L.stack[wv], cnt); return;
      }
    }
  }
  // mixed-octant packets of divergent secondary rays: one walk per lane (LANE_MIXED, FULL A/B knob)
  if (LANE_MIXED && !STATS && TRAV == TRAV_B2_LDS) {
    traverse_lane<ANY, false>(P, r, active, h, found, cnt);
    return;
  }
  trace<ANY, STATS, TRAV>(P, r, active, h, found, L, wv, cnt);
}
template <bool STATS, int TRAV, bool WIDE = false, bool NOCLIP = false>
__device__ __forceinline__ void trace_closest_oct(const DevScene& P, const Ray& r, bool active, Hit& h,
                                                  WaveLds<TRAV, STATS>& L, int wv, uint32_t* cnt) {
  bool found = false;
  trace_oct<false, STATS, TRAV, false, WIDE, false, NOCLIP>(P, r, active, h, found, L, wv, cnt);
}

// FULL mode: primary, reflection and shadow packets also take the octant-specialised loops when the
// wave's rays share an octant (A/B knob)
#ifndef RT_FULL_OCT
#define RT_FULL_OCT 0
#endif
#ifndef RT_FULL_OCT_PRIMARY
#define RT_FULL_OCT_PRIMARY 1
#endif
#ifndef RT_FULL_OCT_SHADOW
#define RT_FULL_OCT_SHADOW 1
#endif
#ifndef RT_FULL_OCT_SHADOW2  // the reflection hits' shadow packets through trace_oct too
#define RT_FULL_OCT_SHADOW2 1
#endif
#ifndef RT_FULL_MIXED_LANE  // FULL secondary packets whose rays span octants walk per lane (traverse_lane)
#define RT_FULL_MIXED_LANE 0
#endif
#ifndef RT_FULL_OCT_REFL  // the reflection packet through trace_oct (octant loops when its rays share one)
#define RT_FULL_OCT_REFL 1
#endif
#ifndef RT_FULL_SPLIT_OCT  // FULL secondary packets spanning several octants: one octant walk per octant
#define RT_FULL_SPLIT_OCT 1       // present (small-scene build; trace_full)
#endif
// RT_FULL_LANE_K > 0: a secondary packet with at most K active lanes walks per lane (traverse_lane)
// instead of as a packet (A/B knob)
#ifndef RT_FULL_LANE_K
#define RT_FULL_LANE_K 0
#endif
template <bool ANY, bool STATS, int TRAV>
__device__ __forceinline__ void trace_full_ray(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                               WaveLds<TRAV, STATS>& L, int wv, uint32_t* cnt) {
  if (RT_FULL_LANE_K > 0 && TRAV == TRAV_B2_LDS && __popcll(ballot(active)) <= RT_FULL_LANE_K) {
    traverse_lane<ANY, STATS>(P, r, active, h, found, cnt);
    return;
  }
  if (RT_FULL_OCT) trace_oct<ANY, STATS, TRAV>(P, r, active, h, found, L, wv, cnt);
  else trace<ANY, STATS, TRAV>(P, r, active, h, found, L, wv, cnt);
}

// ------------------------------------------------------------------------------------------------
// Shading
// ------------------------------------------------------------------------------------------------
struct MatState {  // Flyscene members ka/kd/ks/shininess (flyscene.hpp:179-182)
  f3 ka, kd, ks;
  float ns;
};

__device__ __forceinline__ MatState load_mat(const DevMat& m) {
  return MatState{f3{m.ka[0], m.ka[1], m.ka[2]}, f3{m.kd[0], m.kd[1], m.kd[2]}, f3{m.ks[0], m.ks[1], m.ks[2]}, m.ns};
}

// interpolateNormal (flyscene.cpp:572-600) for the hit triangle of this lane: one contiguous 48-B
// gather of the face's shading record (its three unit vertex normals + material)
// the shading record is indexed by the triangle slot (like the record itself), so its gather does not wait
// for the record's face id: both loads of a hit are issued together
__device__ __forceinline__ f3 hit_normal(const DevScene& P, const TriRec64& tr, uint32_t slot, f3 p, int32_t& mat) {
  const f3 n{tr.nx, tr.ny, tr.nz};
  const f3 w0{tr.w0x, tr.w0y, tr.w0z}, w1{tr.w1x, tr.w1y, tr.w1z}, w2{tr.w2x, tr.w2y, tr.w2z};
  const f3 e0 = sub(w1, w0), e1 = sub(w2, w1), e2 = sub(w0, w2);
  const f3 a0 = cross(e0, sub(p, w0)), a1 = cross(e1, sub(p, w1)), a2 = cross(e2, sub(p, w2));
  const float4* fs = reinterpret_cast<const float4*>(P.fshade + 12 * (size_t)slot);
  const float4 n0 = fs[0];
  mat = __float_as_int(n0.w);
  if (dot(n, a0) < 0 || dot(n, a1) < 0 || dot(n, a2) < 0) return f3{0.0f, 0.0f, 0.0f};
  const float area0 = norm(a0) / 2, area1 = norm(a1) / 2, area2 = norm(a2) / 2;
  const float area = norm(cross(e0, neg(e2))) / 2;
  const float4 n1 = fs[1], n2 = fs[2];
  return blend_normal(f3{n0.x, n0.y, n0.z}, f3{n1.x, n1.y, n1.z}, f3{n2.x, n2.y, n2.z}, area0, area1, area2, area);
}

__device__ __forceinline__ TriRec64 vload_tri(const TriRec64* base, uint32_t i) {
  const float4* p = reinterpret_cast<const float4*>(base + i);
  TriRec64 r;
  float4* q = reinterpret_cast<float4*>(&r);
  q[0] = p[0]; q[1] = p[1]; q[2] = p[2]; q[3] = p[3];
  return r;
}


// Light l of the frame, read from the kernel-argument segment. Every kernel takes FrameParams as its
// first argument, so the lights sit at offsetof(FrameParams, lights) of that segment; indexing them
// there (scalar loads, l is wave-uniform) means a light loop never makes the compiler copy the whole
// FrameParams into private memory for a dynamic index -- which it did in the FULL megakernel once the
// kernel grew (1.7 KB of scratch per lane, 3x slower).
__device__ __forceinline__ Light frame_light(int l) {
  typedef const __attribute__((address_space(4))) char* KArg;
  typedef const __attribute__((address_space(4))) Light* KLight;
  const KArg base = (KArg)__builtin_amdgcn_kernarg_segment_ptr();
  const KLight q = (KLight)(base + offsetof(FrameParams, lights) + (size_t)l * sizeof(Light));
  Light r;
  for (int k = 0; k < 3; k++) {
    r.p[k] = q->p[k];
    r.c[k] = q->c[k];
  }
  r.kind = q->kind;
  return r;
}

// calculateColor's light direction (flyscene.cpp:607-611): point light -(P - pos).normalized(), or a
// directional light's stored vector as is
__device__ __forceinline__ f3 light_dir(f3 p, const Light& l) {
  if (l.kind == RT_LIGHT_DIRECTIONAL) return f3{l.p[0], l.p[1], l.p[2]};
  return neg(normalized(sub(p, f3{l.p[0], l.p[1], l.p[2]})));
}

// Hit information of one lane, gathered once and reused by every light of calculateColor
struct HitInfo {
  f3 p, n;
  int32_t mat;
  uint32_t face;
};

// calcSingleColor body after the shadow test (flyscene.cpp:546-565)
__device__ __forceinline__ f3 phong(const FrameParams& P, MatState& st, const HitInfo& hi, f3 o, f3 L, const float* I) {
  if (hi.mat != -1) st = load_mat(P.sc.mats[hi.mat]);
  const f3 R = phong_r(L, hi.n);
  const f3 E = normalized(sub(o, hi.p));
  const float dif = smax(dot(L, hi.n), 0.0f);
  const float spe = smax(pow_ref(dot(R, E), st.ns), 0.0f);
  return f3{(I[0] * st.ka.x + (I[0] * st.kd.x) * dif) + (I[0] * st.ks.x) * spe,
            (I[1] * st.ka.y + (I[1] * st.kd.y) * dif) + (I[1] * st.ks.y) * spe,
            (I[2] * st.ka.z + (I[2] * st.kd.z) * dif) + (I[2] * st.ks.z) * spe};
}

__device__ __forceinline__ float clamp01(float x) { return smax(smin(x, 1.0f), 0.0f); }

// calculateColor (flyscene.cpp:603-614). SHADOWS: per light, a wave-packet any-hit traversal from
// P + 0.003 L (box predicate from P) decides whether the light contributes (calcSingleColor :543).
template <bool SHADOWS, bool STATS, int TRAV, bool OCTSH = false, bool SPLIT = false>
__device__ __forceinline__ f3 calc_color(const FrameParams& P, MatState& st, const HitInfo& hi, f3 o, bool lane_hit,
                                         WaveLds<TRAV, STATS>* lds, int wv, uint32_t* cnt) {
  f3 sum{0.0f, 0.0f, 0.0f};
  for (int l = 0; l < P.n_lights; l++) {
    const Light lt = frame_light(l);
    const f3 L = light_dir(hi.p, lt);
    bool blocked = false;
    if (SHADOWS) {
      Ray sr;
      sr.o = offset(hi.p, L, 0.003f);
      sr.d = L;
      sr.o2 = affv3(P.Minv, hi.p);
      sr.d2 = normalized(m3v3(P.MS, L));
      setup_cull(sr, P.sc.static_pad);
      Hit hh{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
      if (STATS && lane_hit) cnt[ST_TOTAL]++;
      if (OCTSH)
        trace_oct<true, STATS, TRAV, RT_FULL_MIXED_LANE != 0, false, SPLIT>(P.sc, sr, lane_hit, hh, blocked, *lds, wv, cnt);
      else trace_full_ray<true, STATS, TRAV>(P.sc, sr, lane_hit, hh, blocked, *lds, wv, cnt);
    }
    f3 c{0.0f, 0.0f, 0.0f};
    if (lane_hit && !blocked) c = phong(P, st, hi, o, L, lt.c);
    sum = f3{sum.x + c.x, sum.y + c.y, sum.z + c.z};
  }
  return f3{clamp01(sum.x), clamp01(sum.y), clamp01(sum.z)};
}

// ------------------------------------------------------------------------------------------------
// Frame kernels. One block = one 16x16 pixel tile (2x2 waves of 8x8, one ray per lane).
// XCD-aware order: blocks b and b+8 share an XCD under round-robin dispatch, so each XCD gets a
// contiguous run of tiles (L2 reuse; speed only, any placement is correct).
// ------------------------------------------------------------------------------------------------
struct PixelCoord {
  int px, py, wv, lane;
  int slot;   // this wave's LDS slot within its block
  int qw;     // global wave number (tile-block * 4 + wave): the same for every block shape
  int sub;    // FrameParams::split_k: this block's 16-lane part (rows 2 sub, 2 sub + 1) of its wave, else -1
  bool active;
};

#ifndef RT_ORDER_LPT
#define RT_ORDER_LPT 1
#endif
// WPB = waves per block: 4 (one 256-thread block per 16x16 tile) or 1 (one 64-thread block per 8x8
// quarter, blocks 4t..4t+3 cover tile t; finer-grained dispatch, same pixels and shard assignment)
template <int WPB = 4>
__device__ __forceinline__ PixelCoord pixel_coord(const FrameParams& P) {
  PixelCoord c;
  c.lane = threadIdx.x & 63;
  int nb, b;
  int bid = (int)blockIdx.x;
  c.sub = -1;
  if (RT_ORDER_LPT && WPB == 1 && P.order != nullptr) {
    // longest-first order from an earlier frame's wave costs (k_order_lpt): a permutation of the
    // logical waves that keeps each XCD on its own chunked bands; an out-of-range entry (never
    // produced) falls back to the block's own position, so a wave never leaves the grid.
    // split_k > 0: order positions 0 .. split_k - 1 (the costliest waves) are traced by four blocks
    // each, every one with 16 of the wave's lanes, so the frame's slowest packets shrink to 16 rays
    const uint32_t k = (uint32_t)P.split_k, nlog = gridDim.x - 3u * k;
    uint32_t pos = blockIdx.x;
    if (k > 0) {
      if (pos < 4u * k) {
        c.sub = (int)(pos & 3u);
        pos >>= 2;
      } else {
        pos -= 3u * k;
      }
    }
    const uint32_t o = uniform(P.order[pos]);
    bid = o < nlog ? (int)o : (int)pos;
  } else if (P.xcd_remap >= 2) {
    // chunked XCD order: blocks b and b + 8 share an XCD, so the k-th block of XCD x takes position
    // (k / C) * 8C + x C + k % C -- each XCD receives runs of C consecutive blocks (for one-wave
    // blocks, the four quarters of a tile and its row neighbours) while the runs still interleave
    // over the frame (load balance). The trailing partial group keeps the identity order.
    const int C = P.xcd_remap, G = 8 * C, full = ((int)gridDim.x / G) * G;
    if (bid < full) {
      const int x = bid & 7, k = bid >> 3;
      bid = (k / C) * G + x * C + (k % C);
    }
  }
  if (WPB == 4) {
    c.wv = (int)uniform(threadIdx.x >> 6);
    c.slot = c.wv;
    nb = (int)gridDim.x;
    b = bid;
  } else {
    c.wv = bid & 3;
    c.slot = 0;
    nb = (int)((gridDim.x - 3u * (uint32_t)P.split_k) >> 2);
    b = bid >> 2;
  }
  c.qw = b * 4 + c.wv;
  int L = b;
  if (P.xcd_remap == 1) {
    const int q = nb >> 3, rr = nb & 7, x = b & 7, k = b >> 3;
    L = x < rr ? x * (q + 1) + k : rr * (q + 1) + (x - rr) * q + k;
  }
  int tx, ty;
  shard_tile_xy(P.tiles_x, P.super_tile, P.shard_index, P.shard_count, L, tx, ty);
  c.px = tx * 16 + (c.wv & 1) * 8 + (c.lane & 7);
  c.py = ty * 16 + (c.wv >> 1) * 8 + (c.lane >> 3);
  c.active = c.px < P.W && c.py < P.H && (c.sub < 0 || (c.lane >> 4) == c.sub);
  return c;
}

// traceRayThread: o = getCenter(), d = normalize(screenToWorld(i, j) - o)   (flyscene.cpp:301-308;
// Camera::screenToWorld camera.hpp:155-173 with its fp64 NDC)
__device__ __forceinline__ Ray primary_ray(const FrameParams& P, int px, int py) {
  Ray r;
  const float nx = (float)(2.0 * (double)((float)px - P.vp[0]) / (double)P.vp[2] - 1.0);
  const float ny = (float)(1.0 - 2.0 * (double)((float)py - P.vp[1]) / (double)P.vp[3]);
  const f3 w = affv3(P.vinv, f3{nx * P.xscale, ny * P.yscale, -1.0f});
  r.o = f3{P.eye[0], P.eye[1], P.eye[2]};
  r.d = normalized(sub(w, r.o));
  r.o2 = f3{P.eye_obj[0], P.eye_obj[1], P.eye_obj[2]};
  r.d2 = normalized(m3v3(P.MS, r.d));
  setup_cull(r, P.sc.static_pad);
  return r;
}

// RT_FRAME_TIMELINE: the wave's start / end clocks and where it ran (diagnostics; one uniform branch
// when off). HW_ID / XCC_ID via s_getreg (hwreg ids 4 and 20, all 32 bits).
// The start clocks go to the wave's LDS words rather than staying live in registers for the whole
// kernel (the FULL megakernel's allocation tips into heavy spilling otherwise).
#ifndef RT_WAVE_CLOCK
#define RT_WAVE_CLOCK 1
#endif
__device__ __forceinline__ void wave_clock_start(const FrameParams& P, uint32_t* clk) {
  if (RT_WAVE_CLOCK && (P.timeline || P.cost)) {
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
      clk[0] = (uint32_t)t0;
      clk[1] = (uint32_t)(t0 >> 32);
      clk[2] = r0;
    }
  }
}
// RT_SUBWAVE_COST: how a split wave's cost is refreshed -- 0 kept from the frame that measured it whole,
// 1 sum of its sub-waves' times, 2 their maximum, 3 cost-recording frames run whole waves (no split)
#ifndef RT_SUBWAVE_COST
#define RT_SUBWAVE_COST 2
#endif
__device__ __forceinline__ void wave_clock_end(const FrameParams& P, const uint32_t* clk, int lane, int qw,
                                               bool sub_wave = false) {
  if (!RT_WAVE_CLOCK || (!P.timeline && !P.cost)) return;
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  struct { uint64_t t0; uint32_t r0; } w;
  w.t0 = (uint64_t)uniform(clk[0]) | ((uint64_t)uniform(clk[1]) << 32);
  w.r0 = uniform(clk[2]);
  // this wave's cost for the next frame's dispatch order. The four 16-lane sub-waves of a split wave
  // (sub_wave) write the maximum of their times into the wave's slot, which the host cleared before such
  // a frame (RT_SUBWAVE_COST 2): a split wave's cost is re-measured like every other wave's, so one whose
  // work has become cheap leaves the split range (profiles/ab/r03_subwave_cost_ab.txt: the sum ranks the
  // split waves far above the rest and coarsens the order's buckets, -20% on C5 lone frames; keeping the
  // stale cost is within 1% of the maximum but never refreshes it; running cost-recording frames unsplit
  // costs 6%)
  if (P.cost && lane == 0) {
    const uint64_t dt = t1 - w.t0;
    const uint32_t c = dt > 0x3FFFFFFFull ? 0x3FFFFFFFu : (uint32_t)dt;
    if (!sub_wave) P.cost[qw] = c;
    else if (RT_SUBWAVE_COST == 1) atomicAdd(P.cost + qw, c);
    else if (RT_SUBWAVE_COST == 2) atomicMax(P.cost + qw, c);
  }
  if (!P.timeline) return;
  const uint32_t r1 = (uint32_t)__builtin_amdgcn_s_memrealtime();
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4), xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  if (lane == 0) {
    uint4* o = reinterpret_cast<uint4*>(P.timeline + 8 * (size_t)blockIdx.x);
    o[0] = make_uint4((uint32_t)w.t0, (uint32_t)(w.t0 >> 32), (uint32_t)t1, (uint32_t)(t1 >> 32));
    o[1] = make_uint4(w.r0, r1, hw, (xcc << 28) | ((uint32_t)qw & 0x0FFFFFFFu));
  }
}

__device__ __forceinline__ void flush_stats(const FrameParams& P, const uint32_t* cnt, int lane) {
#pragma unroll
  for (int c = 0; c < ST_COUNT; c++) {
    unsigned long long v = cnt[c];
    if (c == ST_WNODE || c == ST_WTRI || c == ST_WPOP || c == ST_WCULL || c == ST_WWIDE || c == ST_WCAND || c == ST_WPRE ||
        c == ST_WINS || c == ST_WE1 || c == ST_WE2 || c >= ST_WCANDM)
      v = (lane == 0) ? v : 0;  // wave counts once
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane == 0 && v) atomicAdd(P.stats + c, v);
  }
}

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
constexpr int kSplitK = 2048;  // FULL lone frames: waves split into 16-lane sub-waves (FrameParams::split_k)
constexpr int kSplitKPrimary = 1024;  // the same for k_primary_fused (small scenes)
__device__ __forceinline__ uint32_t lpt_bucket(uint32_t c, int shift) {
  // 4 buckets per octave: exponent and 2 mantissa bits of (float)c; costs of 2^10 .. 2^18 shader cycles
  // (0.5 .. 120 us at 2.1 GHz) spread over the buckets, longest first (bucket 0)
  const int q = (int)(__float_as_uint((float)(c | 1u)) >> 21) - ((127 + 10) << 2);
  const int b = (q < 0 ? 0 : (q > 4 * 8 - 1 ? 4 * 8 - 1 : q)) >> shift;
  return (uint32_t)((kLptBuckets >> shift) - 1 - b);
}
__global__ __launch_bounds__(kLptThreads) void k_order_lpt(const uint32_t* cost, uint32_t* order, int n, int C, int shift) {
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
  uint32_t mine[kLptBuckets];
  for (int b = 0; b < kLptBuckets; b++) mine[b] = 0;
  for (int r = r0; r < r1; r++) mine[lpt_bucket(cost[item(r)], shift)]++;
  for (int b = 0; b < nb; b++) cnt[b][t] = mine[b];
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
  if (t == 0) {  // bucket totals -> start ranks, longest bucket first
    uint32_t s = 0;
    for (int b = 0; b < nb; b++) { const uint32_t v = base[b]; base[b] = s; s += v; }
  }
  __syncthreads();
  for (int b = 0; b < nb; b++) mine[b] = base[b] + cnt[b][t];
  for (int r = r0; r < r1; r++) {
    const int j = item(r);
    const uint32_t rr = mine[lpt_bucket(cost[j], shift)]++;
    order[8 * rr + x] = (uint32_t)j;
  }
}

// PRIMARY stage 1: closest hit per pixel (calculateMinimumFace, flyscene.cpp:373-396) -> 8-B hit record.
// Only traversal state is live here, so the kernel fits 8 waves per SIMD.
#ifndef RT_TRACE_WAVES_PER_EU
#define RT_TRACE_WAVES_PER_EU 8  // 8 waves/SIMD: measured +2.5% over the 7 the register count allows
#endif
#ifndef RT_TRACE_WPB
#define RT_TRACE_WPB 1  // waves per block of the traversal kernel (4 or 1; 1 measured 3% faster)
#endif
template <bool STATS, int TRAV>
__global__ __launch_bounds__(64 * RT_TRACE_WPB) __attribute__((amdgpu_waves_per_eu(RT_TRACE_WAVES_PER_EU)))
void k_trace_primary(FrameParams P) {
  __shared__ WaveLds<TRAV, STATS> lds;
  const PixelCoord c = pixel_coord<RT_TRACE_WPB>(P);
  uint32_t cnt[ST_COUNT] = {};
  const Ray r = primary_ray(P, c.px, c.py);
  if (STATS && c.active) { cnt[ST_RAYS]++; cnt[ST_TOTAL]++; }
  Hit h{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
  trace_closest_oct<STATS, TRAV, true>(P.sc, r, c.active, h, lds, c.slot, cnt);
  if (STATS && c.active && h.t != INFINITY) cnt[ST_HITS]++;
  if (c.active) P.hits[(size_t)c.py * P.W + c.px] = make_uint2(__float_as_uint(h.t), h.slot);
  if (P.wcount0 != nullptr) {  // FULL pipeline: per-wave hit count for the list0 compaction
    const uint32_t nh = (uint32_t)__popcll(ballot(c.active && h.t != INFINITY));
    if (c.lane == 0) P.wcount0[c.qw] = nh;
  }
  if (STATS) flush_stats(P, cnt, c.lane);
}

// Persistent-threads form of k_trace_primary (A/B variant bit 2048): one launch of as many one-wave
// blocks as the device holds at 8 waves per SIMD; each wave repeatedly takes the next 8x8 work item
// from its XCD's counter (XCD x owns items [x Q/8, (x+1) Q/8) of the shard's Q = 4 * tiles items, so
// an XCD works through a contiguous band of tiles) and, once that range is exhausted, from the other
// XCDs' counters in turn. The next item's atomic is issued before the current item is traced, so its
// latency overlaps the traversal. Same per-pixel work and outputs as k_trace_primary.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_TRACE_WAVES_PER_EU)))
void k_trace_primary_persistent(FrameParams P, uint32_t* queue, uint32_t max_steal) {
  __shared__ WaveLds<TRAV_B2_LDS, false> lds;
  const int lane = (int)(threadIdx.x & 63);
  const uint32_t Q = 4u * (uint32_t)P.n_tiles_shard;
  const uint32_t x0 = blockIdx.x & 7u;
  uint32_t k = 0;  // counters visited so far (own XCD first)
  auto take = [&](uint32_t x) -> uint32_t {
    uint32_t i = 0;
    if (lane == 0) i = atomicAdd(queue + x, 1u);
    return uniform(i);
  };
  auto item_of = [&](uint32_t x, uint32_t i) -> uint32_t {  // global item or ~0u when x's range is done
    const uint32_t lo = (uint32_t)(((uint64_t)Q * x) / 8), hi = (uint32_t)(((uint64_t)Q * (x + 1)) / 8);
    return lo + i < hi ? lo + i : 0xFFFFFFFFu;
  };
  uint32_t cur = item_of(x0, take(x0));
  for (;;) {
    while (cur == 0xFFFFFFFFu && k < max_steal) {  // steal from the next XCD's range
      k++;
      const uint32_t x = (x0 + k) & 7u;
      cur = item_of(x, take(x));
    }
    if (cur == 0xFFFFFFFFu) break;  // every range exhausted: all waves reach this exit
    const uint32_t xk = (x0 + k) & 7u;
    const uint32_t nxt_i = take(xk);  // the next item from the same counter, requested early
    const int b = (int)(cur >> 2), wv = (int)(cur & 3);
    int tx, ty;
    shard_tile_xy(P.tiles_x, P.super_tile, P.shard_index, P.shard_count, b, tx, ty);
    const int px = tx * 16 + (wv & 1) * 8 + (lane & 7), py = ty * 16 + (wv >> 1) * 8 + (lane >> 3);
    const bool active = px < P.W && py < P.H;
    const Ray r = primary_ray(P, px, py);
    Hit h{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
    trace_closest_oct<false, TRAV_B2_LDS>(P.sc, r, active, h, lds, 0, nullptr);
    if (active) P.hits[(size_t)py * P.W + px] = make_uint2(__float_as_uint(h.t), h.slot);
    cur = item_of(xk, nxt_i);
  }
}

// Two rays per lane (128-ray packets, one 16x8 pixel half-tile per wave): the per-node scalar work
// (fetch, decision, stack) is shared by twice as many rays and each lane carries two independent
// slab / triangle streams. Closest hit only (PRIMARY), LDS stack.
__device__ __forceinline__ void traverse_x2(const DevScene& P, const Ray& ra, const Ray& rb, bool acta, bool actb,
                                            Hit& ha, Hit& hb, uint32_t* lds_stack) {
  if (P.n_nodes == 0) return;
  int sp = 0;
  uint32_t node = P.root;
  const uint64_t ma = ballot(acta), mb = ballot(actb);
  bool dummy = false;
  for (;;) {
    bool pop = true;
    if (!is_leaf(node)) {
      const Node64 nd = sload_node(P.nodes, node);
      const Span a0 = slab(nd.c0lx, nd.c0hx, nd.c0ly, nd.c0hy, nd.c0lz, nd.c0hz, ra, ha.t);
      const Span a1 = slab(nd.c1lx, nd.c1hx, nd.c1ly, nd.c1hy, nd.c1lz, nd.c1hz, ra, ha.t);
      const Span b0 = slab(nd.c0lx, nd.c0hx, nd.c0ly, nd.c0hy, nd.c0lz, nd.c0hz, rb, hb.t);
      const Span b1 = slab(nd.c1lx, nd.c1hx, nd.c1ly, nd.c1hy, nd.c1lz, nd.c1hz, rb, hb.t);
      const uint64_t m0a = mask_le(a0.tmin, a0.tmax) & ma, m1a = mask_le(a1.tmin, a1.tmax) & ma;
      const uint64_t m0b = mask_le(b0.tmin, b0.tmax) & mb, m1b = mask_le(b1.tmin, b1.tmax) & mb;
      const uint64_t v0a = m0a & (~m1a | mask_le(a0.tmin, a1.tmin));
      const uint64_t v0b = m0b & (~m1b | mask_le(b0.tmin, b1.tmin));
      const uint64_t M0 = m0a | m0b, M1 = m1a | m1b;
      const bool first0 = 2 * (__popcll(v0a) + __popcll(v0b)) >= __popcll(m0a | m1a) + __popcll(m0b | m1b);
      lds_stack[sp] = first0 ? nd.child1 : nd.child0;
      sp += ((M0 != 0) & (M1 != 0)) ? 1 : 0;
      node = first0 ? nd.child0 : nd.child1;
      pop = (M0 | M1) == 0;
    } else {
      const uint32_t first = leaf_first(node), count = leaf_count(node);
      for (uint32_t k = 0; k < count; k++) {
        const TriRec64 tr = sload_tri(P.tris, first + k);
        test_tri<false>(P, tr, first + k, ra, ma, ha, dummy);
        test_tri<false>(P, tr, first + k, rb, mb, hb, dummy);
      }
    }
    if (pop) {
      if (sp == 0) break;
      sp--;
      node = uniform(lds_stack[sp]);
    }
  }
}

#ifndef RT_DUAL_WAVES_PER_EU
#define RT_DUAL_WAVES_PER_EU 8
#endif
#ifndef RT_X2_WAVES_PER_EU
#define RT_X2_WAVES_PER_EU 6
#endif
// one 64-thread block per 16x8 half of a 16x16 tile (blocks 2t, 2t+1 cover tile t); lane (x, y) traces
// pixels (x, y) and (x + 8, y) of its half
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_X2_WAVES_PER_EU)))
void k_trace_primary_x2(FrameParams P) {
  __shared__ uint32_t stack[64];
  const int lane = threadIdx.x & 63;
  const int nb = (int)(gridDim.x >> 1), b = (int)(blockIdx.x >> 1), half = (int)(blockIdx.x & 1);
  (void)nb;
  int tx, ty;
  shard_tile_xy(P.tiles_x, P.super_tile, P.shard_index, P.shard_count, b, tx, ty);
  const int pxa = tx * 16 + (lane & 7), pxb = pxa + 8, py = ty * 16 + half * 8 + (lane >> 3);
  const bool acta = pxa < P.W && py < P.H, actb = pxb < P.W && py < P.H;
  const Ray ra = primary_ray(P, pxa, py), rb = primary_ray(P, pxb, py);
  Hit ha{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu}, hb{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
  traverse_x2(P.sc, ra, rb, acta, actb, ha, hb, stack);
  if (acta) P.hits[(size_t)py * P.W + pxa] = make_uint2(__float_as_uint(ha.t), ha.slot);
  if (actb) P.hits[(size_t)py * P.W + pxb] = make_uint2(__float_as_uint(hb.t), hb.slot);
}

// PRIMARY stage 2: traceRay at depth limit 1 without shadows: calculateColor (flyscene.cpp:603-614)
// + traceRay's ks update and clamp (:355-370), or the background on a miss (:327-332), for one pixel
// whose closest hit (t, triangle slot) is known.
// BOXCOL: RENDER_BOUNDINGBOX_COLORED_TRIANGLES (flyscene.cpp:334-348) instead of the shading: the hit
// face's summed box colours (k_face_box_colors), unclamped.
template <bool HITS, bool BOXCOL = false>
__device__ __forceinline__ void shade_primary_pixel(const FrameParams& P, const Ray& r, size_t pix, float t,
                                                    uint32_t slot) {
  const bool hit0 = t != INFINITY;
  f3 col;
  int32_t face = -1;
  if (BOXCOL && hit0) {
    face = (int32_t)P.sc.tris[slot].face;
    const float4 c = reinterpret_cast<const float4*>(P.face_boxcolor)[face];
    col = f3{c.x, c.y, c.z};
  } else if (hit0) {
    const TriRec64 tr0 = vload_tri(P.sc.tris, slot);
    HitInfo hi0;
    hi0.face = tr0.face;
    face = (int32_t)tr0.face;
    hi0.p = f3{r.o.x + t * r.d.x, r.o.y + t * r.d.y, r.o.z + t * r.d.z};
    hi0.n = hit_normal(P.sc, tr0, slot, hi0.p, hi0.mat);
    MatState st = load_mat(P.defmat);
    const f3 direct0 = calc_color<false, false, TRAV_B2_LDS>(P, st, hi0, r.o, true, nullptr, 0, nullptr);
    if (hi0.mat != -1) st.ks = load_mat(P.sc.mats[hi0.mat]).ks;
    col = f3{clamp01(direct0.x + 0.0f * st.ks.x), clamp01(direct0.y + 0.0f * st.ks.y),
             clamp01(direct0.z + 0.0f * st.ks.z)};
  } else {
    col = f3{P.bg[0], P.bg[1], P.bg[2]};
  }
  P.rgb[3 * pix + 0] = col.x;
  P.rgb[3 * pix + 1] = col.y;
  P.rgb[3 * pix + 2] = col.z;
  if (HITS) {
    P.face_out[pix] = face;
    P.t_out[pix] = t;
  }
}

template <bool HITS, bool BOXCOL>
__global__ __launch_bounds__(256) void k_shade_primary(FrameParams P) {
  const PixelCoord c = pixel_coord(P);
  if (!c.active) return;
  const size_t pix = (size_t)c.py * P.W + c.px;
  const uint2 hb = P.hits[pix];
  const float t = __uint_as_float(hb.x);
  Ray r;
  if (t != INFINITY) r = primary_ray(P, c.px, c.py);
  shade_primary_pixel<HITS, BOXCOL>(P, r, pix, t, hb.y);
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

// PRIMARY as one kernel (default; variant bit 32768 selects the two-kernel form k_trace_primary +
// k_shade_primary): the traversal, then the shading of the same lane -- the hit record stays in
// registers instead of a round trip through HBM, and the traversal state is dead by then, so the
// shading's registers do not add to the traversal's (64 VGPR, 8 waves/SIMD, a 112-B spill in the
// shading part). Measured: C3 +2.7% at 4 frames in flight, bunny +4%.
template <bool HITS, bool BOXCOL = false>
__global__ __launch_bounds__(64 * RT_TRACE_WPB) __attribute__((amdgpu_waves_per_eu(RT_TRACE_WAVES_PER_EU)))
void k_primary_fused(FrameParams P) {
  __shared__ WaveLds<TRAV_B2_LDS, false> lds;
  wave_clock_start(P, lds.clk);
  const PixelCoord c = pixel_coord<RT_TRACE_WPB>(P);
#if RT_EYE_VREG
  // the eye (every primary ray's origin) held in VGPRs: origin.dot(facenormal) in each triangle test
  // then reads one SGPR per op and needs no moves
  Ray r = primary_ray(P, c.px, c.py);
  asm("" : "+v"(r.o.x), "+v"(r.o.y), "+v"(r.o.z));
#else
  const Ray r = primary_ray(P, c.px, c.py);
#endif
  Hit h{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
  trace_closest_oct<false, TRAV_B2_LDS, true, true>(P.sc, r, c.active, h, lds, c.slot, nullptr);
#if defined(RT_EXP_NOSHADE)  // timing experiment only: the hit distance instead of the shading
  if (c.active) {
    const size_t pix = (size_t)c.py * P.W + c.px;
    P.rgb[3 * pix] = h.t; P.rgb[3 * pix + 1] = __uint_as_float(h.slot); P.rgb[3 * pix + 2] = 0.0f;
  }
#else
  if (c.active) shade_primary_pixel<HITS, BOXCOL>(P, r, (size_t)c.py * P.W + c.px, h.t, h.slot);
#endif
  wave_clock_end(P, lds.clk, c.lane, c.qw, c.sub >= 0);
}

// PRIMARY with two 8x8 packets per wave (dual-chain traversal, traverse_dual): block b traces pair b
// = the left and right 8x8 quarters of one 8-row half of a 16x16 tile; dispatch order as the one-wave
// kernels (chunked XCD runs, or longest-first over pairs from an earlier frame's pair costs).
struct PairCoord {
  int lane, pair, pxa, py;
  bool acta, actb;
};
__device__ __forceinline__ PairCoord pair_coord(const FrameParams& P) {
  PairCoord c;
  c.lane = threadIdx.x & 63;
  int bid = (int)blockIdx.x;
  if (RT_ORDER_LPT && P.order != nullptr) {
    const uint32_t o = uniform(P.order[blockIdx.x]);
    bid = o < gridDim.x ? (int)o : (int)blockIdx.x;
  } else if (P.xcd_remap >= 2) {
    const int C = P.xcd_remap, G = 8 * C, full = ((int)gridDim.x / G) * G;
    if (bid < full) {
      const int x = bid & 7, k = bid >> 3;
      bid = (k / C) * G + x * C + (k % C);
    }
  }
  c.pair = bid;
  int tx, ty;
  shard_tile_xy(P.tiles_x, P.super_tile, P.shard_index, P.shard_count, bid >> 1, tx, ty);
  c.pxa = tx * 16 + (c.lane & 7);
  c.py = ty * 16 + (bid & 1) * 8 + (c.lane >> 3);
  c.acta = c.pxa < P.W && c.py < P.H;
  c.actb = c.pxa + 8 < P.W && c.py < P.H;
  return c;
}

template <bool HITS, bool BOXCOL = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_DUAL_WAVES_PER_EU)))
void k_primary_dual(FrameParams P) {
  __shared__ WaveLds<TRAV_B2_LDS, false> lds;
  wave_clock_start(P, lds.clk);
  const PairCoord c = pair_coord(P);
  const Ray ra = primary_ray(P, c.pxa, c.py), rb = primary_ray(P, c.pxa + 8, c.py);
  Hit ha{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu}, hb{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
  trace_dual(P.sc, ra, rb, c.acta, c.actb, ha, hb, lds.stack[0], lds.stack[1]);
  if (c.acta) shade_primary_pixel<HITS, BOXCOL>(P, ra, (size_t)c.py * P.W + c.pxa, ha.t, ha.slot);
  if (c.actb) shade_primary_pixel<HITS, BOXCOL>(P, rb, (size_t)c.py * P.W + c.pxa + 8, hb.t, hb.slot);
  wave_clock_end(P, lds.clk, c.lane, c.pair);
}

// FULL: the reference traceRay as-is (max_depth 2): shadow any-hit per light and one reflection
// bounce, all in one kernel (flyscene.cpp:317-371, 510-566, 603-614).
// traceRay(o, d, 0) with max_depth 2 (FULL, flyscene.cpp:317-371): primary hit, per-light shadows, one
// reflection bounce with its own shadows. Shared by the frame megakernel and the ray-list colour query.
// Returns the colour; h0 / face0: the first hit (t, face id).
// SPLIT: mixed-octant secondary packets walk once per octant (trace_oct); the small-scene build only --
// measured C5 +1.5% at 4 frames in flight, +1..3% one at a time, the 1M soup in FULL -5%
// (profiles/ab/r03_full_split_oct_ab.txt)
template <bool STATS, int TRAV, bool SPLIT = false>
__device__ __forceinline__ f3 trace_full(const FrameParams& P, const Ray& r, bool active, WaveLds<TRAV, STATS>& lds, int wv,
                                         uint32_t* cnt, Hit& h, uint32_t& face0) {
  h = Hit{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
  bool dummy = false;
  // the primary packet is coherent: octant-specialised loops for it alone (A/B knob RT_FULL_OCT_PRIMARY)
  if (RT_FULL_OCT_PRIMARY) trace_oct<false, STATS, TRAV>(P.sc, r, active, h, dummy, lds, wv, cnt);
  else trace_full_ray<false, STATS, TRAV>(P.sc, r, active, h, dummy, lds, wv, cnt);
  const bool hit0 = active && h.t != INFINITY;
  if (STATS && hit0) cnt[ST_HITS]++;

  MatState st = load_mat(P.defmat);
  HitInfo hi0;
  hi0.mat = -1;
  hi0.face = 0xFFFFFFFFu;
  hi0.p = f3{0.0f, 0.0f, 0.0f};
  hi0.n = f3{0.0f, 0.0f, 0.0f};
  if (hit0) {
    const TriRec64 tr0 = vload_tri(P.sc.tris, h.slot);
    hi0.face = tr0.face;
    hi0.p = f3{r.o.x + h.t * r.d.x, r.o.y + h.t * r.d.y, r.o.z + h.t * r.d.z};
    hi0.n = hit_normal(P.sc, tr0, h.slot, hi0.p, hi0.mat);
  }
  // the primary hits' shadow packets head for the same light from neighbouring points: octant loops for
  // them too (A/B knob RT_FULL_OCT_SHADOW); the reflection hits' shadows keep the generic loop
  const f3 direct0 = calc_color<true, STATS, TRAV, RT_FULL_OCT_SHADOW != 0, SPLIT>(P, st, hi0, r.o, hit0, &lds, wv, cnt);
  if (hit0 && hi0.mat != -1) st.ks = load_mat(P.sc.mats[hi0.mat]).ks;  // traceRay :355-358

  // reflect(dir.normalized(), interpolateNormal(...)), offset 0.001 (flyscene.cpp:361-363)
  f3 refl{0.0f, 0.0f, 0.0f};
  Ray rr;
  rr.d = reflect(normalized(r.d), hi0.n);
  rr.o = offset(hi0.p, rr.d, 0.001f);
  rr.o2 = affv3(P.Minv, rr.o);
  rr.d2 = normalized(m3v3(P.MS, rr.d));
  setup_cull(rr, P.sc.static_pad);
  if (STATS && hit0) cnt[ST_TOTAL]++;
  Hit h1{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
  if (RT_FULL_OCT_REFL)
    trace_oct<false, STATS, TRAV, RT_FULL_MIXED_LANE != 0, false, SPLIT>(P.sc, rr, hit0, h1, dummy, lds, wv, cnt);
  else trace_full_ray<false, STATS, TRAV>(P.sc, rr, hit0, h1, dummy, lds, wv, cnt);
  const bool hit1 = hit0 && h1.t != INFINITY;
  HitInfo hi1;
  hi1.mat = -1;
  hi1.p = f3{0.0f, 0.0f, 0.0f};
  hi1.n = f3{0.0f, 0.0f, 0.0f};
  if (hit1) {
    const TriRec64 tr1 = vload_tri(P.sc.tris, h1.slot);
    hi1.face = tr1.face;
    hi1.p = f3{rr.o.x + h1.t * rr.d.x, rr.o.y + h1.t * rr.d.y, rr.o.z + h1.t * rr.d.z};
    hi1.n = hit_normal(P.sc, tr1, h1.slot, hi1.p, hi1.mat);
  }
  const f3 direct1 = calc_color<true, STATS, TRAV, RT_FULL_OCT_SHADOW2 != 0, SPLIT>(P, st, hi1, rr.o, hit1, &lds, wv, cnt);
  if (hit1) {
    if (hi1.mat != -1) st.ks = load_mat(P.sc.mats[hi1.mat]).ks;
    // depth 1: direct1 + traceRay(depth 2)=0 * ks, clamped
    refl = f3{clamp01(direct1.x + 0.0f * st.ks.x), clamp01(direct1.y + 0.0f * st.ks.y),
              clamp01(direct1.z + 0.0f * st.ks.z)};
  }
  f3 col;
  if (hit0) {
    col = f3{clamp01(direct0.x + refl.x * st.ks.x), clamp01(direct0.y + refl.y * st.ks.y),
             clamp01(direct0.z + refl.z * st.ks.z)};
  } else {
    col = f3{P.bg[0], P.bg[1], P.bg[2]};
  }
  face0 = hit0 ? hi0.face : 0xFFFFFFFFu;
  return col;
}

// The same traceRay(o, d, 0) as a loop over the two depths, so that the closest-hit and the any-hit
// traversal each appear once in the kernel instead of twice (A/B knob RT_FULL_LOOP). Same expressions
// in the same order as trace_full above, hence the same bits.
#ifndef RT_FULL_LOOP
#define RT_FULL_LOOP 0
#endif
template <bool STATS, int TRAV>
__device__ __forceinline__ f3 trace_full_loop(const FrameParams& P, const Ray& r, bool active, WaveLds<TRAV, STATS>& lds,
                                              int wv, uint32_t* cnt, Hit& h0, uint32_t& face0) {
  MatState st = load_mat(P.defmat);
  Ray cur = r;
  bool act = active, hit0 = false;
  f3 direct0{0.0f, 0.0f, 0.0f}, refl{0.0f, 0.0f, 0.0f};
  face0 = 0xFFFFFFFFu;
#pragma clang loop unroll(disable)
  for (int depth = 0; depth < 2; depth++) {
    Hit h{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
    bool dummy = false;
    trace_full_ray<false, STATS, TRAV>(P.sc, cur, act, h, dummy, lds, wv, cnt);
    const bool hit = act && h.t != INFINITY;
    if (STATS && depth == 0 && hit) cnt[ST_HITS]++;
    HitInfo hi;
    hi.mat = -1;
    hi.face = 0xFFFFFFFFu;
    hi.p = f3{0.0f, 0.0f, 0.0f};
    hi.n = f3{0.0f, 0.0f, 0.0f};
    if (hit) {
      const TriRec64 tr = vload_tri(P.sc.tris, h.slot);
      hi.face = tr.face;
      hi.p = f3{cur.o.x + h.t * cur.d.x, cur.o.y + h.t * cur.d.y, cur.o.z + h.t * cur.d.z};
      hi.n = hit_normal(P.sc, tr, h.slot, hi.p, hi.mat);
    }
    const f3 direct = calc_color<true, STATS, TRAV>(P, st, hi, cur.o, hit, &lds, wv, cnt);
    if (depth == 0) {
      h0 = h;
      hit0 = hit;
      face0 = hit ? hi.face : 0xFFFFFFFFu;
      direct0 = direct;
      if (hit && hi.mat != -1) st.ks = load_mat(P.sc.mats[hi.mat]).ks;  // traceRay :355-358
      // reflect(dir.normalized(), interpolateNormal(...)), offset 0.001 (flyscene.cpp:361-363)
      Ray rr;
      rr.d = reflect(normalized(cur.d), hi.n);
      rr.o = offset(hi.p, rr.d, 0.001f);
      rr.o2 = affv3(P.Minv, rr.o);
      rr.d2 = normalized(m3v3(P.MS, rr.d));
      setup_cull(rr, P.sc.static_pad);
      if (STATS && hit) cnt[ST_TOTAL]++;
      cur = rr;
      act = hit;
    } else if (hit) {
      if (hi.mat != -1) st.ks = load_mat(P.sc.mats[hi.mat]).ks;
      // depth 1: direct1 + traceRay(depth 2)=0 * ks, clamped
      refl = f3{clamp01(direct.x + 0.0f * st.ks.x), clamp01(direct.y + 0.0f * st.ks.y),
                clamp01(direct.z + 0.0f * st.ks.z)};
    }
  }
  if (!hit0) return f3{P.bg[0], P.bg[1], P.bg[2]};
  return f3{clamp01(direct0.x + refl.x * st.ks.x), clamp01(direct0.y + refl.y * st.ks.y),
            clamp01(direct0.z + refl.z * st.ks.z)};
}

// Occupancy of the FULL megakernel, by scene: 8 waves per SIMD (64 VGPR + a 144-B spill) for scenes
// whose node + triangle records exceed the chip's aggregate L2 (the 1M soup: 8 waves beat 5 by 18% and
// 3 by 24% -- the traversal waits on L2 misses and needs the waves), a 6-wave bound (79 VGPR, no
// spill) for smaller ones (bunny, C5: +14% over 8 -- their records are L2-resident; the 5-wave bound
// let the kernel grow to 82 VGPR = 5 waves, 4.6% slower; 7 waves spill 48 B, equal to 6).
#ifndef RT_FULL_WAVES_PER_EU
#define RT_FULL_WAVES_PER_EU 8
#endif
#ifndef RT_FULL_WAVES_PER_EU_SMALL
#define RT_FULL_WAVES_PER_EU_SMALL 6
#endif
constexpr size_t kFullSmallSceneBytes = 32u << 20;  // 8 XCDs x 4 MiB L2
#ifndef RT_FULL_WPB
#define RT_FULL_WPB 1  // waves per block of the FULL megakernel (1: one 8x8 wave per block, measured
                       // +6.5% on bunny FULL and +8% on the soup over 4 = one 16x16 tile per block)
#endif
template <bool STATS, bool HITS, int TRAV, int WPE = RT_FULL_WAVES_PER_EU>
__global__ __launch_bounds__(64 * RT_FULL_WPB) __attribute__((amdgpu_waves_per_eu(WPE)))
void k_render_full(FrameParams P) {
  __shared__ WaveLds<TRAV, STATS> lds;
  wave_clock_start(P, lds.clk);
  const PixelCoord c = pixel_coord<RT_FULL_WPB>(P);
  const bool active = c.active;
  uint32_t cnt[ST_COUNT] = {};
  const Ray r = primary_ray(P, c.px, c.py);
  if (STATS && active) { cnt[ST_RAYS]++; cnt[ST_TOTAL]++; }

  Hit h;
  uint32_t face0;
  const f3 col = RT_FULL_LOOP ? trace_full_loop<STATS, TRAV>(P, r, active, lds, c.slot, cnt, h, face0)
                              : trace_full<STATS, TRAV, RT_FULL_SPLIT_OCT != 0 && WPE == RT_FULL_WAVES_PER_EU_SMALL>(
                                    P, r, active, lds, c.slot, cnt, h, face0);
  const bool hit0 = face0 != 0xFFFFFFFFu;
  if (active) {
    const size_t pix = (size_t)c.py * P.W + c.px;
    P.rgb[3 * pix + 0] = col.x;
    P.rgb[3 * pix + 1] = col.y;
    P.rgb[3 * pix + 2] = col.z;
    if (HITS) {
      P.face_out[pix] = hit0 ? (int32_t)face0 : -1;
      P.t_out[pix] = h.t;
    }
  }
  if (STATS) flush_stats(P, cnt, c.lane);
  wave_clock_end(P, lds.clk, c.lane, c.qw, c.sub >= 0);
}

// traceRay(o, d, 0) for any recursion limit D = P.max_depth (flyscene.cpp:317-371; the reference fixes
// max_depth = 2 at flyscene.hpp:142, SURVEY 8(b) b2 exposes it): level d traces the closest hit of
// the ray from level d-1's reflection, shades it (calculateColor, shadows per P.shadows) and updates
// the sticky ks (traceRay :355-358). The reference combines on the way back up,
//   colour_d = clamp01(direct_d + colour_{d+1} (*) ks),
// reading the ks member AFTER the deeper levels returned, i.e. the last value any level wrote; so the
// kernel keeps each level's direct colour (lane-private array, D <= RT_MAX_TRACE_DEPTH) and folds them
// from the deepest hit level upwards with that final ks. The deepest hit level adds 0 (*) ks (its own
// reflection returned black: a miss below depth 0, or depth == max_depth). D = 0 returns black for
// every pixel without tracing (traceRay :318-320). Same expressions and order as k_render_full for
// D = 2, hence the same bits (tested); this kernel serves the other depths.
template <bool STATS, bool HITS>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_FULL_WAVES_PER_EU_SMALL)))
void k_render_depth(FrameParams P) {
  __shared__ WaveLds<TRAV_B2_LDS, STATS> lds;
  wave_clock_start(P, lds.clk);
  const PixelCoord c = pixel_coord<1>(P);
  const bool active = c.active;
  uint32_t cnt[ST_COUNT] = {};
  Ray cur = primary_ray(P, c.px, c.py);
  const Ray r0 = cur;
  if (STATS && active) { cnt[ST_RAYS]++; cnt[ST_TOTAL]++; }
  MatState st = load_mat(P.defmat);
  f3 direct[RT_MAX_TRACE_DEPTH];
  int levels = 0;  // levels whose closest hit exists (the chain stops at the first miss)
  bool act = active;
  Hit h0{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
  uint32_t face0 = 0xFFFFFFFFu;
  const int D = P.max_depth;
#pragma clang loop unroll(disable)
  for (int d = 0; d < D; d++) {
    Hit h{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
    bool dummy = false;
    if (d == 0) trace_oct<false, STATS, TRAV_B2_LDS>(P.sc, cur, act, h, dummy, lds, c.slot, cnt);
    else trace<false, STATS, TRAV_B2_LDS>(P.sc, cur, act, h, dummy, lds, c.slot, cnt);
    const bool hit = act && h.t != INFINITY;
    if (STATS && d == 0 && hit) cnt[ST_HITS]++;
    HitInfo hi;
    hi.mat = -1;
    hi.face = 0xFFFFFFFFu;
    hi.p = f3{0.0f, 0.0f, 0.0f};
    hi.n = f3{0.0f, 0.0f, 0.0f};
    if (hit) {
      const TriRec64 tr = vload_tri(P.sc.tris, h.slot);
      hi.face = tr.face;
      hi.p = f3{cur.o.x + h.t * cur.d.x, cur.o.y + h.t * cur.d.y, cur.o.z + h.t * cur.d.z};
      hi.n = hit_normal(P.sc, tr, h.slot, hi.p, hi.mat);
    }
    if (d == 0) {
      h0 = h;
      face0 = hit ? hi.face : 0xFFFFFFFFu;
    }
    const f3 dc = P.shadows ? calc_color<true, STATS, TRAV_B2_LDS>(P, st, hi, cur.o, hit, &lds, c.slot, cnt)
                            : calc_color<false, STATS, TRAV_B2_LDS>(P, st, hi, cur.o, hit, &lds, c.slot, cnt);
    if (hit) {
      direct[d] = dc;
      levels = d + 1;
      if (hi.mat != -1) st.ks = load_mat(P.sc.mats[hi.mat]).ks;  // traceRay :355-358
    }
    if (d + 1 == D) break;  // traceRay(depth + 1) returns black without tracing (:318-320)
    // reflect(dir.normalized(), interpolateNormal(...)), offset 0.001 (flyscene.cpp:361-363)
    Ray rr;
    rr.d = reflect(normalized(cur.d), hi.n);
    rr.o = offset(hi.p, rr.d, 0.001f);
    rr.o2 = affv3(P.Minv, rr.o);
    rr.d2 = normalized(m3v3(P.MS, rr.d));
    setup_cull(rr, P.sc.static_pad);
    if (STATS && hit) cnt[ST_TOTAL]++;
    cur = rr;
    act = hit;
    if (ballot(act) == 0) break;  // no lane of the wave continues
  }
  f3 col{0.0f, 0.0f, 0.0f};
  for (int d = levels - 1; d >= 0; d--)
    col = f3{clamp01(direct[d].x + col.x * st.ks.x), clamp01(direct[d].y + col.y * st.ks.y),
             clamp01(direct[d].z + col.z * st.ks.z)};
  if (D > 0 && levels == 0) col = f3{P.bg[0], P.bg[1], P.bg[2]};  // primary miss: BACKGROUND_COLOR (:327-332)
  (void)r0;
  if (active) {
    const size_t pix = (size_t)c.py * P.W + c.px;
    P.rgb[3 * pix + 0] = col.x;
    P.rgb[3 * pix + 1] = col.y;
    P.rgb[3 * pix + 2] = col.z;
    if (HITS) {
      P.face_out[pix] = face0 != 0xFFFFFFFFu ? (int32_t)face0 : -1;
      P.t_out[pix] = h0.t;
    }
  }
  if (STATS) flush_stats(P, cnt, c.lane);
  wave_clock_end(P, lds.clk, c.lane, c.qw);
}

// ------------------------------------------------------------------------------------------------
// FULL as a wavefront pipeline: k_render_full's work cut at every traversal into lean stage kernels
// (each at full occupancy) that hand per-pixel records through HBM:
//   k_trace_primary -> k_full_gen0 -> k_full_shadow(0) -> k_full_refl -> k_full_gen1 -> k_full_shadow(1)
//   -> k_full_final
// Same expressions and the same order of sticky material updates as the megakernel, so the frame is
// bit-identical to it (and to the oracle's traceRay).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ HitState no_hit_state() {
  HitState h;
  h.px = h.py = h.pz = 0.0f;
  h.nx = h.ny = h.nz = 0.0f;
  h.mat = -1;
  h.face = 0xFFFFFFFFu;
  return h;
}
__device__ __forceinline__ HitState to_state(const HitInfo& hi) {
  HitState h;
  h.px = hi.p.x; h.py = hi.p.y; h.pz = hi.p.z;
  h.nx = hi.n.x; h.ny = hi.n.y; h.nz = hi.n.z;
  h.mat = hi.mat;
  h.face = hi.face;
  return h;
}
__device__ __forceinline__ HitInfo from_state(const HitState& h) {
  HitInfo hi;
  hi.p = f3{h.px, h.py, h.pz};
  hi.n = f3{h.nx, h.ny, h.nz};
  hi.mat = h.mat;
  hi.face = h.face;
  return hi;
}
__device__ __forceinline__ size_t pixel_index(const FrameParams& P, const PixelCoord& c) {
  return (size_t)c.py * P.W + c.px;
}

// Compaction without atomics: each producer wave stores its count of selected lanes, one block
// scans the counts (k_scan_counts), and the consumer of the next stage writes its selected lanes to
// list[offset[wave] + rank among the wave's selected lanes]. The list is in wave order, so 64
// consecutive entries come from neighbouring tiles and packets stay coherent.
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// exclusive prefix sum of cnt[0..q) into off[], total into *total (one 1024-thread block)
__global__ __launch_bounds__(1024) void k_scan_counts(const uint32_t* cnt, uint32_t* off, int q, uint32_t* total) {
  __shared__ uint32_t part[1024];
  const int t = (int)threadIdx.x;
  const int per = (q + 1023) / 1024;
  const int b = t * per, e = min(q, b + per);
  uint32_t sum = 0;
  for (int i = b; i < e; i++) sum += cnt[i];
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const uint32_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  for (int i = b; i < e; i++) {
    off[i] = run;
    run += cnt[i];
  }
  if (t == 1023) *total = part[1023];
}

// list wave w of a list-consuming kernel: entries [64 w, 64 w + 64) of a list of n
struct ListLane {
  int w;          // list wave index (uniform)
  uint32_t i;     // this lane's list position
  bool act;       // i < n
  bool any;       // the wave has at least one entry
};
__device__ __forceinline__ ListLane list_lane(uint32_t n) {
  ListLane L;
  L.w = (int)uniform(blockIdx.x * 4 + (threadIdx.x >> 6));
  L.i = (uint32_t)L.w * 64u + (uint32_t)lane_id();
  L.act = L.i < n;
  L.any = (uint32_t)L.w * 64u < n;
  return L;
}

// primary hit record -> hit point, interpolated normal, material; and the reflection ray
// (traceRay flyscene.cpp:336-363)
__global__ __launch_bounds__(256) void k_full_gen0(FrameParams P) {
  const PixelCoord c = pixel_coord(P);
  const size_t pix = c.active ? pixel_index(P, c) : 0;
  const float t = c.active ? __uint_as_float(P.hits[pix].x) : INFINITY;
  // scatter this wave's hit pixels into list0 (offsets from the primary kernel's counts)
  const uint64_t hm = ballot(t != INFINITY);
  if (t != INFINITY) P.list0[P.woff0[c.qw] + lanes_below(hm)] = (uint32_t)pix;
  if (!c.active) return;
  const uint2 hb = P.hits[pix];
  HitState hs = no_hit_state();
  RayRec rq{0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0u, 0u};
  if (t != INFINITY) {
    const Ray r = primary_ray(P, c.px, c.py);
    const TriRec64 tr0 = vload_tri(P.sc.tris, hb.y);
    HitInfo hi0;
    hi0.face = tr0.face;
    hi0.p = f3{r.o.x + t * r.d.x, r.o.y + t * r.d.y, r.o.z + t * r.d.z};
    hi0.n = hit_normal(P.sc, tr0, hb.y, hi0.p, hi0.mat);
    hs = to_state(hi0);
    const f3 d = reflect(normalized(r.d), hi0.n);
    const f3 o = offset(hi0.p, d, 0.001f);
    rq = RayRec{o.x, o.y, o.z, d.x, d.y, d.z, 0u, 0u};
  }
  P.state0[pix] = hs;
  P.refl[pix] = rq;
}

// shadow() for every light from the hits listed for `pass` (0: primary, 1: reflection): per-light
// blocked bits. One wave per 64 list entries.
template <bool STATS, int TRAV>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_TRACE_WAVES_PER_EU)))
void k_full_shadow(FrameParams P, int pass) {
  __shared__ WaveLds<TRAV, STATS> lds;
  const ListLane L = list_lane(P.counters[pass]);
  if (!L.any) return;
  const int wv = (int)uniform(threadIdx.x >> 6);
  const uint32_t pix = L.act ? (pass ? P.list1 : P.list0)[L.i] : 0u;
  const HitState hs = (pass ? P.state1 : P.state0)[pix];
  const f3 p{hs.px, hs.py, hs.pz};
  uint32_t cnt[ST_COUNT] = {};
  uint32_t bits = 0;
  for (int l = 0; l < P.n_lights; l++) {
    const f3 Ld = light_dir(p, frame_light(l));
    Ray sr;
    sr.o = offset(p, Ld, 0.003f);
    sr.d = Ld;
    sr.o2 = affv3(P.Minv, p);
    sr.d2 = normalized(m3v3(P.MS, Ld));
    setup_cull(sr, P.sc.static_pad);
    Hit hh{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
    bool blocked = false;
    if (STATS && L.act) cnt[ST_TOTAL]++;
    trace_full_ray<true, STATS, TRAV>(P.sc, sr, L.act, hh, blocked, lds, wv, cnt);
    bits |= (blocked ? 1u : 0u) << l;
  }
  if (L.act) (pass ? P.blk1 : P.blk0)[pix] = bits;
  if (STATS) flush_stats(P, cnt, lane_id());
}

// the reflection ray's closest hit (traceRay depth 1, flyscene.cpp:361-363) for the list0 pixels;
// per list wave the number of reflection hits (list1 compaction)
template <bool STATS, int TRAV>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_TRACE_WAVES_PER_EU)))
void k_full_refl(FrameParams P) {
  __shared__ WaveLds<TRAV, STATS> lds;
  const ListLane L = list_lane(P.counters[0]);
  if (!L.any) {
    if (L.w < P.n_waves_max && lane_id() == 0) P.wcount1[L.w] = 0;
    return;
  }
  const int wv = (int)uniform(threadIdx.x >> 6);
  const uint32_t pix = L.act ? P.list0[L.i] : 0u;
  const RayRec rq = P.refl[pix];
  Ray rr;
  rr.d = f3{rq.dx, rq.dy, rq.dz};
  rr.o = f3{rq.ox, rq.oy, rq.oz};
  rr.o2 = affv3(P.Minv, rr.o);
  rr.d2 = normalized(m3v3(P.MS, rr.d));
  setup_cull(rr, P.sc.static_pad);
  uint32_t cnt[ST_COUNT] = {};
  if (STATS && L.act) cnt[ST_TOTAL]++;
  Hit h1{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
  bool dummy = false;
  trace_full_ray<false, STATS, TRAV>(P.sc, rr, L.act, h1, dummy, lds, wv, cnt);
  if (L.act) P.hits1[pix] = make_uint2(__float_as_uint(h1.t), h1.slot);
  const uint32_t nh = (uint32_t)__popcll(ballot(L.act && h1.t != INFINITY));
  if (lane_id() == 0) P.wcount1[L.w] = nh;
  if (STATS) flush_stats(P, cnt, lane_id());
}

// reflection hit record -> hit point, interpolated normal, material for every list0 pixel; scatters
// the reflection-hit pixels into list1
__global__ __launch_bounds__(256) void k_full_gen1(FrameParams P) {
  const ListLane L = list_lane(P.counters[0]);
  if (!L.any) return;
  const uint32_t pix = L.act ? P.list0[L.i] : 0u;
  const uint2 hb = P.hits1[pix];
  const float t = L.act ? __uint_as_float(hb.x) : INFINITY;
  const uint64_t hm = ballot(t != INFINITY);
  if (t != INFINITY) P.list1[P.woff1[L.w] + lanes_below(hm)] = pix;
  if (!L.act) return;
  HitState hs = no_hit_state();
  if (t != INFINITY) {
    const RayRec rq = P.refl[pix];
    const TriRec64 tr1 = vload_tri(P.sc.tris, hb.y);
    HitInfo hi1;
    hi1.face = tr1.face;
    hi1.p = f3{rq.ox + t * rq.dx, rq.oy + t * rq.dy, rq.oz + t * rq.dz};
    hi1.n = hit_normal(P.sc, tr1, hb.y, hi1.p, hi1.mat);
    hs = to_state(hi1);
  }
  P.state1[pix] = hs;
}

// calculateColor (flyscene.cpp:603-614) with the shadow() outcomes already known (bit l: light l blocked)
__device__ __forceinline__ f3 calc_color_bits(const FrameParams& P, MatState& st, const HitInfo& hi, f3 o, bool lane_hit,
                                              uint32_t bits) {
  f3 sum{0.0f, 0.0f, 0.0f};
  for (int l = 0; l < P.n_lights; l++) {
    const Light lt = frame_light(l);
    const f3 L = light_dir(hi.p, lt);
    const bool blocked = (bits >> l) & 1u;
    f3 c{0.0f, 0.0f, 0.0f};
    if (lane_hit && !blocked) c = phong(P, st, hi, o, L, lt.c);
    sum = f3{sum.x + c.x, sum.y + c.y, sum.z + c.z};
  }
  return f3{clamp01(sum.x), clamp01(sum.y), clamp01(sum.z)};
}

// traceRay's colour composition (flyscene.cpp:327-370), the megakernel's tail
template <bool HITS>
__global__ __launch_bounds__(256) void k_full_final(FrameParams P) {
  const PixelCoord c = pixel_coord(P);
  if (!c.active) return;
  const size_t pix = pixel_index(P, c);
  const HitState s0 = P.state0[pix];
  const bool hit0 = s0.face != 0xFFFFFFFFu;
  MatState st = load_mat(P.defmat);
  const HitInfo hi0 = from_state(s0);
  const f3 eye{P.eye[0], P.eye[1], P.eye[2]};
  const f3 direct0 = calc_color_bits(P, st, hi0, eye, hit0, hit0 ? P.blk0[pix] : 0u);
  if (hit0 && hi0.mat != -1) st.ks = load_mat(P.sc.mats[hi0.mat]).ks;  // traceRay :355-358
  f3 refl{0.0f, 0.0f, 0.0f};
  // state1 / refl / blk1 exist only for primary-hit pixels (and blk1 only for reflection hits)
  const HitState s1 = hit0 ? P.state1[pix] : no_hit_state();
  const bool hit1 = hit0 && s1.face != 0xFFFFFFFFu;
  const HitInfo hi1 = from_state(s1);
  const RayRec rq = hit0 ? P.refl[pix] : RayRec{0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0u, 0u};
  const f3 direct1 = calc_color_bits(P, st, hi1, f3{rq.ox, rq.oy, rq.oz}, hit1, hit1 ? P.blk1[pix] : 0u);
  if (hit1) {
    if (hi1.mat != -1) st.ks = load_mat(P.sc.mats[hi1.mat]).ks;
    refl = f3{clamp01(direct1.x + 0.0f * st.ks.x), clamp01(direct1.y + 0.0f * st.ks.y),
              clamp01(direct1.z + 0.0f * st.ks.z)};
  }
  f3 col;
  if (hit0) {
    col = f3{clamp01(direct0.x + refl.x * st.ks.x), clamp01(direct0.y + refl.y * st.ks.y),
             clamp01(direct0.z + refl.z * st.ks.z)};
  } else {
    col = f3{P.bg[0], P.bg[1], P.bg[2]};
  }
  P.rgb[3 * pix + 0] = col.x;
  P.rgb[3 * pix + 1] = col.y;
  P.rgb[3 * pix + 2] = col.z;
  if (HITS) {
    P.face_out[pix] = hit0 ? (int32_t)s0.face : -1;
    P.t_out[pix] = __uint_as_float(P.hits[pix].x);
  }
}

// Ray-list kernels (rt_trace_closest / rt_trace_shadow), 64 rays per wave
template <bool ANY, int TRAV>
__global__ __launch_bounds__(256) void k_rays(FrameParams P, RayParams R) {
  __shared__ WaveLds<TRAV, false> lds;
  const int lane = threadIdx.x & 63;
  const int base = (int)uniform((blockIdx.x * 4 + (threadIdx.x >> 6)) * 64);
  if (base >= R.n) return;
  const int i = base + lane;
  const bool active = i < R.n;
  const int j = active ? i : base;
  Ray r;
  if (ANY) {  // shadow(P, L): triangle tests from P + 0.003 L, box tests from P (flyscene.cpp:512-519)
    const f3 p = ld3(R.o + 3 * (size_t)j), L = ld3(R.d + 3 * (size_t)j);
    r.o = offset(p, L, 0.003f);
    r.d = L;
    r.o2 = affv3(P.Minv, p);
  } else {
    r.o = ld3(R.o + 3 * (size_t)j);
    r.d = ld3(R.d + 3 * (size_t)j);
    r.o2 = affv3(P.Minv, r.o);
  }
  r.d2 = normalized(m3v3(P.MS, r.d));
  setup_cull(r, P.sc.static_pad);
  Hit h{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
  bool found = false;
  trace<ANY, false, TRAV>(P.sc, r, active, h, found, lds, (int)uniform(threadIdx.x >> 6), nullptr);
  if (!active) return;
  if (ANY) {
    R.blocked[i] = found ? 1 : 0;
  } else if (h.t != INFINITY) {
    const TriRec64 tr = vload_tri(P.sc.tris, h.slot);
    R.face[i] = (int32_t)tr.face;
    R.t[i] = h.t;
    const f3 p{r.o.x + h.t * r.d.x, r.o.y + h.t * r.d.y, r.o.z + h.t * r.d.z};
    if (R.P) {
      R.P[3 * (size_t)i + 0] = p.x;
      R.P[3 * (size_t)i + 1] = p.y;
      R.P[3 * (size_t)i + 2] = p.z;
    }
    if (R.N) {  // interpolateNormal(face, P) (flyscene.cpp:572-600)
      int32_t mat;
      const f3 nn = hit_normal(P.sc, tr, h.slot, p, mat);
      R.N[3 * (size_t)i + 0] = nn.x;
      R.N[3 * (size_t)i + 1] = nn.y;
      R.N[3 * (size_t)i + 2] = nn.z;
    }
  } else {
    R.face[i] = -1;
    R.t[i] = INFINITY;
    if (R.P) R.P[3 * (size_t)i] = R.P[3 * (size_t)i + 1] = R.P[3 * (size_t)i + 2] = 0.0f;
    if (R.N) R.N[3 * (size_t)i] = R.N[3 * (size_t)i + 1] = R.N[3 * (size_t)i + 2] = 0.0f;
  }
}

// traceRay(o, d, 0) (FULL, max_depth 2) for a list of rays (rt_trace_color): colour, first-hit face and t
template <int TRAV>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_FULL_WAVES_PER_EU)))
void k_rays_color(FrameParams P, RayParams R) {
  __shared__ WaveLds<TRAV, false> lds;
  const int lane = threadIdx.x & 63, wv = (int)uniform(threadIdx.x >> 6);
  const int base = (int)uniform((blockIdx.x * 4 + (threadIdx.x >> 6)) * 64);
  if (base >= R.n) return;
  const int i = base + lane;
  const bool active = i < R.n;
  const int j = active ? i : base;
  Ray r;
  r.o = ld3(R.o + 3 * (size_t)j);
  r.d = ld3(R.d + 3 * (size_t)j);
  r.o2 = affv3(P.Minv, r.o);
  r.d2 = normalized(m3v3(P.MS, r.d));
  setup_cull(r, P.sc.static_pad);
  Hit h;
  uint32_t face0;
  const f3 col = trace_full<false, TRAV>(P, r, active, lds, wv, nullptr, h, face0);
  if (!active) return;
  R.rgb[3 * (size_t)i + 0] = col.x;
  R.rgb[3 * (size_t)i + 1] = col.y;
  R.rgb[3 * (size_t)i + 2] = col.z;
  if (R.face) R.face[i] = face0 != 0xFFFFFFFFu ? (int32_t)face0 : -1;
  if (R.t) R.t[i] = h.t;
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
__global__ __launch_bounds__(256) void k_pack_shard(const float* rgb, uint8_t* out, int W, int H, int tiles_x,
                                                    int si, int sc, int n_tiles, int S) {
  const int L = blockIdx.x;  // one block per tile slot of the shard, one thread per pixel
  if (L >= n_tiles) return;
  int tx, ty;
  shard_tile_xy(tiles_x, S, si, sc, L, tx, ty);
  const int x = tx * 16 + (threadIdx.x & 15), y = ty * 16 + (threadIdx.x >> 4);
  uint8_t* o = out + ((size_t)L * 256 + threadIdx.x) * 3;
  if (x < W && y < H) {
    const float* c = rgb + 3 * ((size_t)y * W + x);
    o[0] = ppm_u8(c[0]);
    o[1] = ppm_u8(c[1]);
    o[2] = ppm_u8(c[2]);
  } else {
    o[0] = o[1] = o[2] = 0;
  }
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

__global__ void k_debug_math(int op, int n, int in_len, int out_len, const float* in, float* out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) debug_math_case(op, in + (size_t)k * in_len, out + (size_t)k * out_len);
}

// ------------------------------------------------------------------------------------------------
// Host glue
// ------------------------------------------------------------------------------------------------
template <typename T>
static int dalloc_copy(T** dst, const void* src, size_t bytes, int64_t& total) {
  *dst = nullptr;
  if (bytes == 0) bytes = 16;
  HIPCHECK(hipMalloc((void**)dst, bytes));
  total += (int64_t)bytes;
  if (src) HIPCHECK(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
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
  HIPCHECK(hipSetDevice(dev));
  s->device = dev;
  s->n_slots = std::max(1, std::min((int)s->opts.frames_in_flight, (int)rt_scene::kMaxSlots));
  for (int k = 0; k < s->n_slots; k++) {
    hipStream_t st;
    HIPCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    s->slots[k].stream = st;
  }
  s->stream = s->slots[0].stream;
  HostScene& hs = s->hs;
  int64_t& tot = s->device_bytes;
  tot = 0;
  int rc;
  s->static_pad = scene_static_pad(hs);
  s->cert_origin_max = cert_origin_max(hs);
  {
    // BVH nodes and triangle records share one allocation (triangles right after the nodes), so one
    // base plus a 32-bit byte offset reaches either: with RT_PREFETCH each uploaded node's pad0 / pad1
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
    std::vector<Node64> nodes(hs.nodes);
    if (RT_PREFETCH) {
      auto pf = [&](uint32_t c) -> uint32_t {
        return (uint32_t)(64 * (is_leaf(c) ? nn + leaf_first(c) : (size_t)c));
      };
      for (Node64& nd : nodes) {
        const uint32_t order = nd.pad0;  // octant_order() (rt_host.cpp), moved into the low offset bits
        nd.pad0 = pf(nd.child0) | (order & 0x3Fu);
        nd.pad1 = pf(nd.child1) | ((order >> 6) & 0x3u);
      }
    }
    if (RT_BYTE_HANDLES) {  // interior children as byte offsets of their records (node_offset)
      for (Node64& nd : nodes) {
        if (!is_leaf(nd.child0)) nd.child0 *= 64u;
        if (!is_leaf(nd.child1)) nd.child1 *= 64u;
      }
    }
    if (nn) HIPCHECK(hipMemcpy(s->d_nodes, nodes.data(), nn * 64, hipMemcpyHostToDevice));
    s->d_tris = reinterpret_cast<TriRec64*>(s->d_nodes + nn);
    if (nt) HIPCHECK(hipMemcpy(s->d_tris, hs.tris.data(), nt * 64, hipMemcpyHostToDevice));
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
      HIPCHECK(hipMemcpy(reinterpret_cast<char*>(s->d_nodes) + wide_base, wide.data(), wide_bytes, hipMemcpyHostToDevice));
    }
  }
  if ((rc = dalloc_copy(&s->d_nodes4, hs.nodes4.data(), hs.nodes4.size() * sizeof(Node4Q), tot))) return rc;
  {
    // per-slot shading record (float4 x 3), in the triangle records' (BVH leaf) order: the unit normals of
    // the slot's face's three vertices (Mesh normals as interpolateNormal normalises them,
    // flyscene.cpp:599) and the material id in the first .w. Indexed by slot, not face id, so a hit's two
    // gathers (triangle record, shading record) are independent and issue together.
    std::vector<float> fsh(12 * hs.tris.size(), 0.0f);
    for (size_t sl = 0; sl < hs.tris.size(); sl++) {
      const uint32_t f = hs.tris[sl].face;
      float* r = fsh.data() + 12 * sl;
      for (int k = 0; k < 3; k++) {
        const f3 n = hs.vnn[hs.fidx[3 * f + k]];
        r[4 * k] = n.x; r[4 * k + 1] = n.y; r[4 * k + 2] = n.z;
      }
      const int32_t m = hs.fmat[f];
      memcpy(&r[3], &m, 4);
    }
    if ((rc = dalloc_copy(&s->d_fshade, fsh.data(), fsh.size() * 4, tot))) return rc;
  }
  std::vector<float> rb(8 * hs.boxes.size());
  for (size_t b = 0; b < hs.boxes.size(); b++) {
    for (int k = 0; k < 3; k++) { rb[8 * b + k] = hs.boxes[b].low[k]; rb[8 * b + 4 + k] = hs.boxes[b].high[k]; }
  }
  if ((rc = dalloc_copy(&s->d_refbox, rb.data(), rb.size() * 4, tot))) return rc;
  std::vector<DevMat> dm(hs.mats.size());
  for (size_t m = 0; m < hs.mats.size(); m++) {
    DevMat& d = dm[m];
    memset(&d, 0, sizeof d);
    for (int k = 0; k < 3; k++) { d.ka[k] = hs.mats[m].ka[k]; d.kd[k] = hs.mats[m].kd[k]; d.ks[k] = hs.mats[m].ks[k]; }
    d.ns = hs.mats[m].shininess;
  }
  if ((rc = dalloc_copy(&s->d_mats, dm.data(), dm.size() * sizeof(DevMat), tot))) return rc;
  if ((rc = dalloc_copy(&s->d_stats, nullptr, kStatSlots * sizeof(unsigned long long), tot))) return rc;
  return RT_OK;
}

void device_release(rt_scene* s) {
  if (s->device == RT_DEVICE_NONE) return;
  (void)hipSetDevice(s->device);
  for (int k = 0; k < s->n_slots; k++)
    if (s->slots[k].stream) (void)hipStreamSynchronize((hipStream_t)s->slots[k].stream);
  void* bufs[] = {s->d_nodes, s->d_nodes4, s->d_fshade, s->d_refbox, s->d_mats, s->d_stats,
                  s->d_face_boxcolor};  // d_tris: inside d_nodes
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  for (int k = 0; k < s->n_slots; k++) {
    rt_scene::FrameSlot& f = s->slots[k];
    void* fb[] = {f.d_rgb, f.d_face, f.d_t, f.d_hits, f.d_rgb8, f.d_full, f.d_queue, f.d_timeline, f.d_cost, f.d_order};
    for (void* b : fb)
      if (b) (void)hipFree(b);
    if (f.stream) (void)hipStreamDestroy((hipStream_t)f.stream);
    f = rt_scene::FrameSlot{};
  }
  for (void* e : s->ev_pool) (void)hipEventDestroy((hipEvent_t)e);
  s->ev_pool.clear();
  s->stream = nullptr;
  s->d_face_boxcolor = nullptr;
  s->face_boxcolor_valid = false;
}

// RT_MODE_BOX_COLORS: (re)computes the per-face box-colour sums when the colours changed. The scene's
// streams are drained first (earlier box-colour frames in flight read the table).
static int ensure_face_boxcolor(rt_scene* s) {
  if (s->face_boxcolor_valid) return RT_OK;
  HostScene& hs = s->hs;
  if (s->box_colors.size() != 3 * hs.boxes.size()) {
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
  P.sc.root = (RT_BYTE_HANDLES && !is_leaf(hs.root)) ? hs.root * 64u : hs.root;
  P.sc.n_nodes = (int32_t)hs.nodes.size();
  P.sc.nodes4 = s->d_nodes4;
  P.sc.root4 = 0;
  P.sc.n_nodes4 = (int32_t)hs.nodes4.size();
  P.sc.static_pad = s->static_pad;
  P.sc.cert_origin_max = s->cert_origin_max;
  P.sc.wide_base = s->wide_base;
  P.sc.wide_copy_bytes = s->wide_copy_bytes;
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
template <bool STATS>
static void launch_trace(const FrameParams& P, int grid, hipStream_t st, int trav) {
  const dim3 g(grid * (4 / RT_TRACE_WPB)), b(64 * RT_TRACE_WPB);
  if (trav == TRAV_B2_VGPR) hipLaunchKernelGGL((k_trace_primary<STATS, TRAV_B2_VGPR>), g, b, 0, st, P);
  else if (trav == TRAV_B2_LDS) hipLaunchKernelGGL((k_trace_primary<STATS, TRAV_B2_LDS>), g, b, 0, st, P);
  else hipLaunchKernelGGL((k_trace_primary<STATS, TRAV_W4>), g, b, 0, st, P);
}
template <bool STATS, bool HITS>
static void launch_full(const FrameParams& P, int grid, hipStream_t st, int trav, bool small) {
  const dim3 g(grid * (4 / RT_FULL_WPB) + 3 * P.split_k), b(64 * RT_FULL_WPB);
  if (trav == TRAV_B2_VGPR) hipLaunchKernelGGL((k_render_full<STATS, HITS, TRAV_B2_VGPR>), g, b, 0, st, P);
  else if (trav == TRAV_B2_LDS && !STATS && small)
    hipLaunchKernelGGL((k_render_full<STATS, HITS, TRAV_B2_LDS, RT_FULL_WAVES_PER_EU_SMALL>), g, b, 0, st, P);
  else if (trav == TRAV_B2_LDS) hipLaunchKernelGGL((k_render_full<STATS, HITS, TRAV_B2_LDS>), g, b, 0, st, P);
  else hipLaunchKernelGGL((k_render_full<STATS, HITS, TRAV_W4>), g, b, 0, st, P);
}

template <bool STATS>
static void launch_shadow(const FrameParams& P, int g, hipStream_t st, int trav, int pass) {
  if (trav == TRAV_B2_VGPR) hipLaunchKernelGGL((k_full_shadow<STATS, TRAV_B2_VGPR>), dim3(g), dim3(256), 0, st, P, pass);
  else if (trav == TRAV_B2_LDS) hipLaunchKernelGGL((k_full_shadow<STATS, TRAV_B2_LDS>), dim3(g), dim3(256), 0, st, P, pass);
  else if (trav == TRAV_W4) hipLaunchKernelGGL((k_full_shadow<STATS, TRAV_W4>), dim3(g), dim3(256), 0, st, P, pass);
  else hipLaunchKernelGGL((k_full_shadow<STATS, TRAV_LANE>), dim3(g), dim3(256), 0, st, P, pass);
}
template <bool STATS>
static void launch_refl(const FrameParams& P, int g, hipStream_t st, int trav) {
  if (trav == TRAV_B2_VGPR) hipLaunchKernelGGL((k_full_refl<STATS, TRAV_B2_VGPR>), dim3(g), dim3(256), 0, st, P);
  else if (trav == TRAV_B2_LDS) hipLaunchKernelGGL((k_full_refl<STATS, TRAV_B2_LDS>), dim3(g), dim3(256), 0, st, P);
  else if (trav == TRAV_W4) hipLaunchKernelGGL((k_full_refl<STATS, TRAV_W4>), dim3(g), dim3(256), 0, st, P);
  else hipLaunchKernelGGL((k_full_refl<STATS, TRAV_LANE>), dim3(g), dim3(256), 0, st, P);
}

// traversal per FULL stage: packets for the coherent primary rays, per-lane walks for the rest unless
// the variant knob says otherwise (32: reflection, 64: shadows of reflection hits, 128: shadows of
// primary hits use packets when set... see kernel_variant)
template <bool STATS>
static void launch_full_pipeline(const FrameParams& P, int grid, hipStream_t st, int trav, int variant, bool hits,
                                 hipEvent_t ev_m) {
  const int q0 = 4 * grid;                    // primary waves (wcount0 entries)
  const int lgrid = (P.W * P.H + 255) / 256;  // list kernels: worst case, every pixel listed
  const int q1 = 4 * lgrid;                   // list waves (wcount1 entries)
  const int t_refl = (variant & 32) ? TRAV_LANE : trav;
  const int t_sh1 = (variant & 64) ? TRAV_LANE : trav;
  const int t_sh0 = (variant & 128) ? TRAV_LANE : trav;
  launch_trace<STATS>(P, grid, st, trav);  // + wcount0
  hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, st, (const uint32_t*)P.wcount0, P.woff0, q0, P.counters + 0);
  hipLaunchKernelGGL(k_full_gen0, dim3(grid), dim3(256), 0, st, P);  // state0, refl, list0
  launch_shadow<STATS>(P, lgrid, st, t_sh0, 0);
  launch_refl<STATS>(P, lgrid, st, t_refl);
  hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, st, (const uint32_t*)P.wcount1, P.woff1, q1, P.counters + 1);
  hipLaunchKernelGGL(k_full_gen1, dim3(lgrid), dim3(256), 0, st, P);  // state1, list1
  launch_shadow<STATS>(P, lgrid, st, t_sh1, 1);
  (void)hipEventRecord(ev_m, st);
  if (hits) hipLaunchKernelGGL(k_full_final<true>, dim3(grid), dim3(256), 0, st, P);
  else hipLaunchKernelGGL(k_full_final<false>, dim3(grid), dim3(256), 0, st, P);
}

static std::atomic<int> g_variant{-1};  // RT_KERNEL_VARIANT, or rt_debug_set_variant()
static int kernel_variant() {
  int v = g_variant.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("RT_KERNEL_VARIANT");
    int want = e ? atoi(e) : 0;
    want = want < 0 ? 0 : want;
    if (g_variant.compare_exchange_strong(v, want)) v = want;  // v: the value another thread set
  }
  return v;
}

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

extern "C" int rt_render_async(rt_scene* s, const rt_camera* cam, const rt_light* lights, int32_t n_lights,
                               const rt_frame* fr) {
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
  if (fr->flags & RT_FRAME_TIMELINE) {  // one record per one-wave block of the render kernel
    const size_t waves = units;
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
  if (fr->mode == RT_MODE_FULL && (variant & 16)) {
    if (sc > 1) { set_error("rt_render: the FULL stage-pipeline variant renders whole frames only"); return RT_ERR_UNSUPPORTED; }
    // sized by the 16x16-padded frame: every wave of the tile grid has a count slot
    const size_t npad = (size_t)P.tiles_x * 16 * (size_t)P.tiles_y * 16;
    if ((rc = ensure_full(slot, npad))) return rc;
    bind_full(slot, P);
  }
  // block order: chunked XCD order with runs of 64 blocks by default (measured -4% trace time on C3:
  // the quarters of a tile and their row neighbours share an XCD's L2); variant bits 512 / 1024 select
  // runs of 4 / 16 blocks, 1536 the plain dispatch order, 4 one contiguous tile range per XCD
  {
    const int sel = (variant >> 9) & 3;
    P.xcd_remap = (variant & 4) ? 1 : (sel == 0 ? 64 : sel == 1 ? 4 : sel == 2 ? 16 : 0);
  }
  const int trav = pick_trav(P, variant);
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
  bool alone = true;
  for (int k = 0; k < s->n_slots; k++)
    if (k != slot_id && s->slots[k].last_done && hipEventQuery((hipEvent_t)s->slots[k].last_done) == hipErrorNotReady)
      alone = false;
  const bool lpt = one_wave_kernel && !(variant & 131072) && P.xcd_remap >= 2 && grid > 0 && (alone || (variant & 524288));
  bool lpt_sort = false;
  if (lpt) {
    const size_t waves = units;
    if (waves > slot.order_waves) {
      HIPCHECK(hipStreamSynchronize(st));
      if (slot.d_cost) (void)hipFree(slot.d_cost);
      if (slot.d_order) (void)hipFree(slot.d_order);
      slot.d_cost = slot.d_order = nullptr;
      slot.order_waves = 0;
      slot.order_valid = false;
      HIPCHECK(hipMalloc((void**)&slot.d_cost, waves * 4));
      HIPCHECK(hipMalloc((void**)&slot.d_order, waves * 4));
      slot.order_waves = waves;
    }
    const int64_t key[8] = {fr->width, fr->height, si, sc, fr->mode, depth0, P.xcd_remap, (int64_t)waves};
    const bool same = slot.order_valid && memcmp(key, slot.order_key, sizeof key) == 0;
    if (same) P.order = slot.d_order;
    // the order is recomputed from this frame's costs after the frame when it is missing or has served
    // kLptRefresh frames (the sort costs a few microseconds on the frame's stream; a static or slowly
    // moving camera keeps its cost map)
    lpt_sort = !same || ++slot.order_age >= kLptRefresh;
    if (lpt_sort) {
      memcpy(slot.order_key, key, sizeof key);
      slot.order_valid = false;  // until this frame's k_order_lpt has been queued
      P.cost = slot.d_cost;
    }
  }
  if (s->ev_used + 3 > s->ev_pool.size()) {
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
      const dim3 g((unsigned)units), b(64);
      if (boxcol) {
        if (hits) hipLaunchKernelGGL((k_primary_dual<true, true>), g, b, 0, st, P);
        else hipLaunchKernelGGL((k_primary_dual<false, true>), g, b, 0, st, P);
      } else {
        if (hits) hipLaunchKernelGGL((k_primary_dual<true, false>), g, b, 0, st, P);
        else hipLaunchKernelGGL((k_primary_dual<false, false>), g, b, 0, st, P);
      }
      HIPCHECK(hipGetLastError());
      HIPCHECK(hipEventRecord(ev_m, st));
    } else if (prim && !stats && !(variant & (32768 | 256 | 2048)) && trav == TRAV_B2_LDS) {
      // lone frames of small scenes: the costliest waves as 16-lane sub-waves, as k_render_full does
      // (RT_SPLIT_KP waves)
      static const int split_p = [] { const char* e = getenv("RT_SPLIT_KP"); return e ? atoi(e) : kSplitKPrimary; }();
      const bool small_p = (s->hs.nodes.size() + s->hs.tris.size()) * 64 <= kFullSmallSceneBytes;
      P.split_k = (P.order && small_p && !P.timeline && RT_TRACE_WPB == 1)
                      ? std::max(0, std::min<int>(split_p, (int)(units / 4))) & ~7 : 0;
      if (P.cost && RT_SUBWAVE_COST == 3) P.split_k = 0;
      if (P.cost && P.split_k && (RT_SUBWAVE_COST == 1 || RT_SUBWAVE_COST == 2))
        HIPCHECK(hipMemsetAsync(P.cost, 0, units * 4, st));  // sub-waves add / take the max
      const dim3 g(grid * (4 / RT_TRACE_WPB) + 3 * P.split_k), b(64 * RT_TRACE_WPB);
      // RT_LDS_PAD (diagnostics): extra dynamic LDS per block, to cap the resident waves per CU in
      // occupancy experiments (160 KiB / (pad + 1 KiB) blocks per CU)
      static const unsigned lds_pad = [] { const char* e = getenv("RT_LDS_PAD"); return e ? (unsigned)atoi(e) : 0u; }();
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
      else if ((variant & 256) && trav == TRAV_B2_LDS)
        hipLaunchKernelGGL(k_trace_primary_x2, dim3(2 * grid), dim3(64), 0, st, P);
      else if ((variant & 2048) && trav == TRAV_B2_LDS && !P.wcount0) {
        if (!slot.d_queue) HIPCHECK(hipMalloc((void**)&slot.d_queue, 8 * sizeof(uint32_t)));
        HIPCHECK(hipMemsetAsync(slot.d_queue, 0, 8 * sizeof(uint32_t), st));
        int cus = 0;
        HIPCHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device));
        const int waves = std::min(4 * grid, std::max(8, cus * 4 * RT_TRACE_WAVES_PER_EU));
        // 4096: no stealing (each XCD's waves finish its own range; needs every XCD to get waves)
        hipLaunchKernelGGL(k_trace_primary_persistent, dim3(std::max(waves, 8)), dim3(64), 0, st, P, slot.d_queue,
                           (variant & 4096) ? 0u : 7u);
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
      static const int split_env = [] { const char* e = getenv("RT_SPLIT_K"); return e ? atoi(e) : kSplitK; }();
      if (P.order && small && !P.timeline && !stats && RT_FULL_WPB == 1 && trav == TRAV_B2_LDS)
        P.split_k = std::max(0, std::min<int>(split_env, (int)(units / 4))) & ~7;
      else
        P.split_k = 0;
      if (P.cost && RT_SUBWAVE_COST == 3) P.split_k = 0;
      if (P.cost && P.split_k && (RT_SUBWAVE_COST == 1 || RT_SUBWAVE_COST == 2))
        HIPCHECK(hipMemsetAsync(P.cost, 0, units * 4, st));  // sub-waves add / take the max
      if (stats) { if (hits) launch_full<true, true>(P, grid, st, trav, small); else launch_full<true, false>(P, grid, st, trav, small); }
      else { if (hits) launch_full<false, true>(P, grid, st, trav, small); else launch_full<false, false>(P, grid, st, trav, small); }
      HIPCHECK(hipEventRecord(ev_m, st));
    } else {
      if (stats) launch_full_pipeline<true>(P, grid, st, trav, variant, hits, ev_m);
      else launch_full_pipeline<false>(P, grid, st, trav, variant, hits, ev_m);
    }
    HIPCHECK(hipGetLastError());
  } else {
    HIPCHECK(hipEventRecord(ev_m, st));
  }
  if (lpt_sort) {  // the next frame of this shape on this slot dispatches longest-first
    hipLaunchKernelGGL(k_order_lpt, dim3(8), dim3(kLptThreads), 0, st, (const uint32_t*)slot.d_cost, slot.d_order,
                       (int)units, P.xcd_remap, (variant & 262144) ? 1 : 0);
    HIPCHECK(hipGetLastError());
    slot.order_valid = true;
    slot.order_age = 0;
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
  // primary rays of this shard: pixels inside the frame of the shard's tiles
  int64_t rays = 0;
  for (int L = 0; L < P.n_tiles_shard; L++) {
    int tx, ty;
    shard_tile_xy(P.tiles_x, P.super_tile, si, sc, L, tx, ty);
    if (tx < P.tiles_x && ty < P.tiles_y)
      rays += (int64_t)std::min(16, fr->width - tx * 16) * std::min(16, fr->height - ty * 16);
  }
  s->last_rays = rays;
  s->pending = true;
  return RT_OK;
}

extern "C" int rt_synchronize(rt_scene* s, rt_stats* out) {
  int rc = check_device_scene(s);
  if (rc) return rc;
  for (int k = 0; k < s->n_slots; k++) HIPCHECK(hipStreamSynchronize((hipStream_t)s->slots[k].stream));
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

extern "C" int rt_frame_download(rt_scene* s, int64_t capacity_pixels, float* rgb, int32_t* face, float* t) {
  int rc = check_device_scene(s);
  if (rc) return rc;
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
                       tiles_x, si, sc, n_tiles, S);
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
  if ((rc = rt_synchronize(s, stats))) return rc;
  if (!out_rgb) return RT_OK;
  const int W = fr->width, H = fr->height;
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
enum { Q_CLOSEST = 0, Q_SHADOW = 1, Q_COLOR = 2 };
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
  if (query == Q_COLOR) {
    if (w4) hipLaunchKernelGGL((k_rays_color<TRAV_W4>), dim3(grid), dim3(256), 0, st, P, R);
    else hipLaunchKernelGGL((k_rays_color<TRAV_B2_LDS>), dim3(grid), dim3(256), 0, st, P, R);
  } else if (w4) {
    if (query == Q_SHADOW) hipLaunchKernelGGL((k_rays<true, TRAV_W4>), dim3(grid), dim3(256), 0, st, P, R);
    else hipLaunchKernelGGL((k_rays<false, TRAV_W4>), dim3(grid), dim3(256), 0, st, P, R);
  } else {
    if (query == Q_SHADOW) hipLaunchKernelGGL((k_rays<true, TRAV_B2_LDS>), dim3(grid), dim3(256), 0, st, P, R);
    else hipLaunchKernelGGL((k_rays<false, TRAV_B2_LDS>), dim3(grid), dim3(256), 0, st, P, R);
  }
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipStreamSynchronize(st));
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
