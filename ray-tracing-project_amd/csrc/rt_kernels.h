// rt_kernels.h -- the gfx950 device code of the MI355X ray-traversal hot path, shared by the product
// library's kernels (rt_device.hip) and the A/B kernel variants (rt_variants.hip, `make variants`).
//
// Hot path (reference: src/flyscene.cpp:299-614):
//   one wave = one 8x8 pixel tile, one ray per lane; rays generated in registers (traceRayThread +
//   Camera::screenToWorld, fp64 NDC as camera.hpp:159-162);
//   wave-packet BVH traversal: every node record is fetched once per wave with a scalar load
//   (s_load_dwordx16 of the 64-B node), each lane slab-tests both children, the wave descends by
//   ballot (near child from the node's order bit for the wave's direction octant) and keeps ONE
//   traversal stack for the wave in LDS; lanes that cannot improve their hit simply vote "no", so the
//   wave stays converged and only visits nodes some lane still needs;
//   triangle test = the reference's calculateDistance/interpolateNormal arithmetic bit for bit
//   (flyscene.cpp:444-478,572-600), tie-break by reference iteration rank (calculateMinimumFace
//   keeps the first minimum, flyscene.cpp:381-391), plus the reference's own object-space box test
//   (intersectBox, flyscene.cpp:484-507) for the candidate's reference box;
//   shading = calculateColor/calcSingleColor (flyscene.cpp:542-614); FULL mode adds the shadow any-hit
//   per light (flyscene.cpp:510-526) and the one reflection bounce of traceRay (flyscene.cpp:317-371).
// No MFMA: there is no dense contraction in this path.
#pragma once
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
// handles keep the (first triangle, count) form.
__device__ __forceinline__ uint32_t node_index(uint32_t h) { return h >> 6; }
__device__ __forceinline__ uint32_t node_offset(uint32_t h) { return h; }
__device__ __forceinline__ Node64 sload_node(const Node64* base, uint32_t h) { return sload64(base, node_index(h)); }
// The node fetch of the production loop, then a prefetch of both children's records into the scalar
// cache, issued the moment the node has arrived so that it overlaps this node's box tests (one dword
// each pulls in the 64-B line). The child offsets come from the record's own registers (Node64::pad0 /
// pad1, words 14 / 15 of the x16 load: the children's node records or, for a leaf child, its first
// triangle record, device_upload). The prefetch sinks pf0 / pf1 are carried from the previous node step
// ("+s"): this load's own s_waitcnt retires the previous step's prefetches, so a step needs no wait of
// its own (the caller waits once at the end of the traversal). The ray's reciprocal direction, passed
// through the prefetch asm as a read-write operand (a loop-carried copy, no move), keeps the box tests
// below it.
// Prefetch-offset check of the RT_CHECK_PREFETCH debug build (`make pfcheck`, DESIGN.md section 5 "scalar
// prefetch offsets"): an offset at or above its limit is recorded in bit `site` of *check and replaced by 0
// (a valid record), so a GPU run of the test suite with that build shows that no product loop issues an
// out-of-range scalar load -- without faulting the GPU. The product build compiles this to the offset.
__device__ __forceinline__ uint32_t pf_off(uint32_t off, uint32_t limit, uint32_t* check, int site) {
#ifdef RT_CHECK_PREFETCH
  if (off >= limit) {
    atomicOr(check, 1u << site);  // (a vector atomic from every active lane)
    return 0u;
  }
#endif
  (void)limit, (void)check, (void)site;
  return off;
}
__device__ __forceinline__ Node64 sload_node_pf_inreg(const DevScene& P, uint32_t h, uint32_t& pf0, uint32_t& pf1,
                                                      f3& id) {
  const uint32_t off = pf_off(node_offset(__builtin_amdgcn_readfirstlane(h)), P.rec_bytes, P.pf_check, 0);
  const uint64_t b = (uint64_t)P.nodes;
  const uint64_t bs = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  i16v v;
  asm volatile("s_load_dwordx16 %0, %3, %4\n\ts_waitcnt lgkmcnt(0)" : "=&s"(v), "+s"(pf0), "+s"(pf1) : "s"(bs), "s"(off) : "memory");
  Node64 r;
  __builtin_memcpy(&r, &v, 64);
  asm volatile("s_load_dword %0, %5, %6\n\ts_load_dword %1, %5, %7"
               : "+s"(pf0), "+s"(pf1), "+v"(id.x), "+v"(id.y), "+v"(id.z)
               : "s"(bs), "s"(pf_off(r.pad0, P.rec_bytes, P.pf_check, 1)), "s"(pf_off(r.pad1, P.rec_bytes, P.pf_check, 2))
               : "memory");
  return r;
}
__device__ __forceinline__ TriRec64 sload_tri(const TriRec64* base, uint32_t i) { return sload64(base, i); }
__device__ __forceinline__ uint32_t uniform(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }
// The lane id recomputed where it is needed (v_mbcnt; volatile, so the compiler cannot reuse the entry's
// thread id and keep it live across the traversal -- in the FULL megakernel that value was spilled).
__device__ __forceinline__ uint32_t lane_id_fresh() {
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// counters of the RT_FRAME_STATS counting run
// ST_WPOP / ST_WCULL (counting run, closest hit): stack pops per wave, and those pops at which no lane
// that wanted the entry still could (every such lane's entry distance into it, recorded at the push,
// now beyond its closest hit) -- what culling at the pop would save (rt_debug_counters)
// ST_WWIDE: 128-B fp32 4-wide node records fetched per wave (ST_WNODE: 64-B binary / quantised records)
// ST_WCAND / ST_WPRE / ST_WINS (counting run, per wave-level triangle test): some lane passed the plane-
// distance stage; some candidate lane's hit point lies inside the triangle's bounding box grown by 1e-3 of
// its extent (what a box prefilter would keep); some lane passed the reference's edge tests. ST_WE1 / ST_WE2:
// the staged edge tests left no candidate after the first / the second edge
enum { ST_NODE = 0, ST_TRI, ST_WNODE, ST_WTRI, ST_RAYS, ST_HITS, ST_TOTAL, ST_WPOP, ST_WCULL, ST_WWIDE,
       ST_WCAND, ST_WPRE, ST_WINS, ST_WE1, ST_WE2,
       // round 4: the same triangle-stage counts with the candidates restricted to the lanes whose ray entered
       // the leaf's box (ST_WCANDM .. ST_WINSM), the triangle tests of leaves reached by descent (ST_WTRID) and
       // their entry-masked candidate count (ST_WCANDD: popped leaves unmasked), and wave-level tests where a
       // lane that never entered the leaf accepted (ST_WACCX: 0 if leaf-entry masking is exact)
       ST_WCANDM, ST_WE1M, ST_WE2M, ST_WINSM, ST_WTRID, ST_WCANDD, ST_WACCX,
       // round 5: the packet -> per-lane hybrid model. ST_HN0 .. ST_HN0 + 6: node steps
       // by the number of lanes whose ray entered the node (bins 0, 1, 2-3, 4-7, 8-15, 16-31, 32-64);
       // ST_HL0 .. + 6: the same for leaf visits. Per threshold k of kHybridK (3 thresholds): once the lanes
       // entering a node fall below k, that node's subtree is a "switched region" (it ends at the first
       // pop below the depth where it began); ST_HPN/ST_HPT + i: the packet's node steps / triangle tests
       // inside such regions, ST_HLN/ST_HLT + i: the per-lane cost of the same regions (the maximum over the
       // wave's lanes of the steps / tests whose node the lane entered, summed over regions) -- what a wave
       // walking those regions one ray per lane would spend
       ST_HN0, ST_HL0 = ST_HN0 + 7, ST_HPN = ST_HL0 + 7, ST_HPT = ST_HPN + 3, ST_HLN = ST_HPT + 3, ST_HLT = ST_HLN + 3,
       // round 6: the FULL megakernel's packet walks by phase p (0 primary, 1 shadows of the
       // primary hits, 2 reflection, 3 shadows of the reflection hits): walks with some active lane (ST_PW + p), the
       // active lanes at their entry summed (ST_PL + p), their node steps (ST_PS + p) and triangle tests (ST_PT + p);
       // ST_PH + b: the secondary phases' node steps by the walk's active lanes at entry (1-8, 9-16, 17-32, 33-48,
       // 49-64)
       ST_PW = ST_HLT + 3, ST_PL = ST_PW + 4, ST_PS = ST_PL + 4, ST_PT = ST_PS + 4, ST_PH = ST_PT + 4,
       ST_COUNT = ST_PH + 5 };
constexpr int kStatSlots = 80;
static_assert(ST_COUNT <= kStatSlots, "stat slots");
constexpr int kHybridK[3] = {4, 8, 16};
__device__ __forceinline__ int lane_bin(uint32_t n) { return n == 0 ? 0 : n == 1 ? 1 : n < 4 ? 2 : n < 8 ? 3 : n < 16 ? 4 : n < 32 ? 5 : 6; }
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off, 64));
  return v;
}

struct Hit {
  float t;
  uint32_t rank;
  uint32_t slot;
};

struct Ray {
  f3 o, d;      // world space (triangle tests)
  f3 id;        // culling: 1/d (zeros nudged)
  f3 oa, ob;    // culling: -(o + p)/d and -(o - p)/d, the lo / hi plane offsets of boxes grown by p
  f3 o2;        // object space (reference intersectBox): Minv*o_box; its direction normalized(MS*d) is
                // formed where the exact box test needs it (ref_box_test), off the traversal's registers
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
constexpr float kCullPadRel = 4e-5f, kCullOriginMax = 1e18f, kCullDirMin = 1e-12f, kCullDirMax = 1e18f;
// The ray's own pad is needed only once it exceeds the static one (every box already carries
// static_pad >= the ray's pad, so the same ~100x margin holds): for origins near the scene -- every
// secondary ray, and primary rays of an eye near it -- the boxes keep exactly their static size.
__device__ __forceinline__ void setup_cull(Ray& r, float static_pad) {
  const float om = fmaxf(fmaxf(fabsf(r.o.x), fabsf(r.o.y)), fabsf(r.o.z));
  const float dm = fmaxf(fmaxf(fabsf(r.d.x), fabsf(r.d.y)), fabsf(r.d.z));
  const bool certified = om <= kCullOriginMax && dm >= kCullDirMin && dm <= kCullDirMax;  // false for NaN
  if (certified) {
    r.id = f3{__builtin_amdgcn_rcpf(nudge(r.d.x)), __builtin_amdgcn_rcpf(nudge(r.d.y)),
              __builtin_amdgcn_rcpf(nudge(r.d.z))};
    const float pr = kCullPadRel * om;
    const float p = pr > static_pad ? pr : 0.0f;
    r.oa = f3{-(r.o.x + p) * r.id.x, -(r.o.y + p) * r.id.y, -(r.o.z + p) * r.id.z};
    r.ob = f3{-(r.o.x - p) * r.id.x, -(r.o.y - p) * r.id.y, -(r.o.z - p) * r.id.z};
  } else {
    // unbounded boxes: lo planes at -inf, hi planes at +inf along the (kept) direction signs
    r.id = f3{copysignf(1.0f, nudge(r.d.x)), copysignf(1.0f, nudge(r.d.y)), copysignf(1.0f, nudge(r.d.z))};
    r.oa = f3{-r.id.x * INFINITY, -r.id.y * INFINITY, -r.id.z * INFINITY};
    r.ob = f3{r.id.x * INFINITY, r.id.y * INFINITY, r.id.z * INFINITY};
  }
}

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
// values -- identical results with 8 fewer min/max per child. OCT < 0: the generic test. (An unclipped
// entry distance for packets starting in front of the scene measured within noise, r03_micro_ab.txt.)
template <int OCT>
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
  s.tmin = fmaxf(fmaxf(__builtin_fmaf(nx, r.id.x, nox), __builtin_fmaf(ny, r.id.y, noy)),
                 fmaxf(__builtin_fmaf(nz, r.id.z, noz), 0.0f));
  // min of the three far planes and tmax_ray in two instructions (the compiler's fminf would first
  // canonicalise tmax_ray, a loop-carried value, with an extra v_max per node)
  asm("v_min3_f32 %0, %1, %2, %3\n\tv_min_f32 %0, %0, %4"
      : "=&v"(s.tmax)
      : "v"(__builtin_fmaf(fx, r.id.x, fox)), "v"(__builtin_fmaf(fy, r.id.y, foy)),
        "v"(__builtin_fmaf(fz, r.id.z, foz)), "v"(tmax_ray));
  return s;
}
// lane masks straight from v_cmp (no bool materialisation): llvm.amdgcn.fcmp predicates
constexpr int kFcmpOLE = 5;
__device__ __forceinline__ uint64_t mask_le(float a, float b) { return __builtin_amdgcn_fcmpf(a, b, kFcmpOLE); }

// The reference's object-space box test, exact (flyscene.cpp:484-507): origin Minv*o (Ray::o2), direction
// (MS*d).normalized() with MS the linear block of Minv (flyscene.cpp:486-487; m3v3's Matrix3f order)
__device__ __forceinline__ bool ref_box_test(const DevScene& S, const Ray& r, const float* bx) {
  const float MS[9] = {S.Minv[0], S.Minv[1], S.Minv[2], S.Minv[4], S.Minv[5], S.Minv[6], S.Minv[8], S.Minv[9], S.Minv[10]};
  const f3 dd = normalized(m3v3(MS, r.d));
  const float lo[3] = {bx[0], bx[1], bx[2]}, hi[3] = {bx[4], bx[5], bx[6]};
  const float o2[3] = {r.o2.x, r.o2.y, r.o2.z}, d2[3] = {dd.x, dd.y, dd.z};
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
  if (tr.box & kBoxCertBit) {
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
  return cand & (ins | ballot(ref_box_test(P, r, bx)));
}

// calculateDistance (flyscene.cpp:444-478) against a wave-uniform triangle record, for the lanes of
// `act`. CLOSEST: update (t, rank, slot) if 0 <= t < best (rank breaks ties as the reference's order
// does). ANY: any valid t >= 0 (shadow(), flyscene.cpp:519).
template <bool ANY, bool STATS = false>
__device__ __forceinline__ void test_tri(const DevScene& P, const TriRec64& tr, uint32_t slot, const Ray& r,
                                         uint64_t act, Hit& h, bool& found, uint32_t* cnt = nullptr,
                                         uint64_t entry = ~0ull, bool desc = false) {
  const f3 n{tr.nx, tr.ny, tr.nz};
  const float dn = dot(n, r.d);                 // facenormal.dot(dir)
  const float orth = tr.dist - dot(r.o, n);     // distancePlane - origin.dot(facenormal)
  const float t = orth / dn;                    // / dir.dot(facenormal)  (same bits as dn)
  uint64_t cand;
  if (!ANY) {
    // dn != 0 && 0 <= t < inf in one class test: t is -0, +0, +denormal or +normal (dn == 0 makes t
    // +-inf or NaN, which the class excludes as the separate tests did)
    uint64_t cls;
    asm("v_cmp_class_f32_e64 %0, %1, %2" : "=s"(cls) : "v"(t), "v"(0x1E0u));
    cand = act & cls &
           (fmask<kFcmpOLT>(t, h.t) | (fmask<kFcmpOEQ>(t, h.t) & __builtin_amdgcn_uicmp(tr.rank, h.rank, kIcmpULT)));
  } else {
    cand = act & fmask<kFcmpUNE>(dn, 0.0f) & fmask<kFcmpOGE>(t, 0.0f);
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
  // the record is wave-uniform (SGPRs) and a VALU op reads at most one SGPR: w0 and w1 copied into
  // VGPRs once serve all three edge differences (6 moves instead of 9; same float operations)
  f3 v0 = w0, v1 = w1;
  asm("" : "+v"(v0.x), "+v"(v0.y), "+v"(v0.z), "+v"(v1.x), "+v"(v1.y), "+v"(v1.z));
  const f3 e0 = sub(w1, v0), e1 = sub(w2, v1), e2 = sub(v0, w2);
  // the reference's three edge tests are independent (interpolateNormal, flyscene.cpp:591: rejected if any is
  // negative), so they run one at a time and the wave stops as soon as no candidate lane is left --
  // the same values, the same set; a packet wholly beyond one edge line skips the other edges' work
  const f3 a0 = cross(e0, sub(p, w0));
  cand &= ~ballot(dot(n, a0) < 0);
  if (STATS) cnt[ST_WE1] += cand == 0;
  if (cand == 0) return;
  const f3 a1 = cross(e1, sub(p, w1));
  cand &= ~ballot(dot(n, a1) < 0);
  if (STATS) cnt[ST_WE2] += cand == 0;
  if (cand == 0) return;
  const f3 a2 = cross(e2, sub(p, w2));
  cand &= ~ballot(dot(n, a2) < 0);
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
// Wave-packet loop with every option: VGPR or LDS stack and the counting run (RT_FRAME_STATS). The
// production closest-hit / any-hit path is traverse_fast() below (same visit order, leaner per-node
// code); this loop serves the counting run and the VGPR-stack A/B variant (rt_variants.hip). Octant-
// specialised loops take the near child from the node's precomputed order bit for the wave's octant
// (split-axis rule, octant_order() in rt_host.cpp) instead of a lane-majority vote: 3 fewer SALU and one
// fewer v_cmp per node step (C3 +3.7% at 4 frames in flight, bunny +2.6%).
// Node64::pad0 / pad1 hold the children's record offsets (multiples of 64, the prefetch targets), so the
// eight octant order bits travel in their low bits: octants 0-5 in pad0 bits 0-5, octants 6-7 in pad1
// bits 0-1. A scalar load ignores the two low offset bits and the rest stays inside the 64-B record,
// so the prefetch still touches the child's cache line.
template <int OCT>
__device__ __forceinline__ uint32_t order_word(const Node64& nd) {
  return OCT < 6 ? nd.pad0 : nd.pad1;
}
template <int OCT>
constexpr int order_bit() {
  return OCT < 6 ? OCT : OCT - 6;
}
template <bool ANY, bool STATS, bool STACK_LDS, int OCT = -1>
__device__ __forceinline__ void traverse(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                         uint32_t* lds_stack, uint32_t* cnt) {
  if (P.n_nodes == 0) return;
  uint32_t stackv = 0;     // lane k holds stack entry k (VGPR stack)
  int sp = 0;              // wave-uniform stack depth (SGPR)
  uint64_t flagstack = 0;  // STATS: per-lane "my ray wanted this entry" bit per stack level
  float tstack[STATS ? 64 : 1];  // STATS: per-lane entry distance into each stack entry
  bool want = active;      // STATS: this lane's ray intersects the current node
  bool desc = false;       // STATS: the current node was reached by descent (not popped)
  uint32_t node = P.root;
  const float tmax_any = INFINITY;
  uint64_t act = ballot(active);  // lanes still tracing (wave-uniform mask)
  // STATS, hybrid model (ST_HPN ..): per threshold, the stack depth where the current switched region began
  // (-1: none) and this lane's node steps / triangle tests inside it
  int hr[3] = {-1, -1, -1};
  uint32_t hln[3] = {0, 0, 0}, hlt[3] = {0, 0, 0};
  auto hybrid_close = [&](int depth) {  // regions that began deeper than `depth` end here
#pragma unroll
    for (int i = 0; i < 3; i++)
      if (hr[i] >= 0 && depth < hr[i]) {
        cnt[ST_HLN + i] += wave_max_u32(hln[i]);
        cnt[ST_HLT + i] += wave_max_u32(hlt[i]);
        hln[i] = hlt[i] = 0;
        hr[i] = -1;
      }
  };
  // one pop site and branch-free pushes keep the per-node control flow to the two uniform branches
  // (interior vs leaf, pop vs descend)
  for (;;) {
    bool pop = true;
    if (STATS) {
      const uint32_t nw = (uint32_t)__popcll(ballot(want) & act);
      cnt[(is_leaf(node) ? ST_HL0 : ST_HN0) + lane_bin(nw)]++;
#pragma unroll
      for (int i = 0; i < 3; i++) {
        if (hr[i] < 0 && nw < (uint32_t)kHybridK[i]) hr[i] = sp;
        if (hr[i] >= 0) {
          if (!is_leaf(node)) {
            cnt[ST_HPN + i]++;
            hln[i] += want ? 1u : 0u;
          } else {
            cnt[ST_HPT + i] += leaf_count(node);
            hlt[i] += want ? leaf_count(node) : 0u;
          }
        }
      }
    }
    if (!is_leaf(node)) {
      const Node64 nd = sload_node(P.nodes, node);  // one scalar 64-B fetch per wave
      if (STATS) {
        if (want) cnt[ST_NODE]++;
        cnt[ST_WNODE]++;
      }
      const float tcut = ANY ? tmax_any : h.t;
      const Span s0 = slab_o<OCT>(nd.c0lx, nd.c0hx, nd.c0ly, nd.c0hy, nd.c0lz, nd.c0hz, r, tcut);
      const Span s1 = slab_o<OCT>(nd.c1lx, nd.c1hx, nd.c1ly, nd.c1hy, nd.c1lz, nd.c1hz, r, tcut);
      const uint64_t m0 = mask_le(s0.tmin, s0.tmax) & act, m1 = mask_le(s1.tmin, s1.tmax) & act;
      bool first0;
      if (OCT >= 0) {
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
        const bool h0 = (m0 >> lane_id()) & 1, h1 = (m1 >> lane_id()) & 1;
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
        hybrid_close(sp);  // the popped entry lies outside regions that began deeper than it
      }
    }
  }
  if (STATS) hybrid_close(-1);
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

// Leaf entry of the binary loops: touch the leaf's triangle records [from, count) (one s_load_dword per 64-B
// record into a prefetch sink; the parent's prefetch already brought record 0), so that their scalar-cache
// misses overlap one another and the first record's instead of following each test (C5 +4%, C3 unchanged:
// profiles/ab/r04_leaf_prefetch_ab.txt). The wide loop's parent prefetch covers records 0 and 1 already.
__device__ __forceinline__ void leaf_prefetch(const DevScene& P, uint64_t bs, uint32_t first, uint32_t from, uint32_t count,
                                              uint32_t& sink) {
  for (uint32_t k = from; k < count; k++)
    asm volatile("s_load_dword %0, %1, %2" : "+s"(sink) : "s"(bs), "s"(pf_off((first + k) * 64u, P.tri_bytes, P.pf_check, 3))
                 : "memory");
}

// the fast loop's wave-stack push as inline asm: a ds_write issued where it stands (the compiler would
// otherwise schedule the store with the decision block at the end of the step)
__device__ __forceinline__ void lds_push(uint32_t* slot, uint32_t v) {
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)slot;
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
// traverse_fast from a given state (node handle, stack depth): the whole traversal starts at the root
// with an empty stack. Per node step (octant loops): the node record arrives with one s_load_dwordx16;
// the same asm then prefetches both children's records into the scalar cache (offsets in the record's
// pad0 / pad1), the sinks carried to the next step, whose own wait retires them; the far child (fixed
// by the node's order bit for this octant) is pushed at once; both slab tests give the lane masks; an
// 8-SALU block picks the next node (near child, the one child needed, or the pop marker) and keeps the
// push only when both children are needed.
template <bool ANY, int OCT>
__device__ __forceinline__ void traverse_fast_from(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                                   uint32_t* lds_stack, uint32_t node, int sp) {
  // lanes still tracing: used by the any-hit triangle tests only (a closest-hit lane without a ray
  // carries t_best = -1, which no candidate t >= -0 passes, so its triangle tests need no mask)
  uint64_t act = ANY ? ballot(active) : ~0ull;
  float tlim = active ? INFINITY : -1.0f;  // ANY: box-test limit (-1 once the lane is blocked)
  if (!ANY && !active) h.t = -1.0f;
  uint32_t cpf0 = 0, cpf1 = 0;  // prefetch sinks, live across the traversal
  f3 rid = r.id;  // loop-carried copy threaded through the prefetch asm
  for (;;) {
    while (!is_leaf(node)) {
      const Node64 nd = sload_node_pf_inreg(P, node, cpf0, cpf1, rid);
      // octant loops: when both children are needed the far one is fixed by the node's order bit for
      // this octant alone, so it is chosen and pushed the moment the node has arrived -- the LDS write
      // completes under the box tests instead of delaying the next node fetch
      uint32_t nearb = 0, farb = 0;
      if (OCT >= 0) {
        sp = (int)uniform((uint32_t)sp);
        asm("s_bitcmp1_b32 %[bits], %[oct]\n\t"
            "s_cselect_b32 %[nb], %[c1], %[c0]\n\t"
            "s_cselect_b32 %[fb], %[c0], %[c1]"
            : [nb] "=&s"(nearb), [fb] "=&s"(farb)
            : [bits] "s"(uniform(order_word<OCT>(nd))), [oct] "i"(order_bit<OCT>()), [c0] "s"(uniform(nd.child0)),
              [c1] "s"(uniform(nd.child1))
            : "scc");
        lds_push(lds_stack + sp, farb);
      }
      const float tcut = ANY ? tlim : h.t;
      Ray rb = r;
      rb.id = rid;
      const Span s0 = slab_o<OCT>(nd.c0lx, nd.c0hx, nd.c0ly, nd.c0hy, nd.c0lz, nd.c0hz, rb, tcut);
      const Span s1 = slab_o<OCT>(nd.c1lx, nd.c1hx, nd.c1ly, nd.c1hy, nd.c1lz, nd.c1hz, rb, tcut);
      const uint64_t m0 = mask_le(s0.tmin, s0.tmax), m1 = mask_le(s1.tmin, s1.tmax);
      uint32_t nxt, far, ta, tb;
      uint64_t tt;
      // (uniform(): inside FULL mode's divergent regions the compiler may otherwise hand the scalar
      // decision block values it keeps in VGPRs; readfirstlane folds away on SGPR values)
      sp = (int)uniform((uint32_t)sp);
      const uint32_t c0 = uniform(nd.child0), c1 = uniform(nd.child1);
      uint32_t* const slot = lds_stack + sp;
      if (OCT >= 0) {
        // both needed: the near child chosen above; one needed: that one; none: the pop marker.
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
        far = farb;
        (void)ta;
        (void)tb;
      } else {
        // mixed-octant packets: near child by lane majority -- each lane that needs a child votes for
        // the one it enters first (v0: lanes voting child 0; 2 * |v0| >= |m0 | m1| picks child 0, which
        // also covers m1 == 0); the far child is written above the top unconditionally and kept only
        // when both are needed
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
      node = nxt;
    }
    if (node != kPopMarker) {
      // leaf: its triangles are fetched once per wave and tested by every lane
      const uint32_t first = leaf_first(node), count = leaf_count(node);
      {
        const uint64_t b = (uint64_t)P.tris;
        const uint64_t bs = ((uint64_t)uniform((uint32_t)(b >> 32)) << 32) | (uint32_t)uniform((uint32_t)b);
        leaf_prefetch(P, bs, first, 1, count, cpf0);
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
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::"s"(cpf0), "s"(cpf1) : "memory");  // the last prefetches landed
  if (!ANY && !active) h.t = INFINITY;
}

template <bool ANY, int OCT>
__device__ __forceinline__ void traverse_fast(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                              uint32_t* lds_stack) {
  if (P.n_nodes == 0) return;
  traverse_fast_from<ANY, OCT>(P, r, active, h, found, lds_stack, P.root, 0);
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

// The production form (octant loops, no counting): node fetch + the prefetch of the nearest child's
// record (both 64-B halves; the measured best of five prefetch forms, profiles/ab/r03_wide_tree_ab.txt),
// the four slab tests, and the decision as one SALU block interleaved with the four stack writes.
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
  uint32_t node = uniform(P.wide_base + (uint32_t)OCT * P.wide_copy_bytes);
  Ray rr = r;
  // the node loop is rotated: the record load that follows a descent sits at the end of the loop body
  // and a separate copy serves the entry after a pop, so a wait the compiler needs after the leaf path
  // (its kernel-argument reloads) stays on that path instead of heading every node step
  auto load = [&](uint32_t off, i16v& lo, i16v& hi) {
    off = pf_off(off, P.all_bytes - 127u, P.pf_check, 5);
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
      asm volatile("s_load_dword %[k], %[b], %[p0]\n\ts_load_dword %[k], %[b], %[p0] offset:0x40"
                   : [k] "+&s"(sink), "+v"(rr.id.x), "+v"(rr.id.y), "+v"(rr.id.z)
                   : [b] "s"(bs), [p0] "s"(pf_off(uniform(nd.pf[0]), P.all_bytes - 64u, P.pf_check, 4))
                   : "memory");
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
  if (!ANY && !active) h.t = INFINITY;
}

// Traversal flavours: binary nodes with the LDS wave stack (the product), and the A/B flavours of
// rt_variants.hip (binary nodes with a VGPR-lane stack, the quantised 4-wide nodes, per-lane walks)
enum { TRAV_B2_VGPR = 0, TRAV_B2_LDS = 1, TRAV_W4 = 2, TRAV_LANE = 3 };

template <int TRAV, bool STATS>
struct WaveLds {
  // binary LDS-stack kernels also run the fp32 4-wide loops (traverse_wide*): kStackW entries
  static constexpr int kEntries = TRAV == TRAV_W4 ? kStack4 : (TRAV == TRAV_LANE ? 1 : (TRAV == TRAV_B2_LDS ? kStackW : 64));
  uint32_t stack[4][kEntries];
  uint64_t mask[4][(STATS && (TRAV == TRAV_W4 || TRAV == TRAV_B2_LDS)) ? kEntries : 1];
  uint32_t clk[4];  // one-wave kernels: the wave's start clocks (wave_clock_start), kept out of registers
};

// the A/B traversal flavours, defined in rt_variants.hip (instantiated only there)
template <bool ANY, bool STATS>
__device__ __forceinline__ void traverse4(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                          uint32_t* lds_stack, uint64_t* lds_mask, uint32_t* cnt);
template <bool ANY, bool STATS>
__device__ __forceinline__ void traverse_lane(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                              uint32_t* cnt);

template <bool ANY, bool STATS, int TRAV>
__device__ __forceinline__ void trace(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                      WaveLds<TRAV, STATS>& L, int wv, uint32_t* cnt) {
  if constexpr (TRAV == TRAV_W4) traverse4<ANY, STATS>(P, r, active, h, found, L.stack[wv], L.mask[STATS ? wv : 0], cnt);
  else if constexpr (TRAV == TRAV_LANE) traverse_lane<ANY, STATS>(P, r, active, h, found, cnt);
  else if constexpr (!STATS && TRAV == TRAV_B2_LDS) traverse_fast<ANY, -1>(P, r, active, h, found, L.stack[wv]);
  else traverse<ANY, STATS, TRAV == TRAV_B2_LDS>(P, r, active, h, found, L.stack[wv], cnt);
}

// Packet traversal specialised by the wave's direction octant when every active ray shares it (coherent
// camera / reflection packets): loops compiled for that octant (known near / far planes, order bits);
// mixed-octant waves take the generic loop.
// WIDE: packets whose rays share an octant walk the fp32 4-wide tree when the scene has one
// (traverse_wide_fast; the counting run traverse_wide); mixed-octant packets keep the binary loop.
// SPLIT (FULL mode's secondary packets, small-scene build): a packet whose rays span several direction
// octants is walked once per octant present, each walk with that octant's lanes only (ballot masks) and
// the octant loop's cheaper slab test, instead of one generic walk of the union; a one-octant packet is
// the loop's single iteration. Each lane is traced by exactly one walk, so results are unchanged.
template <bool ANY, bool STATS, int TRAV, bool WIDE = false, bool SPLIT = false>
__device__ __forceinline__ void trace_oct(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                          WaveLds<TRAV, STATS>& L, int wv, uint32_t* cnt) {
  if (SPLIT && !STATS && TRAV == TRAV_B2_LDS) {
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
  if (TRAV == TRAV_B2_LDS || TRAV == TRAV_B2_VGPR) {
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
      if (!STATS && SL) {
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
  trace<ANY, STATS, TRAV>(P, r, active, h, found, L, wv, cnt);
}
template <bool STATS, int TRAV, bool WIDE = false>
__device__ __forceinline__ void trace_closest_oct(const DevScene& P, const Ray& r, bool active, Hit& h,
                                                  WaveLds<TRAV, STATS>& L, int wv, uint32_t* cnt) {
  bool found = false;
  trace_oct<false, STATS, TRAV, WIDE, false>(P, r, active, h, found, L, wv, cnt);
}
// incoherent FULL-mode packets (the generic loop)
template <bool ANY, bool STATS, int TRAV>
__device__ __forceinline__ void trace_full_ray(const DevScene& P, const Ray& r, bool active, Hit& h, bool& found,
                                               WaveLds<TRAV, STATS>& L, int wv, uint32_t* cnt) {
  trace<ANY, STATS, TRAV>(P, r, active, h, found, L, wv, cnt);
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
      setup_cull(sr, P.sc.static_pad);
      Hit hh{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
      if (STATS && lane_hit) cnt[ST_TOTAL]++;
      if (OCTSH)
        trace_oct<true, STATS, TRAV, false, SPLIT>(P.sc, sr, lane_hit, hh, blocked, *lds, wv, cnt);
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

// WPB = waves per block: 4 (one 256-thread block per 16x16 tile) or 1 (one 64-thread block per 8x8
// quarter, blocks 4t..4t+3 cover tile t; finer-grained dispatch, same pixels and shard assignment)
template <int WPB = 4>
__device__ __forceinline__ PixelCoord pixel_coord(const FrameParams& P) {
  PixelCoord c;
  c.lane = threadIdx.x & 63;
  int nb, b;
  int bid = (int)blockIdx.x;
  c.sub = -1;
  if (WPB == 1 && P.order != nullptr) {
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
      const int x = ((bid & 7) + P.xcd_rot) & 7, k = bid >> 3;
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
  setup_cull(r, P.sc.static_pad);
  return r;
}

// RT_FRAME_TIMELINE: the wave's start / end clocks and where it ran (diagnostics; one uniform branch
// when off). HW_ID / XCC_ID via s_getreg (hwreg ids 4 and 20, all 32 bits).
// The start clocks go to the wave's LDS words rather than staying live in registers for the whole
// kernel (the FULL megakernel's allocation tips into heavy spilling otherwise).
// A kernel argument read at this point of the kernel: the offset passes through an empty asm, so the load
// cannot be hoisted to the kernel's start and its value is not held in registers before it is needed
template <typename T>
__device__ __forceinline__ T late_kernarg(size_t off) {
  uint32_t o = (uint32_t)off;
  asm volatile("" : "+s"(o));
  typedef const __attribute__((address_space(4))) char* KArg;
  const KArg base = (KArg)__builtin_amdgcn_kernarg_segment_ptr();
  return *reinterpret_cast<const __attribute__((address_space(4))) T*>(base + o);
}

__device__ __forceinline__ void wave_clock_start(const FrameParams& P, uint32_t* clk) {
  if (P.timeline || P.cost) {
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
      clk[0] = (uint32_t)t0;
      clk[1] = (uint32_t)(t0 >> 32);
      clk[2] = r0;
    }
  }
}
// tprim (PRIMARY / FULL frame kernels): each lane's primary hit distance (INFINITY: missed or inactive), stored to
// LDS right after the primary hit -- one ds_write per lane, no branch, nothing held in registers -- for a moving
// camera's prediction below (FrameParams::pred)
__device__ __forceinline__ void wave_clock_end(const FrameParams& P, const uint32_t* clk, int lane, int qw,
                                               bool sub_wave = false, const float* tprim = nullptr) {
  if (!P.timeline && !P.cost) return;
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  struct { uint64_t t0; uint32_t r0; } w;
  w.t0 = (uint64_t)uniform(clk[0]) | ((uint64_t)uniform(clk[1]) << 32);
  w.r0 = uniform(clk[2]);
  // this wave's cost for the next frame's dispatch order. The four 16-lane sub-waves of a split wave
  // (sub_wave) write the maximum of their times into the wave's slot, which the host cleared before such
  // a frame: a split wave's cost is re-measured like every other wave's, so one whose
  // work has become cheap leaves the split range (profiles/ab/r03_subwave_cost_ab.txt: the sum ranks the
  // split waves far above the rest and coarsens the order's buckets, -20% on C5 lone frames; keeping the
  // stale cost is within 1% of the maximum but never refreshes it; running cost-recording frames unsplit
  // costs 6%)
  if (P.cost && lane == 0) {
    const uint64_t dt = t1 - w.t0;
    const uint32_t c = dt > 0x3FFFFFFFull ? 0x3FFFFFFFu : (uint32_t)dt;
    if (!sub_wave) P.cost[qw] = c;
    else atomicMax(P.cost + qw, c);
  }
  // a moving camera: lane i raises the map at the i-th wave around the wave's footprint (whole frames: tile qw / 4
  // sits at (tile % tiles_x, tile / tiles_x), its quarters 2 x 2 waves). The fields are read here, from the
  // kernel arguments (late_kernarg), so nothing of this stays live through the traversal: read through P, the
  // compiler loaded them at the kernel's start and held them in SGPRs, spilling more of the kernel's SGPRs to
  // VGPR lanes (C2 with frames in flight -4..-8%, round 6)
  uint32_t* const dil = late_kernarg<uint32_t*>(offsetof(FrameParams, cost_dil));
  if (dil) {
    const uint64_t dt = t1 - w.t0;
    const uint32_t c = dt > 0x3FFFFFFFull ? 0x3FFFFFFFu : (uint32_t)dt;
    const int r = late_kernarg<int32_t>(offsetof(FrameParams, dil_r));
    const int tx = late_kernarg<int32_t>(offsetof(FrameParams, tiles_x)), ty = late_kernarg<int32_t>(offsetof(FrameParams, tiles_y));
    const int t = qw >> 2, q = qw & 3;
    // the wave's pixel origin: its own, or where a moving camera's prediction (FrameParams::pred) expects its
    // content in the next frame -- one hit lane's primary hit (lane 36, the wave's centre, when it hit, else the
    // first hit lane): t along its view-space direction (a px + b, c py + e, -1) (the camera is rigid, so t is a
    // view-space distance), moved by the camera's last step (pred_step: a translation in view space, as the
    // reference's WASD keys make it) and projected back to a pixel; its own when no lane hit
    float ox = (float)(((t % tx) * 2 + (q & 1)) * 8), oy = (float)(((t / tx) * 2 + (q >> 1)) * 8);
    const uint64_t hb = (tprim && late_kernarg<int32_t>(offsetof(FrameParams, pred)))
                            ? ballot(reinterpret_cast<const volatile float*>(tprim)[lane] != INFINITY) : 0;
    if (hb != 0) {
      const int rep = ((hb >> 36) & 1) ? 36 : (int)__builtin_ctzll(hb);
      const float th = reinterpret_cast<const volatile float*>(tprim)[rep];
      const size_t po = offsetof(FrameParams, pred_proj), so = offsetof(FrameParams, pred_step);
      const float a = late_kernarg<float>(po), b = late_kernarg<float>(po + 4), cc = late_kernarg<float>(po + 8),
                  e = late_kernarg<float>(po + 12);
      const float dx = a * (ox + (float)(rep & 7)) + b, dy = cc * (oy + (float)(rep >> 3)) + e;
      const float k = th / sqrtf(dx * dx + dy * dy + 1.0f);
      const float qx = dx * k + late_kernarg<float>(so), qy = dy * k + late_kernarg<float>(so + 4),
                  qz = late_kernarg<float>(so + 8) - k;
      if (qz < 0.0f) {
        const float sx = (qx / -qz - b) / a - (float)(rep & 7), sy = (qy / -qz - e) / cc - (float)(rep >> 3);
        if (sx > -8.0f && sy > -8.0f && sx < 16.0f * (float)tx && sy < 16.0f * (float)ty) {
          ox = sx;
          oy = sy;
        }
      }
    }
    // the waves the 8 x 8 footprint at (ox, oy) overlaps (1 x 1 at the wave's own position, up to 2 x 2 when
    // predicted) take its full cost, a ring of r waves around them 3/4 of it (dil_w: the ring's shift, 2 = 3/4, 1 =
    // 1/2): where the camera stands still the costliest waves still rank first (and take the split), where it
    // moves their neighbours rank next
    const int x0 = (int)floorf(ox * 0.125f), y0 = (int)floorf(oy * 0.125f);
    const int fw = ox * 0.125f != (float)x0 ? 2 : 1, fh = oy * 0.125f != (float)y0 ? 2 : 1;
    const int dw = fw + 2 * r, dh = fh + 2 * r;
    if (lane < dw * dh) {
      const int i = lane % dw, j = lane / dw, x = x0 - r + i, y = y0 - r + j;
      const bool inner = i >= r && i < r + fw && j >= r && j < r + fh;
      const uint32_t v = inner ? c : c - (c >> late_kernarg<int32_t>(offsetof(FrameParams, dil_w)));
      if (x >= 0 && y >= 0 && x < 2 * tx && y < 2 * ty)
        atomicMax(dil + 4 * ((y >> 1) * tx + (x >> 1)) + (y & 1) * 2 + (x & 1), v);
    }
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

// RT_FRAME_WAVE_STATS: this wave's own counts (PRIMARY: node steps, triangle tests, hit lanes; FULL: node steps of
// the four phases, then their triangle tests), for the per-wave time breakdown (tools/wave_breakdown.py)
__device__ __forceinline__ void wave_stats_out(const FrameParams& P, const uint32_t* cnt, int lane, int qw, bool full) {
  if (!P.wave_stats || lane != 0) return;
  uint32_t* o = P.wave_stats + 8 * (size_t)qw;
  if (full) {
    for (int p = 0; p < 4; p++) { o[p] = cnt[ST_PS + p]; o[4 + p] = cnt[ST_PT + p]; }
  } else {
    o[0] = cnt[ST_WNODE]; o[1] = cnt[ST_WTRI]; o[2] = cnt[ST_HITS]; o[3] = 0;
    o[4] = o[5] = o[6] = o[7] = 0;
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


// PRIMARY stage 1: closest hit per pixel (calculateMinimumFace, flyscene.cpp:373-396) -> 8-B hit record.
// Only traversal state is live here, so the kernel fits 8 waves per SIMD.
constexpr int kTraceWavesPerEu = 8;  // 8 waves/SIMD: measured +2.5% over the 7 the register count allows
constexpr int kTraceWPB = 1;  // waves per block of the traversal kernel (4 or 1; 1 measured 3% faster)
template <bool STATS, int TRAV>
__global__ __launch_bounds__(64 * kTraceWPB) __attribute__((amdgpu_waves_per_eu(kTraceWavesPerEu)))
void k_trace_primary(FrameParams P) {
  __shared__ WaveLds<TRAV, STATS> lds;
  const PixelCoord c = pixel_coord<kTraceWPB>(P);
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
  if (STATS) {
    if (P.wave_stats) {  // the wave's hit lanes (ST_HITS counts per lane)
      uint32_t w[ST_COUNT];
      for (int k = 0; k < ST_COUNT; k++) w[k] = cnt[k];
      w[ST_HITS] = (uint32_t)__popcll(ballot(c.active && h.t != INFINITY));
      wave_stats_out(P, w, c.lane, c.qw, false);
    }
    flush_stats(P, cnt, c.lane);
  }
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


// PRIMARY as one kernel (default; variant bit 32768 selects the two-kernel form k_trace_primary +
// k_shade_primary): the traversal, then the shading of the same lane -- the hit record stays in
// registers instead of a round trip through HBM, and the traversal state is dead by then, so the
// shading's registers do not add to the traversal's. Resources of the shipped instantiation
// k_primary_fused<false, false> (make asm -> build/asm/resource.txt, round 5): 59 VGPR, 78 SGPR, no
// scratch, 8 waves/SIMD. Measured: C3 +2.7% at 4 frames in flight, bunny +4%.
template <bool HITS, bool BOXCOL = false>
__global__ __launch_bounds__(64 * kTraceWPB) __attribute__((amdgpu_waves_per_eu(kTraceWavesPerEu)))
void k_primary_fused(FrameParams P) {
  __shared__ WaveLds<TRAV_B2_LDS, false> lds;
  __shared__ float tprim[64];  // the lanes' primary hit distances (wave_clock_end's prediction)
  wave_clock_start(P, lds.clk);
  const PixelCoord c = pixel_coord<kTraceWPB>(P);
  // the eye (every primary ray's origin) held in VGPRs: origin.dot(facenormal) in each triangle test
  // then reads one SGPR per op and needs no moves
  Ray r = primary_ray(P, c.px, c.py);
  asm("" : "+v"(r.o.x), "+v"(r.o.y), "+v"(r.o.z));
  Hit h{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
  trace_closest_oct<false, TRAV_B2_LDS, true>(P.sc, r, c.active, h, lds, c.slot, nullptr);
  tprim[c.lane] = h.t;  // (INFINITY for a miss or an inactive lane)
  if (c.active) shade_primary_pixel<HITS, BOXCOL>(P, r, (size_t)c.py * P.W + c.px, h.t, h.slot);
  wave_clock_end(P, lds.clk, c.lane, c.qw, c.sub >= 0, tprim);
}

// FULL: the reference traceRay as-is (max_depth 2): shadow any-hit per light and one reflection
// bounce, all in one kernel (flyscene.cpp:317-371, 510-566, 603-614).
// traceRay(o, d, 0) with max_depth 2 (FULL, flyscene.cpp:317-371): primary hit, per-light shadows, one
// reflection bounce with its own shadows. Shared by the frame megakernel and the ray-list colour query.
// Returns the colour; h0 / face0: the first hit (t, face id).
// SPLIT: mixed-octant secondary packets walk once per octant (trace_oct); the small-scene build only --
// measured C5 +1.5% at 4 frames in flight, +1..3% one at a time, the 1M soup in FULL -5%
// (profiles/ab/r03_full_split_oct_ab.txt)
// counting run: one phase's packet walk(s) of a wave (ST_PW ..)
struct PhaseMark {
  uint32_t n0, t0;
};
template <bool STATS>
__device__ __forceinline__ PhaseMark phase_begin(const uint32_t* cnt) {
  if (!STATS) return PhaseMark{0, 0};
  return PhaseMark{cnt[ST_WNODE], cnt[ST_WTRI]};
}
template <bool STATS>
__device__ __forceinline__ void phase_end(uint32_t* cnt, int p, const PhaseMark& m, bool act) {
  if (!STATS) return;
  const uint64_t b = ballot(act);
  if (b == 0) return;
  const uint32_t lanes = (uint32_t)__popcll(b), steps = cnt[ST_WNODE] - m.n0;
  cnt[ST_PW + p]++;
  cnt[ST_PL + p] += lanes;
  cnt[ST_PS + p] += steps;
  cnt[ST_PT + p] += cnt[ST_WTRI] - m.t0;
  if (p > 0) cnt[ST_PH + (lanes <= 8 ? 0 : lanes <= 16 ? 1 : lanes <= 32 ? 2 : lanes <= 48 ? 3 : 4)] += steps;
}

template <bool STATS, int TRAV, bool SPLIT = false>
__device__ __forceinline__ f3 trace_full(const FrameParams& P, const Ray& r, bool active, WaveLds<TRAV, STATS>& lds, int wv,
                                         uint32_t* cnt, Hit& h, uint32_t& face0, float* tprim = nullptr) {
  h = Hit{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
  bool dummy = false;
  // the primary packet is coherent: octant-specialised loops
  PhaseMark pm = phase_begin<STATS>(cnt);
  trace_oct<false, STATS, TRAV>(P.sc, r, active, h, dummy, lds, wv, cnt);
  phase_end<STATS>(cnt, 0, pm, active);
  const bool hit0 = active && h.t != INFINITY;
  if (STATS && hit0) cnt[ST_HITS]++;
  if (tprim) tprim[lane_id()] = hit0 ? h.t : INFINITY;

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
  pm = phase_begin<STATS>(cnt);
  const f3 direct0 = calc_color<true, STATS, TRAV, true, SPLIT>(P, st, hi0, r.o, hit0, &lds, wv, cnt);
  phase_end<STATS>(cnt, 1, pm, hit0);
  if (hit0 && hi0.mat != -1) st.ks = load_mat(P.sc.mats[hi0.mat]).ks;  // traceRay :355-358

  // reflect(dir.normalized(), interpolateNormal(...)), offset 0.001 (flyscene.cpp:361-363)
  f3 refl{0.0f, 0.0f, 0.0f};
  Ray rr;
  rr.d = reflect(normalized(r.d), hi0.n);
  rr.o = offset(hi0.p, rr.d, 0.001f);
  rr.o2 = affv3(P.Minv, rr.o);
  setup_cull(rr, P.sc.static_pad);
  if (STATS && hit0) cnt[ST_TOTAL]++;
  Hit h1{INFINITY, 0xFFFFFFFFu, 0xFFFFFFFFu};
  pm = phase_begin<STATS>(cnt);
  trace_oct<false, STATS, TRAV, false, SPLIT>(P.sc, rr, hit0, h1, dummy, lds, wv, cnt);
  phase_end<STATS>(cnt, 2, pm, hit0);
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
  pm = phase_begin<STATS>(cnt);
  const f3 direct1 = calc_color<true, STATS, TRAV, true, SPLIT>(P, st, hi1, rr.o, hit1, &lds, wv, cnt);
  phase_end<STATS>(cnt, 3, pm, hit1);
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

// Occupancy of the FULL megakernel, by scene: 8 waves per SIMD for scenes whose node + triangle records
// exceed the chip's aggregate L2 (the 1M soup: 8 waves beat 5 by 18% and 3 by 24% -- the traversal waits
// on L2 misses and needs the waves), a 6-wave bound for smaller ones (bunny, C5: +14% over 8 -- their
// records are L2-resident). Resources of the shipped instantiations (make asm, round 5, after the pixel
// coordinates moved to LDS): k_render_full<false, false, 1, 6> 80 VGPR, 104 SGPR, no scratch (round 4: 80
// VGPR + 32 B of scratch -- the spill of the thread id and px / py); <false, false, 1, 8> 64 VGPR + 96 B
// scratch. Re-swept in round 5 without the spill: 5 waves (85 VGPR, no scratch) -1..-6%, 7 waves (72 VGPR +
// 48 B scratch) -3..-8% against 6 (profiles/ab/r05_full_waves_ab.txt).
#ifndef RT_FULL_WPE_SMALL  // A/B builds only (make ablib EXTRA=-DRT_FULL_WPE_SMALL=n)
#define RT_FULL_WPE_SMALL 6
#endif
constexpr int kFullWavesPerEu = 8, kFullWavesPerEuSmall = RT_FULL_WPE_SMALL;
constexpr size_t kFullSmallSceneBytes = 32u << 20;  // 8 XCDs x 4 MiB L2
// waves per block of the FULL megakernel (1: one 8x8 wave per block, measured +6.5% on bunny FULL and +8%
// on the soup over 4 = one 16x16 tile per block)
constexpr int kFullWPB = 1;
template <bool STATS, bool HITS, int TRAV, int WPE = kFullWavesPerEu>
__global__ __launch_bounds__(64 * kFullWPB) __attribute__((amdgpu_waves_per_eu(WPE)))
void k_render_full(FrameParams P) {
  static_assert(kFullWPB == 1, "the pixel words below are per one-wave block");
  __shared__ WaveLds<TRAV, STATS> lds;
  // the lane's pixel (x, y; x = ~0 when inactive), parked in LDS across the traversal and re-read by a
  // freshly computed lane id at the end: held in registers, the thread id and the pixel coordinates were
  // spilled to scratch (16 B per lane written at every pixel: ~33 MB of HBM writes per 1080p frame
  // against the 24.9 MB frame itself)
  __shared__ uint32_t pix_xy[2][64];
  __shared__ float tprim[64];  // the lanes' primary hit distances (wave_clock_end's prediction)
  wave_clock_start(P, lds.clk);
  const PixelCoord c = pixel_coord<kFullWPB>(P);
  const bool active = c.active;
  pix_xy[0][c.lane] = active ? (uint32_t)c.px : 0xFFFFFFFFu;
  pix_xy[1][c.lane] = (uint32_t)c.py;
  uint32_t cnt[ST_COUNT] = {};
  const Ray r = primary_ray(P, c.px, c.py);
  if (STATS && active) { cnt[ST_RAYS]++; cnt[ST_TOTAL]++; }

  Hit h;
  uint32_t face0;
  const f3 col = trace_full<STATS, TRAV, WPE == kFullWavesPerEuSmall>(P, r, active, lds, c.slot, cnt, h, face0, tprim);
  const bool hit0 = face0 != 0xFFFFFFFFu;
  const uint32_t lane = lane_id_fresh();
  const uint32_t px = reinterpret_cast<volatile uint32_t*>(pix_xy[0])[lane];
  const uint32_t py = reinterpret_cast<volatile uint32_t*>(pix_xy[1])[lane];
  if (px != 0xFFFFFFFFu) {
    const size_t pix = (size_t)py * P.W + px;
    P.rgb[3 * pix + 0] = col.x;
    P.rgb[3 * pix + 1] = col.y;
    P.rgb[3 * pix + 2] = col.z;
    if (HITS) {
      P.face_out[pix] = hit0 ? (int32_t)face0 : -1;
      P.t_out[pix] = h.t;
    }
  }
  if (STATS) {
    wave_stats_out(P, cnt, (int)lane, c.qw, true);
    flush_stats(P, cnt, (int)lane);
  }
  wave_clock_end(P, lds.clk, (int)lane, c.qw, c.sub >= 0, tprim);
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
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kFullWavesPerEuSmall)))
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
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kFullWavesPerEu)))
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



// ------------------------------------------------------------------------------------------------
// The A/B kernel variants (RT_KERNEL_VARIANT bits, rt_debug_set_variant) live in rt_variants.hip and are
// linked only into the variants library (`make variants` -> lib/librtamd_variants.so): the product
// library's weak default of variant_launch() refuses them with RT_ERR_UNSUPPORTED.
// ------------------------------------------------------------------------------------------------
enum RayQuery { Q_CLOSEST = 0, Q_SHADOW = 1, Q_COLOR = 2 };  // rt_trace_closest / _shadow / _color
enum VariantOp {
  VOP_TRACE_PRIMARY = 0,  // k_trace_primary with a non-default traversal flavour (c.trav)
  VOP_RENDER_FULL,        // k_render_full with a non-default traversal flavour
  VOP_FULL_PIPELINE,      // the FULL stage pipeline (variant bit 16; 32 / 64 / 128 per-lane stages)
  VOP_PRIMARY_DUAL,       // two 8x8 packets per wave (variant bit 1048576)
  VOP_PRIMARY_X2,         // two rays per lane (variant bit 256)
  VOP_PRIMARY_PERSISTENT, // persistent threads (variant bit 2048; 4096: no stealing)
  VOP_RAYS,               // ray-list queries with a non-default traversal flavour
};
struct VariantCall {
  FrameParams P;
  RayParams R;
  int grid = 0, trav = 0, variant = 0, query = 0, device = 0;
  size_t units = 0;
  bool stats = false, hits = false, boxcol = false, small = false;
  hipStream_t st = nullptr;
  hipEvent_t ev_m = nullptr;
  uint32_t* queue = nullptr;  // persistent threads' work counters (8 words)
};
int variant_launch(int op, const VariantCall& c);
bool variants_linked();

}  // namespace rt
