// rt_variants.hip -- the A/B kernel variants of the MI355X ray-traversal library: alternatives measured
// against the product kernels and kept as tested options (every one renders the product's bits,
// tests/test_gpu_parity.py test_kernel_variants_render_identical_bits), built only into the variants
// library (`make variants` -> lib/librtamd_variants.so, selected with RTAMD_LIB). The product library
// (librtamd.so) does not contain them: its weak variant_launch refuses these variant bits.
//   1        binary tree with the wave stack in the lanes of one VGPR (generic loop)
//   2        quantised 4-wide nodes (Node4Q; traverse4)
//   16       FULL as a stage pipeline (k_trace_primary -> ... -> k_full_final); +32 / 64 / 128 per-lane
//            walks (traverse_lane) for the reflection / second / first shadow stage
//   256      two rays per lane (k_trace_primary_x2)
//   2048     persistent threads (k_trace_primary_persistent; +4096: no stealing)
//   1048576  two 8x8 packets per wave (dual-chain, k_primary_dual)
//   4194304  PRIMARY descent by a conservative frustum (interval) test of the packet (k_primary_frustum)
// Their measurements: DESIGN.md section 5 (the "Measured design decisions" table).
#include "rt_kernels.h"

namespace rt {

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
  if ((tr.box & kBoxCertBit) &&
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
  return inside || ref_box_test(P, r, bx);
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


// Persistent-threads form of k_trace_primary (A/B variant bit 2048): one launch of as many one-wave
// blocks as the device holds at 8 waves per SIMD; each wave repeatedly takes the next 8x8 work item
// from its XCD's counter (XCD x owns items [x Q/8, (x+1) Q/8) of the shard's Q = 4 * tiles items, so
// an XCD works through a contiguous band of tiles) and, once that range is exhausted, from the other
// XCDs' counters in turn. The next item's atomic is issued before the current item is traced, so its
// latency overlaps the traversal. Same per-pixel work and outputs as k_trace_primary.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kTraceWavesPerEu)))
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

constexpr int kDualWavesPerEu = 8, kX2WavesPerEu = 6;
// one 64-thread block per 16x8 half of a 16x16 tile (blocks 2t, 2t+1 cover tile t); lane (x, y) traces
// pixels (x, y) and (x + 8, y) of its half
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kX2WavesPerEu)))
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
  if (P.order != nullptr) {
    const uint32_t o = uniform(P.order[blockIdx.x]);
    bid = o < gridDim.x ? (int)o : (int)blockIdx.x;
  } else if (P.xcd_remap >= 2) {
    const int C = P.xcd_remap, G = 8 * C, full = ((int)gridDim.x / G) * G;
    if (bid < full) {
      const int x = ((bid & 7) + P.xcd_rot) & 7, k = bid >> 3;  // the product's band rotation (pixel_coord)
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
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kDualWavesPerEu)))
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
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kTraceWavesPerEu)))
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
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kTraceWavesPerEu)))
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


// ------------------------------------------------------------------------------------------------
// Host side of the variants
// ------------------------------------------------------------------------------------------------
template <bool STATS>
static void launch_trace_v(const FrameParams& P, int grid, hipStream_t st, int trav) {
  const dim3 g(grid * (4 / kTraceWPB)), b(64 * kTraceWPB);
  if (trav == TRAV_B2_VGPR) hipLaunchKernelGGL((k_trace_primary<STATS, TRAV_B2_VGPR>), g, b, 0, st, P);
  else if (trav == TRAV_B2_LDS) hipLaunchKernelGGL((k_trace_primary<STATS, TRAV_B2_LDS>), g, b, 0, st, P);
  else hipLaunchKernelGGL((k_trace_primary<STATS, TRAV_W4>), g, b, 0, st, P);
}
template <bool STATS, bool HITS>
static void launch_full_v(const FrameParams& P, int grid, hipStream_t st, int trav) {
  const dim3 g(grid * (4 / kFullWPB) + 3 * P.split_k), b(64 * kFullWPB);
  if (trav == TRAV_B2_VGPR) hipLaunchKernelGGL((k_render_full<STATS, HITS, TRAV_B2_VGPR>), g, b, 0, st, P);
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
  launch_trace_v<STATS>(P, grid, st, trav);  // + wcount0
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


bool variants_linked() { return true; }

int variant_launch(int op, const VariantCall& c) {
  const FrameParams& P = c.P;
  switch (op) {
    case VOP_TRACE_PRIMARY:
      if (c.stats) launch_trace_v<true>(P, c.grid, c.st, c.trav);
      else launch_trace_v<false>(P, c.grid, c.st, c.trav);
      break;
    case VOP_RENDER_FULL:
      if (c.stats) { if (c.hits) launch_full_v<true, true>(P, c.grid, c.st, c.trav); else launch_full_v<true, false>(P, c.grid, c.st, c.trav); }
      else { if (c.hits) launch_full_v<false, true>(P, c.grid, c.st, c.trav); else launch_full_v<false, false>(P, c.grid, c.st, c.trav); }
      break;
    case VOP_FULL_PIPELINE:
      if (c.stats) launch_full_pipeline<true>(P, c.grid, c.st, c.trav, c.variant, c.hits, c.ev_m);
      else launch_full_pipeline<false>(P, c.grid, c.st, c.trav, c.variant, c.hits, c.ev_m);
      break;
    case VOP_PRIMARY_DUAL: {
      const dim3 g((unsigned)c.units), b(64);
      if (c.boxcol) {
        if (c.hits) hipLaunchKernelGGL((k_primary_dual<true, true>), g, b, 0, c.st, P);
        else hipLaunchKernelGGL((k_primary_dual<false, true>), g, b, 0, c.st, P);
      } else {
        if (c.hits) hipLaunchKernelGGL((k_primary_dual<true, false>), g, b, 0, c.st, P);
        else hipLaunchKernelGGL((k_primary_dual<false, false>), g, b, 0, c.st, P);
      }
      break;
    }
    case VOP_PRIMARY_X2:
      hipLaunchKernelGGL(k_trace_primary_x2, dim3(2 * c.grid), dim3(64), 0, c.st, P);
      break;
    case VOP_PRIMARY_PERSISTENT: {
      int cus = 0;
      HIPCHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c.device));
      const int waves = std::min(4 * c.grid, std::max(8, cus * 4 * kTraceWavesPerEu));
      // 4096: no stealing (each XCD's waves finish its own range; needs every XCD to get waves)
      hipLaunchKernelGGL(k_trace_primary_persistent, dim3(std::max(waves, 8)), dim3(64), 0, c.st, P, c.queue,
                         (c.variant & 4096) ? 0u : 7u);
      break;
    }
    case VOP_RAYS:
      if (c.query == Q_COLOR) hipLaunchKernelGGL((k_rays_color<TRAV_W4>), dim3(c.grid), dim3(256), 0, c.st, P, c.R);
      else if (c.query == Q_SHADOW) hipLaunchKernelGGL((k_rays<true, TRAV_W4>), dim3(c.grid), dim3(256), 0, c.st, P, c.R);
      else hipLaunchKernelGGL((k_rays<false, TRAV_W4>), dim3(c.grid), dim3(256), 0, c.st, P, c.R);
      break;
    default:
      set_error("variant_launch: unknown op %d", op);
      return RT_ERR_INVALID;
  }
  HIPCHECK(hipGetLastError());
  return RT_OK;
}

}  // namespace rt
