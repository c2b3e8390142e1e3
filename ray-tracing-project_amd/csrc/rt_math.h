// rt_math.h -- float arithmetic in the reference's (Eigen 3.3.7) evaluation order, shared by the
// host scene preparation and the gfx950 kernels. Every function is a single fixed sequence of IEEE
// fp32 operations; the build disables FMA contraction (-ffp-contract=off) and keeps hipcc's default
// correctly rounded fp32 division and square root, so host and device produce identical bits.
//
// Order pinned by tests/golden/eigen_kat.bin (generated from the reference's vendored Eigen):
//   size-3 reductions   x0 + (x1 + x2)          Eigen/src/Core/Redux.h:96-110 (halving unroller)
//   Affine3f * Vector3f ((m0 v0 + m1 v1) + m2 v2) + t   Geometry/Transform.h:1372-1392 (4x4 packet)
//   cross               OrthoMethods.h:43-47
//   normalized          x / sqrt(|x|^2) if |x|^2 > 0 else x   Dot.h:124-134
//   std::min/std::max   b<a?b:a / a<b?b:a  (NaN-propagating the reference's way, never v_min/v_max)
#pragma once
#include <cmath>
#include <cstdint>

#if defined(__HIPCC__) || defined(__HIP__)
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD inline
#endif
#if defined(__HIPCC__) || defined(__HIP__)
#define RT_HD_NOINLINE __host__ __device__ __attribute__((noinline)) inline
#else
#define RT_HD_NOINLINE __attribute__((noinline)) inline
#endif

namespace rt {

struct f3 {
  float x, y, z;
};

RT_HD f3 mk(float x, float y, float z) { return f3{x, y, z}; }
RT_HD f3 sub(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
RT_HD f3 neg(f3 a) { return f3{-a.x, -a.y, -a.z}; }
RT_HD float dot(f3 a, f3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
RT_HD float sqnorm(f3 a) { return a.x * a.x + (a.y * a.y + a.z * a.z); }
RT_HD float norm(f3 a) { return sqrtf(sqnorm(a)); }
RT_HD f3 normalized(f3 a) {
  float z = sqnorm(a);
  if (z > 0.0f) {
    float r = sqrtf(z);
    return f3{a.x / r, a.y / r, a.z / r};
  }
  return a;
}
RT_HD f3 cross(f3 a, f3 b) {
  return f3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
RT_HD float smin(float a, float b) { return (b < a) ? b : a; }  // std::min
RT_HD float smax(float a, float b) { return (a < b) ? b : a; }  // std::max

// Affine3f (column-major 4x4 m[16]) * Vector3f
RT_HD f3 affv3(const float* m, f3 v) {
  return f3{((m[0] * v.x + m[4] * v.y) + m[8] * v.z) + m[12],
            ((m[1] * v.x + m[5] * v.y) + m[9] * v.z) + m[13],
            ((m[2] * v.x + m[6] * v.y) + m[10] * v.z) + m[14]};
}
// Matrix3f (column-major m[9]) * Vector3f
RT_HD f3 m3v3(const float* m, f3 v) {
  return f3{m[0] * v.x + (m[3] * v.y + m[6] * v.z), m[1] * v.x + (m[4] * v.y + m[7] * v.z),
            m[2] * v.x + (m[5] * v.y + m[8] * v.z)};
}

// ---- matrix helpers (camera / model matrices), Eigen order -------------------------------------
RT_HD float cof3(const float* m, int i, int j) {  // cofactor_3x3 (InverseImpl.h:124-136), m column-major
  const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
  return m[j1 * 3 + i1] * m[j2 * 3 + i2] - m[j2 * 3 + i1] * m[j1 * 3 + i2];
}
RT_HD void m3inv(const float* m, float* o) {  // compute_inverse<3> (InverseImpl.h:156-171)
  float c0[3] = {cof3(m, 0, 0), cof3(m, 1, 0), cof3(m, 2, 0)};
  float det = c0[0] * m[0] + (c0[1] * m[1] + c0[2] * m[2]);
  float invdet = 1.0f / det;
  float r[9];
  r[0] = c0[0] * invdet; r[3] = c0[1] * invdet; r[6] = c0[2] * invdet;
  r[1] = cof3(m, 0, 1) * invdet; r[4] = cof3(m, 1, 1) * invdet; r[7] = cof3(m, 2, 1) * invdet;
  r[2] = cof3(m, 0, 2) * invdet; r[5] = cof3(m, 1, 2) * invdet; r[8] = cof3(m, 2, 2) * invdet;
  for (int k = 0; k < 9; k++) o[k] = r[k];
}
RT_HD void linear_of(const float* t, float* L) {
  for (int j = 0; j < 3; j++)
    for (int i = 0; i < 3; i++) L[j * 3 + i] = t[j * 4 + i];
}
RT_HD void affinv(const float* t, float* o) {  // Transform.h:1202-1229 (Affine hint)
  float L[9], Li[9];
  linear_of(t, L);
  m3inv(L, Li);
  f3 lt = m3v3(Li, f3{t[12], t[13], t[14]});
  float r[16];
  for (int j = 0; j < 3; j++)
    for (int i = 0; i < 3; i++) r[j * 4 + i] = Li[j * 3 + i];
  r[12] = -lt.x; r[13] = -lt.y; r[14] = -lt.z;
  r[3] = r[7] = r[11] = 0.0f;
  r[15] = 1.0f;
  for (int k = 0; k < 16; k++) o[k] = r[k];
}
RT_HD void identity4(float* m) {
  for (int k = 0; k < 16; k++) m[k] = 0.0f;
  m[0] = m[5] = m[10] = m[15] = 1.0f;
}
RT_HD void scale4(float* m, float s) {  // Transform::scale(Scalar): linearExt() *= s
  for (int j = 0; j < 3; j++)
    for (int i = 0; i < 3; i++) m[j * 4 + i] *= s;
}
RT_HD void translate4(float* m, f3 v) {  // Transform::translate: translation += linear * v
  float L[9];
  linear_of(m, L);
  f3 lv = m3v3(L, v);
  m[12] += lv.x; m[13] += lv.y; m[14] += lv.z;
}
RT_HD void affmul(const float* a, const float* b, float* o) {  // Transform.h:1481-1495
  float La[9], Lb[9], r[16];
  linear_of(a, La);
  linear_of(b, Lb);
  for (int j = 0; j < 3; j++)
    for (int i = 0; i < 3; i++)
      r[j * 4 + i] = La[i] * Lb[j * 3 + 0] + (La[3 + i] * Lb[j * 3 + 1] + La[6 + i] * Lb[j * 3 + 2]);
  f3 tr = m3v3(La, f3{b[12], b[13], b[14]});
  r[12] = tr.x + a[12]; r[13] = tr.y + a[13]; r[14] = tr.z + a[14];
  r[3] = r[7] = r[11] = 0.0f;
  r[15] = 1.0f;
  for (int k = 0; k < 16; k++) o[k] = r[k];
}

// reference expressions built from the primitives above
RT_HD f3 reflect(f3 d, f3 n) {  // Flyscene::reflect (flyscene.cpp:480-482): (d - 2*(d.dot(n)*n)).normalized()
  float dd = dot(d, n);
  return normalized(f3{d.x - 2 * (dd * n.x), d.y - 2 * (dd * n.y), d.z - 2 * (dd * n.z)});
}
RT_HD f3 phong_r(f3 L, f3 n) {  // flyscene.cpp:557: L - 2*(n.dot(L))*n
  float nl2 = 2 * dot(n, L);
  return f3{L.x - nl2 * n.x, L.y - nl2 * n.y, L.z - nl2 * n.z};
}
RT_HD f3 offset(f3 p, f3 v, float k) {  // p + k*v with k = 0.001f / 0.003f (flyscene.cpp:362,512)
  return f3{p.x + k * v.x, p.y + k * v.y, p.z + k * v.z};
}
// interpolateNormal's final blend (flyscene.cpp:599); n* already normalised
RT_HD f3 blend_normal(f3 n0, f3 n1, f3 n2, float area0, float area1, float area2, float area) {
  return normalized(f3{(n0.x * area1 / area + n1.x * area2 / area) + n2.x * area0 / area,
                       (n0.y * area1 / area + n1.y * area2 / area) + n2.y * area0 / area,
                       (n0.z * area1 / area + n1.z * area2 / area) + n2.z * area0 / area});
}

// std::pow(float,float) -> powf (flyscene.cpp:562), evaluated in fp64 and rounded once to float.
// Integer exponents 0..1023 (every material of the configured scenes: MTL Ns is an integer there) take
// binary exponentiation in fp64: at most 20 products, each rounded to 2^-53, so the fp64 value is within
// ~2^-48 relative of x^n and its rounding to float is the correctly rounded x^n except within that distance
// of a float rounding midpoint -- the same exposure as the fp64 library pow. Other exponents call the
// library pow out of line: inlined into a kernel, its fp64 polynomial constants are hoisted into registers
// over the light loop and spilled (112 B per lane of scratch in k_primary_fused, 76-272 B in the FULL
// megakernel builds).
#ifndef RT_POW_INT
#define RT_POW_INT 1
#endif
RT_HD_NOINLINE double pow_generic(double x, double y) { return pow(x, y); }
RT_HD float pow_ref(float x, float y) {
  if (RT_POW_INT && y >= 0.0f && y < 1024.0f && y == truncf(y)) {
    uint32_t n = (uint32_t)y;
    double b = (double)x, r = 1.0;
    while (n != 0u) {
      if (n & 1u) r *= b;
      n >>= 1;
      if (n != 0u) b *= b;
    }
    return (float)r;
  }
  return (float)pow_generic((double)x, (double)y);
}

}  // namespace rt
