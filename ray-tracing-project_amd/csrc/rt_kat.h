// rt_kat.h -- verification hook: one known-answer case of an Eigen-order primitive (op codes of
// oracle/eigen_kat.cpp), evaluated with the product's own rt_math.h on the host or on the device.
// Tests only; the render path never calls it.
#pragma once
#include "rt_math.h"

namespace rt {
RT_HD int debug_math_case(int op, const float* a, float* o) {
  auto put = [&](f3 v) { o[0] = v.x; o[1] = v.y; o[2] = v.z; };
  auto get = [&](const float* p) { return f3{p[0], p[1], p[2]}; };
  switch (op) {
    case 0: o[0] = dot(get(a), get(a + 3)); return 0;
    case 1: put(normalized(get(a))); return 0;
    case 2: put(cross(get(a), get(a + 3))); return 0;
    case 3: put(m3v3(a, get(a + 9))); return 0;
    case 4: put(affv3(a, get(a + 16))); return 0;
    case 5: {
      for (int i = 0; i < 4; i++) o[i] = ((a[i] * a[16] + a[4 + i] * a[17]) + a[8 + i] * a[18]) + a[12 + i] * a[19];
      return 0;
    }
    case 6: m3inv(a, o); return 0;
    case 7: affinv(a, o); return 0;
    case 8: {
      float sh[16], md[16];
      identity4(sh); scale4(sh, a[0]); translate4(sh, f3{-a[1], -a[2], -a[3]});
      identity4(md); affmul(md, sh, o);
      return 0;
    }
    case 9: put(offset(get(a), get(a + 3), 0.001f)); return 0;
    case 10: put(offset(get(a), get(a + 3), 0.003f)); return 0;
    case 11: put(reflect(get(a), get(a + 3))); return 0;
    case 12: put(phong_r(get(a), get(a + 3))); return 0;
    case 13: put(blend_normal(normalized(get(a)), normalized(get(a + 3)), normalized(get(a + 6)), a[9], a[10], a[11], a[12])); return 0;
    case 14: o[0] = norm(get(a)) / 2; return 0;
    case 15: {
      float L[9], Li[9];
      for (int j = 0; j < 3; j++) for (int i = 0; i < 3; i++) L[j * 3 + i] = a[j * 4 + i];
      m3inv(L, Li);
      put(m3v3(Li, f3{-a[12], -a[13], -a[14]}));
      return 0;
    }
    case 16: {  // screenToWorld (camera.hpp:155-173): fp64 NDC, tan in fp64
      f3 nc;
      nc.x = (float)(2.0 * (double)(a[16] - a[18]) / (double)a[20] - 1.0);
      nc.y = (float)(1.0 - 2.0 * (double)(a[17] - a[19]) / (double)a[21]);
      nc.z = -1.0f;
      float persp = (float)((double)1.0f / tan((double)(a[22] / 2.0f) * (3.14159265358979323846 / 180.0)));
      float scale = (float)(1.0 / (double)persp);
      nc.x *= a[23] * scale;
      nc.y *= scale;
      float vinv[16];
      affinv(a, vinv);
      put(affv3(vinv, nc));
      return 0;
    }
    case 17: o[0] = pow_ref(a[0], a[1]); return 0;  // calcSingleColor's std::pow (flyscene.cpp:562)
    default: return -1;
  }
}
}  // namespace rt
