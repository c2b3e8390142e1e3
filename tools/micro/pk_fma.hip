// Issue cost of packed vs single f32 FMA on gfx950 (diagnostic for the node step's 12 box-plane FMAs).
// Each wave runs N iterations of 12 independent FMA chains, either as 12 v_fma_f32 or as 6 v_pk_fma_f32
// (the same 12 products); one SGPR-pair operand per instruction like the node step's box planes.
// Run at 1, 2, 4 and 8 waves per SIMD: the shader clocks per iteration say whether a v_pk_fma_f32 costs
// the VALU pipe one or two single FMAs' time.
//   hipcc --offload-arch=gfx950 -O3 -o pk_fma tools/micro/pk_fma.hip && ./pk_fma
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int PK>
__global__ __launch_bounds__(64) void k_fma(float* out, const float* box, int iters, unsigned long long* clk) {
  f2 a0 = {1.0f + threadIdx.x * 1e-3f, 2.0f}, a1 = {3.0f, 4.0f}, a2 = {5.0f, 6.0f};
  f2 a3 = {7.0f, 8.0f}, a4 = {9.0f, 10.0f}, a5 = {11.0f, 12.0f};
  f2 m = {0.999f, 0.999f}, c = {1e-3f, 2e-3f};
  // a uniform (SGPR) pair like the node record's planes
  const f2 s = {box[0], box[1]};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
    if (PK == 2) {  // src1 broadcast from its low half (op_sel_hi), as the packed box tests use it
#define PKF(r) asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(r) : "s"(s), "v"(m));
      PKF(a0) PKF(a1) PKF(a2) PKF(a3) PKF(a4) PKF(a5)
#undef PKF
    } else if (PK == 3) {  // src1 broadcast from its high half (op_sel)
#define PKF(r) asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(r) : "s"(s), "v"(m));
      PKF(a0) PKF(a1) PKF(a2) PKF(a3) PKF(a4) PKF(a5)
#undef PKF
    } else if (PK == 4) {  // VGPR pairs only
#define PKF(r) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(r) : "v"(m), "v"(c));
      PKF(a0) PKF(a1) PKF(a2) PKF(a3) PKF(a4) PKF(a5)
#undef PKF
    } else if (PK) {
#define PKF(r) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(r) : "s"(s), "v"(m));
      PKF(a0) PKF(a1) PKF(a2) PKF(a3) PKF(a4) PKF(a5)
#undef PKF
    } else {
#define SF(r)                                                                                      \
  asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(r.x) : "s"(s.x), "v"(m.x));            \
  asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(r.y) : "s"(s.y), "v"(m.y));
      SF(a0) SF(a1) SF(a2) SF(a3) SF(a4) SF(a5)
#undef SF
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  f2 r = a0 + a1 + a2 + a3 + a4 + a5 + c;
  out[blockIdx.x * 64 + threadIdx.x] = r.x + r.y;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

int main() {
  const int iters = 4096;
  float *out, *box;
  unsigned long long* clk;
  const int maxb = 256 * 4 * 8;
  hipMalloc(&out, maxb * 64 * 4);
  hipMalloc(&box, 64);
  hipMalloc(&clk, maxb * 8);
  float hb[2] = {0.5f, 0.25f};
  hipMemcpy(box, hb, 8, hipMemcpyHostToDevice);
  unsigned long long* h = (unsigned long long*)malloc(maxb * 8);
  for (int wps : {1, 2, 4, 8}) {
    const int blocks = 256 * 4 * wps;
    for (int pk = 0; pk < 5; pk++) {
      for (int rep = 0; rep < 2; rep++) {
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a);
        if (pk == 1) hipLaunchKernelGGL(k_fma<1>, dim3(blocks), dim3(64), 0, 0, out, box, iters, clk);
        else if (pk == 2) hipLaunchKernelGGL(k_fma<2>, dim3(blocks), dim3(64), 0, 0, out, box, iters, clk);
        else if (pk == 3) hipLaunchKernelGGL(k_fma<3>, dim3(blocks), dim3(64), 0, 0, out, box, iters, clk);
        else if (pk == 4) hipLaunchKernelGGL(k_fma<4>, dim3(blocks), dim3(64), 0, 0, out, box, iters, clk);
        else hipLaunchKernelGGL(k_fma<0>, dim3(blocks), dim3(64), 0, 0, out, box, iters, clk);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        hipMemcpy(h, clk, blocks * 8, hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < blocks; i++) s += (double)h[i];
        if (rep)
          printf("waves/SIMD %d %s: %.1f shader clocks per iteration per wave (12 FMA), kernel %.3f ms\n", wps,
                 pk == 0 ? "12 v_fma_f32" : pk == 1 ? "6 v_pk_fma_f32" : pk == 2 ? "6 v_pk_fma_f32 op_sel_hi" : pk == 3 ? "6 v_pk_fma_f32 op_sel" : "6 v_pk_fma_f32 vgpr", s / blocks / iters, ms);
        hipEventDestroy(a);
        hipEventDestroy(b);
      }
    }
  }
  return 0;
}
