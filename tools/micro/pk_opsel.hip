// What v_pk_fma_f32's op_sel / op_sel_hi select on gfx950 (diagnostic for the packed box tests):
// src0 = SGPR pair {2, 3}, src1 = VGPR pair {5, 7}, src2 = VGPR pair {100, 1000}; prints both result lanes.
//   hipcc --offload-arch=gfx950 -O3 -w -o pk_opsel tools/micro/pk_opsel.hip && ./pk_opsel
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void k(float* out, const float* in) {
  const f2 s = {in[0], in[1]};
  f2 v1 = {in[2] + threadIdx.x * 0.0f, in[3]}, v2 = {in[4], in[5] + threadIdx.x * 0.0f};
  f2 r0, r1, r2, r3;
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(r0) : "s"(s), "v"(v1), "v"(v2));
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r1) : "s"(s), "v"(v1), "v"(v2));
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "=v"(r2) : "s"(s), "v"(v1), "v"(v2));
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,0,1]" : "=v"(r3) : "s"(s), "v"(v1), "v"(v2));
  if (threadIdx.x == 0) {
    out[0] = r0.x; out[1] = r0.y; out[2] = r1.x; out[3] = r1.y;
    out[4] = r2.x; out[5] = r2.y; out[6] = r3.x; out[7] = r3.y;
  }
}

int main() {
  float h[6] = {2, 3, 5, 7, 100, 1000}, o[8];
  float *din, *dout;
  (void)hipMalloc(&din, 64);
  (void)hipMalloc(&dout, 64);
  (void)hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dout, din);
  (void)hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
  printf("s={2,3} v1={5,7} v2={100,1000}\n");
  printf("default                         : %g %g  (expect 110 1021)\n", o[0], o[1]);
  printf("op_sel_hi:[1,0,1]               : %g %g  (broadcast v1.lo: expect 110 1015)\n", o[2], o[3]);
  printf("op_sel:[0,1,0] op_sel_hi:[1,1,1]: %g %g  (broadcast v1.hi: expect 114 1021)\n", o[4], o[5]);
  printf("op_sel:[0,1,0] op_sel_hi:[1,0,1]: %g %g\n", o[6], o[7]);
  return 0;
}
