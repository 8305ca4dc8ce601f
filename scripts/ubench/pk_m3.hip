// Codegen probe (round 5): a 3x3 product chain carried as row pairs (ext_vector_type(2))
// compiles to v_pk_fma_f32 / v_pk_mul_f32 with op_sel broadcasts and few moves:
//   hipcc --offload-arch=gfx950 -O3 -ffast-math -fno-slp-vectorize --cuda-device-only -S pk_m3.hip
#include <hip/hip_runtime.h>
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 bc(float x) { return f2{x, x}; }
// C = A * B, 3x3 row-major; rows as (f2 cols 0,1) + scalar col 2
struct M3p { f2 r01[3]; float r2[3]; };
__global__ void k(const float *in, float *out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  M3p A, B;
  for (int r = 0; r < 3; ++r) {
    A.r01[r] = f2{in[i * 18 + 3 * r], in[i * 18 + 3 * r + 1]}; A.r2[r] = in[i * 18 + 3 * r + 2];
    B.r01[r] = f2{in[i * 18 + 9 + 3 * r], in[i * 18 + 9 + 3 * r + 1]}; B.r2[r] = in[i * 18 + 9 + 3 * r + 2];
  }
  for (int it = 0; it < 8; ++it) {
    M3p C;
    for (int r = 0; r < 3; ++r) {
      const float a0 = r == 0 ? A.r01[0].x : r == 1 ? A.r01[1].x : A.r01[2].x;
      f2 a01 = A.r01[r];
      C.r01[r] = fma2(bc(a01.y), B.r01[1], bc(a01.x) * B.r01[0]);
      C.r01[r] = fma2(bc(A.r2[r]), B.r01[2], C.r01[r]);
      C.r2[r] = __builtin_fmaf(A.r2[r], B.r2[2], __builtin_fmaf(a01.y, B.r2[1], a01.x * B.r2[0]));
      (void)a0;
    }
    A = C;
  }
  for (int r = 0; r < 3; ++r) { out[i * 9 + 3 * r] = A.r01[r].x; out[i * 9 + 3 * r + 1] = A.r01[r].y; out[i * 9 + 3 * r + 2] = A.r2[r]; }
}
