// Micro-benchmark: issue cost of v_fma_f32 vs v_pk_fma_f32 for one wave per
// SIMD (the step kernel's occupancy) and for two.  Prints cycles per
// instruction per wave (clock64 around an unrolled chain of 8 independent ops).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int PK>
__global__ void kern(float *out, long long *cyc, int iters) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float b0 = a0 * 2, b1 = a1 * 2, b2 = a2 * 2, b3 = a3 * 2, b4 = a4 * 2, b5 = a5 * 2, b6 = a6 * 2, b7 = a7 * 2;
    const float m = 0.999f, c = 0.001f;
    __syncthreads();
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
        if constexpr (PK) {
            typedef float f2 __attribute__((ext_vector_type(2)));
            f2 x0 = {a0, b0}, x1 = {a1, b1}, x2 = {a2, b2}, x3 = {a3, b3}, x4 = {a4, b4}, x5 = {a5, b5}, x6 = {a6, b6}, x7 = {a7, b7};
            f2 mm = {m, m}, cc = {c, c};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x0) : "v"(mm), "v"(cc));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x1) : "v"(mm), "v"(cc));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x2) : "v"(mm), "v"(cc));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x3) : "v"(mm), "v"(cc));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x4) : "v"(mm), "v"(cc));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x5) : "v"(mm), "v"(cc));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x6) : "v"(mm), "v"(cc));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x7) : "v"(mm), "v"(cc));
            }
            a0 = x0.x; b0 = x0.y; a1 = x1.x; b1 = x1.y; a2 = x2.x; b2 = x2.y; a3 = x3.x; b3 = x3.y;
            a4 = x4.x; b4 = x4.y; a5 = x5.x; b5 = x5.y; a6 = x6.x; b6 = x6.y; a7 = x7.x; b7 = x7.y;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(m), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a1) : "v"(m), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a2) : "v"(m), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a3) : "v"(m), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a4) : "v"(m), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a5) : "v"(m), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a6) : "v"(m), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a7) : "v"(m), "v"(c));
            }
        }
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + b0 + b1 + b2 + b3 + b4 + b5 + b6 + b7;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

int main() {
    const int iters = 2000;
    float *out;
    long long *cyc;
    hipMalloc(&out, 256 * 512 * sizeof(float));
    hipMalloc(&cyc, 256 * 8 * sizeof(long long));
    long long h[256 * 8];
    for (int threads : {64, 256, 512}) {
        for (int pk = 0; pk < 2; ++pk) {
            for (int rep = 0; rep < 2; ++rep) {
                if (pk) hipLaunchKernelGGL(kern<1>, dim3(256), dim3(threads), 0, 0, out, cyc, iters);
                else hipLaunchKernelGGL(kern<0>, dim3(256), dim3(threads), 0, 0, out, cyc, iters);
            }
            hipDeviceSynchronize();
            const int nw = 256 * threads / 64;
            hipMemcpy(h, cyc, nw * sizeof(long long), hipMemcpyDeviceToHost);
            double s = 0;
            for (int i = 0; i < nw; ++i) s += h[i];
            printf("waves/CU %d %s: %.2f cycles per instruction per wave\n", threads / 64, pk ? "v_pk_fma_f32" : "v_fma_f32   ",
                   s / nw / (iters * 32.0));
        }
    }
    return 0;
}
