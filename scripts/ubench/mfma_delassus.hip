// Micro-benchmark for the MFMA decision (north_star: "MFMA used only for the
// tiny batched mass-matrix/Jacobian contractions where it actually wins").
//
// The GEMM-shaped piece of the step kernel's contact phase is the Delassus
// assembly W = J R: per env, K = 14 contact rows (Thormang: 2 foot boxes x 7
// rows) with a 12-float Jacobian each (6 per contact group, 2 contact groups)
// against the 12 x K impulse responses (column j = the response to a unit
// impulse on row j, held by lane j of the env -- step_par.h "one Delassus
// column per lane").  Layout as in the step kernel: 16 envs per workgroup, 16
// lanes per env, J in LDS.  Two ways to form W into LDS:
//   valu : lane j computes column j, W[i][j] = J_i . R_j (14 x 12 FMAs, J_i an
//          LDS broadcast)
//   mfma : R goes to LDS, then each wave forms its 4 envs' 16 x 16 W tiles
//          with 3 v_mfma_f32_16x16x4_f32 each (K = 12 = 3 k-steps of 4), A and
//          B fragments gathered from LDS, the C fragment stored back
// Both repeat REPS times per launch (the step kernel forms W once per substep;
// the repetition only makes the launch long enough to time).  Prints the
// max |W_valu - W_mfma| and both kernels' times (HIP events); run under
// rocprofv3 --kernel-trace --stats for the per-kernel durations.
//
//   hipcc --offload-arch=gfx950 -O3 -o mfma_delassus mfma_delassus.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

constexpr int EPB = 16, LPE = 16, K = 14, KP = 16, NJ = 12, REPS = 64;
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                 \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 1;                                                            \
        }                                                                        \
    } while (0)

// per env in LDS: J [KP][NJ] (rows >= K zero), R [NJ][KP], W [KP][KP]
struct EnvLds {
    float J[KP][NJ];
    float R[NJ][KP];
    float W[KP][KP];
};

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool MFMA>
__global__ __launch_bounds__(EPB *LPE) void delassus(const float *J, const float *R, float *W, int n, float *sink) {
    __shared__ EnvLds L[EPB];
    const int le = threadIdx.x / LPE, sub = threadIdx.x % LPE;
    const int e = blockIdx.x * EPB + le;
    EnvLds &s = L[le];
    // inputs: J rows of the env into LDS, the lane's response column into registers
    for (int k = sub; k < KP * NJ; k += LPE) s.J[k / NJ][k % NJ] = (k / NJ < K) ? J[(size_t)e * K * NJ + k] : 0.f;
    float r[NJ];
#pragma unroll
    for (int k = 0; k < NJ; ++k) r[k] = sub < K ? R[((size_t)e * NJ + k) * K + sub] : 0.f;
    __syncthreads();
    float acc = 0.f;
    for (int rep = 0; rep < REPS; ++rep) {
        if constexpr (!MFMA) {
            // lane j = column j: W[i][j] = sum_k J[i][k] r[k]
#pragma unroll
            for (int i = 0; i < K; ++i) {
                float w = 0.f;
#pragma unroll
                for (int k = 0; k < NJ; ++k) w = fmaf(s.J[i][k], r[k], w);
                s.W[i][sub] = w;
            }
        } else {
            // responses to LDS in the B layout, then per env of the wave 3 MFMAs
#pragma unroll
            for (int k = 0; k < NJ; ++k) s.R[k][sub] = r[k];
            wave_sync();
            const int lane = threadIdx.x % 64, wbase = (threadIdx.x / 64) * (64 / LPE);
#pragma unroll
            for (int q = 0; q < 64 / LPE; ++q) {
                EnvLds &t = L[wbase + q];
                f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < NJ / 4; ++ks) {
                    const int kk = 4 * ks + (lane >> 4);
                    c = __builtin_amdgcn_mfma_f32_16x16x4f32(t.J[lane & 15][kk], t.R[kk][lane & 15], c, 0, 0, 0);
                }
#pragma unroll
                for (int g = 0; g < 4; ++g) t.W[4 * (lane >> 4) + g][lane & 15] = c[g];
            }
        }
        wave_sync();
        // consume W like the PGS does (lane k reads row k) so neither variant is dead code
        if (sub < K) acc += s.W[sub][(sub + rep) % K];
        wave_sync();
        if constexpr (!MFMA) {
#pragma unroll
            for (int k = 0; k < NJ; ++k) r[k] += 1e-7f * acc;   // keep the columns live across reps
        } else {
#pragma unroll
            for (int k = 0; k < NJ; ++k) r[k] += 1e-7f * acc;
        }
    }
    if (e < n && sub < K)
        for (int i = 0; i < K; ++i) W[((size_t)e * K + i) * K + sub] = s.W[i][sub];
    sink[blockIdx.x * EPB * LPE + threadIdx.x] = acc;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 4096;
    std::vector<float> hJ((size_t)n * K * NJ), hR((size_t)n * NJ * K);
    unsigned x = 12345u;
    auto rnd = [&] { x = x * 1664525u + 1013904223u; return (float)((x >> 8) & 0xFFFF) / 65536.f - 0.5f; };
    for (auto &v : hJ) v = rnd();
    for (auto &v : hR) v = rnd();
    float *J, *R, *W0, *W1, *sink;
    CHECK(hipMalloc(&J, hJ.size() * 4));
    CHECK(hipMalloc(&R, hR.size() * 4));
    CHECK(hipMalloc(&W0, (size_t)n * K * K * 4));
    CHECK(hipMalloc(&W1, (size_t)n * K * K * 4));
    CHECK(hipMalloc(&sink, (size_t)n * LPE * 4));
    CHECK(hipMemcpy(J, hJ.data(), hJ.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(R, hR.data(), hR.size() * 4, hipMemcpyHostToDevice));
    const dim3 grid(n / EPB), block(EPB * LPE);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    float ms[2] = {0, 0};
    for (int it = 0; it < 22; ++it) {   // 2 warm-up rounds, 20 timed
        for (int v = 0; v < 2; ++v) {
            CHECK(hipEventRecord(a));
            if (v == 0) hipLaunchKernelGGL(delassus<false>, grid, block, 0, 0, J, R, W0, n, sink);
            else hipLaunchKernelGGL(delassus<true>, grid, block, 0, 0, J, R, W1, n, sink);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float t = 0;
            CHECK(hipEventElapsedTime(&t, a, b));
            if (it >= 2) ms[v] += t / 20;
        }
    }
    std::vector<float> w0((size_t)n * K * K), w1(w0.size());
    CHECK(hipMemcpy(w0.data(), W0, w0.size() * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(w1.data(), W1, w1.size() * 4, hipMemcpyDeviceToHost));
    double md = 0, mref = 0;
    for (size_t i = 0; i < w0.size(); ++i) {
        md = fmax(md, fabs((double)w0[i] - w1[i]));
        mref = fmax(mref, fabs((double)w0[i]));
    }
    // per env and rep: K*K*NJ FMAs
    const double flops = 2.0 * K * K * NJ * REPS * (double)n;
    printf("{\"envs\": %d, \"reps\": %d, \"K\": %d, \"NJ\": %d, \"valu_ms\": %.4f, \"mfma_ms\": %.4f, "
           "\"valu_gflops\": %.1f, \"mfma_gflops\": %.1f, \"max_abs_diff\": %.3g, \"max_abs\": %.3g}\n",
           n, REPS, K, NJ, ms[0], ms[1], flops / ms[0] * 1e-6, flops / ms[1] * 1e-6, md, mref);
    return md <= 1e-5 * fmax(1.0, mref) ? 0 : 2;
}
