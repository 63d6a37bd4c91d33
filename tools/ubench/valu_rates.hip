// Issue cost of VALU forms on gfx950 with several waves per SIMD (tools only, not shipped):
// each lane runs 8 independent chains of one instruction form; cycles per wave-instruction per SIMD
// = kernel time x clock x SIMDs / (waves x instructions).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 2048;
template <int K>
__global__ void __launch_bounds__(256) kb(float* out, float s, int n) {
    float v[8];
    f2 w[8];
    uint32_t u[8];
    for (int i = 0; i < 8; i++) { v[i] = threadIdx.x * 1e-3f + i; w[i] = (f2){v[i], v[i] + 1}; u[i] = threadIdx.x + i; }
    for (int it = 0; it < n; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (K == 0) v[i] = fmaf(v[i], s, 0.5f);
            if (K == 1) w[i] = w[i] * (f2){s, s} + (f2){0.5f, 0.25f};
            if (K == 2) v[i] = __builtin_amdgcn_exp2f(v[i]);
            if (K == 3) u[i] = u[i] * 0x9E3779B1u + 7;
            if (K == 4) v[i] = __builtin_amdgcn_rcpf(v[i]);
            if (K == 5) u[i] = __builtin_amdgcn_permlane16_swap(u[i], u[(i + 1) & 7], false, false)[0];
            if (K == 6) v[i] = v[i] + s;
        }
    }
    float acc = 0;
    for (int i = 0; i < 8; i++) acc += v[i] + w[i][0] + w[i][1] + (float)u[i];
    if (acc == 1234.5f) out[0] = acc;
}
int main() {
    float* d; hipMalloc(&d, 4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const char* names[] = {"v_fma_f32", "v_pk_fma_f32 (f2 fma)", "v_exp_f32", "v_mul_lo_u32+add", "v_rcp_f32", "v_permlane16_swap", "v_add_f32"};
    for (int wps = 1; wps <= 4; wps *= 2) {
        const int blocks = 256 * wps;  // 4 waves per block, 256 CUs
        for (int k = 0; k < 7; k++) {
            auto launch = [&]() {
                switch (k) {
                    case 0: hipLaunchKernelGGL(kb<0>, blocks, 256, 0, 0, d, 1.0001f, ITER); break;
                    case 1: hipLaunchKernelGGL(kb<1>, blocks, 256, 0, 0, d, 1.0001f, ITER); break;
                    case 2: hipLaunchKernelGGL(kb<2>, blocks, 256, 0, 0, d, 1.0001f, ITER); break;
                    case 3: hipLaunchKernelGGL(kb<3>, blocks, 256, 0, 0, d, 1.0001f, ITER); break;
                    case 4: hipLaunchKernelGGL(kb<4>, blocks, 256, 0, 0, d, 1.0001f, ITER); break;
                    case 5: hipLaunchKernelGGL(kb<5>, blocks, 256, 0, 0, d, 1.0001f, ITER); break;
                    case 6: hipLaunchKernelGGL(kb<6>, blocks, 256, 0, 0, d, 1.0001f, ITER); break;
                }
            };
            launch(); hipDeviceSynchronize();
            hipEventRecord(a); for (int r = 0; r < 5; r++) launch(); hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b); ms /= 5;
            const double insts_per_simd = (double)wps * ITER * 8;  // wave-instructions per SIMD
            printf("waves/SIMD %d  %-24s %8.3f ms  %6.2f ns per wave-instruction per SIMD (%.2f cyc @2.1GHz)\n", wps, names[k], ms,
                   ms * 1e6 / insts_per_simd, ms * 1e6 / insts_per_simd * 2.1);
        }
    }
    return 0;
}
