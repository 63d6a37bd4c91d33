// Do bf16 MFMAs (v_mfma_f32_16x16x32_bf16) and plain VALU of co-resident waves overlap on one SIMD,
// compared with the f32 form (v_mfma_f32_16x16x4_f32)? (tools only, not shipped)
// Each wave runs ITER iterations of M independent MFMAs (4 accumulators) and V independent v_fma_f32.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int ITER = 1024;
template <int BF, int M, int V>
__global__ void __launch_bounds__(256) kb(float* out, float s) {
    f4 acc[4];
    float v[8];
    for (int i = 0; i < 4; i++) acc[i] = (f4){0, 0, 0, 0};
    for (int i = 0; i < 8; i++) v[i] = threadIdx.x * 1e-3f + i;
    const float a = threadIdx.x * 1e-4f, b = 0.5f;
    bf16x8 xa, xb;
    for (int i = 0; i < 8; i++) xa[i] = (__bf16)(a + i), xb[i] = (__bf16)(b - i);
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int m = 0; m < M; m++) {
            if (BF)
                acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa, xb, acc[m & 3], 0, 0, 0);
            else
                acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m & 3], 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < V; k++) v[k & 7] = fmaf(v[k & 7], s, 0.5f);
    }
    float t = 0;
    for (int i = 0; i < 4; i++) t += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    for (int i = 0; i < 8; i++) t += v[i];
    if (t == 1234.5f) out[0] = t;
}
template <int BF, int M, int V>
static void run(float* d, int wps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int blocks = 256 * wps;
    hipLaunchKernelGGL((kb<BF, M, V>), blocks, 256, 0, 0, d, 1.0001f);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL((kb<BF, M, V>), blocks, 256, 0, 0, d, 1.0001f);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    const double cyc = ms * 1e-3 * 2.1e9 / ((double)wps * ITER);  // SIMD cycles per wave-iteration
    printf("%s waves/SIMD %d  M=%2d V=%3d  %.3f ms  %7.1f cyc per wave-iteration per SIMD\n", BF ? "bf16" : "f32 ",
           wps, M, V, ms, cyc);
}
int main() {
    float* d;
    (void)hipMalloc(&d, 4);
    for (int w = 2; w <= 4; w *= 2) {
        run<1, 8, 0>(d, w);
        run<1, 0, 48>(d, w);
        run<1, 8, 48>(d, w);
        run<1, 8, 16>(d, w);
        run<1, 8, 96>(d, w);
        run<0, 4, 0>(d, w);
        run<0, 4, 48>(d, w);
    }
    return 0;
}
