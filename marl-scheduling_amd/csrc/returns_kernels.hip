// returns_kernels.hip — discounted Monte-Carlo returns + per-sequence normalisation
// (PPOmodules.py:128-137) over the rollout's reward rings, on gfx950. Kept apart from the acting
// kernels (policy_kernels.hip), which build with the ILP-first machine scheduler: these are
// memory-bound passes that lose with it (build.sh).
#include <hip/hip_runtime.h>
#include <math.h>

#include "../../include/marlsched.h"
#include "ms_common.h"

namespace ms {

__global__ void __launch_bounds__(256) k_returns(const float* __restrict__ rewards, int T, int64_t M,
                                                 int64_t row_stride, double gamma, float* __restrict__ out) {
    const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= M) return;
    float* o = out + m * T;
    double G = 0.0;
    for (int t = T - 1; t >= 0; t--) {
        // discounted_reward = reward + gamma * discounted_reward (Python floats)
        G = __dadd_rn((double)rewards[(int64_t)t * row_stride + m], __dmul_rn(gamma, G));  // two roundings
        o[t] = (float)G;  // torch.tensor(rewards, dtype=torch.float32)
    }
    double s = 0.0;
    for (int t = 0; t < T; t++) s += (double)o[t];
    const float mean = (float)(s / T);
    double v = 0.0;
    for (int t = 0; t < T; t++) {
        double d = (double)o[t] - (double)mean;
        v += d * d;
    }
    const float sd = T > 1 ? (float)sqrt(v / (T - 1)) : NAN;  // rewards.std() (unbiased)
    const float den = sd + 1e-7f;
    for (int t = 0; t < T; t++) o[t] = (o[t] - mean) / den;
}

// Returns of sequence (e, g) = unit unit_of_group[g] of replica e, gathered from the rollout
// rewards [T][E][U] and written time-major [T][E][G] (coalesced: g is the fastest thread index).
// Same arithmetic as k_returns: float64 scan, f32 values, mean and unbiased std over T.
// The thread's loads are issued kRetBatch at a time (they do not depend on the scan), so a
// sequence costs ~3*T/kRetBatch memory round trips instead of 3*T. G may list the sub-units of
// several update draws at once: the rollout row [t][e][0..U) is then read once for all of them.
constexpr int kRetBatch = 16;

template <bool I32>
__global__ void __launch_bounds__(256) k_unit_returns(const void* __restrict__ rewards, int T, int64_t E, int U,
                                                      const int32_t* __restrict__ unit_of_group, int G, double gamma,
                                                      float* __restrict__ out) {
    const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= E * G) return;
    const int64_t e = m / G;
    const int g = (int)(m - e * G);
    const int u = unit_of_group[g];
    const int64_t EG = E * G;
    const int64_t EU = E * U;
    const size_t src0 = (size_t)e * U + u;
    double Gs = 0.0, s = 0.0, ss = 0.0;
    for (int t1 = T; t1 > 0; t1 -= kRetBatch) {
        double r[kRetBatch];
#pragma unroll
        for (int k = 0; k < kRetBatch; k++) {
            const int t = t1 - 1 - k;
            const size_t idx = src0 + (size_t)(t < 0 ? 0 : t) * EU;
            r[k] = I32 ? (double)static_cast<const int32_t*>(rewards)[idx] : (double)static_cast<const float*>(rewards)[idx];
        }
#pragma unroll
        for (int k = 0; k < kRetBatch; k++) {
            const int t = t1 - 1 - k;
            if (t >= 0) {
                Gs = __dadd_rn(r[k], __dmul_rn(gamma, Gs));  // Python: two roundings, never an fma
                const float f = (float)Gs;
                out[(int64_t)t * EG + m] = f;
                s += (double)f;
                ss += (double)f * (double)f;
            }
        }
    }
    const float mean = (float)(s / T);
    // sum of squared deviations from the f32 mean, from the same pass's sums (no second read):
    // sum (f - m)^2 = ss - 2 m s + T m^2 in double (the f32 inputs leave it well conditioned)
    const double md = (double)mean;
    double v = ss - 2.0 * md * s + (double)T * md * md;
    v = v > 0.0 ? v : 0.0;
    const float sd = T > 1 ? (float)sqrt(v / (T - 1)) : NAN;
    const float den = sd + 1e-7f;
    for (int t0 = 0; t0 < T; t0 += kRetBatch) {
        float f[kRetBatch];
#pragma unroll
        for (int k = 0; k < kRetBatch; k++) f[k] = out[(int64_t)min(t0 + k, T - 1) * EG + m];
#pragma unroll
        for (int k = 0; k < kRetBatch; k++)
            if (t0 + k < T) out[(int64_t)(t0 + k) * EG + m] = (f[k] - mean) / den;
    }
}

// The same returns with the thread's whole sequence held in registers (T == kRetRegT, UPDATE_STEP of the
// BASELINE configs; other lengths take k_unit_returns): the normalised
// values are written once, instead of written, read back and written again (the generic kernel's
// second pass). Same arithmetic, in the same order, as k_unit_returns.
constexpr int kRetRegT = 200;
template <bool I32>
__global__ void __launch_bounds__(256, 2) k_unit_returns_reg(const void* __restrict__ rewards, int64_t E, int U,
                                                          const int32_t* __restrict__ unit_of_group, int G,
                                                          double gamma, float* __restrict__ out) {
    const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= E * G) return;
    const int64_t e = m / G;
    const int g = (int)(m - e * G);
    const int u = unit_of_group[g];
    const int64_t EG = E * G;
    const int64_t EU = E * U;
    const size_t src0 = (size_t)e * U + u;
    float f[kRetRegT];
    double Gs = 0.0, s = 0.0, ss = 0.0;
    constexpr int B = 8;  // loads in flight per batch
    // element t of the sequence at q - (kRetRegT - 1 - t) * EU: q walks down a batch at a time (a running
    // pointer, so the unrolled loop keeps no per-t address)
    const uint32_t* q = static_cast<const uint32_t*>(rewards) + src0 + (size_t)(kRetRegT - 1) * EU;
#pragma unroll
    for (int t1 = kRetRegT; t1 > 0; t1 -= B) {
        double r[B];
#pragma unroll
        for (int k = 0; k < B; k++) {
            const uint32_t w = q[-(int64_t)k * EU];
            r[k] = I32 ? (double)(int32_t)w : (double)__uint_as_float(w);
        }
        q -= (int64_t)B * EU;
#pragma unroll
        for (int k = 0; k < B; k++) {
            const int t = t1 - 1 - k;
            Gs = __dadd_rn(r[k], __dmul_rn(gamma, Gs));  // Python: two roundings, never an fma
            f[t] = (float)Gs;
            s += (double)f[t];
            ss += (double)f[t] * (double)f[t];
        }
    }
    constexpr int T = kRetRegT;
    const float mean = (float)(s / T);
    const double md = (double)mean;
    double v = ss - 2.0 * md * s + (double)T * md * md;
    v = v > 0.0 ? v : 0.0;
    const float sd = (float)sqrt(v / (T - 1));
    const float den = sd + 1e-7f;
    float* o = out + m;
#pragma unroll
    for (int t = 0; t < kRetRegT; t++) {
        *o = (f[t] - mean) / den;
        o += EG;
    }
}

hipError_t launch_unit_returns(const void* rewards, int is_i32, int T, int64_t E, int U, const int32_t* unit_of_group,
                               int G, double gamma, float* out, hipStream_t st) {
    const int64_t M = E * G;
    if (M <= 0) return hipSuccess;
    if (T == kRetRegT) {
        auto kreg = is_i32 ? k_unit_returns_reg<true> : k_unit_returns_reg<false>;
        hipLaunchKernelGGL(kreg, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, st, rewards, E, U, unit_of_group, G,
                           gamma, out);
        return hipGetLastError();
    }
    auto kern = is_i32 ? k_unit_returns<true> : k_unit_returns<false>;
    hipLaunchKernelGGL(kern, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, st, rewards, T, E, U, unit_of_group, G,
                       gamma, out);
    return hipGetLastError();
}

hipError_t launch_returns(const float* rewards, int T, int64_t M, int64_t row_stride, double gamma, float* out,
                          hipStream_t st) {
    if (M <= 0) return hipSuccess;
    const int threads = 256;
    hipLaunchKernelGGL(k_returns, dim3((unsigned)((M + threads - 1) / threads)), dim3(threads), 0, st, rewards, T, M,
                       row_stride, gamma, out);
    return hipGetLastError();
}

}  // namespace ms
