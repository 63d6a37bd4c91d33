// policy_kernels.hip — PPO action selection and return estimation for gfx950.
//
// k_policy_act: fused ActorCritic.act (PPOmodules.py:53-63) for every unit of
// every env replica: Linear(D,H)-tanh-Linear(H,H)-tanh-Linear(H,A)-softmax,
// then torch Categorical semantics (probs renormalised, logits =
// log(clamp(p, eps, 1-eps)), torch/distributions/categorical.py:71,
// utils.py:101-137) and an inverse-CDF sample. One thread per observation
// row; a block only holds rows of one weight group, so the weights are
// wave-uniform and are read through the scalar cache. Observations stay int8
// in HBM (the values are small integers, exact in f32).
//
// k_returns: PPO.update's Monte-Carlo returns (PPOmodules.py:128-137) in
// float64, cast to f32 and normalised per sequence.
#include <hip/hip_runtime.h>
#include <math.h>

#include "../../include/marlsched.h"

namespace ms {

__device__ __forceinline__ uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t& hi) {
    uint64_t p = (uint64_t)a * b;
    hi = (uint32_t)(p >> 32);
    return (uint32_t)p;
}

// Philox4x32-10 (Salmon et al., SC'11): counter-based, one call per row.
__device__ __forceinline__ uint32_t philox_first(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                                  uint32_t k1) {
    for (int r = 0; r < 10; r++) {
        uint32_t hi0, hi1;
        uint32_t lo0 = mulhilo(0xD2511F53u, c0, hi0);
        uint32_t lo1 = mulhilo(0xCD9E8D57u, c2, hi1);
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n1 = lo1;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        uint32_t n3 = lo0;
        c0 = n0;
        c1 = n1;
        c2 = n2;
        c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c0;
}

template <int H, int AMAX>
__global__ void __launch_bounds__(256) k_policy_act(const float* __restrict__ w1, const float* __restrict__ b1,
                                                    const float* __restrict__ w2, const float* __restrict__ b2,
                                                    const float* __restrict__ w3, const float* __restrict__ b3,
                                                    int D, int A, const int8_t* __restrict__ obs, int stride,
                                                    int64_t n_envs, int n_units, int per_group, int blocks_per_group,
                                                    uint64_t seed, uint64_t offset, const float* __restrict__ uniforms,
                                                    int8_t* __restrict__ action, float* __restrict__ logprob) {
    const int g = blockIdx.x / blocks_per_group;  // wave-uniform weight group
    const int64_t item = (int64_t)(blockIdx.x % blocks_per_group) * blockDim.x + threadIdx.x;
    const int64_t n_items = n_envs * per_group;
    if (item >= n_items) return;
    const int64_t e = item / per_group;
    const int u = g * per_group + (int)(item % per_group);
    const int64_t row = e * n_units + u;

    const float* W1 = w1 + (size_t)g * H * D;
    const float* B1 = b1 + (size_t)g * H;
    const float* W2 = w2 + (size_t)g * H * H;
    const float* B2 = b2 + (size_t)g * H;
    const float* W3 = w3 + (size_t)g * A * H;
    const float* B3 = b3 + (size_t)g * A;

    // layer 1: h = tanh(W1 x + b1), x read as dwords of 4 int8 features
    float h[H];
#pragma unroll
    for (int o = 0; o < H; o++) h[o] = 0.f;
    const uint32_t* xr = reinterpret_cast<const uint32_t*>(obs + row * (int64_t)stride);
    const int nd = (D + 3) >> 2;
    for (int q = 0; q < nd; q++) {
        uint32_t w = xr[q];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            int k = q * 4 + j;
            if (k < D) {
                float x = (float)(int8_t)(w >> (8 * j));
#pragma unroll
                for (int o = 0; o < H; o++) h[o] = fmaf(W1[o * D + k], x, h[o]);
            }
        }
    }
#pragma unroll
    for (int o = 0; o < H; o++) h[o] = tanhf(h[o] + B1[o]);
    // layer 2
    float h2[H];
#pragma unroll
    for (int o = 0; o < H; o++) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < H; k++) s = fmaf(W2[o * H + k], h[k], s);
        h2[o] = tanhf(s + B2[o]);
    }
    // layer 3 + softmax (nn.Softmax(dim=-1))
    float z[AMAX];
    float zmax = -INFINITY;
#pragma unroll
    for (int a = 0; a < AMAX; a++) {
        if (a < A) {
            float s = 0.f;
#pragma unroll
            for (int k = 0; k < H; k++) s = fmaf(W3[a * H + k], h2[k], s);
            z[a] = s + B3[a];
            zmax = fmaxf(zmax, z[a]);
        }
    }
    float sum = 0.f;
#pragma unroll
    for (int a = 0; a < AMAX; a++)
        if (a < A) {
            z[a] = expf(z[a] - zmax);
            sum += z[a];
        }
    const float inv = 1.f / sum;
    float psum = 0.f;
#pragma unroll
    for (int a = 0; a < AMAX; a++)
        if (a < A) {
            z[a] = z[a] * inv;  // softmax output
            psum += z[a];
        }
    // Categorical: probs / probs.sum(-1) then inverse-CDF sample
    float uu;
    if (uniforms) {
        uu = uniforms[row];
    } else {
        uint32_t r = philox_first((uint32_t)row, (uint32_t)(row >> 32), (uint32_t)offset, (uint32_t)(offset >> 32),
                                  (uint32_t)seed, (uint32_t)(seed >> 32));
        uu = (float)(r >> 8) * (1.0f / 16777216.0f);
    }
    int chosen = -1;
    float pchosen = 0.f, cum = 0.f;
    int last_nz = 0;
#pragma unroll
    for (int a = 0; a < AMAX; a++)
        if (a < A) {
            float p = z[a] / psum;
            if (p > 0.f) last_nz = a;
            cum += p;
            if (chosen < 0 && uu < cum) {
                chosen = a;
                pchosen = p;
            }
        }
    if (chosen < 0) {
        chosen = last_nz;
        pchosen = z[last_nz] / psum;
    }
    const float eps = 1.1920928955078125e-07f;  // torch.finfo(float32).eps
    float pc = fminf(fmaxf(pchosen, eps), 1.f - eps);
    action[row] = (int8_t)chosen;
    logprob[row] = logf(pc);
}

template <int H, int AMAX>
static hipError_t launch_act_t(const ms_mlp_params* p, const int8_t* obs, int stride, int64_t E, int U, int S,
                               uint64_t seed, uint64_t offset, const float* uniforms, int8_t* action, float* logprob,
                               hipStream_t st) {
    const int threads = 256;
    const int64_t items = E * S;
    const int bpg = (int)((items + threads - 1) / threads);
    const int64_t blocks = (int64_t)bpg * p->n_groups;
    if (blocks <= 0) return hipSuccess;
    hipLaunchKernelGGL((k_policy_act<H, AMAX>), dim3((unsigned)blocks), dim3(threads), 0, st, p->w1, p->b1, p->w2,
                       p->b2, p->w3, p->b3, p->in_dim, p->n_actions, obs, stride, E, U, S, bpg, seed, offset, uniforms,
                       action, logprob);
    return hipGetLastError();
}

hipError_t launch_policy_act(const ms_mlp_params* p, const int8_t* obs, int stride, int64_t E, int U, int S,
                             uint64_t seed, uint64_t offset, const float* uniforms, int8_t* action, float* logprob,
                             hipStream_t st) {
    if (p->hidden != 16) return hipErrorInvalidValue;
    if (p->n_actions <= 16) return launch_act_t<16, 16>(p, obs, stride, E, U, S, seed, offset, uniforms, action, logprob, st);
    if (p->n_actions <= 32) return launch_act_t<16, 32>(p, obs, stride, E, U, S, seed, offset, uniforms, action, logprob, st);
    if (p->n_actions <= 64) return launch_act_t<16, 64>(p, obs, stride, E, U, S, seed, offset, uniforms, action, logprob, st);
    return launch_act_t<16, 128>(p, obs, stride, E, U, S, seed, offset, uniforms, action, logprob, st);
}

// ---------------------------------------------------------------------------

__global__ void __launch_bounds__(256) k_returns(const float* __restrict__ rewards, int T, int64_t M,
                                                 int64_t row_stride, double gamma, float* __restrict__ out) {
    const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= M) return;
    float* o = out + m * T;
    double G = 0.0;
    for (int t = T - 1; t >= 0; t--) {
        // discounted_reward = reward + gamma * discounted_reward (Python floats)
        G = (double)rewards[(int64_t)t * row_stride + m] + gamma * G;
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

hipError_t launch_returns(const float* rewards, int T, int64_t M, int64_t row_stride, double gamma, float* out,
                          hipStream_t st) {
    if (M <= 0) return hipSuccess;
    const int threads = 256;
    hipLaunchKernelGGL(k_returns, dim3((unsigned)((M + threads - 1) / threads)), dim3(threads), 0, st, rewards, T, M,
                       row_stride, gamma, out);
    return hipGetLastError();
}

}  // namespace ms
