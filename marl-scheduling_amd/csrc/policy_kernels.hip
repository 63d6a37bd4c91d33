// policy_kernels.hip — PPO action selection and return estimation for gfx950.
//
// k_act: ActorCritic.act (PPOmodules.py:53-63) for every unit of every env
// replica. A wave takes 16 observation rows at a time and runs
// Linear(D,16)-tanh-Linear(16,16)-tanh-Linear(16,A) on the f32 MFMA
// (v_mfma_f32_16x16x4_f32) with the batch on the lane axis, so each layer's
// accumulator is the next layer's B operand unchanged (the weights are read
// with a permuted k order). Softmax, the Categorical renormalisation and the
// inverse-CDF sample run on the accumulator layout: a row's logits live in 4
// lanes x 4 registers per 16 actions, reduced with two xor-shuffles.
// With a second (price) net the kernel is FreePriceOfferPPO.selectAction
// (PPOmodules.py:312-332): core chooser, then the price chooser on
// [obs[2a:2a+2], obs[-2:]] (or the dummy [-5,-5,-5,-5] for a = 0), in one launch.
//
// k_returns: PPO.update's Monte-Carlo returns (PPOmodules.py:128-137) in
// float64, cast to f32 and normalised per sequence.
#include <hip/hip_runtime.h>
#include <math.h>

#include "../../include/marlsched.h"

namespace ms {

typedef float f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

__device__ __forceinline__ uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t& hi) {
    uint64_t p = (uint64_t)a * b;
    hi = (uint32_t)(p >> 32);
    return (uint32_t)p;
}

// Philox4x32-10 (Salmon et al., SC'11); returns the first two output words.
__device__ __forceinline__ void philox2(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                                        uint32_t& o0, uint32_t& o1) {
    for (int r = 0; r < 10; r++) {
        uint32_t hi0, hi1;
        uint32_t lo0 = mulhilo(0xD2511F53u, c0, hi0);
        uint32_t lo1 = mulhilo(0xCD9E8D57u, c2, hi1);
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    o0 = c0;
    o1 = c1;
}

__device__ __forceinline__ float u24(uint32_t r) { return (float)(r >> 8) * (1.0f / 16777216.0f); }

__device__ __forceinline__ float xsum4g(float v) {
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    return v;
}

// One net's weights staged in LDS: W1 [16][D4] (zero padded), W2 [16][16], W3 [16*NT][16] (zero rows >= A), biases.
struct NetLds {
    float *w1, *w2, *w3, *b1, *b2, *b3;
    int D, D4, A;
};

template <int NT>
__device__ float* stage_net(float* s, const ms_mlp_params& p, int g, int tid, int nthreads, NetLds& n) {
    n.D = p.in_dim;
    n.D4 = (p.in_dim + 3) & ~3;
    n.A = p.n_actions;
    n.w1 = s;
    n.w2 = n.w1 + 16 * n.D4;
    n.w3 = n.w2 + 256;
    n.b1 = n.w3 + 256 * NT;
    n.b2 = n.b1 + 16;
    n.b3 = n.b2 + 16;
    const int D = n.D, D4 = n.D4, A = n.A;
    for (int i = tid; i < 16 * D4; i += nthreads) {
        int r = i / D4, c = i % D4;
        n.w1[i] = c < D ? p.w1[((size_t)g * 16 + r) * D + c] : 0.f;
    }
    for (int i = tid; i < 256; i += nthreads) n.w2[i] = p.w2[(size_t)g * 256 + i];
    for (int i = tid; i < 256 * NT; i += nthreads) {
        int a = i / 16;
        n.w3[i] = a < A ? p.w3[((size_t)g * A + a) * 16 + (i % 16)] : 0.f;
    }
    for (int i = tid; i < 16; i += nthreads) {
        n.b1[i] = p.b1[g * 16 + i];
        n.b2[i] = p.b2[g * 16 + i];
    }
    for (int i = tid; i < 16 * NT; i += nthreads) n.b3[i] = i < A ? p.b3[(size_t)g * A + i] : 0.f;
    return n.b3 + 16 * NT;
}

// Layers 2-3, softmax, Categorical renormalisation and inverse-CDF sample for the
// 16 rows of a tile given layer-1 pre-activations. Returns the action of row
// (lane & 15) in every lane of that row and its log-probability.
template <int NT>
__device__ __forceinline__ void head(const NetLds& n, f4 a1, int j, int g4, float u, int& action, float& logprob) {
    float h1[4];
#pragma unroll
    for (int q = 0; q < 4; q++) h1[q] = tanhf(a1[q] + n.b1[4 * g4 + q]);
    f4 a2 = {0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 4; s++) a2 = mfma4(n.w2[j * 16 + 4 * g4 + s], h1[s], a2);
    float h2[4];
#pragma unroll
    for (int q = 0; q < 4; q++) h2[q] = tanhf(a2[q] + n.b2[4 * g4 + q]);
    float z[NT][4];
    float m = -INFINITY;
#pragma unroll
    for (int t = 0; t < NT; t++) {
        f4 zz = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < 4; s++) zz = mfma4(n.w3[(16 * t + j) * 16 + 4 * g4 + s], h2[s], zz);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            z[t][q] = zz[q] + n.b3[16 * t + 4 * g4 + q];
            if (16 * t + 4 * g4 + q < n.A) m = fmaxf(m, z[t][q]);
        }
    }
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    float s0 = 0.f;
#pragma unroll
    for (int t = 0; t < NT; t++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
            z[t][q] = (16 * t + 4 * g4 + q < n.A) ? expf(z[t][q] - m) : 0.f;
            s0 += z[t][q];
        }
    const float inv0 = 1.f / xsum4g(s0);
    float s1 = 0.f;
#pragma unroll
    for (int t = 0; t < NT; t++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
            z[t][q] *= inv0;  // nn.Softmax output
            s1 += z[t][q];
        }
    const float inv1 = 1.f / xsum4g(s1);
    // Categorical renormalisation, then the inverse CDF over a = 16t + 4*g4 + q in increasing order
    float cum = 0.f, pc = 0.f;
    int found = 0x7fff, last_nz = -1;
#pragma unroll
    for (int t = 0; t < NT; t++) {
        float bs = 0.f;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            z[t][q] *= inv1;
            bs += z[t][q];
        }
        const float gs0 = __shfl(bs, j), gs1 = __shfl(bs, j + 16), gs2 = __shfl(bs, j + 32), gs3 = __shfl(bs, j + 48);
        float c = cum + (g4 > 0 ? gs0 : 0.f) + (g4 > 1 ? gs1 : 0.f) + (g4 > 2 ? gs2 : 0.f);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int a = 16 * t + 4 * g4 + q;
            c += z[t][q];
            if (a < n.A) {
                if (z[t][q] > 0.f) last_nz = a;
                if (u < c && a < found) {
                    found = a;
                    pc = z[t][q];
                }
            }
        }
        cum += gs0 + gs1 + gs2 + gs3;
    }
    // first crossing over the 4 lanes of the row (each lane found its own first one)
    int fmin = min(found, __shfl_xor(found, 16));
    fmin = min(fmin, __shfl_xor(fmin, 32));
    int lmax = max(last_nz, __shfl_xor(last_nz, 16));
    lmax = max(lmax, __shfl_xor(lmax, 32));
    int a_sel = fmin < n.A ? fmin : lmax;
    float mine = 0.f;
    if (fmin < n.A) {
        mine = (found == fmin) ? pc : 0.f;
    } else {
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (16 * t + 4 * g4 + q == a_sel) mine = z[t][q];
    }
    const float pa = xsum4g(mine);
    const float eps = 1.1920928955078125e-07f;  // torch.finfo(float32).eps
    action = a_sel;
    logprob = logf(fminf(fmaxf(pa, eps), 1.f - eps));
}

struct ActArgs {
    ms_mlp_params n1, n2;  // n2 used only with a price net (NT2 > 0)
    const int8_t* obs;
    int stride, U, S, n_cores;
    int E, n_items;
    int tiles_per_wave, blocks_per_group;
    uint64_t seed, offset;
    const uint64_t* offset_dev;
    const float* uniforms;  // [2][E*U] or NULL
    int8_t* action;
    float* logprob;
    int8_t* price_state;   // [E*U][4]
    int8_t* price_action;
    float* price_logprob;
    int8_t* env_price;
};

constexpr int kPreW = 16;  // prefetch dwords per lane: 16 rows x 256 B / 64 lanes

template <int NT, int NT2>
__global__ void __launch_bounds__(256) k_act(ActArgs a) {
    extern __shared__ __align__(16) float sm[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int j = lane & 15, g4 = lane >> 4;
    const int grp = blockIdx.x / a.blocks_per_group;
    const int blk = blockIdx.x % a.blocks_per_group;
    NetLds n1, n2;
    float* s = stage_net<NT>(sm, a.n1, grp, tid, 256, n1);
    if (NT2 > 0) s = stage_net<(NT2 > 0 ? NT2 : 1)>(s, a.n2, grp, tid, 256, n2);
    int8_t* sx = reinterpret_cast<int8_t*>(s) + wave * 16 * a.stride;  // this wave's observation tile
    __syncthreads();
    const uint64_t off = a.offset + (a.offset_dev ? *a.offset_dev : 0ull);
    const int stride4 = a.stride >> 2;
    const int n_rows_total = a.E * a.U;
    const int S1 = n1.D4 / 4;
    // this wave's tiles: [t0, t1)
    const int tiles = (a.n_items + 15) >> 4;
    const int t0 = (blk * 4 + wave) * a.tiles_per_wave;
    const int t1 = min(t0 + a.tiles_per_wave, tiles);
    // lane j copies dwords j-row, columns g4 + 4m; the same lane owns row j's outputs
    auto row_of = [&](int tile) -> int {
        int i = tile * 16 + j;
        if (i >= a.n_items) return -1;
        int e = i / a.S;
        return e * a.U + grp * a.S + (i - e * a.S);
    };
    uint32_t pre[kPreW];
    int row = t0 < t1 ? row_of(t0) : -1;
    auto prefetch = [&](int r) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.obs + (size_t)(r < 0 ? 0 : r) * a.stride);
#pragma unroll
        for (int m = 0; m < kPreW; m++) {
            int cc = g4 + 4 * m;
            pre[m] = (r >= 0 && cc < stride4) ? src[cc] : 0u;
        }
    };
    if (t0 < t1) prefetch(row);
    for (int tile = t0; tile < t1; tile++) {
#pragma unroll
        for (int m = 0; m < kPreW; m++) {
            int cc = g4 + 4 * m;
            if (cc < stride4) reinterpret_cast<uint32_t*>(sx)[j * stride4 + cc] = pre[m];
        }
        const int cur = row;
        if (tile + 1 < t1) {
            row = row_of(tile + 1);
            prefetch(row);
        }
        __builtin_amdgcn_wave_barrier();
        const bool valid = cur >= 0;
        float u1, u2;
        if (a.uniforms) {
            u1 = valid ? a.uniforms[cur] : 0.f;
            u2 = valid && NT2 > 0 ? a.uniforms[n_rows_total + cur] : 0.f;
        } else {
            uint32_t r0, r1;
            philox2((uint32_t)cur, 0u, (uint32_t)off, (uint32_t)(off >> 32), (uint32_t)a.seed, (uint32_t)(a.seed >> 32),
                    r0, r1);
            u1 = u24(r0);
            u2 = u24(r1);
        }
        f4 acc = {0, 0, 0, 0};
        for (int k = 0; k < S1; k++) acc = mfma4(n1.w1[j * n1.D4 + 4 * k + g4], (float)sx[j * a.stride + 4 * k + g4], acc);
        int act;
        float lp;
        head<NT>(n1, acc, j, g4, u1, act, lp);
        if (NT2 > 0) {
            // price chooser input (PPOmodules.py:316-327)
            int8_t pin;
            if (act == 0)
                pin = -5;
            else
                pin = (g4 < 2) ? sx[j * a.stride + 2 * act + g4] : sx[j * a.stride + 2 * a.n_cores + (g4 - 2)];
            f4 acc2 = {0, 0, 0, 0};
            acc2 = mfma4(n2.w1[j * n2.D4 + g4], (float)pin, acc2);
            int pact;
            float plp;
            head<(NT2 > 0 ? NT2 : 1)>(n2, acc2, j, g4, u2, pact, plp);
            if (valid) {
                a.price_state[(size_t)cur * 4 + g4] = pin;
                if (g4 == 0) {
                    a.price_action[cur] = (int8_t)pact;
                    a.price_logprob[cur] = plp;
                    a.env_price[cur] = (int8_t)(act == 0 ? -5 : pact);
                }
            }
        }
        if (valid && g4 == 0) {
            a.action[cur] = (int8_t)act;
            a.logprob[cur] = lp;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

static size_t net_lds_floats(int D, int NT) { return 16 * (size_t)((D + 3) & ~3) + 256 + 256 * NT + 32 + 16 * NT; }

template <int NT, int NT2>
static hipError_t launch_act_t(ActArgs& a, hipStream_t st) {
    size_t lds = sizeof(float) * (net_lds_floats(a.n1.in_dim, NT) + (NT2 > 0 ? net_lds_floats(a.n2.in_dim, NT2) : 0)) +
                 4 * 16 * (size_t)a.stride;
    const int G = a.n1.n_groups;
    const int tiles = (a.n_items + 15) / 16;
    // ~2048 blocks of 4 waves over all groups; each wave walks a contiguous tile range with a prefetch
    int tpw = (int)(((long long)tiles * G + 8191) / 8192);
    a.tiles_per_wave = tpw < 1 ? 1 : tpw;
    a.blocks_per_group = (tiles + 4 * a.tiles_per_wave - 1) / (4 * a.tiles_per_wave);
    hipLaunchKernelGGL((k_act<NT, NT2>), dim3((unsigned)(a.blocks_per_group * G)), dim3(256), lds, st, a);
    return hipGetLastError();
}

static hipError_t dispatch_act(ActArgs& a, hipStream_t st) {
    const int nt = (a.n1.n_actions + 15) / 16;
    const int nt2 = a.n2.n_groups > 0 ? (a.n2.n_actions + 15) / 16 : 0;
#define MS_ACT(T, T2) \
    if (nt <= T && nt2 == T2) return launch_act_t<T, T2>(a, st);
    if (nt2 == 0) {
        MS_ACT(1, 0) MS_ACT(2, 0) MS_ACT(4, 0) MS_ACT(8, 0)
    } else if (nt2 == 1) {
        MS_ACT(1, 1) MS_ACT(2, 1) MS_ACT(4, 1)
    } else if (nt2 == 2) {
        MS_ACT(1, 2) MS_ACT(2, 2) MS_ACT(4, 2)
    } else if (nt2 <= 8) {
        if (nt <= 4) return launch_act_t<4, 8>(a, st);
    }
#undef MS_ACT
    return hipErrorInvalidValue;
}

hipError_t launch_policy_act(const ms_mlp_params* p, const int8_t* obs, int stride, int64_t E, int U, int S,
                             uint64_t seed, uint64_t offset, const uint64_t* offset_dev, const float* uniforms,
                             int8_t* action, float* logprob, hipStream_t st) {
    ActArgs a{};
    a.n1 = *p;
    a.n2.n_groups = 0;
    a.obs = obs;
    a.stride = stride;
    a.U = U;
    a.S = S;
    a.E = (int)E;
    a.n_items = (int)(E * S);
    a.seed = seed;
    a.offset = offset;
    a.offset_dev = offset_dev;
    a.uniforms = uniforms;
    a.action = action;
    a.logprob = logprob;
    return dispatch_act(a, st);
}

hipError_t launch_offer_act_free(const ms_mlp_params* core, const ms_mlp_params* price, const int8_t* obs, int stride,
                                 int64_t E, int U, int S, int n_cores, uint64_t seed, uint64_t offset,
                                 const uint64_t* offset_dev, const float* uniforms, int8_t* core_action,
                                 float* core_logprob, int8_t* price_state, int8_t* price_action, float* price_logprob,
                                 int8_t* env_price, hipStream_t st) {
    ActArgs a{};
    a.n1 = *core;
    a.n2 = *price;
    a.obs = obs;
    a.stride = stride;
    a.U = U;
    a.S = S;
    a.n_cores = n_cores;
    a.E = (int)E;
    a.n_items = (int)(E * S);
    a.seed = seed;
    a.offset = offset;
    a.offset_dev = offset_dev;
    a.uniforms = uniforms;
    a.action = core_action;
    a.logprob = core_logprob;
    a.price_state = price_state;
    a.price_action = price_action;
    a.price_logprob = price_logprob;
    a.env_price = env_price;
    return dispatch_act(a, st);
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
