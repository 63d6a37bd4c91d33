// ms_ppo.h — launch arguments of the fused PPO gradient kernel (ppo_kernels.hip),
// shared with the host ABI (capi.cpp).
#pragma once

#include <stdint.h>

namespace ms {

struct PpoArgs {
    const float *w1, *b1, *w2, *b2, *w3, *b3;        // actor  [G][16][D], [G][16], [G][16][16], [G][16], [G][A][16], [G][A]
    const float *cw1, *cb1, *cw2, *cb2, *cw3, *cb3;  // critic [G][16][D], [G][16], [G][16][16], [G][16], [G][1][16], [G][1]
    const int8_t* states;                            // [R][U][stride]  (R = T*E rows, r = t*E + e)
    const int8_t* actions;                           // [R][U]
    const float* old_lp;                             // [R][U]
    const float* ret;                                // [T][E][ret_ld] normalised returns
    const int32_t* unit_of_group;                    // [G]
    const int8_t* common;                            // [stride] rows equal to it share one forward, or NULL
    float* partials;                                 // [G][n_chunks][P]
    int D, A, stride, T, U, G, ret_ld;
    long long E, R;
    int chunk_tiles, n_chunks, P;
    float eps_clip, inv_R;
};

constexpr int kAdamMaxTensors = 16, kAdamMaxGroups = 4;
struct AdamTensor {  // layout of ms_adam_tensor
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    int64_t numel;
    int32_t lr_group;
};

struct GradOut {
    float *w1, *b1, *w2, *b2, *w3, *b3, *cw1, *cb1, *cw2, *cb2, *cw3, *cb3, *loss;
};

// parameter offsets inside one group's gradient vector
struct POff {
    int w1, b1, w2, b2, w3, b3, cw1, cb1, cw2, cb2, cw3, cb3, loss, total;
};

#if defined(__HIPCC__)
__host__ __device__
#endif
inline POff poff(int D, int A) {
    POff o;
    o.w1 = 0;
    o.b1 = o.w1 + 16 * D;
    o.w2 = o.b1 + 16;
    o.b2 = o.w2 + 256;
    o.w3 = o.b2 + 16;
    o.b3 = o.w3 + 16 * A;
    o.cw1 = o.b3 + A;
    o.cb1 = o.cw1 + 16 * D;
    o.cw2 = o.cb1 + 16;
    o.cb2 = o.cw2 + 256;
    o.cw3 = o.cb2 + 16;
    o.cb3 = o.cw3 + 16;
    o.loss = o.cb3 + 1;
    o.total = o.loss + 3;
    return o;
}

}  // namespace ms
