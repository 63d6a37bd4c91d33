// ms_dqn.h — launch arguments of the DQN kernels (dqn_kernels.hip), shared with capi.cpp.
#pragma once

#include <stddef.h>
#include <stdint.h>

namespace ms {

constexpr int kQH = 16;  // DQNEntity hidden width (DQNmodules.py:41-46)

struct QArgs {  // one unit type's nets, stacked over groups (nn.Linear layouts)
    const float *w1, *b1, *w2, *b2;  // [G][16][D], [G][16], [G][A][16], [G][A]
    int D, A, G, upg;                // upg = units per group
};

struct DqnActArgs {
    QArgs q;
    const int8_t* obs;  // [E][U][stride]
    int stride, U;
    long long E;
    double eps;              // exploration threshold of this round
    const double* uniforms;  // [2][E*U] or NULL (Philox keyed by seed, counter (row, offset))
    uint64_t seed, offset;
    const uint64_t* offset_dev;
    int8_t* action;  // [E][U]
    int8_t* greedy;  // [E][U] argmax or NULL
};

struct DqnGradArgs {
    QArgs q, t;  // policy and target nets (same shapes)
    const int8_t *states, *next_states;  // memory [E][U][cap][stride]
    const int8_t* actions;               // [E][U][cap]
    const float* rewards;                // [E][U][cap]
    const int32_t* samples;              // [E][U][B]
    int stride, U, cap, B, xpitch, P;
    long long E, rows;  // rows per group = upg * E * B
    float gamma, inv_rows;
    float* partials;  // [G][nblk][P]
};

struct DqnReduceArgs {
    const float* partials;
    int nblk, P, D, A;
    float clip, inv_rows;
    float *w1, *b1, *w2, *b2, *loss;
};

size_t dqn_act_lds(const QArgs& q);
size_t dqn_grad_lds(const QArgs& q, int xpitch);

}  // namespace ms
