// ms_wide.h — launch arguments of the wide-net PPO kernels (wide_kernels.hip), shared with capi.cpp.
// "Wide" nets are the aggregated agents' ActorCritics (PPOmodules.py:177-232): 32 or 64 hidden units
// and (O+1)^C, (C+1)^L or their product actions, one net per agent (group).
#pragma once

#include <stddef.h>
#include <stdint.h>

namespace ms {

constexpr int kWideRowsPerTile = 16;
constexpr int kWideThreads = 256;
constexpr int kWideStats = 16;  // per-row scalars in a row record (see WideRows)

// Net pointers: group g's tensors start at w1 + g*H*D, b1 + g*H, w2 + g*H*H, b2 + g*H,
// w3 + g*A*H, b3 + g*A (A = 1 for the critic).
struct WideNet {
    const float *w1, *b1, *w2, *b2, *w3, *b3;
};

struct WideAct {
    WideNet actor;
    int D, H, A, G;
    const int8_t* obs;  // row (e, g) at obs + (e * G + g) * stride
    int stride;
    long long E;
    const float* uniforms;  // [E][G]
    int32_t* action;        // [E][G]
    float* logprob;         // [E][G]
};

// Offsets (floats) of one group's gradient in the flat partial vectors: o[i] for the tensors in
// ms_ppo_grads order, o[kWideSegs] = the vector's length.
enum { kOW1 = 0, kOB1, kOW2, kOB2, kOW3, kOB3, kOCW1, kOCB1, kOCW2, kOCB2, kOCW3, kOCB3, kWideSegs };
struct WideOffsets {
    long long o[kWideSegs + 1];
};

// Row record (floats, RW = 8H + kWideStats per row, [G][R][RW]):
//   h1 | h2 | hc1 | hc2 | d1 | d2 | c1 | c2 | stats
// d = d loss / d (pre-activation) of the actor's layers 1, 2; c the critic's. stats:
//   0 M (max logit) 1 rS (1 / sum exp) 2 inv1 (1 / sum softmax) 3 x1 4 x2 5 g_lp 6 g_h 7 g_v 8 act (int bits)
enum { kStM = 0, kStRS, kStInv1, kStX1, kStX2, kStGlp, kStGh, kStGv, kStAct };

struct WideRows {
    WideNet actor, critic;
    int D, H, A, G;
    const int8_t* states;  // row (r, g) at states + (r * G + g) * stride
    int stride;
    long long R;
    const int32_t* actions;     // [R][G]
    const float* old_logprob;   // [R][G]
    const float* returns;       // [G][R]
    float eps_clip, inv_R;
    int NB;                     // blocks per group
    float* zbuf;                // [G][NB][16][A]
    float* rec;                 // [G][R][RW]
    float* loss_part;           // [G][NB][3]
};

struct WideGrads {  // split partials and the reduce
    WideNet actor, critic;
    int D, H, A, G;
    const int8_t* states;
    int stride;
    long long R;
    int RS;              // row splits
    long long rows_per_split;  // multiple of 16
    const float* rec;
    float* part;         // [RS][G][total]
    WideOffsets off;
};

struct WideReduce {
    const float* part;  // [RS][G][total]
    int RS, G, NB;
    WideOffsets off;
    float* dst[kWideSegs];  // grads in WideOffsets order, each [G][count]
    const float* loss_part;
    float* loss;        // [G][3]
    float inv_R;
};

}  // namespace ms
