// ms_bdqn.h — launch arguments of the Branching DQN acting kernels (bdqn_kernels.hip), shared with capi.cpp.
#pragma once

#include <stddef.h>
#include <stdint.h>

namespace ms {

constexpr int kBH = 128;     // BranchingQNetwork hidden width (BranchingDQNModules.py:85)
constexpr int kBPitch = 132; // LDS row pitch (floats) of staged 128-wide weight rows: 16 lanes' b128 reads hit 64 banks

struct BdqnNet {  // one BranchingQNetwork, heads stacked (head b = rows b*n .. b*n+n-1 of wa / ba)
    const float *w1, *b1, *w2, *b2, *wv, *bv, *wa, *ba;
    int obs, ac_dim, n;
};

// layer 1 of the aggregated acceptor rows from compact observations (h1 = base + sum of owned cores' W1_c (R_c - F))
struct BdqnL1Compact {
    const uint16_t* w1s;       // [3][128][C][Dp] bf16 bit patterns: W1 = hi + mid + lo exactly, zero for k >= D
    const float* base;         // [128]: b1 + sum_c W1_c F
    const float* cF;           // [C][128]: W1_c F
    const int8_t* core_rows;   // [E][C][stride]
    const int8_t* core_owner;  // [E][C]
    long long E;
    int N, C, D, Dp, stride;
    float* P;                  // [E][C][128] scratch: W1_c (R_c - F)
    float* h1;                 // [E*N][128]
};

struct BdqnAct {
    BdqnNet q;
    const float* h1;       // [rows][128] layer-1 pre-activations, or NULL: layer 1 from x in the kernel
    const int8_t* x;       // [rows][x_stride] int8 inputs (h1 == NULL)
    const uint16_t* w1s;   // [3][128][Kp] split W1 (h1 == NULL)
    int x_stride, Kp;
    long long rows;
    const uint8_t* explore;  // [rows] nonzero: take rnd (or NULL)
    const int8_t* rnd;       // [rows][ac_dim]
    int8_t* action;          // [rows][ac_dim]
    // compact acceptor rows (P != NULL, h1 == NULL): layer 1 of agent row r = e * N + a is
    // base + the P rows of the cores agent a owns, in core order (k_bdqn_l1_gather's sum, in the kernel)
    const float* P;            // [E][C][128] W1_c (R_c - F)
    const float* base;         // [128]
    const int8_t* core_owner;  // [E][C]
    int N, C;
    // with a row list (list != NULL, compact rows): the kernel runs rows list[0 .. 1 + *n_owning) only,
    // entry -1 being the common row (an agent owning no core: layer 1 = base), whose greedy actions go
    // to common[ac_dim]; k_bdqn_common_fill then writes them to every row of an agent owning no core
    const int32_t* list;
    const int32_t* n_owning;
    int8_t* common;
    unsigned long long* own_mask;  // [E] agents owning a core, bit a (N <= 64)
};

// update_policy of one role (bdqn_update_kernels.hip)
struct BdqnGrads {
    float *w1, *b1, *w2, *b2, *wv, *bv, *wa, *ba;  // clamped gradients of the online net
    float* loss;                                   // [1]
};
struct BdqnUpd {
    BdqnNet q, t;             // online and target nets
    const int8_t* xs;         // [B][ld] state rows (int8 observations)
    const int8_t* xn;         // [B][ld] next-state rows
    int ld;
    const int8_t* act;        // [B][act_ld] the taken actions, one per branch
    int act_ld;
    const float* rew;         // [B]
    const float* mask;        // [B] 0 at an episode end
    int B;                    // <= 128
    float gamma, clip;
    int nK;                   // layer-1 K chunks of 128 inputs
    int Mp;                   // head rows (ac_dim * n advantage rows, then the value row) padded to 64
    float* l1p;               // [3][nK][128][128] layer-1 partial sums of the three forwards
    float* out1;              // [128][128] ReLU output of layer 1 of q(s)
    float* out2;              // [3][128][128] ReLU outputs of layer 2 of q(s), q(s'), target(s')
    float* q3;                // [3][128][Mp] head outputs (advantages, then the value) of the three forwards
    float* dq;                // [128][Mp] d loss / d head outputs of q(s) (zero rows past B)
    float* d2p;               // [Mp / 64][128][128] d out2 partial sums per chunk of 64 head rows
    float *dpre2, *dpre1;     // [128][128] d loss / d pre-activations of layers 2 and 1
    float* lossb;             // [128] squared errors of a row (summed over the branches)
    BdqnGrads g;
};
constexpr int kUpdMaxHeadRows = 5440;  // Mp * 3 floats of one row's head outputs in 64 KB of LDS

}  // namespace ms
