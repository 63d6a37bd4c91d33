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
};

}  // namespace ms
