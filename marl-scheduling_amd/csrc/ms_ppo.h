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
    int64_t rrs, rus;                                // row (r, u) of states / actions / old_lp at r*rrs + u*rus:
                                                     //   (U, 1) for [R][U], (1, unit stride) unit-major
    const float* ret;                                // [T][E][ret_ld] normalised returns
    const int32_t* unit_of_group;                    // [G]
    const int8_t* common;                            // [stride] rows equal to it share one forward, or NULL
    const int8_t* owner;                             // compact acceptor rows: states [R][owner_C][stride],
    int owner_C;                                     //   owner [R][owner_C] (unit u = a*C + c), or NULL
    float* partials;                                 // [G][n_chunks][P]
    int D, A, stride, T, U, G, ret_ld;
    long long E, R;
    int chunk_tiles, n_chunks, P;
    float eps_clip, inv_R;
    int part_rows, part_off;  // partial vectors per group, this launch's first one
    int blocks_per_group;     // blocks per group of this launch (set by the launcher)
    // keyed rows (rows of <= 4 bytes whose values lie in [-8, 24), ppo_kernels.hip): a row's dense
    // index packs its bytes 5 bits each; the distinct rows of a group, ranked by dense index, get
    // one forward and one backward pass, and every row adds its loss derivatives to its rank's
    // int64 fixed-point sums (per scan block, in LDS)
    uint8_t* key_mark;     // [G][kKeyDense] dense index occurs
    uint32_t* key_idx;     // [G][R] the rows' dense indices, actions, old log-probs, returns (contiguous)
    int8_t* key_act;
    float* key_olp;
    float* key_ret;
    int32_t* key_rank;     // [G][kKeyDense] dense index -> rank
    uint32_t* key_sorted;  // [G][kKeyMaxRanks] rank -> row word
    int32_t* key_n;        // [G] distinct rows, -1: the group takes the tile path
    int32_t* key_flag;     // [G] set when a row is out of range or its terms too large (tile path)
    long long* key_part;   // [G][scan blocks][kKeyMaxRanks][16*NT + 1] per scan block: sums of
                           //   d min(surr) / d ratio * ratio per action, of V - G
    uint32_t* key_pcnt;    // [G][scan blocks][kKeyMaxRanks] rows per rank
    float* key_ploss;      // [G][scan blocks][4] the scan blocks' loss sums
    float* key_fwd;        // [G][kKeyMaxRanks][16*NT + 4] clamped log-probs, V, entropy per rank
    float key_bound;       // a larger |term| sends the group to the tile path (keeps the sums in int64)
    int key_nbs;           // scan blocks per group
    int key_cap;           // ranks per scan pass (LDS)
    // compact acceptor rows of many groups (G >= kOwnMinGroups, the divided acceptors): k_own_scan
    // reads every row once for 64 groups at a time (lane = group), sums the common rows' loss
    // derivatives and marks the rest; the tile kernel (kMaskRow) runs only the marked rows
    uint32_t* own_mask;    // [G][own_words] bit r of word w: row 32w + r goes to the tiles
    int own_words;         // ceil(R / 32)
    int own_nb;            // scan blocks per group (kOwnScanRows * 4 rows each)
    long long* own_part;   // [G][own_nb][A] int64 fixed-point sums of d min(surr)/d ratio * ratio
    float* own_wpart;      // [G][4 * own_nb][8] per scan wave: sum of (V - G)/R, count, loss sums
    float* own_cfwd;       // [G][16*NT + 4] the common row's clamped log-probs, V, entropy
    float* own_csum;       // [G][16*NT + 8] the group's common-row sums (k_own_common)
    float own_qbound;      // a larger |term| marks the row for the tiles (|sum| * 2^28 < 2^63)
};

constexpr int kOwnMinGroups = 64;     // groups from which compact rows take k_own_scan + kMaskRow
constexpr int kOwnScanRows = 1024;    // rows per scan wave (a multiple of 32: whole mask words)

// row (r, u) of the rollout arrays (states rows, actions, old log-probs): [R][U] or unit-major
__device__ __forceinline__ size_t ru_index(const PpoArgs& p, long long r, int u) {
    return (size_t)r * (size_t)p.rrs + (size_t)u * (size_t)p.rus;  // no branch: loads batch as before
}

constexpr int kKeyDense = 1 << 20;   // 4 bytes x 5 bits
constexpr int kKeyMaxRanks = 4096;   // distinct rows per group, more: tile path
constexpr int kKeyBlocks = 32;       // blocks per group of the rank passes (forward, backward)
constexpr int kKeyScanBlocks = 32;   // blocks per group of the row scan
// 2^20: fixed-point scale of the keyed sums. A term's rounding is 2^-21 (a 21-bit mantissa at |term| ~ 1;
// the integer sums themselves are exact), and terms up to 2^42 / R stay in range (1.3e6 at cfg3's
// R = 3.3M rows: a ratio far from 1 with a negative advantage after an earlier draw's update; at
// 2^28 the bound was 5242, and one such row sent its whole group to the tile path)
constexpr double kKeyFx = 1048576.0;

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
