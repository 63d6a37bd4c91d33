// ms_common.h — the cooperative row scan shared by the common-row act and PPO-gradient kernels.
//
// A 64-row scan step asks, for every row, whether it equals the common row (the acceptor row of
// a core the agent does not own, Agent.py:167-212). LPR lanes read one row with 16-byte loads:
// chunk c of a row starts at dword min(4c, stride4 - 4) (the last chunk overlaps its neighbour
// instead of running past the row), so a load instruction covers 64 / LPR rows and the step
// needs LPR instructions instead of one per dword. Needs stride4 >= 4.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ms {

typedef uint32_t u4a __attribute__((ext_vector_type(4), aligned(4)));  // 4-byte aligned 16-byte load

template <int LPR>
struct CommonScan {
    static constexpr int RPI = 64 / LPR;  // rows per load instruction
    u4a tc;                               // the common row's dwords of this lane's chunk
    int start;                            // the chunk's first dword, -1: no chunk for this lane
    u4a nx[LPR];                          // the next step's chunks: instruction i -> row i*RPI + lane/LPR

    __device__ __forceinline__ void init(const uint32_t* crow, int stride4, int lane) {
        const int c = lane % LPR, nch = (stride4 + 3) / 4;
        start = c < nch ? min(4 * c, stride4 - 4) : -1;
        tc = start >= 0 ? *reinterpret_cast<const u4a*>(crow + start) : u4a{0, 0, 0, 0};
    }
    // rowptr(k): dword pointer of step row k in [0, 64) (a valid row for rows past the range)
    template <class RowPtr>
    __device__ __forceinline__ void load_into(u4a (&dst)[LPR], RowPtr rowptr, int lane) const {
#pragma unroll
        for (int i = 0; i < LPR; i++) {
            const uint32_t* src = rowptr(i * RPI + lane / LPR);
            dst[i] = start >= 0 ? *reinterpret_cast<const u4a*>(src + start) : tc;
        }
    }
    template <class RowPtr>
    __device__ __forceinline__ void load(RowPtr rowptr, int lane) {
        load_into(nx, rowptr, lane);
    }
    __device__ __forceinline__ bool lane_row_common(int lane) const { return common_of(nx, lane); }
    // whether step row `lane` of the chunks in src equals the common row
    __device__ __forceinline__ bool common_of(const u4a (&src)[LPR], int lane) const {
        uint64_t sel = 0;
#pragma unroll
        for (int i = 0; i < LPR; i++) {
            const u4a d = src[i] ^ tc;
            const uint64_t m = __ballot((d[0] | d[1] | d[2] | d[3]) != 0u);
            sel = (lane / RPI == i) ? m : sel;
        }
        const uint64_t grp = LPR == 64 ? ~0ull : ((1ull << LPR) - 1ull);
        return ((sel >> ((lane % RPI) * LPR)) & grp) == 0;
    }
};

}  // namespace ms
