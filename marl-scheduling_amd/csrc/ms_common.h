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

// ---- the four 16-lane rows of a wave without LDS: v_permlane16_swap / v_permlane32_swap (gfx950).
// With both operands the same register, permlane16_swap returns rows (0, 0, 2, 2) and (1, 1, 3, 3)
// and permlane32_swap halves (lo, lo) and (hi, hi): each lane gets its partner's value beside its
// own. The reductions below equal the __shfl_xor(16) / (32) forms bit for bit (add and max are
// commutative), without the LDS crossbar round trips.
__device__ __forceinline__ void swap16(uint32_t v, uint32_t& a, uint32_t& b) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    a = r[0];
    b = r[1];
}
__device__ __forceinline__ void swap32(uint32_t v, uint32_t& a, uint32_t& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    a = r[0];
    b = r[1];
}
// v(l) + v(l ^ 16), then + the same of l ^ 32: the sum over lanes j, j+16, j+32, j+48 (j = l % 16)
__device__ __forceinline__ float rows_sum(float v) {
    uint32_t a, b;
    swap16(__float_as_uint(v), a, b);
    const float s = __uint_as_float(a) + __uint_as_float(b);
    swap32(__float_as_uint(s), a, b);
    return __uint_as_float(a) + __uint_as_float(b);
}
// rows_sum of two values at once (three swaps instead of four, bit-identical to rows_sum of each):
// swap16(x, y) leaves rows (x0, y0, x2, y2) and (x1, y1, x3, y3), whose sum holds x's pair sums in
// rows 0 / 2 and y's in rows 1 / 3; swap32 + add gives the totals (x, y, x, y), and one more swap16
// spreads each over all four rows
__device__ __forceinline__ void rows_sum2(float& x, float& y) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    const float s = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    uint32_t a, b;
    swap32(__float_as_uint(s), a, b);
    const float t = __uint_as_float(a) + __uint_as_float(b);
    swap16(__float_as_uint(t), a, b);
    x = __uint_as_float(a);
    y = __uint_as_float(b);
}
__device__ __forceinline__ void rows_max2(float& x, float& y) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    const float s = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    uint32_t a, b;
    swap32(__float_as_uint(s), a, b);
    const float t = fmaxf(__uint_as_float(a), __uint_as_float(b));
    swap16(__float_as_uint(t), a, b);
    x = __uint_as_float(a);
    y = __uint_as_float(b);
}
__device__ __forceinline__ void rows_sum2_i(int& x, int& y) {
    const auto r = __builtin_amdgcn_permlane16_swap((uint32_t)x, (uint32_t)y, false, false);
    const int s = (int)r[0] + (int)r[1];
    uint32_t a, b;
    swap32((uint32_t)s, a, b);
    const int t = (int)a + (int)b;
    swap16((uint32_t)t, a, b);
    x = (int)a;
    y = (int)b;
}
__device__ __forceinline__ float rows_max(float v) {
    uint32_t a, b;
    swap16(__float_as_uint(v), a, b);
    const float s = fmaxf(__uint_as_float(a), __uint_as_float(b));
    swap32(__float_as_uint(s), a, b);
    return fmaxf(__uint_as_float(a), __uint_as_float(b));
}
__device__ __forceinline__ int rows_sum_i(int v) {
    uint32_t a, b;
    swap16((uint32_t)v, a, b);
    const int s = (int)a + (int)b;
    swap32((uint32_t)s, a, b);
    return (int)a + (int)b;
}
__device__ __forceinline__ int rows_max_i(int v) {
    uint32_t a, b;
    swap16((uint32_t)v, a, b);
    const int s = max((int)a, (int)b);
    swap32((uint32_t)s, a, b);
    return max((int)a, (int)b);
}
// r[k] = v of lane l % 16 + 16 k (= __shfl(v, l % 16 + 16 k)) for k = 0..3
__device__ __forceinline__ void rows_bcast(uint32_t v, uint32_t (&r)[4]) {
    uint32_t a, b;
    swap16(v, a, b);          // a: rows (0, 0, 2, 2), b: rows (1, 1, 3, 3)
    swap32(a, r[0], r[2]);    // rows 0 and 2 everywhere
    swap32(b, r[1], r[3]);    // rows 1 and 3
}

// ---- an array addressed as a raw buffer: a wave-uniform base in scalar registers and 32-bit per-lane
// byte offsets (no 64-bit address arithmetic per access; a 32-bit multiply is a quarter-rate VALU
// op, __umul24 a full-rate one). Accesses at or past `bytes` read 0 / are dropped.
struct RawBuf {
    __amdgpu_buffer_rsrc_t r;
    __device__ __forceinline__ RawBuf(const void* base, long long bytes) {
        r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0,
                                              (int)(bytes < 0 ? 0 : (bytes > 0x7fffffffll ? 0x7fffffffll : bytes)),
                                              0x00020000);
    }
    __device__ __forceinline__ uint32_t ld32(uint32_t off) const {
        return __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0);
    }
    __device__ __forceinline__ float ldf(uint32_t off) const { return __uint_as_float(ld32(off)); }
    __device__ __forceinline__ int ld8s(uint32_t off) const {
        return (int)(int8_t)__builtin_amdgcn_raw_buffer_load_b8(r, (int)off, 0, 0);
    }
    __device__ __forceinline__ void st8(uint32_t off, int v) const {
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, r, (int)off, 0, 0);
    }
    __device__ __forceinline__ void stf(uint32_t off, float v) const {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)off, 0, 0);
    }
};

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
