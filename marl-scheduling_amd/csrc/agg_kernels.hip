// agg_kernels.hip — aggregated agents (Agent.py:73-140, :359-492) around the divided env step.
//
// The aggregated / fully-aggregated agents see the same world as the divided ones: their
// observations are concatenations of the divided rows, and their one action per agent is a
// number whose base-(O+1) / base-(C+1) digits are the divided actions. So the env step runs
// unchanged (ms_env_step; its aggregated reward outputs come from the same settlement) and two
// small kernels convert at its boundary:
//  * k_aggregate_obs: divided acceptor rows [E][N][C][acc_stride] and offer rows
//    [E][N][L][off_stride] -> per agent
//      acceptor  = concat_c row(a, c)[0 : D_acc]                          (Agent.py:82-124)
//      offer     = [(prio, rem) of every core] + [(prio, rem) of every slot]
//                = row(a, 0)[0 : 2C] + concat_s row(a, s)[2C : 2C + 2]     (Agent.py:126-134)
//      fully     = concat(offer, acceptor)                                (Agent.py:464)
//    rows zero-padded to a multiple of 4 bytes;
//  * k_decode_aggregated: agent action numbers -> acceptor actions [E][N][C] and offer actions
//    [E][N][L] (numberToNDimensionalAction Agent.py:644-666: digit i in base b is the action of
//    core / slot i), with the fully aggregated split a // (C+1)^L, a % (C+1)^L (Agent.py:469-473).
// Both are byte reshuffles of a few bytes per agent: one thread per output dword / agent.
#include <hip/hip_runtime.h>

#include "../../include/marlsched.h"
#include "ms_layout.h"

namespace ms {


// byte k of agent a's aggregated offer row (k < 2C + 2L)
__device__ __forceinline__ int8_t agg_off_byte(const AggArgs& g, const int8_t* off_a, int k) {
    const int C2 = 2 * g.C;
    if (k < C2) return off_a[k];  // the cores' (prio, rem): the first 2C bytes of any slot's row
    const int s = (k - C2) >> 1;
    return off_a[(size_t)s * g.off_stride + C2 + ((k - C2) & 1)];  // slot s's (prio, rem)
}
// byte k of agent a's aggregated acceptor row (k < C * D_acc)
__device__ __forceinline__ int8_t agg_acc_byte(const AggArgs& g, const int8_t* acc_a, int k) {
    const int c = k / g.d_acc;
    return acc_a[(size_t)c * g.acc_stride + (k - c * g.d_acc)];
}

__global__ void __launch_bounds__(256) k_aggregate_obs(AggArgs g) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;  // output dword
    const int wa = g.out_acc ? g.agg_acc_stride / 4 : 0;
    const int wo = g.out_off ? g.agg_off_stride / 4 : 0;
    const int wf = g.out_full ? g.full_stride / 4 : 0;
    const int per = wa + wo + wf;
    const long long ea = i / per;  // (env, agent)
    if (ea >= g.E * g.N) return;
    int w = (int)(i - ea * per);
    const int8_t* acc_a = g.acc + (size_t)ea * g.C * g.acc_stride;
    const int8_t* off_a = g.off + (size_t)ea * g.L * g.off_stride;
    const int d_off = 2 * g.C + 2 * g.L, d_acc_all = g.C * g.d_acc;
    uint32_t v = 0;
    int8_t* dst;
    if (w < wa) {
        for (int b = 0; b < 4; b++) {
            const int k = 4 * w + b;
            if (k < d_acc_all) v |= (uint32_t)(uint8_t)agg_acc_byte(g, acc_a, k) << (8 * b);
        }
        dst = g.out_acc + (size_t)ea * g.agg_acc_stride + 4 * w;
    } else if ((w -= wa) < wo) {
        for (int b = 0; b < 4; b++) {
            const int k = 4 * w + b;
            if (k < d_off) v |= (uint32_t)(uint8_t)agg_off_byte(g, off_a, k) << (8 * b);
        }
        dst = g.out_off + (size_t)ea * g.agg_off_stride + 4 * w;
    } else {
        w -= wo;
        for (int b = 0; b < 4; b++) {
            const int k = 4 * w + b;
            int8_t x = 0;
            if (k < d_off)
                x = agg_off_byte(g, off_a, k);
            else if (k < d_off + d_acc_all)
                x = agg_acc_byte(g, acc_a, k - d_off);
            v |= (uint32_t)(uint8_t)x << (8 * b);
        }
        dst = g.out_full + (size_t)ea * g.full_stride + 4 * w;
    }
    *reinterpret_cast<uint32_t*>(dst) = v;
}

hipError_t launch_aggregate_obs(const AggArgs& g, hipStream_t st) {
    const long long per = (g.out_acc ? g.agg_acc_stride / 4 : 0) + (g.out_off ? g.agg_off_stride / 4 : 0) +
                          (g.out_full ? g.full_stride / 4 : 0);
    const long long n = g.E * g.N * per;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_aggregate_obs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g);
    return hipGetLastError();
}

// One thread per (env, agent). A number outside the action range raises ValueError in the
// reference (Agent.py:651-652): it is counted in *bad (device int, may be NULL) and decodes as
// reject everything / offer nothing.
__global__ void __launch_bounds__(256) k_decode_aggregated(const int32_t* __restrict__ actions, long long EN, int C,
                                                           int L, int O, int fully, int8_t* __restrict__ acc,
                                                           int8_t* __restrict__ off, int* bad) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= EN) return;
    long long n_off = 1, n_acc = 1;
    for (int s = 0; s < L; s++) n_off *= (C + 1);
    for (int c = 0; c < C; c++) n_acc *= (O + 1);
    long long a_acc, a_off;
    bool ok;
    if (fully) {
        const long long a = actions[i];
        ok = a >= 0 && a < n_acc * n_off;
        a_acc = a / n_off;
        a_off = a % n_off;
    } else {  // acceptor numbers [E][N], then offer numbers [E][N]
        a_acc = actions[i];
        a_off = actions[EN + i];
        ok = a_acc >= 0 && a_acc < n_acc && a_off >= 0 && a_off < n_off;
    }
    if (!ok && bad) atomicAdd(bad, 1);
    for (int c = 0; c < C; c++) {
        acc[i * C + c] = (int8_t)(ok ? a_acc % (O + 1) : O);
        a_acc /= (O + 1);
    }
    for (int s = 0; s < L; s++) {
        off[i * L + s] = (int8_t)(ok ? a_off % (C + 1) : C);
        a_off /= (C + 1);
    }
}

hipError_t launch_decode_aggregated(const int32_t* actions, long long EN, int C, int L, int O, int fully, int8_t* acc,
                                    int8_t* off, int* bad, hipStream_t st) {
    if (EN <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_aggregated, dim3((unsigned)((EN + 255) / 256)), dim3(256), 0, st, actions, EN, C, L, O,
                       fully, acc, off, bad);
    return hipGetLastError();
}


// Agent rows regenerated from the compact observations of a replay memory (ms_regen_agent_rows):
// sample b reads compact record frame[b] (core rows [C][acc_stride], owners [C], slot pairs
// [N][L][2]) as agent agent[b]. Acceptor byte k = byte k % D_acc of core k / D_acc's row if the
// agent owns that core, else of the constant foreign row [0, -1, -1, (-2, -2) * O] (Agent.py:167-212);
// offer bytes = the cores' (prio, rem) (bytes 1, 2 of every core row) then the agent's slot pairs.
__global__ void __launch_bounds__(256) k_regen_agent_rows(RegenArgs g) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    const int wa = g.acc ? g.acc_ld / 4 : 0, wo = g.off ? g.off_ld / 4 : 0;
    const int per = wa + wo;
    const long long b = i / per;
    if (b >= g.n) return;
    int w = (int)(i - b * per);
    const long long m = g.frame[b];
    const int a = g.agent[b];
    const int8_t* rows = g.core_rows + (size_t)m * g.C * g.acc_stride;
    const int8_t* own = g.core_owner + (size_t)m * g.C;
    uint32_t v = 0;
    int8_t* dst;
    if (w < wa) {
        for (int q = 0; q < 4; q++) {
            const int k = 4 * w + q;
            if (k >= g.C * g.d_acc) break;
            const int c = k / g.d_acc, col = k - c * g.d_acc;
            int8_t x;
            if (own[c] == a + 1)
                x = rows[(size_t)c * g.acc_stride + col];
            else
                x = col == 0 ? 0 : (col < 3 ? -1 : -2);
            v |= (uint32_t)(uint8_t)x << (8 * q);
        }
        dst = g.acc + (size_t)b * g.acc_ld + 4 * w;
    } else {
        w -= wa;
        const int8_t* sp = g.slot_pairs + ((size_t)m * g.N + a) * g.L * 2;
        for (int q = 0; q < 4; q++) {
            const int k = 4 * w + q;
            if (k >= 2 * g.C + 2 * g.L) break;
            const int8_t x = k < 2 * g.C ? rows[(size_t)(k >> 1) * g.acc_stride + 1 + (k & 1)] : sp[k - 2 * g.C];
            v |= (uint32_t)(uint8_t)x << (8 * q);
        }
        dst = g.off + (size_t)b * g.off_ld + 4 * w;
    }
    *reinterpret_cast<uint32_t*>(dst) = v;
}

hipError_t launch_regen_agent_rows(const RegenArgs& g, hipStream_t s) {
    const int per = (g.acc ? g.acc_ld / 4 : 0) + (g.off ? g.off_ld / 4 : 0);
    const long long n = g.n * per;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_regen_agent_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g);
    return hipGetLastError();
}
}  // namespace ms
