// env_kernels.hip — the batched marl-scheduling round as one HIP kernel for gfx950.
//
// One 64-lane wave steps one env replica per round. The env's packed state
// record (ms_layout.h) is staged in LDS and the round runs as wave-parallel
// phases. The offer set of a round (at most N*L <= 126 offers, one per slot,
// offer-ID order = slot order) is indexed by 128-bit masks, one per core and
// one per recipient, built with LDS atomic ORs: every ordered selection of the
// reference — the idx-th offer of (recipient, core) behind an acceptor action,
// the auctioneer's tied maxima, the offers listed in an acceptor observation —
// is a walk over the set bits of mask(core) & mask(recipient). The loads the
// round depends on (MT19937 window, liability chains of cores that may
// terminate) are issued right after staging so their latency overlaps the
// selection phases. Observations are assembled in LDS (prefilled with the -2
// pad by dword stores) and streamed out with dword stores. Reference semantics
// (paths relative to /root/reference/src) are cited per phase; the CPU
// restatement that checks this kernel bit-for-bit is oracle/ms_oracle.c.
#include <hip/hip_runtime.h>

#include "ms_layout.h"

namespace ms {

// Every env kernel runs one 64-lane wave per block, so a phase boundary only has to order the
// wave's own memory operations: LDS operations of one wave complete in issue order, so the
// compiler barrier is enough. A __syncthreads would also drain every outstanding load (s_waitcnt)
// at each of the round's ~20 phase boundaries.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------------------
// CPython MT19937 (Modules/_randommodule.c) — tempering and wave-cooperative twist

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// In-place twist of 624 words held in LDS by one wave. The three parallel
// phases respect the sequential recurrence: words [0,227) read only old words,
// [227,454) read new [0,227), [454,623) read new [227,396), 623 reads new 0/396.
__device__ void mt_twist_lds(uint32_t* mt, int lane) {
    auto step = [&](int i, uint32_t hi_src, uint32_t lo_src, uint32_t xsrc) -> uint32_t {
        uint32_t y = (hi_src & 0x80000000u) | (lo_src & 0x7fffffffu);
        return xsrc ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    };
    const int ranges[3][2] = {{0, kMtN - kMtM}, {kMtN - kMtM, 2 * (kMtN - kMtM)}, {2 * (kMtN - kMtM), kMtN - 1}};
    for (int ph = 0; ph < 3; ph++) {
        uint32_t v[4];
        int cnt = 0;
        for (int i = ranges[ph][0] + lane; i < ranges[ph][1]; i += kWave) {
            int x = (ph == 0) ? i + kMtM : i + (kMtM - kMtN);
            v[cnt++] = step(i, mt[i], mt[i + 1], mt[x]);
        }
        wave_sync();
        cnt = 0;
        for (int i = ranges[ph][0] + lane; i < ranges[ph][1]; i += kWave) mt[i] = v[cnt++];
        wave_sync();
    }
    if (lane == 0) mt[kMtN - 1] = step(kMtN - 1, mt[kMtN - 1], mt[0], mt[kMtM - 1]);
    wave_sync();
}

// A 64-word window of the env's stream held one word per lane. Stream
// positions are relative to the env's mti at kernel entry; positions at or
// beyond 624 - mti0 come from the twisted state (computed at most once per
// launch, only when a consumer actually needs such a word, so the stored
// state always equals CPython's after the same draws).
struct MtStream {
    uint32_t* gmt;    // env's 624 state words in HBM
    uint32_t* lds;    // 624-word LDS scratch (valid after the twist)
    int mti0;         // mti at entry
    int wb, wend;     // window covers stream positions [wb, wend)
    int p;            // next unconsumed stream position
    bool twisted;
    uint32_t v;       // this lane's tempered word (position wb + lane)

    // Window at stream position pos. need = words the caller is about to
    // consume; need == 0 only peeks (never twists; the window may be empty).
    __device__ void load(int pos, int need, int lane) {
        int limit = twisted ? 0x3fffffff : (kMtN - mti0);  // old words end here
        if (!twisted && need > 0 && pos + need > limit) {
            // read the old words of this window before the state is replaced
            int g = mti0 + pos + lane;
            uint32_t old = (g < kMtN) ? gmt[g] : 0u;
            for (int i = lane; i < kMtN; i += kWave) lds[i] = gmt[i];
            wave_sync();
            mt_twist_lds(lds, lane);
            for (int i = lane; i < kMtN; i += kWave) gmt[i] = lds[i];
            twisted = true;
            v = mt_temper((g < kMtN) ? old : lds[g - kMtN]);
            wb = pos;
            wend = pos + kWave;
            return;
        }
        int g = mti0 + pos + lane;
        uint32_t raw = 0;
        if (twisted)
            raw = (g >= kMtN && g < 2 * kMtN) ? lds[g - kMtN] : 0u;
        else if (g < kMtN)
            raw = gmt[g];
        v = mt_temper(raw);
        wb = pos;
        wend = twisted ? pos + kWave : min(pos + kWave, limit);
    }

    // Random._randbelow_with_getrandbits(n) (random.py:239-249), wave-uniform result
    __device__ uint32_t randbelow(uint32_t n, int lane) {
        int k = 32 - __clz(n);  // n.bit_length()
        int sh = 32 - k;
        for (;;) {
            if (p >= wend) load(p, 1, lane);
            int pos = wb + lane;
            bool ok = pos >= p && pos < wend && ((v >> sh) < n);
            uint64_t m = __ballot(ok);
            if (m) {
                int q = __ffsll((unsigned long long)m) - 1;
                uint32_t r = __shfl(v, q) >> sh;
                p = wb + q + 1;
                return r;
            }
            p = wend;
        }
    }

    // final mti (CPython's index after the same draws)
    __device__ int final_index() const { return twisted ? (mti0 + p - kMtN) : (mti0 + p); }
};

// ---------------------------------------------------------------------------
// record accessors (LDS copy of the env record)

struct Rec {
    uint8_t* b;
    const Params* P;
    __device__ int32_t& round() { return *reinterpret_cast<int32_t*>(b + 0); }
    __device__ uint32_t& flags() { return *reinterpret_cast<uint32_t*>(b + 4); }
    __device__ int32_t& mti() { return *reinterpret_cast<int32_t*>(b + 8); }
    __device__ int8_t* core_owner() { return reinterpret_cast<int8_t*>(b + P->o_core_owner); }
    __device__ int8_t* core_kind() { return reinterpret_cast<int8_t*>(b + P->o_core_kind); }
    __device__ int8_t* core_rem() { return reinterpret_cast<int8_t*>(b + P->o_core_rem); }
    __device__ uint8_t* liab_n() { return b + P->o_liab_n; }
    __device__ int32_t* core_birth() { return reinterpret_cast<int32_t*>(b + P->o_core_birth); }
    __device__ int8_t* slot_kind() { return reinterpret_cast<int8_t*>(b + P->o_slot_kind); }
    __device__ int8_t* slot_rem() { return reinterpret_cast<int8_t*>(b + P->o_slot_rem); }
    __device__ int8_t* slot_wait() { return reinterpret_cast<int8_t*>(b + P->o_slot_wait); }
    __device__ int8_t* offer_core() { return reinterpret_cast<int8_t*>(b + P->o_offer_core); }
    __device__ int8_t* offer_recip() { return reinterpret_cast<int8_t*>(b + P->o_offer_recip); }
    __device__ int8_t* offer_price() { return reinterpret_cast<int8_t*>(b + P->o_offer_price); }
    __device__ int32_t* slot_birth() { return reinterpret_cast<int32_t*>(b + P->o_slot_birth); }
};

__device__ __forceinline__ void copy_dwords(uint32_t* dst, const uint32_t* src, int n, int lane) {
    for (int i = lane; i < n; i += kWave) dst[i] = src[i];
}

// calculateRewardRatio (HardcodedModules.py:5-13) as an exact fraction; the
// double comparisons of the reference agree with exact rational comparisons
// for int8 operands (distinct ratios differ by >= 1/16129 >> 1 ulp).
__device__ __forceinline__ void ratio_of(int p, int n, int& num, int& den) {
    if (p == -1 || n == -1 || p == -2 || n == -2) {
        num = -1;
        den = 1;
    } else {
        num = n < 0 ? -p : p;
        den = n < 0 ? -n : n;
    }
}

// ---------------------------------------------------------------------------
// offer-set masks (bit i = the offer of slot i; slot order is offer-ID order)

struct M128 {
    uint64_t lo, hi;
};

__device__ __forceinline__ M128 mand(const M128& a, const M128& b) { return M128{a.lo & b.lo, a.hi & b.hi}; }

// index of the k-th (k >= 0) set bit of m, -1 if m has fewer bits
__device__ __forceinline__ int kth_bit(const M128& m, int k) {
    uint64_t w = m.lo;
    int base = 0;
    const int c = __popcll(m.lo);
    if (k >= c) {
        k -= c;
        w = m.hi;
        base = 64;
        if (k >= __popcll(w)) return -1;
    }
    for (; k > 0; k--) w &= w - 1;
    return base + __ffsll((unsigned long long)w) - 1;
}

// Iterate the set bits of m in increasing order: for (MaskIter it(m); it.more(); ) { int i = it.next(); ... }
struct MaskIter {
    uint64_t lo, hi;
    __device__ __forceinline__ explicit MaskIter(const M128& m) : lo(m.lo), hi(m.hi) {}
    __device__ __forceinline__ bool more() const { return (lo | hi) != 0; }
    __device__ __forceinline__ int next() {
        if (lo) {
            const int i = __ffsll((unsigned long long)lo) - 1;
            lo &= lo - 1;
            return i;
        }
        const int i = __ffsll((unsigned long long)hi) - 1;
        hi &= hi - 1;
        return 64 + i;
    }
};

__device__ __forceinline__ void mask_set(M128* m, int i) {
    unsigned long long* w = reinterpret_cast<unsigned long long*>(m) + (i >> 6);
    atomicOr(w, 1ull << (i & 63));
}

// Masks of the current offers: mc[c] = offers to core c, mr[r] = offers to
// recipient r (0 = auctioneer). Ends with a barrier.
__device__ void build_masks(Rec& R, const Params& P, M128* mc, M128* mr, int lane) {
    for (int i = lane; i < P.C; i += kWave) mc[i] = M128{0, 0};
    for (int i = lane; i <= P.N; i += kWave) mr[i] = M128{0, 0};
    wave_sync();
    const int8_t* oc = R.offer_core();
    const int8_t* orc = R.offer_recip();
    for (int i = lane; i < P.NL; i += kWave) {
        const int c = oc[i];
        if (c >= 0) {
            mask_set(&mc[c], i);
            mask_set(&mr[orc[i]], i);
        }
    }
    wave_sync();
}

// ---------------------------------------------------------------------------
// observations of the current (LDS) state: Agent.py:167-212 (acceptor),
// Agent.py:271-300 (offer), Auctioneer.py:34-77 (auctioneer)

// One acceptor/auctioneer row over a scratch row prefilled with -2 bytes.
__device__ __forceinline__ void acceptor_row(Rec& R, const Params& P, const M128* mc, const M128* mr, int recipient,
                                             int c, int8_t* row) {
    const bool own = R.core_owner()[c] == recipient;
    const int kind = R.core_kind()[c];
    row[0] = own ? 1 : 0;
    row[1] = (int8_t)(own ? (kind >= 0 ? P.prio[kind] : -1) : -1);
    row[2] = (int8_t)(own ? R.core_rem()[c] : -1);
    const int8_t* op = R.offer_price();
    const int8_t* sr = R.slot_rem();
    int w = 3;
    for (MaskIter it(mand(mc[c], mr[recipient])); it.more();) {  // (price, necT) in offer-ID order
        const int i = it.next();
        row[w] = op[i];
        row[w + 1] = sr[i];
        w += 2;
    }
    for (int z = P.d_acc; z < P.acc_stride; z++) row[z] = 0;
}

// Acceptor rows (KIND 0, row g = agent g / C, core g % C) or auctioneer rows
// (KIND 2, row g = core g), staged in LDS chunks and streamed to dst.
template <int KIND>
__device__ void emit_acc_rows(Rec& R, const Params& P, const M128* mc, const M128* mr, uint8_t* scratch, int8_t* dst,
                              int n_rows, int lane) {
    if (!dst) return;
    const int stride = P.acc_stride;
    const int per_chunk = P.obs_chunk / stride;
    uint32_t* sw = reinterpret_cast<uint32_t*>(scratch);
    for (int r0 = 0; r0 < n_rows; r0 += per_chunk) {
        const int nr = min(per_chunk, n_rows - r0);
        const int nd = nr * stride / 4;
        for (int i = lane; i < nd; i += kWave) sw[i] = 0xFEFEFEFEu;  // -2 pads
        wave_sync();
        for (int r = lane; r < nr; r += kWave) {
            const int g = r0 + r;
            int8_t* row = reinterpret_cast<int8_t*>(scratch) + r * stride;
            if (KIND == 0)
                acceptor_row(R, P, mc, mr, g / P.C + 1, g - (g / P.C) * P.C, row);
            else
                acceptor_row(R, P, mc, mr, 0, g, row);
        }
        wave_sync();
        copy_dwords(reinterpret_cast<uint32_t*>(dst + (size_t)r0 * stride), sw, nd, lane);
        wave_sync();
    }
}

// Offer rows: the (prio, rem) pairs of all cores — the same for every row of
// the env — then the slot's own pair, zero padded to the stride. Built one
// dword per lane (strides are multiples of 4, so a dword never spans rows).
__device__ void emit_off_rows(Rec& R, const Params& P, uint8_t* scratch, int8_t* dst, int lane) {
    if (!dst) return;
    const int stride = P.off_stride;
    const int per_chunk = P.obs_chunk / stride;
    const int8_t* ck = R.core_kind();
    const int8_t* cr = R.core_rem();
    const int8_t* sk = R.slot_kind();
    const int8_t* srem = R.slot_rem();
    uint32_t* sw = reinterpret_cast<uint32_t*>(scratch);
    for (int r0 = 0; r0 < P.NL; r0 += per_chunk) {
        const int nr = min(per_chunk, P.NL - r0);
        const int nd = nr * stride / 4;
        for (int d = lane; d < nd; d += kWave) {
            const int r = (4 * d) / stride;
            const int col0 = 4 * d - r * stride;
            const int s = r0 + r;
            uint32_t word = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int col = col0 + b;
                int v = 0;
                if (col < 2 * P.C) {
                    const int c = col >> 1, k = ck[c];
                    v = k < 0 ? -1 : ((col & 1) ? cr[c] : P.prio[k]);
                } else if (col < P.d_off) {
                    const int k = sk[s];
                    v = k < 0 ? -1 : ((col & 1) ? srem[s] : P.prio[k]);
                }
                word |= (uint32_t)(uint8_t)v << (8 * b);
            }
            sw[d] = word;
        }
        wave_sync();
        copy_dwords(reinterpret_cast<uint32_t*>(dst + (size_t)r0 * stride), sw, nd, lane);
        wave_sync();
    }
}

__device__ void emit_obs(Rec& R, const Params& P, const M128* mc, const M128* mr, uint8_t* scratch, int8_t* acc,
                         int8_t* off, int8_t* auct, int64_t e, int lane) {
    emit_acc_rows<0>(R, P, mc, mr, scratch, acc ? acc + e * (int64_t)P.N * P.C * P.acc_stride : nullptr, P.N * P.C,
                     lane);
    emit_off_rows(R, P, scratch, off ? off + e * (int64_t)P.NL * P.off_stride : nullptr, lane);
    emit_acc_rows<2>(R, P, mc, mr, scratch, auct ? auct + e * (int64_t)P.C * P.acc_stride : nullptr, P.C, lane);
}

// HardcodedAuctioneerAcceptor.selectAction for every core (HardcodedModules.py:54-78,
// Auctioneer.getAuctioneerAction Auctioneer.py:95-102) on the staged state: per core the max
// ratio over the auctioneer's offers and the count of offers attaining it, then one
// _randbelow(count) per tied core in core order on the env stream. Writes s_auct[c] (O = reject).
__device__ void hardcoded_auctioneer(Rec& R, const Params& P, const M128* s_mc, const M128* s_mr, MtStream& rs,
                                     int16_t* s_auct, int16_t* s_tie_n, int16_t* s_pick, int lane) {
    const int C = P.C, O = P.O;
    const int8_t* c_owner = R.core_owner();
    const int8_t* o_price = R.offer_price();
    const int8_t* s_rem = R.slot_rem();
    // per core: the max ratio over the auctioneer's offers (the padded list's -1 entries and the
    // own empty job bound it from below) and how many offers attain it
    int mn = -1, md = 1;
    if (lane < C) {
        int nt = 0;
        if (c_owner[lane] == 0) {
            const M128 cand = mand(s_mc[lane], s_mr[0]);
            for (MaskIter it(cand); it.more();) {
                const int i = it.next();
                int num, den;
                ratio_of(o_price[i], s_rem[i], num, den);
                if (num * md > mn * den) {
                    mn = num;
                    md = den;
                }
            }
            if (mn > -md) {  // max(ratios) > own ratio (-1, the auctioneer's empty job)
                for (MaskIter it(cand); it.more();) {
                    const int i = it.next();
                    int num, den;
                    ratio_of(o_price[i], s_rem[i], num, den);
                    nt += (num * md == mn * den);
                }
            }
        }
        s_auct[lane] = (int16_t)O;
        s_tie_n[lane] = (int16_t)nt;
    }
    wave_sync();
    // tie-break draws in core order on the env stream (Auctioneer.getAuctioneerAction
    // Auctioneer.py:95-102)
    bool any = false;
    for (int c = 0; c < C; c++) {
        const int nt = s_tie_n[c];
        if (nt > 0) {
            const uint32_t pick = rs.randbelow((uint32_t)nt, lane);
            if (lane == 0) s_pick[c] = (int16_t)pick;
            any = true;
        }
    }
    if (any) {
        wave_sync();
        // the pick-th maximal candidate's position in the padded list
        if (lane < C && s_tie_n[lane] > 0) {
            const int pick = s_pick[lane];
            int k = 0, t = 0;
            for (MaskIter it(mand(s_mc[lane], s_mr[0])); it.more(); k++) {
                const int i = it.next();
                int num, den;
                ratio_of(o_price[i], s_rem[i], num, den);
                if (num * md == mn * den) {
                    if (t == pick) s_auct[lane] = (int16_t)k;
                    t++;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// kernels


// Initial state (world.py:247, Core.__init__ world.py:30-37, JobCollection
// world.py:118-121) and random.seed(seed + e) (init_by_array of the seed's
// 32-bit words).
__global__ void __launch_bounds__(64) k_env_init(Params P, uint8_t* recs, uint32_t* mt, Liab* liab,
                                                 uint64_t seed) {
    extern __shared__ __align__(16) uint8_t smem[];
    const int lane = threadIdx.x;
    const int64_t e = blockIdx.x;
    uint8_t* rec = smem;
    uint32_t* st = reinterpret_cast<uint32_t*>(smem + P.s_scratch);
    for (int i = lane; i < P.rec_bytes / 4; i += kWave) reinterpret_cast<uint32_t*>(rec)[i] = 0;
    wave_sync();
    Rec R{rec, &P};
    for (int c = lane; c < P.C; c += kWave) {
        R.core_owner()[c] = 0;
        R.core_kind()[c] = -1;
        R.core_rem()[c] = -1;
        R.liab_n()[c] = 0;
        R.core_birth()[c] = -1;
    }
    for (int i = lane; i < P.NL; i += kWave) {
        R.slot_kind()[i] = -1;
        R.slot_rem()[i] = -1;
        R.slot_wait()[i] = 0;
        R.offer_core()[i] = -1;
        R.offer_recip()[i] = 0;
        R.offer_price()[i] = 0;
        R.slot_birth()[i] = -1;
    }
    if (lane == 0) {
        uint64_t s = seed + (uint64_t)e;
        uint32_t key[2] = {(uint32_t)s, (uint32_t)(s >> 32)};
        int len = key[1] ? 2 : 1;
        st[0] = 19650218u;
        for (int i = 1; i < kMtN; i++) st[i] = 1812433253u * (st[i - 1] ^ (st[i - 1] >> 30)) + (uint32_t)i;
        int i = 1, j = 0;
        for (int k = (kMtN > len ? kMtN : len); k; k--) {
            st[i] = (st[i] ^ ((st[i - 1] ^ (st[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
            i++;
            j++;
            if (i >= kMtN) {
                st[0] = st[kMtN - 1];
                i = 1;
            }
            if (j >= len) j = 0;
        }
        for (int k = kMtN - 1; k; k--) {
            st[i] = (st[i] ^ ((st[i - 1] ^ (st[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
            i++;
            if (i >= kMtN) {
                st[0] = st[kMtN - 1];
                i = 1;
            }
        }
        st[0] = 0x80000000u;
        R.mti() = kMtN;
    }
    wave_sync();
    copy_dwords(mt + e * kMtN, st, kMtN, lane);
    copy_dwords(reinterpret_cast<uint32_t*>(recs + e * (int64_t)P.rec_bytes), reinterpret_cast<uint32_t*>(rec),
                P.rec_bytes / 4, lane);
}

__global__ void __launch_bounds__(64) k_env_reset(Params P, const uint8_t* recs, int8_t* obs_acc, int8_t* obs_off,
                                                  int8_t* obs_auct) {
    extern __shared__ __align__(16) uint8_t smem[];
    M128* s_mc = reinterpret_cast<M128*>(smem + P.s_mc);
    M128* s_mr = reinterpret_cast<M128*>(smem + P.s_mr);
    const int lane = threadIdx.x;
    const int64_t e = blockIdx.x;
    uint8_t* rec = smem + P.s_rec;
    copy_dwords(reinterpret_cast<uint32_t*>(rec), reinterpret_cast<const uint32_t*>(recs + e * (int64_t)P.rec_bytes),
                P.rec_bytes / 4, lane);
    wave_sync();
    Rec R{rec, &P};
    build_masks(R, P, s_mc, s_mr, lane);
    emit_obs(R, P, s_mc, s_mr, smem + P.s_scratch, obs_acc, obs_off, obs_auct, e, lane);
}

constexpr int kLiabPrefetch = 4;  // newest chain entries loaded ahead per core that may terminate

// One round of SchedulingEnv.step (SchedulingEnvironment.py:32-83) for env blockIdx.x.
__global__ void __launch_bounds__(64) k_env_step(Params P, uint8_t* recs, uint32_t* mt, Liab* liab, StepIO io) {
    extern __shared__ __align__(16) uint8_t smem[];
    M128* s_mc = reinterpret_cast<M128*>(smem + P.s_mc);          // offers per core
    M128* s_mr = reinterpret_cast<M128*>(smem + P.s_mr);          // offers per recipient (0 = auctioneer)
    Liab* s_newle = reinterpret_cast<Liab*>(smem + P.s_newle);    // liability entry appended this round per core
    int16_t* s_exec = reinterpret_cast<int16_t*>(smem + P.s_exec);  // per core: executed offer's slot, -1 none
    int16_t* s_key = reinterpret_cast<int16_t*>(smem + P.s_key);    // execution order key
    int8_t* s_by_rank = reinterpret_cast<int8_t*>(smem + P.s_rank); // cores in execution order
    int8_t* s_fresh = reinterpret_cast<int8_t*>(smem + P.s_fresh);  // s_newle[c] is the chain's newest entry
    int16_t* s_auct = reinterpret_cast<int16_t*>(smem + P.s_auct);  // auctioneer action per core
    int16_t* s_tie_n = reinterpret_cast<int16_t*>(smem + P.s_tie);  // tied maxima count (auctioneer)
    int16_t* s_pick = reinterpret_cast<int16_t*>(smem + P.s_pick);  // tie-break draw per core
    int32_t* s_agent_r = reinterpret_cast<int32_t*>(smem + P.s_agentr);  // agentReward
    int32_t* s_auct_r = reinterpret_cast<int32_t*>(smem + P.s_auctr);    // auctioneerReward
    uint32_t& s_flags = *reinterpret_cast<uint32_t*>(smem + P.s_misc);
    int& s_n_exec = *reinterpret_cast<int*>(smem + P.s_misc + 4);

    const int lane = threadIdx.x;
    const int64_t e = blockIdx.x;
    const int N = P.N, C = P.C, L = P.L, NL = P.NL, O = P.O;

    uint8_t* rec = smem + P.s_rec;
    int8_t* a_acc = reinterpret_cast<int8_t*>(smem + P.s_act_acc);
    int8_t* a_off = reinterpret_cast<int8_t*>(smem + P.s_act_off);
    int8_t* a_price = reinterpret_cast<int8_t*>(smem + P.s_act_price);
    int8_t* a_auct = reinterpret_cast<int8_t*>(smem + P.s_act_auct);
    int32_t* acc_r = reinterpret_cast<int32_t*>(smem + P.s_accr);
    float* off_r = reinterpret_cast<float*>(smem + P.s_offr);
    float* price_r = reinterpret_cast<float*>(smem + P.s_pricer);
    int8_t* spawn_kind = reinterpret_cast<int8_t*>(smem + P.s_spawn_kind);
    uint8_t* scratch = smem + P.s_scratch;

    // ---- stage state and actions in LDS
    copy_dwords(reinterpret_cast<uint32_t*>(rec), reinterpret_cast<const uint32_t*>(recs + e * (int64_t)P.rec_bytes),
                P.rec_bytes / 4, lane);
    for (int i = lane; i < N * C; i += kWave) a_acc[i] = io.act_acc[e * N * C + i];
    for (int i = lane; i < NL; i += kWave) {
        a_off[i] = io.act_off[e * NL + i];
        a_price[i] = io.act_price ? io.act_price[e * NL + i] : 0;
    }
    for (int i = lane; i < C; i += kWave) a_auct[i] = io.act_auct ? io.act_auct[e * C + i] : 0;
    for (int i = lane; i < N * C; i += kWave) acc_r[i] = 0;
    for (int i = lane; i < NL; i += kWave) {
        off_r[i] = 0.f;
        price_r[i] = 0.f;
    }
    for (int i = lane; i < C; i += kWave) {
        s_auct_r[i] = 0;
        s_exec[i] = -1;
        s_fresh[i] = 0;
    }
    for (int i = lane; i < N; i += kWave) s_agent_r[i] = 0;
    if (lane == 0) {
        s_flags = 0;
        s_n_exec = 0;
    }
    wave_sync();
    Rec R{rec, &P};
    const int round = R.round();
    int8_t* c_owner = R.core_owner();
    int8_t* c_kind = R.core_kind();
    int8_t* c_rem = R.core_rem();
    int32_t* c_birth = R.core_birth();
    uint8_t* l_n = R.liab_n();
    int8_t* s_kind = R.slot_kind();
    int8_t* s_rem = R.slot_rem();
    int8_t* s_wait = R.slot_wait();
    int32_t* s_birth = R.slot_birth();
    int8_t* o_core = R.offer_core();
    int8_t* o_recip = R.offer_recip();
    int8_t* o_price = R.offer_price();
    Liab* my_liab = liab + e * (int64_t)C * P.cap;

    // ---- issue the dependent loads early: the MT window at mti (a peek: no twist
    //      yet) and the newest liability entries of every core that may terminate
    //      this round, i.e. whose current job or one of the jobs offered to it has
    //      one round left (its chain is settled in the tick below)
    MtStream rs;
    rs.gmt = mt + e * kMtN;
    rs.lds = reinterpret_cast<uint32_t*>(scratch);
    rs.mti0 = R.mti();
    rs.p = 0;
    rs.twisted = false;
    rs.load(0, 0, lane);
    build_masks(R, P, s_mc, s_mr, lane);
    Liab pf[kLiabPrefetch];
    int pf_n = 0;
    if (lane < C) {
        bool maybe = c_kind[lane] >= 0 && c_rem[lane] == 1;
        for (MaskIter it(s_mc[lane]); it.more() && !maybe;) maybe = s_rem[it.next()] == 1;
        if (maybe) {
            const int n = l_n[lane];
            pf_n = min(n, kLiabPrefetch);
            const Liab* chain = my_liab + lane * P.cap;
#pragma unroll
            for (int q = 0; q < kLiabPrefetch; q++)
                if (q < pf_n) pf[q] = chain[n - 1 - q];
        }
    }

    // ---- auctioneer actions: HardcodedAuctioneerAcceptor (HardcodedModules.py:54-78), asked by the
    //      driver before env.step (trainPPO.py:162); ties broken with random.sample -> _randbelow
    if (!io.act_auct) {
        hardcoded_auctioneer(R, P, s_mc, s_mr, rs, s_auct, s_tie_n, s_pick, lane);
    } else {
        for (int c = lane; c < C; c += kWave) s_auct[c] = a_auct[c];
    }
    wave_sync();

    // ---- which offer each core executes (executeAgentAcceptions1 world.py:391-404,
    //      executeAuctioneerAcceptions world.py:378-389): offers to core c are all addressed to c's
    //      owner (created after the tick with recipient = owner, world.py:428), so only the owner's
    //      acceptor (or the auctioneer) can pick one, and each core executes at most once per round.
    for (int i = lane; i < N * C; i += kWave) {
        int a = a_acc[i];
        if (a < 0 || a > O) atomicOr(&s_flags, MS_FLAG_BAD_ACTION);
    }
    for (int c = lane; c < C; c += kWave) {
        int owner = c_owner[c];
        int idx = owner > 0 ? a_acc[(owner - 1) * C + c] : s_auct[c];
        if (owner == 0 && (idx < 0 || idx > O)) atomicOr(&s_flags, MS_FLAG_BAD_ACTION);
        int slot = -1;
        if (idx >= 0 && idx < O) slot = kth_bit(mand(s_mc[c], s_mr[owner]), idx);
        s_exec[c] = (int16_t)slot;
        s_key[c] = (int16_t)(owner > 0 ? (owner - 1) * C + c : N * C + c);
    }
    wave_sync();
    for (int c = lane; c < C; c += kWave) {
        if (s_exec[c] >= 0) {
            int r = 0;
            for (int d = 0; d < C; d++) r += (s_exec[d] >= 0 && s_key[d] < s_key[c]);
            s_by_rank[r] = (int8_t)c;
            atomicAdd(&s_n_exec, 1);
        }
    }
    wave_sync();

    // ---- apply executions in reference order (World.executeAnOffer world.py:261-293)
    if (lane == 0) {
        int n_exec = s_n_exec;
        for (int r = 0; r < n_exec; r++) {
            int c = s_by_rank[r];
            int i = s_exec[c];
            int offerer = i / L + 1, slot = i % L;
            int recip = o_recip[i];
            int nk = s_kind[i], nrem = s_rem[i], nbirth = s_birth[i];
            int price = o_price[i];
            // removeAndReturnEntry (world.py:135-141); newJob.wait = False (world.py:276)
            s_kind[i] = -1;
            s_rem[i] = -1;
            s_wait[i] = 0;
            s_birth[i] = -1;
            // dispatchNewJobAndReturnOldOne (world.py:61-76)
            int ok = c_kind[c], orem = c_rem[c], obirth = c_birth[c];
            c_kind[c] = (int8_t)nk;
            c_rem[c] = (int8_t)nrem;
            c_birth[c] = nbirth;
            c_owner[c] = (int8_t)offerer;
            if (recip != 0) {  // insertJob into the recipient's first empty slot (world.py:123-133)
                int base = (recip - 1) * L, placed = 0;
                for (int s = 0; s < L; s++)
                    if (s_kind[base + s] < 0) {
                        s_kind[base + s] = (int8_t)ok;
                        s_rem[base + s] = (int8_t)orem;
                        s_wait[base + s] = 0;
                        s_birth[base + s] = obirth;
                        placed = 1;
                        break;
                    }
                if (!placed) s_flags |= MS_FLAG_COLLECTION_FULL;
            }
            // liability entry (deepcopy, round = world.round), appendleft (world.py:285-289)
            int n = l_n[c];
            if (n < P.cap) {
                Liab le;
                le.offerer = (int8_t)offerer;
                le.recipient = (int8_t)recip;
                le.price = (int8_t)price;
                le.nec = (int8_t)nrem;
                le.round = round;
                my_liab[c * P.cap + n] = le;
                s_newle[c] = le;
                s_fresh[c] = 1;
                l_n[c] = (uint8_t)(n + 1);
            } else {
                s_flags |= MS_FLAG_LIABILITY_OVERFLOW;
            }
            // offer-side rewards from world.acceptedOffers (Reward.py:164-170 / :23-49)
            int prio1 = P.prio[nk];
            if (!P.free_prices) {
                off_r[i] = (float)prio1;
            } else {
                int diff = prio1 - price;
                float pc;
                if (P.commercial)
                    pc = diff == 0 ? P.net_zero : (float)diff;
                else
                    pc = diff >= 0 ? (float)prio1 : (float)diff;
                off_r[i] = (float)prio1;
                price_r[i] = pc;
            }
            if (io.ev_acc) {
                ms_accept_rec ar;
                ar.valid = 1;
                ar.offerer = (int8_t)offerer;
                ar.recipient = (int8_t)recip;
                ar.slot = (int8_t)slot;
                ar.price = (int8_t)price;
                ar.nec_time = (int8_t)nrem;
                ar.prio = (int8_t)prio1;
                ar.kind = (int8_t)nk;
                ar.order = (int8_t)r;
                ar.pad[0] = ar.pad[1] = ar.pad[2] = 0;
                ar.round = round;
                io.ev_acc[e * C + c] = ar;
            }
        }
    }
    wave_sync();

    // ---- tick (processOneTimestepAndUpdateOwnership world.py:336-367) and liability settlement
    //      (getDividedFixedPricesReward Reward.py:187-210 / getDividedFreePricesReward Reward.py:59-82)
    for (int c = lane; c < C; c += kWave) {
        ms_term_rec tr = {0, 0, 0, 0, 0};
        if (c_kind[c] >= 0) {
            int rem = c_rem[c] - 1;
            c_rem[c] = (int8_t)rem;
            if (rem == 0) {
                int owner = c_owner[c];
                int kind = c_kind[c];
                int gen = P.mult * P.prio[kind];
                int ts = round + 1;
                tr.valid = 1;
                tr.owner = (int8_t)owner;
                tr.prio = (int8_t)P.prio[kind];
                tr.init_len = (int8_t)P.len[kind];
                tr.dwell = round - c_birth[c];
                // Core.assignCoreToAuctioneer (world.py:57-59)
                c_kind[c] = -1;
                c_rem[c] = -1;
                c_birth[c] = -1;
                c_owner[c] = 0;
                // settlement, newest entry first: this round's entry from LDS, the next
                // kLiabPrefetch from the registers loaded at staging, older ones from HBM
                acc_r[(owner - 1) * C + c] = gen;
                if (!P.free_prices) atomicAdd(&s_agent_r[owner - 1], gen);
                const int n = l_n[c];
                const int fresh = s_fresh[c];
                int last = ts, tm = 0;
                for (int k = n - 1; k >= 0; k--) {
                    const int q = n - 1 - k - fresh;  // index among the entries older than this round's
                    Liab le;
                    if (q < 0) {
                        le = s_newle[c];
                    } else if (q < pf_n) {
                        le = pf[0];
#pragma unroll
                        for (int j = 1; j < kLiabPrefetch; j++)
                            if (q == j) le = pf[j];
                    } else {
                        le = my_liab[c * P.cap + k];
                    }
                    tm += last - le.round;
                    last = le.round;
                    double ratio = (double)le.price / (double)le.nec;  // Python true division
                    int traded = (int)rint(ratio * (double)tm);        // Python round(): half-even
                    acc_r[(le.offerer - 1) * C + c] -= traded;
                    atomicAdd(&s_agent_r[le.offerer - 1], -traded);
                    if (le.recipient > 0) {
                        atomicAdd(&s_agent_r[le.recipient - 1], traded);
                        acc_r[(le.recipient - 1) * C + c] += traded;
                    } else {
                        s_auct_r[c] = traded;
                    }
                }
                l_n[c] = 0;  // resetLiabilityListForACore
            }
        }
        if (io.ev_term) io.ev_term[e * C + c] = tr;
        if (io.ev_acc && s_exec[c] < 0) {
            ms_accept_rec ar = {};
            io.ev_acc[e * C + c] = ar;
        }
    }
    wave_sync();

    // ---- offers from offer actions (createFixPriceOfferObjectsFromActions world.py:406-443,
    //      createFreePriceOfferObjectsFromActions world.py:445-478); IDs = slot order
    for (int i = lane; i < NL; i += kWave) {
        int act = a_off[i];
        int cidx = (act >= 0 && act < C) ? act : -1;
        int kind = s_kind[i];
        int price;
        if (P.free_prices)
            price = a_price[i];
        else
            price = P.fix[kind >= 0 ? kind : P.n_fix - 1];
        if (cidx >= 0 && kind >= 0 && !s_wait[i]) {
            o_core[i] = (int8_t)cidx;
            o_recip[i] = c_owner[cidx];
            o_price[i] = (int8_t)price;
            s_wait[i] = 1;
        } else {
            o_core[i] = -1;
            o_recip[i] = 0;
            o_price[i] = 0;
            s_wait[i] = 0;
        }
    }
    wave_sync();

    // ---- spawn (fillQueuesWithNewRandomJobs world.py:369-376, fillCollectionRandomly Agent.py:50-70)
    {
        const int k = P.new_jobs;
        bool sp = false;
        if (lane < N) {
            int owned = 0, free_slots = 0;
            for (int c = 0; c < C; c++) owned += (c_owner[c] == lane + 1);
            for (int s = 0; s < L; s++) free_slots += (s_kind[lane * L + s] < 0);
            sp = owned + k <= free_slots;
        }
        uint64_t spm = __ballot(sp);
        int n_sp = __popcll(spm);
        int total_pairs = n_sp * k;
        int done = 0;
        while (done < total_pairs) {
            if (rs.wend - rs.p < 2) rs.load(rs.p, 2, lane);
            int avail = (rs.wend - rs.p) / 2;
            int cnt = min(avail, total_pairs - done);
            int off0 = rs.p - rs.wb;
            uint32_t wa = __shfl(rs.v, (off0 + 2 * lane) & 63);
            uint32_t wb2 = __shfl(rs.v, (off0 + 2 * lane + 1) & 63);
            if (lane < cnt) {
                // random(): (a>>5 * 2^26 + b>>6) / 2^53 (Modules/_randommodule.c)
                double u = ((double)(wa >> 5) * 67108864.0 + (double)(wb2 >> 6)) * (1.0 / 9007199254740992.0);
                int kind = -1;
                for (int q = 0; q < P.K; q++)
                    if (u < P.acc[q]) {
                        kind = q;
                        break;
                    }
                if (kind < 0) {
                    kind = P.K - 1;
                    atomicOr(&s_flags, MS_FLAG_SPAWN_EDGE);
                }
                spawn_kind[done + lane] = (int8_t)kind;
            }
            rs.p += 2 * cnt;
            done += cnt;
        }
        wave_sync();
        if (sp) {
            int rank = __popcll(spm & ((1ull << lane) - 1ull));
            int base = lane * L;
            for (int j = 0; j < k; j++) {
                int kind = spawn_kind[rank * k + j];
                int placed = 0;
                for (int s = 0; s < L; s++)
                    if (s_kind[base + s] < 0) {
                        s_kind[base + s] = (int8_t)kind;
                        s_rem[base + s] = (int8_t)P.len[kind];
                        s_wait[base + s] = 0;
                        s_birth[base + s] = round;
                        placed = 1;
                        break;
                    }
                if (!placed) atomicOr(&s_flags, MS_FLAG_COLLECTION_FULL);
            }
        }
    }
    wave_sync();
    if (lane == 0) {
        R.round() = round + 1;
        R.mti() = rs.final_index();
        R.flags() |= s_flags;
    }
    wave_sync();

    // ---- outputs: state record, rewards, observations of the new offer set
    copy_dwords(reinterpret_cast<uint32_t*>(recs + e * (int64_t)P.rec_bytes), reinterpret_cast<uint32_t*>(rec),
                P.rec_bytes / 4, lane);
    if (io.rew_acc) copy_dwords(reinterpret_cast<uint32_t*>(io.rew_acc + e * N * C), reinterpret_cast<uint32_t*>(acc_r), N * C, lane);
    if (io.rew_offer) copy_dwords(reinterpret_cast<uint32_t*>(io.rew_offer + e * NL), reinterpret_cast<uint32_t*>(off_r), NL, lane);
    if (io.rew_price) copy_dwords(reinterpret_cast<uint32_t*>(io.rew_price + e * NL), reinterpret_cast<uint32_t*>(price_r), NL, lane);
    if (io.rew_agent)
        for (int a = lane; a < N; a += kWave) io.rew_agent[e * N + a] = s_agent_r[a];
    if (io.rew_auct)
        for (int c = lane; c < C; c += kWave) io.rew_auct[e * C + c] = s_auct_r[c];
    build_masks(R, P, s_mc, s_mr, lane);
    emit_obs(R, P, s_mc, s_mr, scratch, io.obs_acc, io.obs_off, io.obs_auct, e, lane);
}

// Auctioneer.getAuctioneerAction (Auctioneer.py:95-102) on its own, as the driver calls it
// before env.step (trainPPO.py:162): writes actions [E][C] and advances the env stream by the
// tie-break draws; a following ms_env_step with these actions then draws only the spawn.
__global__ void __launch_bounds__(64) k_env_auctioneer(Params P, uint8_t* recs, uint32_t* mt, int8_t* actions) {
    extern __shared__ __align__(16) uint8_t smem[];
    M128* s_mc = reinterpret_cast<M128*>(smem + P.s_mc);
    M128* s_mr = reinterpret_cast<M128*>(smem + P.s_mr);
    int16_t* s_auct = reinterpret_cast<int16_t*>(smem + P.s_auct);
    int16_t* s_tie_n = reinterpret_cast<int16_t*>(smem + P.s_tie);
    int16_t* s_pick = reinterpret_cast<int16_t*>(smem + P.s_pick);
    const int lane = threadIdx.x;
    const int64_t e = blockIdx.x;
    uint8_t* rec = smem + P.s_rec;
    copy_dwords(reinterpret_cast<uint32_t*>(rec), reinterpret_cast<const uint32_t*>(recs + e * (int64_t)P.rec_bytes),
                P.rec_bytes / 4, lane);
    wave_sync();
    Rec R{rec, &P};
    MtStream rs;
    rs.gmt = mt + e * kMtN;
    rs.lds = reinterpret_cast<uint32_t*>(smem + P.s_scratch);
    rs.mti0 = R.mti();
    rs.p = 0;
    rs.twisted = false;
    rs.load(0, 0, lane);
    build_masks(R, P, s_mc, s_mr, lane);
    hardcoded_auctioneer(R, P, s_mc, s_mr, rs, s_auct, s_tie_n, s_pick, lane);
    wave_sync();
    for (int c = lane; c < P.C; c += kWave) actions[e * P.C + c] = (int8_t)s_auct[c];
    if (lane == 0) *reinterpret_cast<int32_t*>(recs + e * (int64_t)P.rec_bytes + 8) = rs.final_index();
}

// random._randbelow(n) on env e's stream (random.randint in the update schedulers,
// Agent.py:718,725, SchedulingEnvironment.py:317-326).
__global__ void __launch_bounds__(64) k_env_randbelow(Params P, uint8_t* recs, uint32_t* mt, int64_t e, uint32_t n,
                                                      uint32_t* out) {
    extern __shared__ __align__(16) uint8_t smem[];
    const int lane = threadIdx.x;
    uint8_t* rec = recs + e * (int64_t)P.rec_bytes;
    int32_t* mti = reinterpret_cast<int32_t*>(rec + 8);
    MtStream rs;
    rs.gmt = mt + e * kMtN;
    rs.lds = reinterpret_cast<uint32_t*>(smem + P.s_scratch);
    rs.mti0 = *mti;
    rs.wb = rs.wend = rs.p = 0;
    rs.twisted = false;
    rs.v = 0;
    uint32_t r = rs.randbelow(n, lane);
    wave_sync();
    if (lane == 0) {
        *out = r;
        *mti = rs.final_index();
    }
}

}  // namespace ms

// launch wrappers used by capi.cpp
namespace ms {
hipError_t launch_env_init(const Params& P, int64_t E, uint8_t* recs, uint32_t* mt, Liab* liab, uint64_t seed,
                           hipStream_t s) {
    hipLaunchKernelGGL(k_env_init, dim3((unsigned)E), dim3(kWave), P.s_total, s, P, recs, mt, liab, seed);
    return hipGetLastError();
}
hipError_t launch_env_reset(const Params& P, int64_t E, const uint8_t* recs, int8_t* a, int8_t* o, int8_t* u,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_env_reset, dim3((unsigned)E), dim3(kWave), P.s_total, s, P, recs, a, o, u);
    return hipGetLastError();
}
hipError_t launch_env_step(const Params& P, int64_t E, uint8_t* recs, uint32_t* mt, Liab* liab, const StepIO& io,
                           hipStream_t s) {
    hipLaunchKernelGGL(k_env_step, dim3((unsigned)E), dim3(kWave), P.s_total, s, P, recs, mt, liab, io);
    return hipGetLastError();
}
hipError_t launch_env_auctioneer(const Params& P, int64_t E, uint8_t* recs, uint32_t* mt, int8_t* actions,
                                 hipStream_t s) {
    hipLaunchKernelGGL(k_env_auctioneer, dim3((unsigned)E), dim3(kWave), P.s_total, s, P, recs, mt, actions);
    return hipGetLastError();
}
hipError_t launch_env_randbelow(const Params& P, uint8_t* recs, uint32_t* mt, int64_t e, uint32_t n, uint32_t* out,
                                hipStream_t s) {
    hipLaunchKernelGGL(k_env_randbelow, dim3(1), dim3(kWave), P.s_total, s, P, recs, mt, e, n, out);
    return hipGetLastError();
}
}  // namespace ms
