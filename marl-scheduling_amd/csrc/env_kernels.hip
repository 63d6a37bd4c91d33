// env_kernels.hip — the batched marl-scheduling round as one HIP kernel for gfx950.
//
// A group of LPE lanes (a power of two >= max(C, N), at least 16; 64 / LPE
// groups per 64-lane wave) steps one env replica per round, so the wave's
// scalar control flow and the lane-serial parts (the offer executions, the
// MT19937 draws) are shared by several envs. The env's packed state record
// (ms_layout.h) is staged in the group's LDS slice with one batch of loads and
// the round runs as group-parallel phases. The offer set of a round (at most
// N*L <= 126 offers, one per slot, offer-ID order = slot order) is indexed by
// 128-bit masks, one per core and one per recipient, built with LDS atomic ORs:
// every ordered selection of the reference — the idx-th offer of (recipient,
// core) behind an acceptor action, the auctioneer's tied maxima, the offers
// listed in an acceptor observation — is a walk over the set bits of
// mask(core) & mask(recipient). The MT19937 stream reads two state blocks (the
// current one and its precomputed successor), so no draw waits for a twist.
// Observations are built from per-core owner rows in LDS and streamed with
// 16-byte write-through stores. Reference semantics (paths relative to
// /root/reference/src) are cited per phase; the CPU restatement that checks
// this kernel bit-for-bit is oracle/ms_oracle.c.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include "ms_layout.h"
#include "ms_act.h"  // the fused next-round acting (fused_act); it sets its own contraction, restored here:

#pragma clang fp contract(off)  // the env round reproduces Python's float64 arithmetic (build.sh: -ffp-contract=off)

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

// Phase timing for the separate profiling build only (tools/build_phase_probe.sh defines
// MS_PHASE_TIMING): lane 0 of every wave adds the cycles since the previous mark to a per-phase
// counter. The product library is built without it and the marks compile to nothing.
#ifdef MS_PHASE_TIMING
constexpr int kProbeSlots = 65536;
__device__ unsigned long long g_phase_cycles[kProbeSlots][16];  // per block, summed on the host
__device__ unsigned long long g_wave_span[kProbeSlots][2];      // last launch: s_memrealtime at entry / exit
__device__ unsigned long long g_free_cycles[kProbeSlots][5];    // k_env_rollout_act_free: env, wait, offers, acceptors, wait
#define MS_MARK(k)                                                     \
    do {                                                               \
        const uint64_t t_now = __builtin_amdgcn_s_memtime();          \
        t_acc[k] += t_now - t_prev;                                    \
        t_prev = t_now;                                                \
    } while (0)
#else
#define MS_MARK(k) \
    do {           \
    } while (0)
#endif

// The LPE lanes of one env within the wave.
template <int LPE>
struct Lanes {
    int gl;     // lane within the group
    int gbase;  // the group's first lane in the wave
    __device__ explicit Lanes(int lane) : gl(lane & (LPE - 1)), gbase(lane & ~(LPE - 1)) {}
    __device__ __forceinline__ uint64_t ballot(bool p) const {
        const uint64_t m = __ballot(p);
        return LPE == 64 ? m : (m >> gbase) & ((1ull << (LPE & 63)) - 1ull);
    }
    __device__ __forceinline__ uint32_t shfl(uint32_t v, int src) const { return (uint32_t)__shfl((int)v, gbase + src); }
};

// ---------------------------------------------------------------------------
// CPython MT19937 (Modules/_randommodule.c) — tempering and group-cooperative twist

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ uint32_t mt_step(uint32_t hi_src, uint32_t lo_src, uint32_t xsrc) {
    const uint32_t y = (hi_src & 0x80000000u) | (lo_src & 0x7fffffffu);
    return xsrc ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// The twist's three phases respect the sequential recurrence: words [0,227) read only old words,
// [227,454) read new [0,227), [454,623) read new [227,396), 623 reads new 0/396. Inside a phase a
// chunk of lanes computes from old words (i, i+1 not yet written), then stores.
__device__ __forceinline__ void mt_phase_range(int ph, int& lo, int& hi) {
    lo = ph * (kMtN - kMtM);
    hi = ph < 2 ? (ph + 1) * (kMtN - kMtM) : kMtN - 1;
}

// Twist of 624 words in LDS by a whole wave.
__device__ void mt_twist_lds_wave(uint32_t* st, int lane) {
    for (int ph = 0; ph < 3; ph++) {
        int lo, hi;
        mt_phase_range(ph, lo, hi);
        for (int c0 = lo; c0 < hi; c0 += kWave) {
            const int i = c0 + lane;
            uint32_t v = 0;
            if (i < hi) v = mt_step(st[i], st[i + 1], st[ph == 0 ? i + kMtM : i + (kMtM - kMtN)]);
            wave_sync();
            if (i < hi) st[i] = v;
            wave_sync();
        }
    }
    if (lane == 0) st[kMtN - 1] = mt_step(st[kMtN - 1], st[0], st[kMtM - 1]);
    wave_sync();
}

// successor half := twist(current half) of one env's blocks, by the whole wave in LDS
__device__ void mt_twist_into_successor(uint32_t* mt_env, uint32_t sel, uint8_t* lds, int lane) {
    uint32_t* st = reinterpret_cast<uint32_t*>(lds);
    const uint32_t h = sel & 1u;
    const uint32_t* cur = mt_env + h * kMtN;
    uint32_t* nxt = mt_env + (h ^ 1u) * kMtN;
    for (int i = lane; i < kMtN; i += kWave) st[i] = cur[i];
    wave_sync();
    mt_twist_lds_wave(st, lane);
    for (int i = lane; i < kMtN; i += kWave) nxt[i] = st[i];
    // the stores complete before this wave's later loads of the successor (other lanes' words)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    wave_sync();
}

// Each env keeps two 624-word blocks in HBM ([E][2][624]): its current CPython state words and
// their successor twist(current), so the round's draws never wait for a twist. Header word 3 of
// the record (mt_sel) says which half is current (bit 0) and whether the other half holds its
// successor (bit 1). An env whose stream crossed into the successor block in the previous round
// gets the next successor at the start of the round: the whole wave twists it in LDS (the LDS is
// not staged yet), once per ~40 rounds of an env.
// successor := twist(current) for every group whose leader lane is set in the wave-uniform mask
// `need` (sel = that leader's mt_sel); the whole wave twists each env in turn in `lds`
template <int LPE>
__device__ void mt_refill_groups(uint32_t* mt, int64_t e0, uint64_t need, uint32_t sel, uint8_t* lds, int lane) {
    while (need) {
        const int src = __ffsll((unsigned long long)need) - 1;
        need &= need - 1;
        mt_twist_into_successor(mt + (e0 + src / LPE) * 2 * kMtN, (uint32_t)__shfl((int)sel, src), lds, lane);
    }
}

template <int LPE>
__device__ void mt_refill_next(uint32_t* mt, const uint8_t* recs, const Geom& P, int64_t slot, bool active,
                               uint8_t* lds, int lane) {
    const int gl = lane & (LPE - 1);
    const int64_t e0 = slot * (kWave / LPE);
    uint32_t sel = 0;
    if (active && gl == 0) sel = *reinterpret_cast<const uint32_t*>(recs + (e0 + lane / LPE) * P.rec_bytes + 12);
    mt_refill_groups<LPE>(mt, e0, __ballot(active && gl == 0 && !(sel & 2u)), sel, lds, lane);
}

// New (mt_sel, mti) after a round whose draws ended at stream index fin (relative to the current
// block): CPython's state is the block holding index fin - 1 with mti = the index within it.
__device__ __forceinline__ void mt_commit(int fin, int32_t* mti, uint32_t* sel) {
    const uint32_t h = *sel & 1u;
    if (fin > 2 * kMtN) {  // fallback: the current half holds twist(successor), no successor yet
        *sel = h;
        *mti = fin - 2 * kMtN;
    } else if (fin > kMtN) {  // crossed into the successor; its own successor comes next round
        *sel = h ^ 1u;
        *mti = fin - kMtN;
    } else {
        *sel = h | 2u;
        *mti = fin;
    }
}

// Fallback for a round that needs more than the current block's rest plus the successor (never
// for the shipped configs): cur := twist(nxt), in place in HBM by one lane group. The loads bypass
// the CU's L1 (agent-scope relaxed atomics read the XCD's L2, where this wave's stores land) and
// workgroup-scope fences order each chunk's stores before the group's next loads.
__device__ __forceinline__ uint32_t mt_ld(const uint32_t* p) {
    return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void mt_st(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int LPE>
__device__ void mt_twist_from(uint32_t* cur, const uint32_t* nxt, int gl) {
    for (int i = gl; i < kMtN; i += LPE) mt_st(cur + i, nxt[i]);
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    for (int ph = 0; ph < 3; ph++) {
        int lo, hi;
        mt_phase_range(ph, lo, hi);
        for (int c0 = lo; c0 < hi; c0 += LPE) {
            const int i = c0 + gl;
            uint32_t v = 0;
            if (i < hi) v = mt_step(mt_ld(cur + i), mt_ld(cur + i + 1), mt_ld(cur + (ph == 0 ? i + kMtM : i + (kMtM - kMtN))));
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
            if (i < hi) mt_st(cur + i, v);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        }
    }
    if (gl == 0) mt_st(cur + kMtN - 1, mt_step(mt_ld(cur + kMtN - 1), mt_ld(cur), mt_ld(cur + kMtM - 1)));
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
}

// A window of LPE words of the env's stream held one word per group lane. Stream positions are
// relative to the env's mti at kernel entry; index mti0 + pos < 624 reads the current block,
// < 1248 its successor, beyond that the fallback block.
template <int LPE>
struct MtStream {
    uint32_t* cur;    // current block (CPython's state words)
    uint32_t* nxt;    // its successor (mt_refill_next made it valid)
    int mti0;         // mti at entry
    int wb, wend;     // window covers stream positions [wb, wend)
    int p;            // next unconsumed stream position
    bool fell_back;   // cur was overwritten with twist(nxt)
    bool overrun;     // a draw needed words past the third block (MS_FLAG_RNG_WINDOW)
    bool store;       // false for a padding group: never write (its draws are discarded)
    uint32_t v;       // this lane's raw state word (position wb + gl); tempered where it is used, so
                      // the load's wait lands at the first draw, not at the load

    __device__ void init(uint32_t* mt_env, uint32_t sel, int mti, bool active) {
        cur = mt_env + (sel & 1u) * kMtN;
        nxt = mt_env + ((sel & 1u) ^ 1u) * kMtN;
        mti0 = mti;
        wb = wend = p = 0;
        fell_back = false;
        overrun = false;
        store = active;
        v = 0;
    }

    __device__ __forceinline__ uint32_t word() const { return mt_temper(v); }  // the window's tempered word

    // Window at stream position pos. need = words the caller is about to consume; need == 0
    // only peeks (never falls back; the window may be empty).
    __device__ void load(int pos, int need, const Lanes<LPE>& L) {
        if (!fell_back && need > 0 && mti0 + pos + need > 2 * kMtN) {
            if (store) mt_twist_from<LPE>(cur, nxt, L.gl);
            fell_back = true;
        }
        if (need > 0 && mti0 + pos + need > 3 * kMtN) overrun = true;
        const int g = mti0 + pos + L.gl;
        uint32_t w = 0;
        if (g < kMtN)
            w = cur[g];
        else if (g < 2 * kMtN)
            w = nxt[g - kMtN];
        else if (g < 3 * kMtN)
            w = mt_ld(cur + g - 2 * kMtN);
        v = w;
        wb = pos;
        wend = fell_back ? pos + LPE : min(pos + LPE, 2 * kMtN - mti0);
    }

    // Random._randbelow_with_getrandbits(n) (random.py:239-249), group-uniform result
    __device__ uint32_t randbelow(uint32_t n, const Lanes<LPE>& L) {
        const int k = 32 - __clz(n);  // n.bit_length()
        const int sh = 32 - k;
        for (;;) {
            if (p >= wend) load(p, 1, L);
            const int pos = wb + L.gl;
            const uint32_t tv = word();
            const bool ok = pos >= p && pos < wend && ((tv >> sh) < n);
            const uint64_t m = L.ballot(ok);
            if (m) {
                const int q = __ffsll((unsigned long long)m) - 1;
                const uint32_t r = L.shfl(tv, q) >> sh;
                p = wb + q + 1;
                return r;
            }
            p = wend;
        }
    }

    // stream index after the draws, relative to the entry block (see mt_commit)
    __device__ int end_index() const { return mti0 + p; }
};

// ---------------------------------------------------------------------------
// record accessors (LDS copy of the env record)

struct Rec {
    uint8_t* b;
    const Geom* P;  // record offsets
    const int32_t* kt;  // kind tables in LDS: prio[16], len[16], fix[16] (per-lane lookups must not
                        // index the kernel-argument struct: that is a memory load per access)
    __device__ int prio(int k) const { return kt[k]; }
    __device__ int len(int k) const { return kt[16 + k]; }
    __device__ int fix(int k) const { return kt[32 + k]; }
    __device__ int32_t& round() { return *reinterpret_cast<int32_t*>(b + 0); }
    __device__ uint32_t& flags() { return *reinterpret_cast<uint32_t*>(b + 4); }
    __device__ int32_t& mti() { return *reinterpret_cast<int32_t*>(b + 8); }
    __device__ uint32_t& mt_sel() { return *reinterpret_cast<uint32_t*>(b + 12); }
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

// the kind tables of Params copied to LDS once per wave (read back by every group)
__device__ __forceinline__ void load_kind_tables(const Params& P, int32_t* kt, int lane) {
    if (lane < 16) {
        kt[lane] = P.prio[lane];
        kt[16 + lane] = P.len[lane];
        kt[32 + lane] = P.fix[lane];
    }
}

template <int LPE>
__device__ __forceinline__ void copy_dwords(uint32_t* dst, const uint32_t* src, int n, int gl) {
#pragma unroll 8
    for (int i = gl; i < n; i += LPE) dst[i] = src[i];
}

// Output arrays written with 16-byte write-through stores (sc1): the line leaves the XCD's L2
// with the store, so the kernel ends without megabytes of dirty L2 lines to write back at its
// boundary (the next kernel reads them from another XCD's side anyway). Addressed as a raw buffer
// over the whole array (wave-uniform base, per-lane 31-bit byte offsets).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
struct WtOut {
    __amdgpu_buffer_rsrc_t r;
    bool ok;  // 16-B aligned base and an array that fits the buffer range
    __device__ WtOut(void* base, int64_t bytes) {
        ok = base != nullptr && (reinterpret_cast<uintptr_t>(base) & 15) == 0 && bytes <= 0x7fffffff;
        r = __builtin_amdgcn_make_buffer_rsrc(base, 0, ok ? (int)bytes : 0, 0x00020000);
    }
    __device__ __forceinline__ void st4(int64_t off, uint32_t a, uint32_t b, uint32_t c, uint32_t d) const {
        const u32x4 v = {a, b, c, d};
        __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 16 /* sc1 */);
    }
};

// n_dw dwords from LDS to env e's block (env_off bytes into the array): write-through 16-B stores
// when the block allows, else plain dword stores to dst.
template <int LPE>
__device__ __forceinline__ void copy_out(const WtOut& o, int64_t env_off, uint32_t* dst, const uint32_t* src, int n_dw,
                                         int gl) {
    if (o.ok && (n_dw & 3) == 0 && (env_off & 15) == 0) {
        for (int k = gl; 4 * k < n_dw; k += LPE)
            o.st4(env_off + 16 * k, src[4 * k], src[4 * k + 1], src[4 * k + 2], src[4 * k + 3]);
    } else {
        copy_dwords<LPE>(dst, src, n_dw, gl);
    }
}

// Up to R dwords per lane of n from global to LDS, all loads issued before the first LDS store
// (with stage_dwords_rest for n > R * LPE): the staged arrays then cost one memory round trip.
template <int LPE, int R>
struct DwordBatch {
    uint32_t v[R];
    __device__ __forceinline__ void load(const uint32_t* src, int n, int gl) {
#pragma unroll
        for (int i = 0; i < R; i++) {
            const int k = gl + i * LPE;
            v[i] = k < n ? src[k] : 0u;
        }
    }
    __device__ __forceinline__ void store(uint32_t* dst, int n, int gl) const {
#pragma unroll
        for (int i = 0; i < R; i++) {
            const int k = gl + i * LPE;
            if (k < n) dst[k] = v[i];
        }
    }
};

// n bytes from global src to LDS dst: dword loads when both sides allow (issued together, then
// the LDS stores), else byte loads. LDS destinations are 4-byte aligned (ms_layout.h).
template <int LPE>
__device__ __forceinline__ void stage_bytes(int8_t* dst, const int8_t* src, int n, int gl) {
    if ((n & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 3) == 0) {
        const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
        uint32_t* d4 = reinterpret_cast<uint32_t*>(dst);
#pragma unroll 4
        for (int i = gl; i < n / 4; i += LPE) d4[i] = s4[i];
    } else {
#pragma unroll 4
        for (int i = gl; i < n; i += LPE) dst[i] = src[i];
    }
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

// Episode metrics (ms_env_metrics): no-return device atomics on the env's own accumulators (one
// group per env, so nothing contends across envs and each replica's order is fixed). The vector
// atomics leave no wait in the round's chain; the adds land before the kernel ends.
__device__ __forceinline__ void m_add(int32_t* p, int v) {
    if (v) __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void m_add(int64_t* p, long long v) {
    if (v) __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void m_add(double* p, double v) {
    if (v != 0.0) unsafeAtomicAdd(p, v);
}

// Masks of the current offers: mc[c] = offers to core c, mr[r] = offers to
// recipient r (0 = auctioneer). Ends with a phase boundary.
// With last1 != NULL also last1[c] = 1 when an offer to core c holds a job with one round left.
template <int LPE>
__device__ void build_masks(Rec& R, const Geom& P, M128* mc, M128* mr, int gl, uint8_t* last1 = nullptr) {
    for (int i = gl; i < P.C; i += LPE) {
        mc[i] = M128{0, 0};
        if (last1) last1[i] = 0;
    }
    for (int i = gl; i <= P.N; i += LPE) mr[i] = M128{0, 0};
    wave_sync();
    const int8_t* oc = R.offer_core();
    const int8_t* orc = R.offer_recip();
    for (int i = gl; i < P.NL; i += LPE) {
        const int c = oc[i];
        if (c >= 0) {
            mask_set(&mc[c], i);
            mask_set(&mr[orc[i]], i);
            if (last1 && R.slot_rem()[i] == 1) last1[c] = 1;
        }
    }
    wave_sync();
}

// ---------------------------------------------------------------------------
// observations of the current (LDS) state: Agent.py:167-212 (acceptor),
// Agent.py:271-300 (offer), Auctioneer.py:34-77 (auctioneer)

// Observations. At emission time every offer to core c is addressed to c's owner: offers are
// created after the tick with recipient = the core's owner (world.py:428) and ownership changes
// only in the next round's executions (ms_env_import checks the same invariant). So the acceptor
// row of (agent a, core c) (Agent.py:167-212) is the core's "owner row"
//   [1, prio, rem, (price, necT) per offer to c in offer-ID order, (-2, -2) pad, 0 stride pad]
// when a owns c, and otherwise the constant "foreign row" [0, -1, -1, (-2, -2) * O, 0 pad]; the
// auctioneer row of core c (Auctioneer.py:34-77) is the same with the auctioneer as owner. An
// offer row (Agent.py:271-300) is the env's core-pair template with the slot's own pair merged.
//
// The source rows are built in LDS; then each of the env's observation blocks is streamed as a
// flat dword array. The strides are multiples of 4, so every dword lies in one row and is a
// dword of that row's source. With 16-B aligned blocks each lane stores 4 consecutive dwords
// with one global_store_dwordx4: the store-instruction count per CU, not the bytes, bounded the
// row-at-a-time emission.

// dword k of the foreign row
__device__ __forceinline__ uint32_t foreign_dword(int k, int d_acc) {
    uint32_t w = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
        const int col = 4 * k + b;
        const uint32_t v = col == 0 ? 0x00u : (col < 3 ? 0xFFu : (col < d_acc ? 0xFEu : 0x00u));
        w |= v << (8 * b);
    }
    return w;
}

// The LDS sources of env e's observations:
//   crow [C+1][acc_stride]: the owner rows of the C cores, then the foreign row;
//   rowsrc [N*C] u16: dword offset in crow of acceptor row (a, c)'s source: row c if agent a owns
//                     core c, else the foreign row C;
//   otmpl [off_stride]: offer-row template (the (prio, rem) pairs of all cores, zero tail);
//   slot_pair [NL]: (prio, rem) of every slot.
template <int LPE>
__device__ void build_obs_sources(Rec& R, const Geom& P, const M128* mc, const M128* mr, uint8_t* scratch, bool acc,
                                  bool auct, bool off, int gl) {
    const int C = P.C, nw = P.acc_stride / 4;
    uint32_t* crow = reinterpret_cast<uint32_t*>(scratch);
    const int8_t* owner = R.core_owner();
    const int8_t* ck = R.core_kind();
    const int8_t* cr = R.core_rem();
    if (acc || auct) {
        // lane-fixed column: one foreign dword per lane, stored to all C + 1 rows (no division)
        for (int k = gl; k < nw; k += LPE) {
            const uint32_t v = foreign_dword(k, P.d_acc);
            for (int r = 0; r <= C; r++) crow[r * nw + k] = v;
        }
    }
    if (acc) {
        uint16_t* rowsrc = reinterpret_cast<uint16_t*>(scratch + P.s_rowsel);
        for (int r = gl; r < P.N * C; r += LPE) {
            const int a = r / C, c = r - a * C;
            rowsrc[r] = (uint16_t)((owner[c] == a + 1 ? c : C) * nw);
        }
    }
    if (off) {
        uint32_t* otmpl = reinterpret_cast<uint32_t*>(scratch + P.s_otmpl);
        for (int k = gl; k < P.off_stride / 4; k += LPE) {
            uint32_t cw = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int col = 4 * k + b;
                if (col < 2 * C) {
                    const int c = col >> 1, kk = ck[c];
                    const int v = kk < 0 ? -1 : ((col & 1) ? cr[c] : R.prio(kk));
                    cw |= (uint32_t)(uint8_t)v << (8 * b);
                }
            }
            otmpl[k] = cw;
        }
        uint16_t* slot_pair = reinterpret_cast<uint16_t*>(scratch + P.s_slotpair);
        for (int s = gl; s < P.NL; s += LPE) {
            const int k = R.slot_kind()[s];
            const uint32_t pr = (uint8_t)(k < 0 ? -1 : R.prio(k));
            const uint32_t rm = (uint8_t)(k < 0 ? -1 : R.slot_rem()[s]);
            slot_pair[s] = (uint16_t)(pr | (rm << 8));
        }
    }
    wave_sync();
    if (acc || auct) {
        const int8_t* op = R.offer_price();
        const int8_t* sr = R.slot_rem();
        const int8_t* oc = R.offer_core();
        const int8_t* orc = R.offer_recip();
        for (int c = gl; c < C; c += LPE) {
            int8_t* row = reinterpret_cast<int8_t*>(crow) + c * P.acc_stride;
            const int kind = ck[c];
            row[0] = 1;
            row[1] = (int8_t)(kind >= 0 ? R.prio(kind) : -1);
            row[2] = cr[c];
        }
        // the (price, necT) pairs of the offers to c addressed to c's owner, in offer-ID order
        // (Agent.py:180-200): one lane per offer, placed at its rank among those offers (no serial
        // walk of the core's mask)
        for (int i = gl; i < P.NL; i += LPE) {
            const int c = oc[i];
            if (c >= 0 && orc[i] == owner[c]) {
                const M128 m = mand(mc[c], mr[owner[c]]);
                const int rank = i < 64 ? __popcll(m.lo & ((1ull << i) - 1ull))
                                        : __popcll(m.lo) + __popcll(m.hi & ((1ull << (i - 64)) - 1ull));
                int8_t* row = reinterpret_cast<int8_t*>(crow) + c * P.acc_stride;
                row[3 + 2 * rank] = op[i];
                row[4 + 2 * rank] = sr[i];
            }
        }
    }
    wave_sync();
}

__device__ __forceinline__ int div_mag(uint32_t w, uint32_t mag, int d) { return d == 1 ? (int)w : (int)__umulhi(w, mag); }

// x / d for 0 <= x < 256 and 1 <= d < 256 without the integer-division sequence: floor((x + 1/2) * rcp(d)).
// (x + 1/2) / d lies at least 1/(2d) >= 2^-9 from an integer and the product's error is below
// 256 * 2^-21 = 2^-13 (rcp within 2 ulp), so the floor is exact; checked exhaustively over the range
// with the reciprocal perturbed by +-2 ulp (tests/test_env_helpers.py).
__device__ __forceinline__ int small_div(int x, int d) {
    return (int)(((float)x + 0.5f) * __builtin_amdgcn_rcpf((float)d));
}

// Block e of an [E][n_dw] dword array: dword w = val(w / nw, w % nw), LPE lanes, 4 dwords per
// lane-store (write-through) when aligned.
template <int LPE, class F>
__device__ __forceinline__ void emit_flat(uint32_t* base, int64_t e, int64_t E, int n_dw, int nw, uint32_t mag, int gl,
                                          F val) {
    const WtOut o(base, E * n_dw * 4);
    if (o.ok && (n_dw & 3) == 0) {
        const int64_t env_off = e * n_dw * 4;
        for (int k = gl; 4 * k < n_dw; k += LPE) {
            const int w0 = 4 * k;
            int r = div_mag(w0, mag, nw), col = w0 - r * nw;
            uint32_t v[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                v[i] = val(r, col);
                if (++col == nw) {
                    col = 0;
                    r++;
                }
            }
            o.st4(env_off + 4 * w0, v[0], v[1], v[2], v[3]);
        }
    } else {
        uint32_t* dst = base + e * n_dw;
        for (int w = gl; w < n_dw; w += LPE) {
            const int r = div_mag(w, mag, nw);
            dst[w] = val(r, w - r * nw);
        }
    }
}

// Block e of an [E][n_rows][nw] dword array, streamed in row groups: RG = lcm(nw, 4) / nw rows
// are CG = lcm(nw, 4) / 4 16-byte chunks. Lane l < GPI * CG (GPI = LPE / CG row groups per pass)
// owns chunk j = l % CG of every GPI-th row group, so the (row in group, column) of its four
// dwords are fixed per lane: src(row, col, i) is one lookup per dword. Other shapes (CG > LPE,
// unaligned arrays) take emit_flat.
template <int LPE, class Src>
__device__ __forceinline__ void emit_rows(uint32_t* base, int64_t e, int64_t E, int n_rows, int nw, uint32_t mag,
                                          int gl, Src src) {
    const int n_dw = n_rows * nw;
    const int lg4 = (nw & 1) ? 2 : ((nw & 2) ? 1 : 0);
    const int g4 = 1 << lg4;  // RG
    const int CG = (nw << lg4) >> 2;
    const WtOut o(base, E * n_dw * 4);
    if (!o.ok || (n_dw & 3) != 0 || CG > LPE) {
        emit_flat<LPE>(base, e, E, n_dw, nw, mag, gl, [&](int r, int col) { return src(r, col, 0); });
        return;
    }
    const int GPI = small_div(LPE, CG);  // CG <= LPE <= 64
    const int q0 = small_div(gl, CG), j = gl - q0 * CG;
    if (q0 >= GPI) return;
    int ri[4], col[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int d = 4 * j + i;
        ri[i] = div_mag(d, mag, nw);
        col[i] = d - ri[i] * nw;
    }
    const int64_t env_off = e * n_dw * 4;
    const int n_groups = n_rows >> lg4;
    for (int q = q0; q < n_groups; q += GPI) {
        const int r0 = q * g4;
        o.st4(env_off + 4 * (r0 * nw + 4 * j), src(r0 + ri[0], col[0], 0), src(r0 + ri[1], col[1], 1),
              src(r0 + ri[2], col[2], 2), src(r0 + ri[3], col[3], 3));
    }
}

// All observations of env e (dst == NULL skips a kind; a padding group passes write = false).
template <int LPE>
__device__ void emit_obs(Rec& R, const Geom& P, const M128* mc, const M128* mr, uint8_t* scratch, int8_t* acc,
                         int8_t* off, int8_t* auct, int8_t* crows, int8_t* cown, int64_t e, int64_t E, bool write,
                         int gl) {
    build_obs_sources<LPE>(R, P, mc, mr, scratch, acc != nullptr, auct != nullptr || crows != nullptr, off != nullptr,
                           gl);
    if (!write) return;
    const int C = P.C, nw = P.acc_stride / 4, nwo = P.off_stride / 4;
    const uint32_t* crow = reinterpret_cast<const uint32_t*>(scratch);
    if (acc) {
        const uint16_t* rowsrc = reinterpret_cast<const uint16_t*>(scratch + P.s_rowsel);
        emit_rows<LPE>(reinterpret_cast<uint32_t*>(acc), e, E, P.N * C, nw, P.mag_acc, gl,
                       [&](int r, int col, int) { return crow[rowsrc[r] + col]; });
    }
    if (auct) {
        const int8_t* owner = R.core_owner();
        emit_rows<LPE>(reinterpret_cast<uint32_t*>(auct), e, E, C, nw, P.mag_acc, gl,
                       [&](int c, int col, int) { return crow[(owner[c] == 0 ? c : C) * nw + col]; });
    }
    // compact acceptor observations: the owner row of every core and the owners; acceptor row (a, c)
    // is core row c when a + 1 == owner[c], else the constant foreign row (regenerated on demand)
    if (crows) emit_rows<LPE>(reinterpret_cast<uint32_t*>(crows), e, E, C, nw, P.mag_acc, gl,
                              [&](int c, int col, int) { return crow[c * nw + col]; });
    if (cown) {
        const int8_t* owner = R.core_owner();
        for (int c = gl; c < C; c += LPE) cown[e * C + c] = owner[c];
    }
    if (off) {
        const uint32_t* otmpl = reinterpret_cast<const uint32_t*>(scratch + P.s_otmpl);
        const uint16_t* slot_pair = reinterpret_cast<const uint16_t*>(scratch + P.s_slotpair);
        const int pcol = (2 * C) >> 2, pshift = 8 * ((2 * C) & 3);
        emit_rows<LPE>(reinterpret_cast<uint32_t*>(off), e, E, P.NL, nwo, P.mag_off, gl, [&](int s, int col, int) {
            uint32_t v = otmpl[col];
            if (col == pcol) v |= (uint32_t)slot_pair[s] << pshift;
            return v;
        });
    }
}

// HardcodedAuctioneerAcceptor.selectAction for every core (HardcodedModules.py:54-78,
// Auctioneer.getAuctioneerAction Auctioneer.py:95-102) on the staged state: per core the max
// ratio over the auctioneer's offers and the count of offers attaining it (in registers), then
// one _randbelow(count) per tied core in core order on the env stream. Writes s_auct[c] (O = reject).
// Needs LPE >= C (group lane c owns core c).
template <int LPE>
__device__ void hardcoded_auctioneer(Rec& R, const Geom& P, const M128* s_mc, const M128* s_mr, MtStream<LPE>& rs,
                                     int16_t* s_auct, const Lanes<LPE>& L) {
    const int C = P.C, O = P.O, gl = L.gl;
    const int8_t* c_owner = R.core_owner();
    const int8_t* o_price = R.offer_price();
    const int8_t* s_rem = R.slot_rem();
    // per core, in one pass over the auctioneer's offers: the max ratio (the padded list's -1
    // entries and the own empty job bound it from below), how many offers attain it and their
    // positions in the padded list (a new maximum restarts the count)
    int mn = -1, md = 1, nt = 0;
    M128 ties{0, 0};
    if (gl < C) {
        if (c_owner[gl] == 0) {
            int k = 0;
            for (MaskIter it(mand(s_mc[gl], s_mr[0])); it.more(); k++) {
                const int i = it.next();
                int num, den;
                ratio_of(o_price[i], s_rem[i], num, den);
                const int lhs = num * md, rhs = mn * den;
                if (lhs >= rhs) {
                    if (lhs > rhs) {
                        mn = num;
                        md = den;
                        nt = 0;
                        ties = M128{0, 0};
                    }
                    nt++;
                    if (k < 64)
                        ties.lo |= 1ull << k;
                    else
                        ties.hi |= 1ull << (k - 64);
                }
            }
            if (!(mn > -md)) nt = 0;  // max(ratios) must exceed the own ratio (-1, the empty job)
        }
        s_auct[gl] = (int16_t)O;
    }
    // tie-break draws in core order on the env stream (Auctioneer.getAuctioneerAction
    // Auctioneer.py:95-102), only for the cores with a candidate. The draws run on the words the
    // window already holds: each draw takes the first word from the stream position at which its
    // _randbelow accepts (MtStream::randbelow's rule), the chain carried in registers, and each
    // core lane reads its accepted word once at the end; a draw the window cannot finish and the
    // ones after it go through MtStream::randbelow.
    const uint64_t need = L.ballot(gl < C && nt > 0);
    int my_pick = 0;
    if (need) {
        if (rs.p >= rs.wend) rs.load(rs.p, 1, L);
        const uint32_t tv = rs.word();
        const int wpos = rs.wb + gl;
        const bool live = wpos < rs.wend;
        int p = rs.p, my_q = -1, my_sh = 0;
        uint64_t rest = need;
        for (uint64_t m = need; m; m &= m - 1) {
            const int c = __ffsll((unsigned long long)m) - 1;
            const uint32_t n = L.shfl((uint32_t)nt, c);
            const int sh = __clz(n);  // 32 - n.bit_length()
            const uint64_t acc = L.ballot(live && wpos >= p && (tv >> sh) < n);
            if (!acc) break;
            const int q = __ffsll((unsigned long long)acc) - 1;
            if (gl == c) {
                my_q = q;
                my_sh = sh;
            }
            p = rs.wb + q + 1;
            rest &= rest - 1;
        }
        const uint32_t w = L.shfl(tv, my_q < 0 ? 0 : my_q);
        if (my_q >= 0) my_pick = (int)(w >> my_sh);
        rs.p = p;
        for (uint64_t m = rest; m; m &= m - 1) {
            const int c = __ffsll((unsigned long long)m) - 1;
            const uint32_t pick = rs.randbelow(L.shfl((uint32_t)nt, c), L);
            if (gl == c) my_pick = (int)pick;
        }
    }
    // the pick-th maximal candidate's position in the padded list
    if (gl < C && nt > 0) s_auct[gl] = (int16_t)kth_bit(ties, my_pick);
}

// The hard-coded agents of HardcodedFixPriceEnvironment (SchedulingEnvironment.py:439-456):
// DividedHardcodedAgent.getActions (Agent.py:630-641) asks, per agent, its HardcodedOfferer of
// every slot (HardcodedModules.py:81-109: a core of minimal ratio, random.sample over the tied
// cores) and then its HardcodedAcceptor of every core (:16-45: reject unless the agent owns the core
// and the best offered ratio beats its own job's; random.sample over the tied maxima), all on the
// env stream before the auctioneer draws. The offer rows of all slots hold the same core pairs, so
// one candidate mask serves every offerer. Writes the staged action arrays (LDS). Needs LPE >= C.
template <int LPE>
__device__ void hardcoded_agents(Rec& R, const Geom& P, const M128* s_mc, const M128* s_mr, MtStream<LPE>& rs,
                                 int8_t* a_acc, int8_t* a_off, const Lanes<LPE>& L) {
    const int C = P.C, N = P.N, NL = P.NL, O = P.O, gl = L.gl;
    const int8_t* c_owner = R.core_owner();
    const int8_t* c_kind = R.core_kind();
    const int8_t* c_rem = R.core_rem();
    const int8_t* o_price = R.offer_price();
    const int8_t* s_rem = R.slot_rem();
    // offerers: the cores of minimal calculateRewardRatio(prio, rem) (empty cores: -1)
    uint64_t cand = 0;
    int mn = 0, md = 1;
    for (int c = 0; c < C; c++) {
        const int k = c_kind[c];
        int num, den;
        ratio_of(k >= 0 ? R.prio(k) : -1, c_rem[c], num, den);
        const int lhs = num * md, rhs = mn * den;
        if (c == 0 || lhs < rhs) {
            mn = num;
            md = den;
            cand = 1ull << c;
        } else if (lhs == rhs) {
            cand |= 1ull << c;
        }
    }
    const uint32_t nc = (uint32_t)__popcll(cand);
    // acceptors: group lane c evaluates core c for its owner (an agent's own job is never empty)
    int nt = 0;
    M128 ties{0, 0};
    if (gl < C && c_owner[gl] > 0) {
        const int k = c_kind[gl];
        int on, od;
        ratio_of(R.prio(k), c_rem[gl], on, od);
        int bn = 0, bd = 1, kk = 0;
        bool any = false;
        for (MaskIter it(mand(s_mc[gl], s_mr[c_owner[gl]])); it.more(); kk++) {
            const int i = it.next();
            int num, den;
            ratio_of(o_price[i], s_rem[i], num, den);
            const int lhs = num * bd, rhs = bn * den;
            if (!any || lhs > rhs) {
                bn = num;
                bd = den;
                nt = 0;
                ties = M128{0, 0};
                any = true;
            }
            if (lhs >= rhs || nt == 0) {
                nt++;
                if (kk < 64)
                    ties.lo |= 1ull << kk;
                else
                    ties.hi |= 1ull << (kk - 64);
            }
        }
        // the (-2, -2) pads of the padded list rate -1 (calculateRewardRatio)
        if (kk < O && (!any || -bd >= bn)) {
            if (!any || -bd > bn) {
                bn = -1;
                bd = 1;
                nt = 0;
                ties = M128{0, 0};
            }
            for (int q = kk; q < O; q++) {
                nt++;
                if (q < 64)
                    ties.lo |= 1ull << q;
                else
                    ties.hi |= 1ull << (q - 64);
            }
        }
        if (!(bn * od > on * bd)) nt = 0;  // max(listOfOfferdRatios) > ownRewardRatio
    }
    for (int i = gl; i < N * C; i += LPE) a_acc[i] = (int8_t)O;
    wave_sync();
    // the draws, in getActions order
    for (int a = 0; a < N; a++) {
        for (int j = 0; j < P.L; j++) {
            const uint32_t pick = rs.randbelow(nc, L);
            uint64_t m = cand;
            for (uint32_t q = 0; q < pick; q++) m &= m - 1;
            if (gl == 0) a_off[a * P.L + j] = (int8_t)(__ffsll((unsigned long long)m) - 1);
        }
        const uint64_t mine = L.ballot(gl < C && nt > 0 && c_owner[gl] == a + 1);
        for (uint64_t m = mine; m; m &= m - 1) {
            const int c = __ffsll((unsigned long long)m) - 1;
            const uint32_t pick = rs.randbelow(L.shfl((uint32_t)nt, c), L);
            if (gl == c) a_acc[a * C + c] = (int8_t)kth_bit(ties, (int)pick);
        }
    }
    (void)NL;
}

// ---------------------------------------------------------------------------
// kernels (the host picks LPE; init / reset / auctioneer / randbelow run one env per wave)

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
    Rec R{rec, &P, nullptr};
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
        const uint64_t s = seed + (uint64_t)e;
        const uint32_t key[2] = {(uint32_t)s, (uint32_t)(s >> 32)};
        const int len = key[1] ? 2 : 1;
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
        R.mt_sel() = 2u;  // current = half 0, half 1 = its successor
    }
    wave_sync();
    copy_dwords<kWave>(mt + e * 2 * kMtN, st, kMtN, lane);
    wave_sync();
    mt_twist_lds_wave(st, lane);
    copy_dwords<kWave>(mt + e * 2 * kMtN + kMtN, st, kMtN, lane);
    copy_dwords<kWave>(reinterpret_cast<uint32_t*>(recs + e * (int64_t)P.rec_bytes), reinterpret_cast<uint32_t*>(rec),
                       P.rec_bytes / 4, lane);
}

__global__ void __launch_bounds__(64) k_env_reset(Params P, const uint8_t* recs, int8_t* obs_acc, int8_t* obs_off,
                                                  int8_t* obs_auct, int8_t* obs_crow, int8_t* obs_cown) {
    extern __shared__ __align__(16) uint8_t smem[];
    M128* s_mc = reinterpret_cast<M128*>(smem + P.s_mc);
    M128* s_mr = reinterpret_cast<M128*>(smem + P.s_mr);
    const int lane = threadIdx.x;
    const int64_t e = blockIdx.x;
    uint8_t* rec = smem + P.s_rec;
    __shared__ int32_t s_kt[48];
    load_kind_tables(P, s_kt, lane);
    copy_dwords<kWave>(reinterpret_cast<uint32_t*>(rec),
                       reinterpret_cast<const uint32_t*>(recs + e * (int64_t)P.rec_bytes), P.rec_bytes / 4, lane);
    wave_sync();
    Rec R{rec, &P, s_kt};
    build_masks<kWave>(R, P, s_mc, s_mr, lane);
    emit_obs<kWave>(R, P, s_mc, s_mr, smem + P.s_scratch, obs_acc, obs_off, obs_auct, obs_crow, obs_cown, e, gridDim.x,
                    true, lane);
}

// Shape tags of env_round: DynShape reads the geometry from the kernel arguments; FixShape<N, C,
// L, J> compiles it in (the BASELINE shapes, launch_env_step picks them when the config matches).
struct DynShape {
    static constexpr bool kStatic = false;
    static constexpr int kN = 0, kC = 0, kL = 0, kJ = 0;
};
template <int N_, int C_, int L_, int J_>
struct FixShape {
    static constexpr bool kStatic = true;
    static constexpr int kN = N_, kC = C_, kL = L_, kJ = J_;
};

constexpr int kLiabPrefetch = 4;  // newest chain entries loaded ahead per core that may terminate

// One round of SchedulingEnv.step (SchedulingEnvironment.py:32-83): group g of block b steps env
// b * (64 / LPE) + g. Each group owns a P.s_total-byte slice of the block's LDS. EXT: the kernel
// variant with the optional features (hard-coded agents when io.act_acc == NULL, episode metrics,
// compact acceptor observations); the plain training round is compiled without them, so it carries
// none of their registers (the compact emission beside the full rows costs ~90 spilled SGPRs). CMP:
// the plain round that emits the compact acceptor observations instead of the [N][C] rows (the
// training loop's form: its act and gradient kernels read core rows + owners).
template <int LPE, bool EXT, bool CMP, class SH>
__device__ __forceinline__ void env_round(const Params& P, int64_t E, uint8_t* recs, uint32_t* mt, Liab* liab,
                                          const StepIO& io, int64_t slot, int lane_arg = -1,
                                          uint8_t* wave_lds = nullptr, const int8_t* acc_lds = nullptr) {
    // wave_lds: the wave's part of a multi-wave workgroup's LDS (k_env_rollout_act_free), else the block's;
    // acc_lds: the acceptor actions of the wave's replicas in the LDS ([kWave / LPE][N * C]; read instead of
    // io.act_acc, which then serves the padding replicas only)
    extern __shared__ __align__(16) uint8_t smem_dyn[];
    uint8_t* const smem_all = wave_lds ? wave_lds : smem_dyn;
    // the shape: a compile-time constant for the BASELINE shapes (offsets fold into immediates,
    // loops over agents / cores / slots get constant trip counts), else the kernel arguments
    Geom g;
    if constexpr (SH::kStatic) {
        constexpr Geom kg = make_geom(SH::kN, SH::kC, SH::kL, SH::kJ);
        g = kg;
    } else {
        g = P;
    }
    const int lane = lane_arg >= 0 ? lane_arg : (int)threadIdx.x;  // (k_env_rollout_act: opaque per round)
    const Lanes<LPE> Lg(lane);
    const int gl = Lg.gl;
    const int64_t e_raw = slot * (kWave / LPE) + (lane / LPE);
    const bool active = e_raw < E;  // padding groups of the last wave replay env E-1 without writing
    const int64_t e = active ? e_raw : E - 1;
    uint8_t* smem = smem_all + (lane / LPE) * g.s_total;
    M128* s_mc = reinterpret_cast<M128*>(smem + g.s_mc);          // offers per core
    M128* s_mr = reinterpret_cast<M128*>(smem + g.s_mr);          // offers per recipient (0 = auctioneer)
    Liab* s_newle = reinterpret_cast<Liab*>(smem + g.s_newle);    // liability entry appended this round per core
    int16_t* s_exec = reinterpret_cast<int16_t*>(smem + g.s_exec);  // per core: executed offer's slot, -1 none
    int16_t* s_key = reinterpret_cast<int16_t*>(smem + g.s_key);    // execution order key
    int8_t* s_by_rank = reinterpret_cast<int8_t*>(smem + g.s_rank); // cores in execution order
    int8_t* s_fresh = reinterpret_cast<int8_t*>(smem + g.s_fresh);  // s_newle[c] is the chain's newest entry
    int16_t* s_auct = reinterpret_cast<int16_t*>(smem + g.s_auct);  // auctioneer action per core
    int32_t* s_agent_r = reinterpret_cast<int32_t*>(smem + g.s_agentr);  // agentReward
    int32_t* s_auct_r = reinterpret_cast<int32_t*>(smem + g.s_auctr);    // auctioneerReward
    int32_t* s_credit = reinterpret_cast<int32_t*>(smem + g.s_credit);   // chain credits per recipient
    uint32_t& s_flags = *reinterpret_cast<uint32_t*>(smem + g.s_misc);
    int& s_n_exec = *reinterpret_cast<int*>(smem + g.s_misc + 4);

    const int N = g.N, C = g.C, L = g.L, NL = g.NL, O = g.O;
#ifdef MS_PHASE_TIMING
    uint64_t t_prev = __builtin_amdgcn_s_memtime();
    uint64_t t_acc[16] = {};
#endif

    uint8_t* rec = smem + g.s_rec;
    int8_t* a_acc = reinterpret_cast<int8_t*>(smem + g.s_act_acc);
    int8_t* a_off = reinterpret_cast<int8_t*>(smem + g.s_act_off);
    int8_t* a_price = reinterpret_cast<int8_t*>(smem + g.s_act_price);
    int8_t* a_auct = reinterpret_cast<int8_t*>(smem + g.s_act_auct);
    int32_t* acc_r = reinterpret_cast<int32_t*>(smem + g.s_accr);
    float* off_r = reinterpret_cast<float*>(smem + g.s_offr);
    float* price_r = reinterpret_cast<float*>(smem + g.s_pricer);
    int8_t* spawn_kind = reinterpret_cast<int8_t*>(smem + g.s_spawn_kind);
    uint8_t* scratch = smem + g.s_scratch;

    // ---- stage state and actions in LDS; the successor MT blocks of the envs that crossed into
    //      theirs last round are made while the staged words wait in registers (whole wave in LDS)
    __shared__ int32_t s_kt[48];
    {
        // the record and the dword-aligned action arrays: one batch of loads, then the LDS stores
        const uint32_t* src_rec = reinterpret_cast<const uint32_t*>(recs + e * (int64_t)g.rec_bytes);
        const int rec_dw = g.rec_bytes / 4;
        const int8_t* a_src[4] = {acc_lds && active ? acc_lds + (lane / LPE) * N * C
                                                    : (io.act_acc ? io.act_acc + e * N * C : nullptr),
                                  io.act_off ? io.act_off + e * NL : nullptr,
                                  io.act_price ? io.act_price + e * NL : nullptr,
                                  io.act_auct ? io.act_auct + e * C : nullptr};
        int8_t* a_dst[4] = {a_acc, a_off, a_price, a_auct};
        const int a_len[4] = {N * C, NL, NL, C};
        int a_dw[4];
#pragma unroll
        for (int i = 0; i < 4; i++)
            a_dw[i] = (a_src[i] && (a_len[i] & 3) == 0 && (reinterpret_cast<uintptr_t>(a_src[i]) & 3) == 0)
                          ? a_len[i] / 4
                          : 0;
        constexpr int RB = (96 + LPE - 1) / LPE;  // records up to 384 B in the batch
        DwordBatch<LPE, RB> br;
        DwordBatch<LPE, 1> ba[4];
        br.load(src_rec, rec_dw, gl);
#pragma unroll
        for (int i = 0; i < 4; i++) ba[i].load(reinterpret_cast<const uint32_t*>(a_src[i]), a_dw[i], gl);
        // record dword 3 (mt_sel) is group lane 3's first staged word: the refill test costs no load
        // round trip of its own (the LDS is not written yet, so the twist may use all of it)
        const uint32_t sel = Lg.shfl(br.v[0], 3);
        const uint64_t need = __ballot(active && gl == 0 && !(sel & 2u));
        if (need) mt_refill_groups<LPE>(mt, slot * (kWave / LPE), need, sel, smem_all, lane);
        load_kind_tables(P, s_kt, lane);
        br.store(reinterpret_cast<uint32_t*>(rec), rec_dw, gl);
#pragma unroll
        for (int i = 0; i < 4; i++) ba[i].store(reinterpret_cast<uint32_t*>(a_dst[i]), a_dw[i], gl);
        // the rest (large records / action arrays, unaligned arrays)
        for (int k = gl + RB * LPE; k < rec_dw; k += LPE) reinterpret_cast<uint32_t*>(rec)[k] = src_rec[k];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            for (int k = gl + LPE; k < a_dw[i]; k += LPE)
                reinterpret_cast<uint32_t*>(a_dst[i])[k] = reinterpret_cast<const uint32_t*>(a_src[i])[k];
            if (a_src[i] && a_dw[i] == 0) stage_bytes<LPE>(a_dst[i], a_src[i], a_len[i], gl);
        }
    }
    for (int i = gl; i < N * C; i += LPE) acc_r[i] = 0;
    for (int i = gl; i < NL; i += LPE) {
        off_r[i] = 0.f;
        price_r[i] = 0.f;
    }
    for (int i = gl; i < C; i += LPE) {
        s_auct_r[i] = 0;
        s_exec[i] = -1;
        s_fresh[i] = 0;
    }
    for (int i = gl; i < N; i += LPE) {
        s_agent_r[i] = 0;
        s_credit[i] = 0;
    }
    if (gl == 0) {
        s_flags = 0;
        s_n_exec = 0;
    }
    wave_sync();
    MS_MARK(1);
    Rec R{rec, &g, s_kt};
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
    // this round's episode accumulators (trainPPO.py:172-187): slot of episode round / episodeLength
    const bool HC = EXT && io.act_acc == nullptr;
    constexpr bool MX = EXT;
    ms_env_metrics* mx = (MX && io.metrics && active)
                             ? io.metrics + (int64_t)((round / P.ep_len) % io.metrics_slots) * E + e
                             : nullptr;

    // ---- issue the dependent loads early: the MT window at mti (a peek: no twist
    //      yet) and the newest liability entries of every core that may terminate
    //      this round, i.e. whose current job or one of the jobs offered to it has
    //      one round left (its chain is settled in the tick below)
    MtStream<LPE> rs;
    rs.init(mt + e * 2 * kMtN, R.mt_sel(), R.mti(), active);
    rs.load(0, 0, Lg);
    // the scratch is free until the executions: per core, "an offer to it has one round left"
    build_masks<LPE>(R, g, s_mc, s_mr, gl, scratch);
    Liab pf[kLiabPrefetch];
    int pf_n = 0;
    if (gl < C) {
        const bool maybe = (c_kind[gl] >= 0 && c_rem[gl] == 1) || scratch[gl];
        if (maybe) {
            const int n = l_n[gl];
            pf_n = min(n, kLiabPrefetch);
            const Liab* chain = my_liab + gl * P.cap;
#pragma unroll
            for (int q = 0; q < kLiabPrefetch; q++)
                if (q < pf_n) pf[q] = chain[n - 1 - q];
        }
    }

    MS_MARK(2);
    // ---- auctioneer actions: HardcodedAuctioneerAcceptor (HardcodedModules.py:54-78), asked by the
    //      driver before env.step (trainPPO.py:162); ties broken with random.sample -> _randbelow
    if (HC) {  // HardcodedFixPriceEnvironment: the agents' actions come from the kernel
        hardcoded_agents<LPE>(R, g, s_mc, s_mr, rs, a_acc, a_off, Lg);
        wave_sync();
    }
    if (!io.act_auct) {
        hardcoded_auctioneer<LPE>(R, g, s_mc, s_mr, rs, s_auct, Lg);
    } else {
        for (int c = gl; c < C; c += LPE) s_auct[c] = a_auct[c];
    }
    // the spawn's words, peeked now at the stream position the tie-breaks left: the load's latency
    // hides behind the executions and the tick (a window short of the spawn reloads there)
    if (rs.wend - rs.p < 2 * P.new_jobs * N) rs.load(rs.p, 0, Lg);
    wave_sync();
    MS_MARK(3);

    // ---- which offer each core executes (executeAgentAcceptions1 world.py:391-404,
    //      executeAuctioneerAcceptions world.py:378-389): offers to core c are all addressed to c's
    //      owner (created after the tick with recipient = owner, world.py:428), so only the owner's
    //      acceptor (or the auctioneer) can pick one, and each core executes at most once per round.
    for (int i = gl; i < N * C; i += LPE) {
        const int a = a_acc[i];
        if (a < 0 || a > O) atomicOr(&s_flags, MS_FLAG_BAD_ACTION);
    }
    for (int c = gl; c < C; c += LPE) {
        const int owner = c_owner[c];
        const int idx = owner > 0 ? a_acc[(owner - 1) * C + c] : s_auct[c];
        if (owner == 0 && (idx < 0 || idx > O)) atomicOr(&s_flags, MS_FLAG_BAD_ACTION);
        int slot = -1;
        if (idx >= 0 && idx < O) slot = kth_bit(mand(s_mc[c], s_mr[owner]), idx);
        s_exec[c] = (int16_t)slot;
        s_key[c] = (int16_t)(owner > 0 ? (owner - 1) * C + c : N * C + c);
    }
    wave_sync();
    for (int c = gl; c < C; c += LPE) {
        if (s_exec[c] >= 0) {
            // branch-free, so the unrolled loop issues its LDS reads together
            const int kc = s_key[c];
            int r = 0;
#pragma unroll 8
            for (int d = 0; d < C; d++) r += (int)(s_exec[d] >= 0) & (int)(s_key[d] < kc);
            s_by_rank[r] = (int8_t)c;
            atomicAdd(&s_n_exec, 1);
        }
    }
    wave_sync();
    MS_MARK(4);

    // ---- apply executions in reference order (World.executeAnOffer world.py:261-293). Executions
    //      of different cores touch different cores, offer slots, liability chains and reward
    //      entries; only the placement of a dispatched job in its recipient's first empty slot
    //      (world.py:123-133) depends on the earlier executions, through that one collection. So the
    //      plain round runs each execution's core part on the core's lane, then replays the
    //      removals and insertions of every collection, in rank order, on the collection owner's
    //      lane. With episode metrics or event records (their rank-ordered sums) the groups' leaders
    //      run the executions one after another instead.
    if (!EXT && io.ev_acc == nullptr) {
        // per core, in the scratch (free between the staging and the observation emission): the
        // job its execution dispatched away (for the insertion), the offerer and the recipient
        int32_t* x_birth = reinterpret_cast<int32_t*>(scratch);
        int8_t* x_kind = reinterpret_cast<int8_t*>(scratch + 4 * C);
        int8_t* x_rem = x_kind + C;
        int8_t* x_off = x_kind + 2 * C;
        int8_t* x_recip = x_kind + 3 * C;
        if (gl < C && s_exec[gl] >= 0) {
            const int c = gl;
            const int i = s_exec[c];
            const int offerer = small_div(i, L) + 1;  // i < NL <= 128
            const int recip = o_recip[i];
            if (recip != c_owner[c]) atomicOr(&s_flags, MS_FLAG_GUARD);  // executeAnOffer's check (world.py:266)
            const int nk = s_kind[i], nrem = s_rem[i], nbirth = s_birth[i];
            const int price = o_price[i];
            // dispatchNewJobAndReturnOldOne (world.py:61-76)
            x_kind[c] = c_kind[c];
            x_rem[c] = c_rem[c];
            x_birth[c] = c_birth[c];
            x_off[c] = (int8_t)offerer;
            x_recip[c] = (int8_t)recip;
            c_kind[c] = (int8_t)nk;
            c_rem[c] = (int8_t)nrem;
            c_birth[c] = nbirth;
            c_owner[c] = (int8_t)offerer;
            // liability entry (deepcopy, round = world.round), appendleft (world.py:285-289)
            const int n = l_n[c];
            if (n < P.cap) {
                Liab le;
                le.offerer = (int8_t)offerer;
                le.recipient = (int8_t)recip;
                le.price = (int8_t)price;
                le.nec = (int8_t)nrem;
                le.round = round;
                if (active) my_liab[c * P.cap + n] = le;
                s_newle[c] = le;
                s_fresh[c] = 1;
                l_n[c] = (uint8_t)(n + 1);
            } else {
                atomicOr(&s_flags, MS_FLAG_LIABILITY_OVERFLOW);
            }
            // offer-side rewards from world.acceptedOffers (Reward.py:164-170 / :23-49)
            const int prio1 = R.prio(nk);
            off_r[i] = (float)prio1;
            if (P.free_prices) {
                const int diff = prio1 - price;
                price_r[i] = P.commercial ? (diff == 0 ? P.net_zero : (float)diff) : (diff >= 0 ? (float)prio1 : (float)diff);
            }
        }
        wave_sync();
        // per collection (agent a = lane): removeAndReturnEntry of its executed offers (world.py:135-141,
        // newJob.wait = False world.py:276) and insertJob of the jobs dispatched to it, in rank order
        if (gl < N) {
            const int a1 = gl + 1, base = gl * L, n_exec = s_n_exec;
            for (int r = 0; r < n_exec; r++) {
                const int c = s_by_rank[r];
                if (x_off[c] == a1) {
                    const int i = s_exec[c];
                    s_kind[i] = -1;
                    s_rem[i] = -1;
                    s_wait[i] = 0;
                    s_birth[i] = -1;
                }
                if (x_recip[c] == a1) {
                    int placed = 0;
                    for (int q = 0; q < L; q++)
                        if (s_kind[base + q] < 0) {
                            s_kind[base + q] = x_kind[c];
                            s_rem[base + q] = x_rem[c];
                            s_wait[base + q] = 0;
                            s_birth[base + q] = x_birth[c];
                            placed = 1;
                            break;
                        }
                    if (!placed) atomicOr(&s_flags, MS_FLAG_COLLECTION_FULL);
                }
            }
        }
    } else if (gl == 0) {
        const int n_exec = s_n_exec;
        double q_sum = 0.0;  // calculateAverageAcceptionQuality (SchedulingEnvironment.py:174-192)
        int n_q = 0;
        for (int r = 0; r < n_exec; r++) {
            const int c = s_by_rank[r];
            const int i = s_exec[c];
            const int offerer = small_div(i, L) + 1, slot = i - (offerer - 1) * L;  // i < NL <= 128
            const int recip = o_recip[i];
            if (recip != c_owner[c]) s_flags |= MS_FLAG_GUARD;  // executeAnOffer's ownership check (world.py:266)
            const int nk = s_kind[i], nrem = s_rem[i], nbirth = s_birth[i];
            const int price = o_price[i];
            // removeAndReturnEntry (world.py:135-141); newJob.wait = False (world.py:276)
            s_kind[i] = -1;
            s_rem[i] = -1;
            s_wait[i] = 0;
            s_birth[i] = -1;
            // dispatchNewJobAndReturnOldOne (world.py:61-76)
            const int ok = c_kind[c], orem = c_rem[c], obirth = c_birth[c];
            c_kind[c] = (int8_t)nk;
            c_rem[c] = (int8_t)nrem;
            c_birth[c] = nbirth;
            c_owner[c] = (int8_t)offerer;
            if (recip != 0) {  // insertJob into the recipient's first empty slot (world.py:123-133)
                const int base = (recip - 1) * L;
                int placed = 0;
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
            const int n = l_n[c];
            if (n < P.cap) {
                Liab le;
                le.offerer = (int8_t)offerer;
                le.recipient = (int8_t)recip;
                le.price = (int8_t)price;
                le.nec = (int8_t)nrem;
                le.round = round;
                if (active) my_liab[c * P.cap + n] = le;
                s_newle[c] = le;
                s_fresh[c] = 1;
                l_n[c] = (uint8_t)(n + 1);
            } else {
                s_flags |= MS_FLAG_LIABILITY_OVERFLOW;
            }
            // offer-side rewards from world.acceptedOffers (Reward.py:164-170 / :23-49)
            const int prio1 = R.prio(nk);
            if (!P.free_prices) {
                off_r[i] = (float)prio1;
            } else {
                const int diff = prio1 - price;
                float pc;
                if (P.commercial)
                    pc = diff == 0 ? P.net_zero : (float)diff;
                else
                    pc = diff >= 0 ? (float)prio1 : (float)diff;
                off_r[i] = (float)prio1;
                price_r[i] = pc;
            }
            if (MX && mx) {
                m_add(&mx->price_sum[nk], price);  // prices.append((offeredReward, jobKind)) trainPPO.py:172-174
                m_add(&mx->price_count[nk], 1);
                if (recip != 0) {  // formerCore* = the core's job before this round's execution
                    const double former = ok >= 0 ? (double)R.prio(ok) / (double)orem : 0.0;
                    q_sum += ((double)price / (double)nrem - former) * 10.0;
                    n_q++;
                }
            }
            if (io.ev_acc && active) {
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
        if (MX && mx && n_q > 0) {  // statistics.mean of the round's qualities, then collected per round
            m_add(&mx->quality_sum, q_sum / n_q);
            m_add(&mx->quality_rounds, 1);
            m_add(&mx->acception_amount, n_q);
        }
    }
    wave_sync();
    MS_MARK(5);

    // ---- tick (processOneTimestepAndUpdateOwnership world.py:336-367) and liability settlement
    //      (getDividedFixedPricesReward Reward.py:187-210 / getDividedFreePricesReward Reward.py:59-82)
    if (gl < C) {
        const int c = gl;
        ms_term_rec tr = {0, 0, 0, 0, 0};
        if (c_kind[c] >= 0) {
            const int rem = c_rem[c] - 1;
            c_rem[c] = (int8_t)rem;
            if (rem == 0) {
                const int owner = c_owner[c];
                const int kind = c_kind[c];
                const int gen = P.mult * R.prio(kind);
                const int ts = round + 1;
                tr.valid = 1;
                tr.owner = (int8_t)owner;
                tr.prio = (int8_t)R.prio(kind);
                tr.init_len = (int8_t)R.len(kind);
                tr.dwell = round - c_birth[c];
                if (MX && mx) {  // verweilzeiten (world.py:350-357); env.terminationRevenues (Reward.py:193)
                    m_add(&mx->dwell_sum[kind], tr.dwell - 1);
                    m_add(&mx->dwell_count[kind], 1);
                    if (!P.free_prices) m_add(&mx->termination_revenue, (long long)gen);
                }
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
                    const double ratio = (double)le.price / (double)le.nec;  // Python true division
                    const int traded = (int)rint(ratio * (double)tm);        // Python round(): half-even
                    acc_r[(le.offerer - 1) * C + c] -= traded;
                    atomicAdd(&s_agent_r[le.offerer - 1], -traded);
                    if (le.recipient > 0) {
                        atomicAdd(&s_agent_r[le.recipient - 1], traded);
                        acc_r[(le.recipient - 1) * C + c] += traded;
                        if (io.rew_agg_acc) atomicAdd(&s_credit[le.recipient - 1], traded);
                    } else {
                        s_auct_r[c] = traded;
                    }
                }
                l_n[c] = 0;  // resetLiabilityListForACore
            }
        }
        if (active) {
            if (io.ev_term) io.ev_term[e * C + c] = tr;
            if (io.ev_acc && s_exec[c] < 0) {
                ms_accept_rec ar = {};
                io.ev_acc[e * C + c] = ar;
            }
        }
    }
    wave_sync();
    MS_MARK(6);

    // ---- ownership is final for the round: stream every acceptor chunk with no owner-row dword
    //      now (the stores drain while the offers, spawn, outputs and owner rows are computed)
    // ---- offers from offer actions (createFixPriceOfferObjectsFromActions world.py:406-443,
    //      createFreePriceOfferObjectsFromActions world.py:445-478); IDs = slot order
    for (int i = gl; i < NL; i += LPE) {
        const int act = a_off[i];
        const int cidx = (act >= 0 && act < C) ? act : -1;
        const int kind = s_kind[i];
        int price;
        if (P.free_prices)
            price = a_price[i];
        else
            price = R.fix(kind >= 0 ? kind : P.n_fix - 1);
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
    MS_MARK(7);

    // ---- spawn (fillQueuesWithNewRandomJobs world.py:369-376, fillCollectionRandomly Agent.py:50-70)
    {
        const int k = P.new_jobs;
        bool sp = false;
        if (gl < N) {
            int owned = 0, free_slots = 0;
            for (int c = 0; c < C; c++) owned += (c_owner[c] == gl + 1);
            for (int s = 0; s < L; s++) free_slots += (s_kind[gl * L + s] < 0);
            sp = owned + k <= free_slots;
        }
        const uint64_t spm = Lg.ballot(sp);
        const int total_pairs = __popcll(spm) * k;
        int done = 0;
        while (done < total_pairs) {
            if (rs.wend - rs.p < 2) rs.load(rs.p, 2, Lg);
            const int avail = (rs.wend - rs.p) / 2;
            const int cnt = min(avail, total_pairs - done);
            const int off0 = rs.p - rs.wb;
            const uint32_t tv = rs.word();
            const uint32_t wa = Lg.shfl(tv, (off0 + 2 * gl) & (LPE - 1));
            const uint32_t wb2 = Lg.shfl(tv, (off0 + 2 * gl + 1) & (LPE - 1));
            if (gl < cnt) {
                // random(): (a>>5 * 2^26 + b>>6) / 2^53 (Modules/_randommodule.c)
                const double u = ((double)(wa >> 5) * 67108864.0 + (double)(wb2 >> 6)) * (1.0 / 9007199254740992.0);
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
                spawn_kind[done + gl] = (int8_t)kind;
            }
            rs.p += 2 * cnt;
            done += cnt;
        }
        wave_sync();
        if (sp) {
            const int rank = __popcll(spm & ((1ull << gl) - 1ull));
            const int base = gl * L;
            for (int j = 0; j < k; j++) {
                const int kind = spawn_kind[rank * k + j];
                int placed = 0;
                for (int s = 0; s < L; s++)
                    if (s_kind[base + s] < 0) {
                        s_kind[base + s] = (int8_t)kind;
                        s_rem[base + s] = (int8_t)R.len(kind);
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
    MS_MARK(8);
    if (gl == 0) {
        if (rs.overrun) s_flags |= MS_FLAG_RNG_WINDOW;
        R.round() = round + 1;
        mt_commit(rs.end_index(), &R.mti(), &R.mt_sel());
        R.flags() |= s_flags;
        // the host sees a fatal flag at its next ms_env_step without synchronising (plain store to
        // host-coherent memory; any nonzero value will do, so racing groups need no atomic)
        if ((s_flags & MS_FATAL_FLAGS) && io.err_word && active) *io.err_word = 1u;
    }
    wave_sync();
    MS_MARK(9);

    // ---- outputs: state record, rewards, observations of the new offer set
    if (active) {
        copy_out<LPE>(WtOut(recs, E * g.rec_bytes), e * g.rec_bytes, reinterpret_cast<uint32_t*>(recs + e * (int64_t)g.rec_bytes),
                      reinterpret_cast<const uint32_t*>(rec), g.rec_bytes / 4, gl);
        // rewards: write-through (consumed by the update, rounds later)
        auto rew = [&](void* base, int per_env, const void* src) {
            if (!base) return;
            copy_out<LPE>(WtOut(base, E * per_env * 4), e * per_env * 4, reinterpret_cast<uint32_t*>(base) + e * per_env,
                          reinterpret_cast<const uint32_t*>(src), per_env, gl);
        };
        if (MX && mx) {  // the driver's reward accumulators (trainPPO.py:176-183)
            if (gl < N) {
                int ar = 0, orw = 0;
                float pr = 0.f;
                for (int c = 0; c < C; c++) ar += acc_r[gl * C + c];
                for (int j = 0; j < L; j++) {
                    orw += (int)off_r[gl * L + j];
                    pr += price_r[gl * L + j];
                }
                m_add(&mx->agent_reward[gl], (long long)s_agent_r[gl]);
                m_add(&mx->acceptor_reward, (long long)ar);
                m_add(&mx->offer_reward, (long long)orw);
                if (P.free_prices) m_add(&mx->price_reward, (double)pr);
            }
            if (gl < C) m_add(&mx->auctioneer_reward, (long long)s_auct_r[gl]);
            if (gl == 0) m_add(&mx->rounds, 1);
        }
        rew(io.rew_acc, N * C, acc_r);
        rew(io.rew_offer, NL, off_r);
        rew(io.rew_price, NL, price_r);
        rew(io.rew_agent, N, s_agent_r);
        rew(io.rew_auct, C, s_auct_r);
        // getAggregatedFixedPricesReward (Reward.py:92-143): offer = sum of the agent's slot rewards
        // (prio1 of its accepted offers); acceptor = its divided acceptor rewards without the chain
        // credits it received as a recipient
        if (io.rew_agg_off || io.rew_agg_acc) {
            for (int a = gl; a < N; a += LPE) {
                if (io.rew_agg_off) {
                    int v = 0;
                    for (int j = 0; j < L; j++) v += (int)off_r[a * L + j];
                    io.rew_agg_off[e * N + a] = v;
                }
                if (io.rew_agg_acc) {
                    int v = -s_credit[a];
                    for (int c = 0; c < C; c++) v += acc_r[a * C + c];
                    io.rew_agg_acc[e * N + a] = v;
                }
            }
        }
    }
    MS_MARK(10);
    build_masks<LPE>(R, g, s_mc, s_mr, gl);
    MS_MARK(11);
    emit_obs<LPE>(R, g, s_mc, s_mr, scratch, CMP ? nullptr : io.obs_acc, io.obs_off, io.obs_auct,
                  (EXT || CMP) ? io.obs_crow : nullptr, (EXT || CMP) ? io.obs_cown : nullptr, e, E, active, gl);
    MS_MARK(12);
#ifdef MS_PHASE_TIMING
    if (lane == 0)
        for (int k = 0; k < 16; k++) g_phase_cycles[blockIdx.x % kProbeSlots][k] += t_acc[k];
#endif
}

// ---- the next round's acting of the wave's envs (ms_env_step_act): ActorCritic.act of the offer units and
//      the compact acceptors (PPOmodules.py:53-63, SchedulingEnvironment.py:150-172) on the observations the
//      round just built in its LDS, with the arithmetic and the Philox draws of k_act / k_act_common
//      (ms_act.h), so the outputs equal ms_act_round_free(offer net, NULL, ...) on the emitted rows. One
//      offer net and one acceptor net (n_groups 1), each one 32-input k-step and <= 16 actions
//      (env_step_act_supported); item i of a net is row i (e * units + u), its uniform word (i >> 6) & 1 of
//      the draw countered by row (i & ~64) + row_base, as in k_act_common's scan.
template <int LPE, class SH>
__device__ __forceinline__ void fused_act(const Params& P, int64_t E, const FusedAct& fa, int64_t slot,
                                          int lane_arg = -1) {
    constexpr int EPW = kWave / LPE;  // envs per wave
    extern __shared__ __align__(16) uint8_t smem_all[];
    __shared__ float s_cum[16], s_lp[16];
    __shared__ uint32_t s_tab[2];  // the common row's S (f32 bits) and last nonzero action
    __shared__ uint32_t s_tmpl[8];
    Geom g;
    if constexpr (SH::kStatic) {
        constexpr Geom kg = make_geom(SH::kN, SH::kC, SH::kL, SH::kJ);
        g = kg;
    } else {
        g = P;
    }
    const int lane = lane_arg >= 0 ? lane_arg : (int)threadIdx.x, j = lane & 15, g4 = lane >> 4;
    const int C = g.C, Ua = g.N * C, Uo = g.NL;
    const int64_t e0 = slot * EPW;
    const uint64_t dev_off = fa.offset_dev ? *fa.offset_dev : 0ull;
    // weights: the act fragment blocks (ms_act_prepare), else derived from the f32 weights (bit-identical)
    W1Split<1> wo, wa;
    Head<1> ho, ha;
    using FL = FragLayout<1, 1>;
    const uint32_t* fo = frag_groups<1, 1>(fa.off, false);
    const uint32_t* fc = frag_groups<1, 1>(fa.acc, true);
    if (fo) {
        wo.load_frag(fo + lane * FL::LW);
        ho.load_frag(reinterpret_cast<const float*>(fo + lane * FL::LW + 12));
    } else {
        wo.load(fa.off.w1, fa.off.in_dim, j, g4);
        ho.load(fa.off, 0, j, g4);
    }
    if (fc) {
        wa.load_frag(fc + lane * FL::LW);
        ha.load_frag(reinterpret_cast<const float*>(fc + lane * FL::LW + 12));
        if (lane < 34) {
            const uint32_t v = fc[64 * FL::LW + lane];  // [16 running sums][16 log-probs][S][last nonzero]
            if (lane < 16)
                s_cum[lane] = __uint_as_float(v);
            else if (lane < 32)
                s_lp[lane - 16] = __uint_as_float(v);
            else
                s_tab[lane - 32] = v;
        }
    } else {
        wa.load(fa.acc.w1, fa.acc.in_dim, j, g4);
        ha.load(fa.acc, 0, j, g4);
        float S0;
        int lnz0;
        common_table<1, 1>(wa, ha, fa.common, g.acc_stride >> 2, s_tmpl, s_cum, s_lp, &S0, &lnz0, lane);
        if (lane == 0) {
            s_tab[0] = __float_as_uint(S0);
            s_tab[1] = (uint32_t)lnz0;
        }
    }
    wave_sync();  // the table, and the round's observation sources in every group's LDS slice
    const int Aa = fa.acc.n_actions, Ao = fa.off.n_actions;
    const int nw = g.acc_stride >> 2, nwo = g.off_stride >> 2;
    auto philox_u = [&](int64_t item, int64_t row_base, uint64_t off) {  // item i's uniform (k_act_common's rule)
        uint32_t r0, r1;
        philox2((uint32_t)(item & ~64ll) + (uint32_t)row_base, off + dev_off, fa.seed, r0, r1);
        return u24((item & 64) ? r1 : r0);
    };
    // ---- the MFMA rows, all issued before either head runs (the three tiles' chains are independent):
    //      offers: every slot's row (template + pair), 16-row tiles; acceptors: the row of each owned core,
    //      which is the owner's acceptor row (item (owner - 1) * C + c); every other acceptor row is the
    //      common row (sampled from its table below). EPW * C <= 16: one tile.
    const int pcol = (2 * C) >> 2, pshift = 8 * ((2 * C) & 3);
    auto offer_rows = [&](int t0, f4* acc, int* row, float* u2) {
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int r = t0 + 16 * i + j;
            const int ge = r / Uo, s = r - ge * Uo;
            const int64_t e = e0 + ge;
            const bool v = r < EPW * Uo && e < E;
            const uint8_t* sc = smem_all + (size_t)(v ? ge : 0) * g.s_total + g.s_scratch;
            const uint32_t* otmpl = reinterpret_cast<const uint32_t*>(sc + g.s_otmpl);
            const uint16_t pair = reinterpret_cast<const uint16_t*>(sc + g.s_slotpair)[v ? s : 0];
            uint32_t d[2];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int cc = 2 * g4 + h, wd = cc < nwo ? cc : nwo - 1;
                d[h] = otmpl[wd] | (wd == pcol ? (uint32_t)pair << pshift : 0u);
            }
            const u4v x = bytes_to_bf16(d[0], d[1]);
            acc[i] = (f4){0, 0, 0, 0};
            acc[i] = mfma_bf16(wo.hi[0], x, acc[i]);
            acc[i] = mfma_bf16(wo.mid[0], x, acc[i]);
            acc[i] = mfma_bf16(wo.lo[0], x, acc[i]);
            const int64_t item = e * Uo + s;
            u2[i] = philox_u(item, fa.off.row_base, fa.off_offset);
            row[i] = v ? (int)item : -1;
        }
    };
    auto store = [&](int8_t* act_out, float* lp_out, const int* row, const int* act, const float* lp) {
#pragma unroll
        for (int i = 0; i < 2; i++)
            if (g4 == 0 && row[i] >= 0) {
                act_out[row[i]] = (int8_t)act[i];
                lp_out[row[i]] = lp[i];
            }
    };
    f4 acc_o[2], acc_a[2];
    int row_o[2], row_a[2], act_o[2], act_a[2];
    float u_o[2], u_a[2], lp_o[2], lp_a[2];
    offer_rows(0, acc_o, row_o, u_o);
    {
        const int ge = j / C, c = j - ge * C;
        const int64_t e = e0 + ge;
        const uint8_t* sl = smem_all + (size_t)(ge < EPW ? ge : 0) * g.s_total;
        const int owner = (int)reinterpret_cast<const int8_t*>(sl + g.s_rec + g.o_core_owner)[c];
        const bool v = ge < EPW && e < E && owner > 0;
        const uint32_t* crow = reinterpret_cast<const uint32_t*>(sl + g.s_scratch) + c * nw;
        const int c0 = 2 * g4, c1 = 2 * g4 + 1;
        const u4v x = bytes_to_bf16(crow[c0 < nw ? c0 : nw - 1], crow[c1 < nw ? c1 : nw - 1]);
        acc_a[0] = (f4){0, 0, 0, 0};
        acc_a[0] = mfma_bf16(wa.hi[0], x, acc_a[0]);
        acc_a[0] = mfma_bf16(wa.mid[0], x, acc_a[0]);
        acc_a[0] = mfma_bf16(wa.lo[0], x, acc_a[0]);
        acc_a[1] = acc_a[0];  // (an empty partner tile: no row of it is written)
        const int64_t item = e * Ua + (owner - 1) * C + c;
        u_a[0] = philox_u(item, fa.acc.row_base, fa.acc_offset);
        u_a[1] = 0.f;
        row_a[0] = v ? (int)item : -1;
        row_a[1] = -1;
    }
    ho.run2(acc_o, Ao, g4, u_o, act_o, lp_o);
    ha.run2(acc_a, Aa, g4, u_a, act_a, lp_a);
    store(fa.off_action, fa.off_logprob, row_o, act_o, lp_o);
    store(fa.acc_action, fa.acc_logprob, row_a, act_a, lp_a);
    for (int t0 = 32; t0 < EPW * Uo; t0 += 32) {  // (LPE 16: four replicas' offers)
        offer_rows(t0, acc_o, row_o, u_o);
        ho.run2(acc_o, Ao, g4, u_o, act_o, lp_o);
        store(fa.off_action, fa.off_logprob, row_o, act_o, lp_o);
    }
    // ---- acceptors whose row is the common row (a core the agent does not own): one lane per item, sampled
    //      from the common row's table (k_act_common's scan)
    const float S = __uint_as_float(s_tab[0]);
    const int last_nz = (int)s_tab[1];
    {
        const int ge = lane / Ua, u = lane - ge * Ua, a = u / C, c = u - a * C;
        const int64_t e = e0 + ge;
        const uint8_t* sl = smem_all + (size_t)(ge < EPW ? ge : 0) * g.s_total;
        const bool in = lane < EPW * Ua && e < E;
        const int owner = (int)reinterpret_cast<const int8_t*>(sl + g.s_rec + g.o_core_owner)[c];
        if (in && owner != a + 1) {
            const int64_t item = e * Ua + u;
            const float target = philox_u(item, fa.acc.row_base, fa.acc_offset) * S;
            int cnt = 0;
#pragma unroll
            for (int step = 16; step >= 1; step >>= 1)
                if (cnt + step <= 16 && s_cum[cnt + step - 1] <= target) cnt += step;
            const int act = cnt >= Aa ? last_nz : cnt;
            fa.acc_action[item] = (int8_t)act;
            fa.acc_logprob[item] = s_lp[act];
        }
    }
}

// One round for the 64 / LPE envs of wave slot blockIdx.x. (A persistent loop over several slots
// per wave would let one slot's observation stores drain under the next slot's compute, but the
// compiler then keeps the whole round's state live across iterations: 3x the VGPRs.)
template <int LPE, bool EXT, bool CMP, class SH>
__global__ void __launch_bounds__(64, 4) k_env_step(Params P, int64_t E, uint8_t* recs, uint32_t* mt, Liab* liab,
                                                 StepIO io) {
#ifdef MS_PHASE_TIMING
    const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();
#endif
    // per-wave start / end for the bench's launch span (optional; plain stores, no shared address,
    // nothing held across the round: the kernel sits at 4 waves per SIMD with no register to spare)
    // (with the shader clock beside the 100 MHz one: the launch's effective clock, which differs box to box)
    if (io.span && threadIdx.x == 0) {
        io.span[4 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
        io.span[4 * blockIdx.x + 2] = __builtin_amdgcn_s_memtime();
    }
    env_round<LPE, EXT, CMP, SH>(P, E, recs, mt, liab, io, blockIdx.x);
    if (io.span && threadIdx.x == 0) {
        io.span[4 * blockIdx.x + 3] = __builtin_amdgcn_s_memtime();
        io.span[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
#ifdef MS_PHASE_TIMING
    if (threadIdx.x == 0) {
        g_wave_span[blockIdx.x % kProbeSlots][0] = rt_start;
        g_wave_span[blockIdx.x % kProbeSlots][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

// the round of k_env_step (compact acceptor observations) and then the next round's acting (fused_act)
template <int LPE, class SH>
__global__ void __launch_bounds__(64, 4) k_env_step_act(Params P, int64_t E, uint8_t* recs, uint32_t* mt, Liab* liab,
                                                     StepIO io, FusedAct fa) {
    if (io.span && threadIdx.x == 0) {
        io.span[4 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
        io.span[4 * blockIdx.x + 2] = __builtin_amdgcn_s_memtime();
    }
    env_round<LPE, false, true, SH>(P, E, recs, mt, liab, io, blockIdx.x);
    fused_act<LPE, SH>(P, E, fa, blockIdx.x);
    if (io.span && threadIdx.x == 0) {
        io.span[4 * blockIdx.x + 3] = __builtin_amdgcn_s_memtime();
        io.span[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

template <class T>
__device__ __forceinline__ T* advance(T* p, int64_t bytes) {
    return p ? reinterpret_cast<T*>(reinterpret_cast<uintptr_t>(p) + bytes) : p;
}
// n_rounds rounds of k_env_step_act in one launch: each wave steps its replicas, then samples their next
// actions, round after round; round t's arrays are the given ones advanced by t strides. A round reads what
// the wave's lanes wrote in the round before (records, MT blocks, liabilities, actions): a workgroup-scope
// fence (the wave is its workgroup) orders those writes before the next round's loads.
// Every round re-reads its arguments from the kernel-argument segment through a pointer the compiler cannot
// see through, and takes the lane index the same way: otherwise the loop-invariant argument loads and
// lane arithmetic are hoisted out of the round loop and held across it (hundreds of spilled registers).
struct RolloutArgs {
    Params P;
    int64_t E;
    uint8_t* recs;
    uint32_t* mt;
    Liab* liab;
    StepIO io;
    FusedAct fa;
    RoundStride st;
    int n_rounds, act_last;
};
template <int LPE, class SH>
__global__ void __launch_bounds__(64, 2) k_env_rollout_act(RolloutArgs A0) {
    unsigned long long* span = A0.io.span;
    if (span && threadIdx.x == 0) {
        span[4 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
        span[4 * blockIdx.x + 2] = __builtin_amdgcn_s_memtime();
    }
    const int n_rounds = A0.n_rounds;
    for (int t = 0; t < n_rounds; t++) {
        auto ka = __builtin_amdgcn_kernarg_segment_ptr();  // (constant address space)
        asm volatile("" : "+s"(ka));
        const RolloutArgs& A = *(const RolloutArgs*)ka;
        int lane = threadIdx.x;
        asm volatile("" : "+v"(lane));
        const RoundStride& st = A.st;
        StepIO io = A.io;
        io.span = nullptr;
        io.act_acc = advance(io.act_acc, t * st.act_acc);
        io.act_off = advance(io.act_off, t * st.act_off);
        io.obs_crow = advance(io.obs_crow, t * st.obs_crow);
        io.obs_cown = advance(io.obs_cown, t * st.obs_cown);
        io.obs_off = advance(io.obs_off, t * st.obs_off);
        io.rew_offer = advance(io.rew_offer, t * st.rew_offer);
        io.rew_acc = advance(io.rew_acc, t * st.rew_acc);
        io.rew_agent = advance(io.rew_agent, t * st.rew_agent);
        io.rew_auct = advance(io.rew_auct, t * st.rew_auct);
        env_round<LPE, false, true, SH>(A.P, A.E, A.recs, A.mt, A.liab, io, blockIdx.x, lane);
        if (t + 1 < n_rounds || A.act_last) {
            FusedAct fa = A.fa;
            fa.off_action = advance(fa.off_action, t * st.off_action);
            fa.off_logprob = advance(fa.off_logprob, t * st.off_logprob);
            fa.acc_action = advance(fa.acc_action, t * st.acc_action);
            fa.acc_logprob = advance(fa.acc_logprob, t * st.acc_logprob);
            fa.off_offset += (uint64_t)t * st.offset_step;
            fa.acc_offset += (uint64_t)t * st.offset_step;
            fused_act<LPE, SH>(A.P, A.E, fa, blockIdx.x, lane);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        wave_sync();
    }
    if (span && threadIdx.x == 0) {
        span[4 * blockIdx.x + 3] = __builtin_amdgcn_s_memtime();
        span[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

// ---- locally shared free-price rollouts (BASELINE cfg3; ms_env_rollout_act_free): the next round's
//      getActionForAllAgents (SchedulingEnvironment.py:150-172) of a workgroup's replicas, one wave per agent,
//      from the observations the workgroup's env round just built in its LDS: the agent's offer units
//      (FreePriceOfferPPO.selectAction PPOmodules.py:312-332: core chooser, then the price chooser on
//      [obs[2a:2a+2], obs[-2:]] or the dummy [-5] * 4) and its acceptors (LocallySharedPPO.selectAction
//      PPOmodules.py:532-543, Agent.py:682-699) on the compact acceptor rows. The arithmetic and the Philox draws
//      are k_act_pair's (act_tiles' core + price choosers with the price table, act_common_rows' compact
//      acceptors), so the outputs equal ms_act_round_free's on the emitted observations bit for bit:
//      a row's MFMA column, its four lanes' reductions and its draw depend on the row alone, not on the rows
//      that share its tile.
constexpr int kPriceTW1 = 36;  // floats per price-table entry of <= 16 actions (policy_kernels.hip PriceTW<1>)

__device__ __forceinline__ uint32_t pick4u(const uint32_t (&v)[4], int k) {
    return k == 0 ? v[0] : (k == 1 ? v[1] : (k == 2 ? v[2] : v[3]));
}

// The acceptors of cores the agent does not own are left to k_acc_common_fill (after the launch, or later on
// another stream): the env reads only the owner's acceptor action (world.py:391-404), so their sampling is off the
// round's chain. (Sampling them here as well, k_act_common's table search per item: 50.2 us per round against
// 47.4, profiles/r7g.)
template <class SH, int PART = 3>  // PART bit 0: the offer units, bit 1: the acceptors (the probe build times them apart)
__device__ __forceinline__ void act_free(const Geom& g, int64_t E, const FusedActFree& fa, int64_t e0, int a, int lane,
                                         uint8_t* lds, const FreeLds& fl, bool pace_on = false) {
    const int j = lane & 15, g4 = lane >> 4;
    // pace_on: waves a and a ^ 4 share a SIMD, where issue goes to the older wave first, so one of them finishes
    // its acting well before the other and waits at the round's barrier. After each step (a tile pair, a 64-item
    // scan) a wave counts it in the LDS and raises its issue priority while it is behind its partner.
    const int partner = a ^ 4;
    const bool pacing = pace_on && partner < g.N;
    auto pace = [&]() {
        if (!pacing) return;
        volatile int* pg = reinterpret_cast<volatile int*>(lds + fl.pace);
        const int mine = pg[a] + 1;
        pg[a] = mine;
        const int other = __builtin_amdgcn_readfirstlane(pg[partner]);
        if (other > __builtin_amdgcn_readfirstlane(mine))
            __builtin_amdgcn_s_setprio(1);
        else
            __builtin_amdgcn_s_setprio(0);
    };
    const int N = g.N, C = g.C, L = g.L, Uo = g.NL, Ua = N * C;
    const int EW = kFreeEPW * N;  // the workgroup's replicas
    const uint64_t dev_off = fa.offset_dev ? *fa.offset_dev : 0ull;
    const int16_t* pdig = reinterpret_cast<const int16_t*>(lds + fl.pdig);
    auto slice = [&](int k) -> const uint8_t* { return lds + k * g.s_total; };

    // ---------------- the offer units: agent a's L slots of every replica, rows r = k * L + s
    if constexpr ((PART & 1) != 0) {
        using FL = FragLayout<1, 1>;
        constexpr int TW = kPriceTW1;
        W1Split<1> w1;
        Head<1> h1;
        if (const uint32_t* fg = frag_groups<1, 1>(fa.core, false)) {
            const uint32_t* lf = fg + (size_t)a * FL::GB + lane * FL::LW;
            w1.load_frag(lf);
            h1.load_frag(reinterpret_cast<const float*>(lf + 12));
        } else {
            w1.load(fa.core.w1 + (size_t)a * 16 * fa.core.in_dim, fa.core.in_dim, j, g4);
            h1.load(fa.core, a, j, g4);
        }
        const int n_rows = EW * L, tiles = (n_rows + 15) >> 4;
        const uint64_t off = fa.off_offset + dev_off;
        const uint32_t rbase = (uint32_t)fa.core.row_base;
        const long long rows_all = E * Uo;
        const RawBuf ca_b(fa.core_action, rows_all), cl_b(fa.core_logprob, 4 * rows_all),
            ps_b(fa.price_state, 4 * rows_all), pa_b(fa.price_action, rows_all), pl_b(fa.price_logprob, 4 * rows_all),
            ep_b(fa.env_price, rows_all);
        const RawBuf tab_b(fa.ptab + (size_t)a * fa.pkeys * TW, 4ll * fa.pkeys * TW);
        const int nwo = g.off_stride >> 2, pcol = (2 * C) >> 2, pshift = 8 * ((2 * C) & 3);
        const int A1 = fa.core.n_actions, A2 = fa.price.n_actions;
        // the call row (e * N*L + a*L + s) of the agent's row r, -1 past the replicas; k, s: its replica in
        // the workgroup and its slot (0 for rows past the end: their LDS reads stay in range)
        auto row_of = [&](int r, int& k, int& s) -> int {
            k = r / L;
            s = r - k * L;
            const bool v = r < n_rows && e0 + k < E;
            const int row = (int)((e0 + k) * Uo) + a * L + s;
            if (r >= n_rows) k = s = 0;
            return v ? row : -1;
        };
        uint32_t rb0[4] = {0, 0, 0, 0}, rb1[4] = {0, 0, 0, 0};
        // one tile pair up to the price chooser's input: the rows' core choices, the price inputs and their
        // key digits (act_tiles: core2 + price_in2)
        auto core_pair = [&](int tile, int (&cur)[2], int (&act)[2], float (&lp)[2], float (&u2)[2], int (&pin)[2],
                             int (&dg)[2]) {
            if ((tile & 3) == 0) {  // Philox for 4 tiles: lane (j, g4) draws row j of tile tile + g4
                int k, s;
                const int r = row_of(16 * (tile + g4) + j, k, s);
                uint32_t r0, r1;
                philox2((uint32_t)r + rbase, off, fa.seed, r0, r1);
                rows_bcast(r1, rb1);
                rows_bcast(r0, rb0);
            }
            const int kq = tile & 3;
            int kk[2], ss[2];
            f4 acc[2];
            float u1[2];
#pragma unroll
            for (int i = 0; i < 2; i++) {
                cur[i] = row_of(16 * (tile + i) + j, kk[i], ss[i]);
                const uint8_t* sc = slice(kk[i]) + g.s_scratch;
                const uint32_t* otmpl = reinterpret_cast<const uint32_t*>(sc + g.s_otmpl);
                const uint32_t pr = reinterpret_cast<const uint16_t*>(sc + g.s_slotpair)[a * L + ss[i]];
                uint32_t d[2];
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int cc = 2 * g4 + h, wd = cc < nwo ? cc : nwo - 1;
                    d[h] = otmpl[wd] | (wd == pcol ? pr << pshift : 0u);
                }
                const u4v x = bytes_to_bf16(d[0], d[1]);
                acc[i] = (f4){0, 0, 0, 0};
                acc[i] = mfma_bf16(w1.hi[0], x, acc[i]);
                acc[i] = mfma_bf16(w1.mid[0], x, acc[i]);
                acc[i] = mfma_bf16(w1.lo[0], x, acc[i]);
                u1[i] = u24(pick4u(rb0, kq + i));
                u2[i] = u24(pick4u(rb1, kq + i));
            }
            h1.run2(acc, A1, g4, u1, act, lp);
#pragma unroll
            for (int i = 0; i < 2; i++) {
                // byte kb of the row: the chosen core's (prio, rem) for g4 < 2, the slot's pair obs[-2:] for g4 >= 2
                const int kb = g4 < 2 ? 2 * act[i] + g4 : 2 * C + (g4 - 2);
                const int8_t* sc = reinterpret_cast<const int8_t*>(slice(kk[i]) + g.s_scratch);
                const int byte = kb < 2 * C ? sc[g.s_otmpl + kb] : sc[g.s_slotpair + 2 * (a * L + ss[i]) + (kb - 2 * C)];
                pin[i] = act[i] == 0 ? -5 : byte;
                dg[i] = cur[i] >= 0 ? (int)pdig[g4 * 256 + pin[i] + 128] : 0;
            }
        };
        // the price chooser's outputs of a pair (PPOmodules.py:316-332; env price -5 for core action 0)
        auto price_out = [&](const int (&cur)[2], const int (&act)[2], const int (&pin)[2], const int (&pact)[2],
                             const float (&plp)[2]) {
#pragma unroll
            for (int i = 0; i < 2; i++)
                if (cur[i] >= 0) {
                    const uint32_t pc = (uint32_t)cur[i];
                    ps_b.st8(4 * pc + g4, pin[i]);
                    if (g4 == 0) {
                        pa_b.st8(pc, pact[i]);
                        pl_b.stf(4 * pc, plp[i]);
                        ep_b.st8(pc, act[i] == 0 ? -5 : pact[i]);
                    }
                }
        };
        bool any_miss = false;
        for (int tile = 0; tile < tiles; tile += 2) {
            int cur[2], act[2], pin[2], dg[2];
            float lp[2], u2[2];
            core_pair(tile, cur, act, lp, u2, pin, dg);
            if (__ballot(dg[0] < 0 || dg[1] < 0) == 0ull) {
                // every row of the pair is tabulated: sample from the table (act_tiles' arithmetic)
                rows_sum2_i(dg[0], dg[1]);
                float cum[2][4], S2[2];
                int lnz[2], cnt[2], pact[2];
                float plp[2];
                uint32_t te[2];
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    te[i] = __umul24((uint32_t)dg[i], 4u * TW);
                    const auto c4 = __builtin_amdgcn_raw_buffer_load_b128(tab_b.r, (int)(te[i] + 4 * (4 * g4)), 0, 0);
#pragma unroll
                    for (int q = 0; q < 4; q++) cum[i][q] = __uint_as_float(c4[q]);
                    S2[i] = tab_b.ldf(te[i] + 4 * 32);
                    lnz[i] = (int)tab_b.ld32(te[i] + 4 * 33);
                }
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    const float target = u2[i] * S2[i];
                    cnt[i] = 0;
#pragma unroll
                    for (int q = 0; q < 4; q++) cnt[i] += (cum[i][q] <= target) ? 1 : 0;
                }
                rows_sum2_i(cnt[0], cnt[1]);
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    pact[i] = cnt[i] >= A2 ? lnz[i] : cnt[i];
                    plp[i] = tab_b.ldf(te[i] + 4 * (16 + pact[i]));
                }
                price_out(cur, act, pin, pact, plp);
            } else {
                any_miss = true;
            }
#pragma unroll
            for (int i = 0; i < 2; i++)
                if (cur[i] >= 0 && g4 == 0) {
                    ca_b.st8((uint32_t)cur[i], act[i]);
                    cl_b.stf(4 * (uint32_t)cur[i], lp[i]);
                }
            pace();
        }
        if (any_miss) {
            // the pairs the table could not serve: the same pairs and draws again, the core chooser recomputed
            // (bit-identical), then the price net itself (act_tiles' second loop)
            Head<1> h2;
            h2.load(fa.price, a, j, g4);
            const float pw1 = fa.price.w1[((size_t)a * 16 + j) * 4 + g4];  // W1p[j][g4] (K = 4 inputs)
            for (int tile = 0; tile < tiles; tile += 2) {
                int cur[2], act[2], pin[2], dg[2];
                float lp[2], u2[2];
                core_pair(tile, cur, act, lp, u2, pin, dg);
                if (__ballot(dg[0] < 0 || dg[1] < 0) == 0ull) continue;  // priced from the table above
                int pact[2];
                float plp[2];
                f4 acc2[2];
#pragma unroll
                for (int i = 0; i < 2; i++) acc2[i] = mfma4(pw1, (float)pin[i], (f4){0, 0, 0, 0});
                h2.run2(acc2, A2, g4, u2, pact, plp);
                price_out(cur, act, pin, pact, plp);
            }
        }
    }

    // ---------------- the acceptors: agent a's C items of every replica, item m = k * C + c (group item
    //                  i = e * C + c): the cores it does not own sample the common row's table, the owned ones
    //                  are listed and run in 16-row MFMA tiles (act_common_rows with compact rows)
    if constexpr ((PART & 2) != 0) {
        using FL = FragLayout<2, 2>;
        const uint32_t* const fg = frag_groups<2, 2>(fa.acc, true);
        int16_t* lm = reinterpret_cast<int16_t*>(lds + fl.list + a * kFreeListCap * 6);
        float* lu = reinterpret_cast<float*>(lds + fl.list + a * kFreeListCap * 6 + 2 * kFreeListCap);
        const int nw = g.acc_stride >> 2, Aa = fa.acc.n_actions;
        const int n_items = EW * C;
        const uint64_t off = fa.acc_offset + dev_off;
        const uint32_t rbase = (uint32_t)fa.acc.row_base;
        const long long rows_all = E * Ua;
        const RawBuf aa_b(fa.acc_action, rows_all), al_b(fa.acc_logprob, 4 * rows_all);
        const RawBuf oa_b(fa.own_action, E * C), ol_b(fa.own_logprob, 4 * E * C);
        // the listed rows [0, cnt) (cnt <= 32) as two 16-row tiles (a lone or partial tile: rows past cnt
        // are computed on entry 0 and not written)
        auto tiles2 = [&](int cnt) {
            // the net's fragments only for the tiles (52 registers not held through the scan): loaded per call
            // through a pointer the compiler cannot see through, so the loads are not hoisted out of the scan loop
            W1Split<2> w1;
            Head<2> h1;
            if (fg) {
                const uint32_t* lf = fg + (size_t)a * FL::GB + lane * FL::LW;
                asm volatile("" : "+v"(lf));
                w1.load_frag(lf);
                h1.load_frag(reinterpret_cast<const float*>(lf + 24));
            } else {
                w1.load(fa.acc.w1 + (size_t)a * 16 * fa.acc.in_dim, fa.acc.in_dim, j, g4);
                h1.load(fa.acc, a, j, g4);
            }
            f4 acc[2];
            int row[2], orow[2], lrow[2];
            float uu[2];
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int t = 16 * i + j;
                const bool v = t < cnt;
                const int mm = lm[v ? t : 0];
                uu[i] = lu[v ? t : 0];
                const int kk = mm / C, cc = mm - kk * C;
                row[i] = v ? (int)((e0 + kk) * Ua) + a * C + cc : -1;
                orow[i] = (int)(e0 * C) + mm;  // (e0 + kk) * C + cc
                lrow[i] = fl.accx + kk * Ua + a * C + cc;
                const uint32_t* crow = reinterpret_cast<const uint32_t*>(slice(kk) + g.s_scratch) + cc * nw;
                acc[i] = (f4){0, 0, 0, 0};
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    const int c0 = 8 * s + 2 * g4, c1 = c0 + 1;
                    const u4v x = bytes_to_bf16(crow[c0 < nw ? c0 : nw - 1], crow[c1 < nw ? c1 : nw - 1]);
                    acc[i] = mfma_bf16(w1.hi[s], x, acc[i]);
                    acc[i] = mfma_bf16(w1.mid[s], x, acc[i]);
                    acc[i] = mfma_bf16(w1.lo[s], x, acc[i]);
                }
            }
            int act[2];
            float lp[2];
            h1.run2(acc, Aa, g4, uu, act, lp);
#pragma unroll
            for (int i = 0; i < 2; i++)
                if (row[i] >= 0 && g4 == 0) {
                    if (fa.own_action) {
                        // by core (the fill writes the rings' rows whole), and into the replica's LDS staging of
                        // acceptor actions, where the next env round reads its owners' (StepIO::acc_in_lds)
                        oa_b.st8((uint32_t)orow[i], act[i]);
                        ol_b.stf(4 * (uint32_t)orow[i], lp[i]);
                        reinterpret_cast<int8_t*>(lds)[lrow[i]] = (int8_t)act[i];
                    } else {
                        aa_b.st8((uint32_t)row[i], act[i]);
                        al_b.stf(4 * (uint32_t)row[i], lp[i]);
                    }
                }
        };
        // item i's uniform: word (i >> 6) & 1 of the draw countered by the row of item i & ~64 (k_act_common's
        // rule), so a lane's draw serves its item and the item 64 further when both are in this wave
        const uint32_t i_base = (uint32_t)(e0 * C);
        uint32_t last_ib = 0xffffffffu, wd0 = 0, wd1 = 0;
        const uint64_t below = (1ull << lane) - 1ull;
        int n_list = 0;
        for (int m0 = 0; m0 < n_items; m0 += 64) {
            const int m = m0 + lane;
            const bool in = m < n_items;
            const int k = in ? m / C : 0, c = in ? m - (m / C) * C : 0;
            const bool valid = in && e0 + k < E;
            const uint32_t i = i_base + (uint32_t)m, ib = i & ~64u;
            const int own = reinterpret_cast<const int8_t*>(slice(k) + g.s_rec + g.o_core_owner)[c];
            const bool owned = valid && own == a + 1;
            // (only the owned items' uniforms: the common ones are sampled after the launch)
            const bool need = owned && ib != last_ib;
            if (__ballot(need)) {
                const uint32_t eb = ib / (uint32_t)C;
                uint32_t r0, r1;
                philox2(eb * (uint32_t)Ua + (uint32_t)(a * C) + (ib - eb * (uint32_t)C) + rbase, off, fa.seed, r0, r1);
                if (need) {
                    last_ib = ib;
                    wd0 = r0;
                    wd1 = r1;
                }
            }
            const float u = u24((i & 64u) ? wd1 : wd0);
            const uint64_t mo = __ballot(owned);
            if (owned) {
                const int p = n_list + __popcll(mo & below);
                lm[p] = (int16_t)m;
                lu[p] = u;
            }
            n_list += __popcll(mo);
            pace();
            wave_sync();
            while (n_list >= 32) {
                tiles2(32);
                const int rest = n_list - 32;  // < 64: carried to the front of the list
                int16_t vm = 0;
                float vu = 0.f;
                if (lane < rest) {
                    vm = lm[32 + lane];
                    vu = lu[32 + lane];
                }
                wave_sync();
                if (lane < rest) {
                    lm[lane] = vm;
                    lu[lane] = vu;
                }
                wave_sync();
                n_list = rest;
            }
        }
        if (n_list > 0) tiles2(n_list);
    }
}

// The acceptor items the one-launch rollout leaves (ms_env_rollout_act_free; k_env_rollout_act_free acts with
// act_free<SH, false>): for every acting round t and every (replica e, agent a, core c) whose core a does not own,
// k_act_common's sample from agent a's common-row table (Head::table, ms_act_prepare) with the item's uniform,
// word (i >> 6) & 1 of the draw countered by the row of item i & ~64 (i = e * C + c): the outputs
// ms_act_round_free writes for those items, bit for bit. One thread per item, lanes along the [E][N*C] rows
// (coalesced byte / f32 stores), rounds on blockIdx.y; the N tables in LDS once per block.
struct CommonFillArgs {
    const int8_t* owner;     // round 0's owners [E][C] (the observation the acting of ring slot 1 read)
    int8_t* action;          // round 0's outputs [E][N*C]
    float* logprob;
    int64_t owner_stride, action_stride, logprob_stride;  // bytes per round
    const int8_t* own_action;  // round 0's owned items by core [E][C] (NULL: already in action / logprob)
    const float* own_logprob;
    int64_t own_action_stride, own_logprob_stride;
    const uint32_t* frag;    // the acceptor net's act fragment groups (frag_groups<2, 2>)
    int E, N, C, A;
    uint32_t row_base;
    uint64_t seed, offset, offset_step;
    const uint64_t* offset_dev;
};
constexpr int kFillPer = 8;  // items per thread of k_acc_common_fill: their owner loads in flight together
__global__ void __launch_bounds__(256) k_acc_common_fill(CommonFillArgs p) {
    __shared__ float tabs[8 * kFreeTabDw];
    using FL = FragLayout<2, 2>;
    const int t = blockIdx.y;
    for (int k = threadIdx.x; k < p.N * kFreeTabDw; k += blockDim.x) {
        const int a = k / kFreeTabDw;
        tabs[k] = __uint_as_float(p.frag[(size_t)a * FL::GB + 64 * FL::LW + (k - a * kFreeTabDw)]);
    }
    const int C = p.C, U = p.N * C;
    const int64_t n = (int64_t)p.E * U;
    const uint32_t mag_u = magic_div((uint32_t)U), mag_c = magic_div((uint32_t)C);
    const RawBuf own_b(advance(p.owner, t * p.owner_stride), (int64_t)p.E * C);
    const RawBuf act_b(advance(p.action, t * p.action_stride), n), lp_b(advance(p.logprob, t * p.logprob_stride), 4 * n);
    const uint64_t off = p.offset + (uint64_t)t * p.offset_step + (p.offset_dev ? *p.offset_dev : 0ull);
    // item r = e * U + a * C + c (the [E][N*C] output row): block b takes kFillPer * 256 consecutive items
    const uint32_t r0 = (uint32_t)blockIdx.x * (kFillPer * 256) + threadIdx.x;
    int own[kFillPer];
#pragma unroll
    for (int k = 0; k < kFillPer; k++) {
        const uint32_t r = r0 + 256 * k;
        const uint32_t e = U == 1 ? r : __umulhi(r, mag_u);
        const int u = (int)(r - e * (uint32_t)U);
        const int c = u - small_div(u, C) * C;
        own[k] = own_b.ld8s(e * (uint32_t)C + (uint32_t)c);  // (past the end: 0, the item is skipped below)
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kFillPer; k++) {
        const uint32_t r = r0 + 256 * k;
        const uint32_t e = U == 1 ? r : __umulhi(r, mag_u);
        const int u = (int)(r - e * (uint32_t)U);
        const int a = small_div(u, C), c = u - a * C;
        if ((int64_t)r >= n) continue;
        if (own[k] == a + 1) {  // the owner's row: acted in the rollout launch (by core: copied here)
            if (p.own_action) {
                const size_t oc = (size_t)e * C + c;
                act_b.st8(r, advance(p.own_action, t * p.own_action_stride)[oc]);
                lp_b.stf(4 * r, advance(p.own_logprob, t * p.own_logprob_stride)[oc]);
            }
            continue;
        }
        const uint32_t i = e * (uint32_t)C + (uint32_t)c, ib = i & ~64u;
        const uint32_t eb = C == 1 ? ib : __umulhi(ib, mag_c);
        uint32_t w0, w1;
        philox2(eb * (uint32_t)U + (uint32_t)(a * C) + (ib - eb * (uint32_t)C) + p.row_base, off, p.seed, w0, w1);
        const float* tab = tabs + a * kFreeTabDw;
        const float target = u24((i & 64u) ? w1 : w0) * tab[64];
        int cnt = 0;
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1)
            if (cnt + step <= 32 && tab[cnt + step - 1] <= target) cnt += step;
        const int act = cnt >= p.A ? __float_as_int(tab[65]) : cnt;
        act_b.st8(r, act);
        lp_b.stf(4 * r, tab[32 + act]);
    }
}

// k_acc_common_fill for C % 4 == 0 (the shipped shapes): a thread takes 4 consecutive items (one replica, one
// agent, cores c0..c0+3) of kFillRounds rounds, so the items' index math and Philox rows are computed once, the
// owners come as one dword per round (all rounds' loads in flight together), and a quad none of whose cores its
// agent owns is stored as one dword of actions and one 16-byte vector of log-probs (the per-item kernel: a byte
// and a dword store per item, and the tables loaded once per round per block). PAIR (64 % C == 0): items i and
// i ^ 64 take the two words of one draw, and i ^ 64 is the same agent's core c of replica e ^ (64 / C), so the
// thread also takes that replica's quad and each draw is computed once (the Philox rounds are the kernel's
// largest VALU cost: 32-bit multiplies at quarter rate). Same values bit for bit.
constexpr int kFillRounds = 8;
template <bool PAIR>
__global__ void __launch_bounds__(256) k_acc_common_fill4(CommonFillArgs p, int n_acts, int merge) {  // merge: fill_merge()
    __shared__ __align__(16) float tabs[8 * kFreeTabDw];
    using FL = FragLayout<2, 2>;
    for (int k = threadIdx.x; k < p.N * kFreeTabDw; k += blockDim.x) {
        const int a = k / kFreeTabDw;
        tabs[k] = __uint_as_float(p.frag[(size_t)a * FL::GB + 64 * FL::LW + (k - a * kFreeTabDw)]);
    }
    __syncthreads();
    const int C = p.C, U = p.N * C, QR = U >> 2;  // quads per replica row
    const uint32_t g = (uint32_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t pr = __umulhi(g, magic_div((uint32_t)QR)), uq = g - pr * (uint32_t)QR;
    const uint32_t S = PAIR ? 64u / (uint32_t)C : 1u;  // the partner replica's distance
    const uint32_t e0 = PAIR ? (((pr & ~(S - 1u)) << 1) | (pr & (S - 1u))) : pr, e1 = e0 + S;
    if (e0 >= (uint32_t)p.E) return;
    const bool has1 = PAIR && e1 < (uint32_t)p.E;
    const int u = 4 * (int)uq, a = small_div(u, C), c0 = u - a * C;
    uint32_t row[4], hi = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {  // item i = e * C + c: its uniform is word (i >> 6) & 1 of row(i & ~64)'s draw
        if constexpr (PAIR) {      // (i & 64 == 0 for replica e0: row(i) is its own)
            row[k] = e0 * (uint32_t)U + (uint32_t)(u + k) + p.row_base;
        } else {
            const uint32_t i = e0 * (uint32_t)C + (uint32_t)(c0 + k), ib = i & ~64u;
            const uint32_t eb = C == 1 ? ib : __umulhi(ib, magic_div((uint32_t)C));
            row[k] = eb * (uint32_t)U + (uint32_t)(a * C) + (ib - eb * (uint32_t)C) + p.row_base;
            hi |= ((i >> 6) & 1u) << k;
        }
    }
    const float* tab = tabs + a * kFreeTabDw;
    const float tmax = tab[64];
    float bm[3];  // the maxima of the first three blocks of 8 running sums
#pragma unroll
    for (int b = 0; b < 3; b++) bm[b] = tab[8 * b + 7];
    const int t0 = (int)blockIdx.y * kFillRounds;
    uint32_t own0[kFillRounds], own1[kFillRounds];
#pragma unroll
    for (int j = 0; j < kFillRounds; j++) {
        const int8_t* ob = advance(p.owner, (int64_t)(t0 + j) * p.owner_stride);
        own0[j] = t0 + j < n_acts ? *reinterpret_cast<const uint32_t*>(ob + (size_t)e0 * C + c0) : 0u;
        own1[j] = has1 && t0 + j < n_acts ? *reinterpret_cast<const uint32_t*>(ob + (size_t)e1 * C + c0) : 0u;
    }
    const uint64_t off0 = p.offset + (p.offset_dev ? *p.offset_dev : 0ull);
    const uint32_t mine = 0x01010101u * (uint32_t)(a + 1);
    auto store = [&](uint32_t e, int t, int owned, uint32_t acts, const float (&lps)[4]) {
        const size_t r = (size_t)e * U + u;
        int8_t* ad = advance(p.action, (int64_t)t * p.action_stride) + r;
        float* ld = advance(p.logprob, (int64_t)t * p.logprob_stride) + r;
        if (owned == 0 || merge || p.own_action) {
            uint32_t a4 = acts;
            float4 l4 = make_float4(lps[0], lps[1], lps[2], lps[3]);
            if (owned != 0) {  // merge the owned items the rollout wrote: whole quads, no partially written lines
                // (by core [E][C]: cores c0..c0 + 3 of replica e; else the rings' own quad)
                const size_t oc = (size_t)e * C + c0;
                const uint32_t old_a = p.own_action
                                           ? *reinterpret_cast<const uint32_t*>(advance(p.own_action, (int64_t)t * p.own_action_stride) + oc)
                                           : *reinterpret_cast<const uint32_t*>(ad);
                const float4 old_l = p.own_action
                                         ? *reinterpret_cast<const float4*>(advance(p.own_logprob, (int64_t)t * p.own_logprob_stride) + oc)
                                         : *reinterpret_cast<const float4*>(ld);
                uint32_t m = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) m |= ((owned >> k) & 1) ? 0xffu << (8 * k) : 0u;
                a4 = (acts & ~m) | (old_a & m);
                if (owned & 1) l4.x = old_l.x;
                if (owned & 2) l4.y = old_l.y;
                if (owned & 4) l4.z = old_l.z;
                if (owned & 8) l4.w = old_l.w;
            }
            *reinterpret_cast<uint32_t*>(ad) = a4;
            *reinterpret_cast<float4*>(ld) = l4;
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (!((owned >> k) & 1)) {
                    ad[k] = (int8_t)(acts >> (8 * k));
                    ld[k] = lps[k];
                }
        }
    };
#pragma unroll
    for (int j = 0; j < kFillRounds; j++) {
        const int t = t0 + j;
        if (t >= n_acts) break;
        const uint64_t off = off0 + (uint64_t)t * p.offset_step;
        // byte k == 0: the agent owns core c0 + k (acted in the rollout launch); replica e1 absent: all owned
        const uint32_t x0 = own0[j] ^ mine, x1 = has1 ? own1[j] ^ mine : 0u;
        int owned0 = 0, owned1 = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            owned0 |= ((x0 >> (8 * k)) & 0xffu) == 0u ? 1 << k : 0;
            owned1 |= ((x1 >> (8 * k)) & 0xffu) == 0u ? 1 << k : 0;
        }
        // every item's draw and search, owned or not (the owned ones are replaced at the store), branch-free and
        // in lockstep: the NI searches' dependent LDS reads of one step issue together instead of one search
        // after the other behind the ownership branches (the kernel is bound by that latency, not by its stores)
        constexpr int NI = PAIR ? 8 : 4;
        float tg[NI];
        int cnt[NI];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint32_t w0, w1;
            philox2(row[k], off, p.seed, w0, w1);
            tg[k] = u24(PAIR ? w0 : (((hi >> k) & 1u) ? w1 : w0)) * tmax;
            if constexpr (PAIR) tg[4 + k] = u24(w1) * tmax;
        }
        // the count of running sums <= target (the binary search's result: the sums are non-decreasing) in two
        // levels: the block of 8 from the 4 block maxima held in registers, then that block's 8 sums (two 16-byte
        // LDS reads, every item's issued together) -- instead of 6 dependent LDS reads per item
#pragma unroll
        for (int i = 0; i < NI; i++) {
            int nb = 0;
#pragma unroll
            for (int b = 0; b < 3; b++) nb += bm[b] <= tg[i] ? 1 : 0;
            cnt[i] = nb;  // block 0..3 (block 3 also when all of its sums are <= target: its count is then 8)
        }
        float4 blo[NI], bhi[NI];
#pragma unroll
        for (int i = 0; i < NI; i++) {
            blo[i] = *reinterpret_cast<const float4*>(tab + 8 * cnt[i]);
            bhi[i] = *reinterpret_cast<const float4*>(tab + 8 * cnt[i] + 4);
        }
#pragma unroll
        for (int i = 0; i < NI; i++) {
            const float t = tg[i];
            cnt[i] = 8 * cnt[i] + (blo[i].x <= t) + (blo[i].y <= t) + (blo[i].z <= t) + (blo[i].w <= t) + (bhi[i].x <= t) +
                     (bhi[i].y <= t) + (bhi[i].z <= t) + (bhi[i].w <= t);
        }
        const int lnz = __float_as_int(tab[65]);
        uint32_t acts0 = 0, acts1 = 0;
        float lps0[4], lps1[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int a0 = cnt[k] >= p.A ? lnz : cnt[k];
            acts0 |= (uint32_t)(uint8_t)a0 << (8 * k);
            lps0[k] = tab[32 + a0];
            if constexpr (PAIR) {
                const int a1 = cnt[4 + k] >= p.A ? lnz : cnt[4 + k];
                acts1 |= (uint32_t)(uint8_t)a1 << (8 * k);
                lps1[k] = tab[32 + a1];
            } else {
                lps1[k] = 0.f;
            }
        }
        store(e0, t, owned0, acts0, lps0);
        if (has1) store(e1, t, owned1, acts1, lps1);
    }
}

struct RolloutFreeArgs {
    Params P;
    int64_t E;
    uint8_t* recs;
    uint32_t* mt;
    Liab* liab;
    StepIO io;
    FusedActFree fa;
    RoundStrideFree st;
    int n_rounds, act_last;
    int prio;  // bit 0: the workgroup's waves 4.. at raised issue priority while acting, bit 1: during the env round,
               // bit 2: the acting's waves paced against their SIMD partners (act_free pace_on)
};
// The locally shared free-price rollout in one launch: workgroup b holds replicas kFreeEPW * N * b .. in its LDS,
// and wave w steps kFreeEPW of them (k_env_step's round, 16 lanes per replica) and then acts for agent w of all
// of them (act_free), round after round, with a workgroup barrier between the phases: every agent's nets
// act from registers and LDS on the rows the round just built, instead of an act launch re-reading them from
// HBM. Round t's arrays are the given ones advanced by t strides. The round re-reads its arguments through
// the opaque kernel-argument pointer (k_env_rollout_act). Two workgroups per CU: 4 waves per SIMD (<= 128 VGPRs).
template <class SH>
__global__ void __launch_bounds__(512, 4) k_env_rollout_act_free(RolloutFreeArgs A0) {
    extern __shared__ __align__(16) uint8_t smem_free[];
    Geom g;
    if constexpr (SH::kStatic) {
        constexpr Geom kg = make_geom(SH::kN, SH::kC, SH::kL, SH::kJ);
        g = kg;
    } else {
        g = A0.P;
    }
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane0 = (int)threadIdx.x & 63;
    const FreeLds fl = free_lds(g);
    const int64_t wslot = (int64_t)blockIdx.x * g.N + wave;  // the wave's slot of kFreeEPW replicas
    unsigned long long* span = A0.io.span;
    if (span && lane0 == 0) {
        span[4 * wslot] = __builtin_amdgcn_s_memrealtime();
        span[4 * wslot + 2] = __builtin_amdgcn_s_memtime();
    }
    // once per launch (the acting nets do not change within a rollout): the price table's key digits, one copy
    // per workgroup
    {
        uint32_t* pd = reinterpret_cast<uint32_t*>(smem_free + fl.pdig);
        const uint32_t* src = reinterpret_cast<const uint32_t*>(A0.fa.pdigit);
        for (int k = (int)threadIdx.x; k < 512; k += (int)blockDim.x) pd[k] = src[k];
        // (by-core mode) the acceptor actions the env rounds stage from the LDS: the acting writes the owners'
        // items only, and the env checks every item's range (k_env_step: they are all sampled), so the others
        // hold a valid action (0, "reject") instead of whatever the LDS held
        uint32_t* ax = reinterpret_cast<uint32_t*>(smem_free + fl.accx);
        for (int k = (int)threadIdx.x; k < (fl.total - fl.accx) / 4; k += (int)blockDim.x) ax[k] = 0u;  // (+ pace)
    }
    __syncthreads();
#ifdef MS_PHASE_TIMING
    // probe build: per wave, the shader cycles of the env rounds, the wait at the barrier after them, the acting,
    // and the wait at the barrier after it (tools/env_phase_probe.py --free)
    uint64_t f_prev = __builtin_amdgcn_s_memtime(), f_acc[5] = {0, 0, 0, 0, 0};
#define FREE_MARK(k)                                                   \
    do {                                                               \
        const uint64_t f_now = __builtin_amdgcn_s_memtime();          \
        if ((k) >= 0) f_acc[(k) < 0 ? 0 : (k)] += f_now - f_prev;      \
        f_prev = f_now;                                                \
    } while (0)
#else
#define FREE_MARK(k) \
    do {             \
    } while (0)
#endif
    const int n_rounds = A0.n_rounds;
    for (int t = 0; t < n_rounds; t++) {
        auto ka = __builtin_amdgcn_kernarg_segment_ptr();  // (constant address space)
        asm volatile("" : "+s"(ka));
        const RolloutFreeArgs& A = *(const RolloutFreeArgs*)ka;
        int lane = (int)threadIdx.x & 63;
        asm volatile("" : "+v"(lane));
        const RoundStrideFree& st = A.st;
        StepIO io = A.io;
        io.span = nullptr;
        io.act_acc = advance(io.act_acc, t * st.act_acc);
        io.act_off = advance(io.act_off, t * st.act_off);
        io.obs_crow = advance(io.obs_crow, t * st.obs_crow);
        io.obs_cown = advance(io.obs_cown, t * st.obs_cown);
        io.obs_off = advance(io.obs_off, t * st.obs_off);
        io.rew_offer = advance(io.rew_offer, t * st.rew_offer);
        io.rew_price = advance(io.rew_price, t * st.rew_price);
        io.rew_acc = advance(io.rew_acc, t * st.rew_acc);
        io.rew_agent = advance(io.rew_agent, t * st.rew_agent);
        io.rew_auct = advance(io.rew_auct, t * st.rew_auct);
        FREE_MARK(-1);
        // (the younger half of the workgroup's waves otherwise trails the older at every barrier: issue goes by
        //  priority, then age)
        const bool up = wave >= 4 && (A.prio & 2);
        if (up) __builtin_amdgcn_s_setprio(1);
        // rounds after the first (by-core mode): the owners' acceptor actions are where this launch's acting left
        // them in the LDS (the rings' acceptor rows are written after the launch, by the fill)
        const int8_t* acc_lds = t > 0 && A.fa.own_action
                                    ? reinterpret_cast<const int8_t*>(smem_free + fl.accx) + wave * kFreeEPW * g.N * g.C
                                    : nullptr;
        env_round<kWave / kFreeEPW, false, true, SH>(A.P, A.E, A.recs, A.mt, A.liab, io, wslot, lane,
                                                     smem_free + wave * kFreeEPW * g.s_total, acc_lds);
        if (up) __builtin_amdgcn_s_setprio(0);
        FREE_MARK(0);
        if (t + 1 < n_rounds || A.act_last) {
            __syncthreads();  // every replica's observation sources are in the LDS
            FREE_MARK(1);
            FusedActFree fa = A.fa;
            fa.core_action = advance(fa.core_action, t * st.core_action);
            fa.core_logprob = advance(fa.core_logprob, t * st.core_logprob);
            fa.price_state = advance(fa.price_state, t * st.price_state);
            fa.price_action = advance(fa.price_action, t * st.price_action);
            fa.price_logprob = advance(fa.price_logprob, t * st.price_logprob);
            fa.acc_action = advance(fa.acc_action, t * st.acc_action);
            fa.acc_logprob = advance(fa.acc_logprob, t * st.acc_logprob);
            fa.own_action = advance(fa.own_action, t * st.own_action);
            fa.own_logprob = advance(fa.own_logprob, t * st.own_logprob);
            fa.off_offset += (uint64_t)t * st.offset_step;
            fa.acc_offset += (uint64_t)t * st.offset_step;
            const bool up_act = wave >= 4 && (A.prio & 1);
            if (up_act) __builtin_amdgcn_s_setprio(1);
            const bool pace_on = (A.prio & 4) != 0;
#ifdef MS_PHASE_TIMING
            act_free<SH, 1>(g, A.E, fa, (int64_t)blockIdx.x * kFreeEPW * g.N, wave, lane, smem_free, fl, pace_on);
            FREE_MARK(2);
            act_free<SH, 2>(g, A.E, fa, (int64_t)blockIdx.x * kFreeEPW * g.N, wave, lane, smem_free, fl, pace_on);
#else
            act_free<SH>(g, A.E, fa, (int64_t)blockIdx.x * kFreeEPW * g.N, wave, lane, smem_free, fl, pace_on);
#endif
            if (up_act || pace_on) __builtin_amdgcn_s_setprio(0);
            FREE_MARK(3);
            __syncthreads();  // the actions are stored and the LDS is free for the next round
            FREE_MARK(4);
        }
    }
    if (span && lane0 == 0) {
        span[4 * wslot + 3] = __builtin_amdgcn_s_memtime();
        span[4 * wslot + 1] = __builtin_amdgcn_s_memrealtime();
    }
#ifdef MS_PHASE_TIMING
    if (lane0 == 0)
        for (int k = 0; k < 5; k++) g_free_cycles[wslot % kProbeSlots][k] += f_acc[k];
#endif
}

// Auctioneer.getAuctioneerAction (Auctioneer.py:95-102) on its own, as the driver calls it
// before env.step (trainPPO.py:162): writes actions [E][C] and advances the env stream by the
// tie-break draws; a following ms_env_step with these actions then draws only the spawn.
__global__ void __launch_bounds__(64) k_env_auctioneer(Params P, uint8_t* recs, uint32_t* mt, int8_t* actions) {
    extern __shared__ __align__(16) uint8_t smem[];
    M128* s_mc = reinterpret_cast<M128*>(smem + P.s_mc);
    M128* s_mr = reinterpret_cast<M128*>(smem + P.s_mr);
    int16_t* s_auct = reinterpret_cast<int16_t*>(smem + P.s_auct);
    const int lane = threadIdx.x;
    const Lanes<kWave> Lg(lane);
    const int64_t e = blockIdx.x;
    uint8_t* rec = smem + P.s_rec;
    __shared__ int32_t s_kt[48];
    mt_refill_next<kWave>(mt, recs, P, blockIdx.x, true, smem, lane);
    load_kind_tables(P, s_kt, lane);
    copy_dwords<kWave>(reinterpret_cast<uint32_t*>(rec),
                       reinterpret_cast<const uint32_t*>(recs + e * (int64_t)P.rec_bytes), P.rec_bytes / 4, lane);
    wave_sync();
    Rec R{rec, &P, s_kt};
    MtStream<kWave> rs;
    rs.init(mt + e * 2 * kMtN, R.mt_sel(), R.mti(), true);
    rs.load(0, 0, Lg);
    build_masks<kWave>(R, P, s_mc, s_mr, lane);
    hardcoded_auctioneer<kWave>(R, P, s_mc, s_mr, rs, s_auct, Lg);
    wave_sync();
    for (int c = lane; c < P.C; c += kWave) actions[e * P.C + c] = (int8_t)s_auct[c];
    if (lane == 0) {
        int32_t* hdr = reinterpret_cast<int32_t*>(recs + e * (int64_t)P.rec_bytes);
        mt_commit(rs.end_index(), hdr + 2, reinterpret_cast<uint32_t*>(hdr + 3));
    }
}

// random._randbelow(n) on env e's stream (random.randint in the update schedulers,
// Agent.py:718,725, SchedulingEnvironment.py:317-326).
__global__ void __launch_bounds__(64) k_env_randbelow(Params P, uint8_t* recs, uint32_t* mt, int64_t e, uint32_t n,
                                                      uint32_t* out) {
    extern __shared__ __align__(16) uint8_t smem[];
    const int lane = threadIdx.x;
    const Lanes<kWave> Lg(lane);
    uint8_t* rec = recs + e * (int64_t)P.rec_bytes;
    int32_t* mti = reinterpret_cast<int32_t*>(rec + 8);
    uint32_t* sel = reinterpret_cast<uint32_t*>(rec + 12);
    if (!(*sel & 2u)) mt_twist_into_successor(mt + e * 2 * kMtN, *sel, smem, lane);
    MtStream<kWave> rs;
    rs.init(mt + e * 2 * kMtN, *sel, *mti, true);
    const uint32_t r = rs.randbelow(n, Lg);
    wave_sync();
    if (lane == 0) {
        *out = r;
        mt_commit(rs.end_index(), mti, sel);
    }
}

}  // namespace ms

#ifdef MS_PHASE_TIMING
// profiling build only: read (and optionally clear) the per-phase cycle counters
extern "C" int ms_probe_phase_cycles(unsigned long long* out, int clear) {
    static unsigned long long host[ms::kProbeSlots][16];
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(ms::g_phase_cycles), sizeof(host)) != hipSuccess) return -1;
    for (int k = 0; k < 16; k++) {
        out[k] = 0;
        for (int b = 0; b < ms::kProbeSlots; b++) out[k] += host[b][k];
    }
    if (clear) {
        memset(host, 0, sizeof(host));
        if (hipMemcpyToSymbol(HIP_SYMBOL(ms::g_phase_cycles), host, sizeof(host)) != hipSuccess) return -1;
    }
    return 0;
}
// the per-phase cycles of every block (summed over the launches since the last clear): out[16 * n_blocks]
extern "C" int ms_probe_phase_blocks(unsigned long long* out, int n_blocks) {
    static unsigned long long host[ms::kProbeSlots][16];
    if (n_blocks > ms::kProbeSlots) return -1;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(ms::g_phase_cycles), sizeof(host)) != hipSuccess) return -1;
    memcpy(out, host, sizeof(unsigned long long) * 16 * n_blocks);
    return 0;
}
// k_env_rollout_act_free's per-wave cycles (env rounds, barrier wait, acting, barrier wait) summed over the
// launches since the last clear: out[4 * n_waves]
extern "C" int ms_probe_free_cycles(unsigned long long* out, int n_waves, int clear) {
    static unsigned long long host[ms::kProbeSlots][5];
    if (n_waves > ms::kProbeSlots) return -1;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(ms::g_free_cycles), sizeof(host)) != hipSuccess) return -1;
    memcpy(out, host, sizeof(unsigned long long) * 5 * n_waves);
    if (clear) {
        memset(host, 0, sizeof(host));
        if (hipMemcpyToSymbol(HIP_SYMBOL(ms::g_free_cycles), host, sizeof(host)) != hipSuccess) return -1;
    }
    return 0;
}
// entry / exit s_memrealtime (100 MHz) of every block of the last launch: out[2 * n_blocks]
extern "C" int ms_probe_wave_spans(unsigned long long* out, int n_blocks) {
    static unsigned long long host[ms::kProbeSlots][2];
    if (n_blocks > ms::kProbeSlots) return -1;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(ms::g_wave_span), sizeof(host)) != hipSuccess) return -1;
    memcpy(out, host, sizeof(unsigned long long) * 2 * n_blocks);
    return 0;
}
#endif

// launch wrappers used by capi.cpp
namespace ms {
hipError_t launch_env_init(const Params& P, int64_t E, uint8_t* recs, uint32_t* mt, Liab* liab, uint64_t seed,
                           hipStream_t s) {
    // the seeding runs in the scratch, which k_env_init needs at MT-state size
    const size_t lds = (size_t)P.s_scratch + 4 * kMtN > (size_t)P.s_total ? (size_t)P.s_scratch + 4 * kMtN : P.s_total;
    hipLaunchKernelGGL(k_env_init, dim3((unsigned)E), dim3(kWave), lds, s, P, recs, mt, liab, seed);
    return hipGetLastError();
}
hipError_t launch_env_reset(const Params& P, int64_t E, const uint8_t* recs, int8_t* a, int8_t* o, int8_t* u,
                            int8_t* crow, int8_t* cown, hipStream_t s) {
    hipLaunchKernelGGL(k_env_reset, dim3((unsigned)E), dim3(kWave), P.s_total, s, P, recs, a, o, u, crow, cown);
    return hipGetLastError();
}

// lanes per env: the smallest power of two >= max(C, N) and >= 16 (a 16-word MT window), so a
// wave steps 4 (cfg2/cfg3), 2 (cfg4) or 1 (cfg5) envs
#ifndef MS_MIN_LPE
#define MS_MIN_LPE 16
#endif
// A launch of >= 1024 replicas in fewer than MS_ENV_MIN_WAVES waves (env variable, default 2048: two per
// SIMD) widens the lane groups up to that many waves, so the chip's SIMDs each hold two waves
// whose waits can hide each other: cfg2 (4096 replicas, 4 x 4) runs 32 lanes per env, 2048 waves,
// instead of 16 lanes, 1024 waves (one per SIMD, every wait exposed).
static int lanes_per_env(const Params& P, int64_t E) {
    int need = P.C > P.N ? P.C : P.N;
    int lpe = MS_MIN_LPE;
    while (lpe < need) lpe *= 2;
    static const long long min_waves = [] {
        const char* v = getenv("MS_ENV_MIN_WAVES");
        return v ? atoll(v) : 2048LL;
    }();
    while (E >= 1024 && lpe < kWave && (E * lpe + kWave - 1) / kWave < min_waves &&
           (E * 2 * lpe + kWave - 1) / kWave <= min_waves)
        lpe *= 2;
    return lpe;
}

template <int LPE, class SH>
static hipError_t launch_step_sh(const Params& P, int64_t E, uint8_t* recs, uint32_t* mt, Liab* liab, const StepIO& io,
                                 hipStream_t s) {
    constexpr int G = kWave / LPE;
    const int64_t blocks = (E + G - 1) / G;
    const size_t lds = (size_t)P.s_total * G > 4 * kMtN ? (size_t)P.s_total * G : 4 * kMtN;  // >= one MT block
    const bool compact = io.obs_crow != nullptr || io.obs_cown != nullptr;
    const bool ext = io.act_acc == nullptr || io.metrics != nullptr || (compact && io.obs_acc != nullptr);
    auto kern = ext ? k_env_step<LPE, true, false, DynShape>
                    : (compact ? k_env_step<LPE, false, true, SH> : k_env_step<LPE, false, false, SH>);
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kWave), lds, s, P, E, recs, mt, liab, io);
    return hipGetLastError();
}

template <int N, int C, int L, int J>
static bool is_shape(const Params& P) {
    return P.N == N && P.C == C && P.L == L && P.new_jobs == J;
}

// The BASELINE shapes (cfg2 4x4x3, cfg3 8x8x3, cfg4 16x16x3, cfg5 32x32x3, one new job per agent and
// round) run the kernel compiled for their geometry; every other shape the generic one.
template <int LPE>
static hipError_t launch_step_t(const Params& P, int64_t E, uint8_t* recs, uint32_t* mt, Liab* liab, const StepIO& io,
                                hipStream_t s) {
#ifndef MS_NO_FIXED_SHAPES
    if constexpr (LPE == 16) {
        if (is_shape<8, 8, 3, 1>(P)) return launch_step_sh<LPE, FixShape<8, 8, 3, 1>>(P, E, recs, mt, liab, io, s);
        if (is_shape<16, 16, 3, 1>(P)) return launch_step_sh<LPE, FixShape<16, 16, 3, 1>>(P, E, recs, mt, liab, io, s);
    }
    if constexpr (LPE == 32) {
        if (is_shape<4, 4, 3, 1>(P)) return launch_step_sh<LPE, FixShape<4, 4, 3, 1>>(P, E, recs, mt, liab, io, s);
        if (is_shape<32, 32, 3, 1>(P)) return launch_step_sh<LPE, FixShape<32, 32, 3, 1>>(P, E, recs, mt, liab, io, s);
    }
#endif
    return launch_step_sh<LPE, DynShape>(P, E, recs, mt, liab, io, s);
}

hipError_t launch_env_step(const Params& P, int64_t E, uint8_t* recs, uint32_t* mt, Liab* liab, const StepIO& io,
                           hipStream_t s) {
    switch (lanes_per_env(P, E)) {
#if MS_MIN_LPE <= 8
        case 8: return launch_step_t<8>(P, E, recs, mt, liab, io, s);
#endif
        case 16: return launch_step_t<16>(P, E, recs, mt, liab, io, s);
        case 32: return launch_step_t<32>(P, E, recs, mt, liab, io, s);
        default: return launch_step_t<64>(P, E, recs, mt, liab, io, s);
    }
}
// ms_env_step_act: a wave's acceptor items one per lane (<= 64), its offer rows in 16-row tiles (<= 64) and
// its owned cores' rows in one
bool env_step_act_supported(const Params& P, int64_t E) {
    const int epw = kWave / lanes_per_env(P, E);
    return epw * P.N * P.C <= kWave && epw * P.NL <= kWave && epw * P.C <= 16;
}
template <int LPE, class SH>
static hipError_t launch_step_act_sh(const Params& P, int64_t E, uint8_t* recs, uint32_t* mt, Liab* liab,
                                     const StepIO& io, const FusedAct& fa, hipStream_t s) {
    constexpr int G = kWave / LPE;
    const int64_t blocks = (E + G - 1) / G;
    const size_t lds = (size_t)P.s_total * G > 4 * kMtN ? (size_t)P.s_total * G : 4 * kMtN;
    hipLaunchKernelGGL((k_env_step_act<LPE, SH>), dim3((unsigned)blocks), dim3(kWave), lds, s, P, E, recs, mt, liab, io,
                       fa);
    return hipGetLastError();
}
hipError_t launch_env_step_act(const Params& P, int64_t E, uint8_t* recs, uint32_t* mt, Liab* liab, const StepIO& io,
                               const FusedAct& fa, hipStream_t s) {
    if (!env_step_act_supported(P, E) || io.act_acc == nullptr || io.metrics != nullptr || io.obs_acc != nullptr)
        return hipErrorInvalidValue;
    switch (lanes_per_env(P, E)) {
        case 16: return launch_step_act_sh<16, DynShape>(P, E, recs, mt, liab, io, fa, s);
        case 32:
#ifndef MS_NO_FIXED_SHAPES
            if (is_shape<4, 4, 3, 1>(P)) return launch_step_act_sh<32, FixShape<4, 4, 3, 1>>(P, E, recs, mt, liab, io, fa, s);
#endif
            return launch_step_act_sh<32, DynShape>(P, E, recs, mt, liab, io, fa, s);
        default: return launch_step_act_sh<64, DynShape>(P, E, recs, mt, liab, io, fa, s);
    }
}
template <int LPE, class SH>
static hipError_t launch_rollout_act_sh(const Params& P, int64_t E, uint8_t* recs, uint32_t* mt, Liab* liab,
                                        const StepIO& io, const FusedAct& fa, const RoundStride& st, int n_rounds,
                                        int act_last, hipStream_t s) {
    constexpr int G = kWave / LPE;
    const int64_t blocks = (E + G - 1) / G;
    const size_t lds = (size_t)P.s_total * G > 4 * kMtN ? (size_t)P.s_total * G : 4 * kMtN;
    const RolloutArgs A{P, E, recs, mt, liab, io, fa, st, n_rounds, act_last};
    hipLaunchKernelGGL((k_env_rollout_act<LPE, SH>), dim3((unsigned)blocks), dim3(kWave), lds, s, A);
    return hipGetLastError();
}
hipError_t launch_env_rollout_act(const Params& P, int64_t E, uint8_t* recs, uint32_t* mt, Liab* liab,
                                  const StepIO& io, const FusedAct& fa, const RoundStride& st, int n_rounds,
                                  int act_last, hipStream_t s) {
    if (!env_step_act_supported(P, E) || io.act_acc == nullptr || io.metrics != nullptr || io.obs_acc != nullptr ||
        n_rounds < 1)
        return hipErrorInvalidValue;
    switch (lanes_per_env(P, E)) {
        case 16: return launch_rollout_act_sh<16, DynShape>(P, E, recs, mt, liab, io, fa, st, n_rounds, act_last, s);
        case 32:
#ifndef MS_NO_FIXED_SHAPES
            if (is_shape<4, 4, 3, 1>(P))
                return launch_rollout_act_sh<32, FixShape<4, 4, 3, 1>>(P, E, recs, mt, liab, io, fa, st, n_rounds,
                                                                       act_last, s);
#endif
            return launch_rollout_act_sh<32, DynShape>(P, E, recs, mt, liab, io, fa, st, n_rounds, act_last, s);
        default: return launch_rollout_act_sh<64, DynShape>(P, E, recs, mt, liab, io, fa, st, n_rounds, act_last, s);
    }
}
// ms_env_rollout_act_free: 16 lanes per replica (max(N, C) <= 16), one wave per agent (N <= 8: a 512-lane
// workgroup), the core chooser one k-step with <= 16 actions, the acceptor two k-steps with 17..32 actions
// (k_act_pair<1, 1, 1, 2, 2>'s shapes), the price chooser <= 16 actions, two workgroups' LDS per CU
bool env_rollout_free_supported(const Params& P) {
    return P.free_prices && P.N >= 1 && P.N <= 8 && P.C >= 1 && P.C <= 16 && P.off_stride <= 32 &&
           P.C + 1 <= 16 && P.acc_stride > 32 && P.acc_stride <= 64 && P.O + 1 > 16 && P.O + 1 <= 32 &&
           2 * (free_lds(P).total + 256) <= 160 * 1024;
}
template <class SH>
static hipError_t launch_rollout_free_sh(const Params& P, int64_t E, uint8_t* recs, uint32_t* mt, Liab* liab,
                                         const StepIO& io, const FusedActFree& fa, const RoundStrideFree& st,
                                         int n_rounds, int act_last, hipStream_t s) {
    const int64_t epb = (int64_t)kFreeEPW * P.N;
    const int64_t blocks = (E + epb - 1) / epb;
    static const int prio = [] {
        const char* v = getenv("MS_FREE_PRIO");  // (measurement knob, tools/gpu_job.sh envab)
        // measured: 1 (acting) 49.6 -> 49.0 us per round, 3 (and env) 49.1 (profiles/r7c); 4 (paced acting)
        // 47.07 -> 46.66 us against 1 over three A/B pairs, wait after acting 9.0k -> 4.5k cycles (profiles/r7)
        return v ? atoi(v) : 4;
    }();
    const RolloutFreeArgs A{P, E, recs, mt, liab, io, fa, st, n_rounds, act_last, prio};
    hipLaunchKernelGGL((k_env_rollout_act_free<SH>), dim3((unsigned)blocks), dim3(64 * P.N), (size_t)free_lds(P).total, s,
                       A);
    return hipGetLastError();
}
// quads with owned items stored whole, merged with the values the rollout wrote: every line of the outputs is
// written whole (the per-item stores left every line partial): 501 -> 425 us per 199-round fill (profiles/r7s).
// MS_FILL_MERGE=0: the per-item stores (A/B measurements)
static int fill_merge() {
    static const int v = [] {
        const char* e = getenv("MS_FILL_MERGE");
        return e && e[0] == '0' ? 0 : 1;
    }();
    return v;
}
// MS_FILL_PAIR=0: the quad fill without the draw pairing (A/B measurements)
static bool fill_pair_enabled() {
    static const bool v = [] {
        const char* e = getenv("MS_FILL_PAIR");
        return !(e && e[0] == '0');
    }();
    return v;
}
// MS_FILL_QUAD=0: the per-item fill kernel (A/B measurements)
static bool fill_quad_enabled() {
    static const bool v = [] {
        const char* e = getenv("MS_FILL_QUAD");
        return !(e && e[0] == '0');
    }();
    return v;
}
// the acceptor items of cores their agent does not own, every acting round of a k_env_rollout_act_free launch
// with the same arguments (its outputs' other items are untouched)
hipError_t launch_env_fill_common(const Params& P, int64_t E, const StepIO& io, const FusedActFree& fa,
                                  const RoundStrideFree& st, int n_rounds, int act_last, hipStream_t s) {
    const int n_acts = act_last ? n_rounds : n_rounds - 1;
    if (!env_rollout_free_supported(P) || io.obs_cown == nullptr || fa.acc.act_frag == nullptr) return hipErrorInvalidValue;
    if (n_acts < 1) return hipSuccess;
    const CommonFillArgs c{io.obs_cown, fa.acc_action, fa.acc_logprob, st.obs_cown, st.acc_action, st.acc_logprob,
                           fa.own_action, fa.own_logprob, st.own_action, st.own_logprob,
                           static_cast<const uint32_t*>(fa.acc.act_frag) + 4, (int)E, P.N, P.C, fa.acc.n_actions,
                           (uint32_t)fa.acc.row_base, fa.seed, fa.acc_offset, st.offset_step, fa.offset_dev};
    const int64_t items = E * P.N * P.C;
    // the quad kernel: C % 4 == 0 and every round's owners / actions 4-byte, log-probs 16-byte aligned
    const bool quad = P.C % 4 == 0 && fill_quad_enabled() &&
                      ((reinterpret_cast<uintptr_t>(c.owner) | (uintptr_t)c.owner_stride) & 3) == 0 &&
                      ((reinterpret_cast<uintptr_t>(c.action) | (uintptr_t)c.action_stride) & 3) == 0 &&
                      ((reinterpret_cast<uintptr_t>(c.logprob) | (uintptr_t)c.logprob_stride) & 15) == 0 &&
                      ((reinterpret_cast<uintptr_t>(c.own_action) | (uintptr_t)c.own_action_stride) & 3) == 0 &&
                      ((reinterpret_cast<uintptr_t>(c.own_logprob) | (uintptr_t)c.own_logprob_stride) & 15) == 0;
    if (quad) {
        const unsigned by = (unsigned)((n_acts + kFillRounds - 1) / kFillRounds);
        const int64_t qr = (int64_t)P.N * P.C / 4;
        if (64 % P.C == 0 && fill_pair_enabled()) {  // threads: quads of the replicas e with e & (64 / C) == 0
            const int64_t S = 64 / P.C, pairs = (E + 2 * S - 1) / (2 * S) * S;
            hipLaunchKernelGGL(k_acc_common_fill4<true>, dim3((unsigned)((pairs * qr + 255) / 256), by), dim3(256), 0, s,
                               c, n_acts, fill_merge());
        } else {
            hipLaunchKernelGGL(k_acc_common_fill4<false>, dim3((unsigned)((E * qr + 255) / 256), by), dim3(256), 0, s, c,
                               n_acts, fill_merge());
        }
        return hipGetLastError();
    }
    const unsigned bx = (unsigned)((items + kFillPer * 256 - 1) / (kFillPer * 256));
    hipLaunchKernelGGL(k_acc_common_fill, dim3(bx, (unsigned)n_acts), dim3(256), 0, s, c);
    return hipGetLastError();
}
hipError_t launch_env_rollout_act_free(const Params& P, int64_t E, uint8_t* recs, uint32_t* mt, Liab* liab,
                                       const StepIO& io, const FusedActFree& fa, const RoundStrideFree& st,
                                       int n_rounds, int act_last, hipStream_t s) {
    if (!env_rollout_free_supported(P) || io.act_acc == nullptr || io.metrics != nullptr || io.obs_acc != nullptr ||
        n_rounds < 1)
        return hipErrorInvalidValue;
#ifndef MS_NO_FIXED_SHAPES
    if (is_shape<8, 8, 3, 1>(P))
        return launch_rollout_free_sh<FixShape<8, 8, 3, 1>>(P, E, recs, mt, liab, io, fa, st, n_rounds, act_last, s);
#endif
    return launch_rollout_free_sh<DynShape>(P, E, recs, mt, liab, io, fa, st, n_rounds, act_last, s);
}
hipError_t launch_env_auctioneer(const Params& P, int64_t E, uint8_t* recs, uint32_t* mt, int8_t* actions,
                                 hipStream_t s) {
    const size_t lds = (size_t)P.s_total > 4 * kMtN ? (size_t)P.s_total : 4 * kMtN;
    hipLaunchKernelGGL(k_env_auctioneer, dim3((unsigned)E), dim3(kWave), lds, s, P, recs, mt, actions);
    return hipGetLastError();
}
hipError_t launch_env_randbelow(const Params& P, uint8_t* recs, uint32_t* mt, int64_t e, uint32_t n, uint32_t* out,
                                hipStream_t s) {
    hipLaunchKernelGGL(k_env_randbelow, dim3(1), dim3(kWave), 4 * kMtN, s, P, recs, mt, e, n, out);
    return hipGetLastError();
}
}  // namespace ms
