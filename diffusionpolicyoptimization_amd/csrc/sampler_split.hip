// sampler_split.hip — a9: VPGDiffusion.call (model/diffusion/diffusion_vpg.py:250-339), DDPM branch,
// as a register-resident SPLIT kernel (the default for the bf16 denoiser at <= 512 envs per GPU).
//
// Why: the weight-streaming kernel (sampler.hip) gives each 16-env tile one CU, which must pull the
// whole 1.1 MB bf16 actor through its 64 B/clk load path every denoising step (~8 us a step at 64
// envs). Here each 16-env tile is owned by a GROUP of P = 8 workgroups (one per CU), and member c
// keeps 1/8 of the actor in its register file for the whole launch:
//   in-Dense   all 512 outputs (64 KB, replicated: its input is tiny and local)
//   l1         output columns [64c, 64c+64)                      (W_l1[:, slice],  64 KB)
//   l2         input rows     [64c, 64c+64), all 512 outputs     (W_l2[slice, :],  64 KB)
//   out-Dense  all of it (16 KB), applied to the member's PARTIAL l2 sum
// so the only cross-CU traffic of a denoising step is one exchange of 16 x XD fp32 out-layer
// partial sums between the 8 members (mlp.py:186-206 is linear from the l2 product to the
// out-Dense: eps = sum_c (P_c [+ b_l2 + h1 on member 0]) W_out + b_out). Every member then runs
// the same fp32 DDPM epilogue on the same sum (fixed member order: bit-identical x on all eight).
//
// The exchange is in-launch (MI355X_MICROARCH.md "handoff-1to1"/R2 granules): each member stores
// its partials as 8-byte {tag, value} granules and every wave sweeps its slice of the group's
// granules with agent-scope (sc1, L1-bypassing) loads until every tag matches. Tags carry a
// per-launch sequence number and the step index, so nothing is zeroed between launches; slots
// alternate by step parity (a member can be at most one step ahead of a peer). The wait is
// bounded (100 ms): a launch that times out writes NaN actions and flags bit 31 of *done.
// Store flavour, chosen per group at run time (never assumed from blockIdx):
//   * every member reads its XCD from HW_REG_XCC_ID and announces it (sc1 granule) in the
//     prologue; the members sweep the announcements and agree on the mode;
//   * all on one XCD -> "L2-local": workgroup-scope (sc0) granule stores, which keep the line in
//     that XCD's L2, where the peers' sc1 loads find it (tools/xchg_probe2.hip: 1.55 vs 2.21 us
//     per exchange step; sc0 across XCDs never becomes visible: the probe's spread row times out).
//     These granules live in a region owned by that XCD alone ([xcc][slot][G][P][NV], fixed
//     stride), so no other XCD's L2 ever holds a copy of those lines;
//   * otherwise -> write-through agent-scope (sc1) stores into the shared region, the
//     placement-independent form.
//
// Layout per step (member c, 8 waves; all GEMMs computed TRANSPOSED, W^T x^T, so an MFMA result
// lane holds 4 consecutive features of one env):
//   in-layer   wave w: h1 features [64w, 64w+64)    -> u1 = bf16 relu(h1) to LDS (8-B stores)
//   l1         wave w: l1 n-tile (w % 4), K-half (w / 4) -> fp32 partial to LDS
//   l2         wave w: h3 features [64w, 64w+64) of this member's K-slice (+ b_l2 + h1 on c = 0)
//   out-Dense  wave w: its own h3 registers as the B operand (hi/lo bf16 split: fp32-accurate),
//              W_out fragments pre-permuted to the MFMA result lane order -> partial to LDS
//   wave 0: sum the 8 wave partials, publish, sweep the group, DDPM epilogue; waves 1-7 write
//   the next step's time embedding.
// Block -> (group, member): members of a group share blockIdx % 8 (one XCD under the observed
// round-robin placement: a speed choice only; correctness does not depend on placement).
#include <mutex>
#include <type_traits>
#include <stdlib.h>
#include <string.h>
#include "dppo_common.cuh"
#include "dppo_internal.h"
#include "dppo_sampler.h"

// phase timing for tuning builds (-DDPPO_SAMPLER_TIMING): thread 0 of every workgroup adds the
// shader-clock cycles of each phase (0 prologue, 1 actor switch, 2 in-Dense, 3 l1, 4 l2 + out,
// 5 publish + sweep, 6 epilogue); 11-15 split phases 2-5 at the point wave 0 reaches the barrier
// (11 in-Dense, 12 l1, 13 l2 GEMM, 14 out-Dense + partial store, 15 partial sum + publish)
#ifdef DPPO_SAMPLER_TIMING
__device__ unsigned long long dppo_split_cycles[16 + 64 * 8];
// [0, 16): phase sums over all workgroups; [16 + 8 i + k): phase k of step i of workgroup 0 alone
#define XPHASE(k)                                                                 \
    do {                                                                          \
        if (threadIdx.x == 0) {                                                   \
            const unsigned long long now_ = __builtin_readcyclecounter();         \
            atomicAdd(&dppo_split_cycles[(k)], now_ - t_phase_);                  \
            if (blockIdx.x == 0 && t_step_ < 64 && (k) < 8) dppo_split_cycles[16 + 8 * t_step_ + (k)] = now_ - t_phase_; \
            t_phase_ = now_;                                                      \
        }                                                                         \
    } while (0)
#define XPHASE_START unsigned long long t_phase_ = __builtin_readcyclecounter(); int t_step_ = 0
#define XSTEP(i) t_step_ = (i)
// groups that ran the exchange L2-local ([1]) or shared ([0]), summed over launches
__device__ unsigned dppo_split_xmode_groups[2];
extern "C" DPPO_API int dppo_debug_split_xmode(unsigned* out, int reset) {
    DPPO_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(dppo_split_xmode_groups), sizeof(unsigned) * 2));
    if (reset) {
        unsigned z[2] = {};
        DPPO_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dppo_split_xmode_groups), z, sizeof(z)));
    }
    return DPPO_OK;
}
extern "C" DPPO_API int dppo_debug_split_cycles(unsigned long long* out, int reset) {
    DPPO_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(dppo_split_cycles), sizeof(unsigned long long) * (16 + 64 * 8)));
    if (reset) {
        unsigned long long z[16 + 64 * 8] = {};
        DPPO_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dppo_split_cycles), z, sizeof(z)));
    }
    return DPPO_OK;
}
#else
#define XPHASE(k) do {} while (0)
#define XPHASE_START do {} while (0)
#define XSTEP(i) do {} while (0)
#endif

// Host hand-off of a pipelined step (DPPO_SPLIT_SIGNAL, tuning knob):
//   0: acquire poll of go per iteration; plain output stores; __threadfence_system() + release add
//   1: relaxed poll of go + one system acquire after it matches
//   2: 1 + the launch's device outputs stored write-through (sc1), so the final system release
//      has no dirty L2 lines to write back
#ifndef DPPO_SPLIT_SIGNAL
#define DPPO_SPLIT_SIGNAL 2
#endif

// exchange sweeps in flight per wave (DPPO_SPLIT_POLL, tuning knob): 1 = load, check, repeat;
// 2 = the next sweep is issued before the previous one is checked. Measured: 2 is SLOWER (81 vs
// 67 us per launch): the extra polls queue in front of the granules' own arrival at the consumer.
// DPPO_SPLIT_POLL_SLEEP > 0 inserts s_sleep(N) between serial sweeps
#ifndef DPPO_SPLIT_POLL
#define DPPO_SPLIT_POLL 1
#endif
// timing probes (tools/variant_build.sh ... -DDPPO_PROBE_NOSYNC=k, results wrong): drop barrier k of a
// folded-kernel step (1 in-Dense, 2 partial sums, 3 step end)
#ifndef DPPO_PROBE_NOSYNC
#define DPPO_PROBE_NOSYNC 0
#endif
#ifndef DPPO_SPLIT_POLL_SLEEP
#define DPPO_SPLIT_POLL_SLEEP 0
#endif

namespace {

// a store of a kernel output that leaves no dirty line in L2 (write-through; see DPPO_SPLIT_SIGNAL)
__device__ inline void store_out(float* p, float v) {
#if DPPO_SPLIT_SIGNAL >= 2
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    *p = v;
#endif
}

constexpr int SW = 8;              // waves per workgroup
constexpr int SPLIT_P = 8;         // workgroups (CUs) per 16-env group
constexpr int SPLIT_H = 512;       // actor hidden width the split layout is built for
constexpr int XMAX_NV = 16 * 32;   // granules per member per step at XD <= 32
constexpr int XMAX_G = 32;         // groups per launch (512 envs): 8*P*G/8 = 256 workgroups

constexpr size_t XREGION = (size_t)2 * XMAX_G * SPLIT_P * XMAX_NV;   // granules of one exchange region
// after the 9 exchange regions: the XCD announcements [XMAX_G * SPLIT_P], then the dual-set x
// hand-off [XMAX_G][XMAX_NV]
constexpr size_t XANN = 9 * XREGION;
constexpr size_t XHOFF = XANN + (size_t)XMAX_G * SPLIT_P;
constexpr size_t XTOTAL = XHOFF + (size_t)XMAX_G * XMAX_NV;

struct SplitArgs {
    SampleArgs a;
    uint64_t* xbuf;   // shared (sc1) region [2 slots][G][P][NV], then 8 XCD-owned (sc0) regions of
                      // XREGION granules each, then the XCD announcements [XMAX_G][P]
    uint32_t seq;     // launch sequence number (tag high bits)
    int G;            // 16-env groups
    int force_shared; // DPPO_SPLIT_XCHG=shared: always the placement-independent sc1 form (A/B knob)
    uint32_t* xfail_host;  // mapped host word: set by a launch whose exchange timed out (lost
                           // co-residency); the next launch on the stream reports it as an error
    int dual;         // P = 4 kernel: the base actor's steps and the fine-tuned actor's steps run on
                      // two member sets, each with its actor resident for the whole launch
};

__device__ inline int xcc_id() {
    int x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x;
}

// one k-slot -> feature map of the transposed-result lane order: slot (j, e) of a 32-wide
// k-step holds feature e < 4 ? 4j + e : 16 + 4j + (e - 4)
__device__ inline int slot_feature(int j, int e) { return e < 4 ? 4 * j + e : 16 + 4 * j + (e - 4); }


// tuning knobs of the split kernel (tools/variant_build.sh <tag> "-D..." + tools/ab_variants.sh)
#ifndef DPPO_S4_L1D
#define DPPO_S4_L1D 4        // l1: u1 fragment reads kept in flight ahead of the MFMA chain
#endif
#ifndef DPPO_S4_INREADY
#define DPPO_S4_INREADY 1    // in-Dense: all LDS operands in one round trip
#endif
#ifndef DPPO_S4_PUBREADY
#define DPPO_S4_PUBREADY 1   // publish: the 8 wave partials in one round trip
#endif
#ifndef DPPO_S4_EPIEARLY
#define DPPO_S4_EPIEARLY 1   // epilogue inputs read at the step start (else after the publish)
#endif

// relu as one v_max_i32 on the bits (fmaxf(x, 0) canonicalises its MFMA-produced input first: two
// VALU ops per element); negative values and -0 map to +0, as fmaxf(x, 0) does up to the sign of 0
__device__ inline float relu_f(float x) { return __int_as_float(max(__float_as_int(x), 0)); }
// LDS_READY(...): an empty asm statement that "uses" its operands: every one of them is loaded
// before it, so their loads issue together and pay one LDS round trip (left alone, hipcc sank each
// read next to its use)

template <int CTRL>
__device__ inline float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

// XQ = XD / 4 (compile time: the sweep's loads must all be in flight before the first wait)
// Pol: the 2-byte operand policy (PolicyBF16, or PolicyF16 for BASELINE config 5)
template <class Pol, int P, int XQ, int KSI, bool INJ>
__global__ __launch_bounds__(SW * 64) void sample_split_kernel(SplitArgs sa) {
    constexpr int NO = (4 * XQ + 15) / 16;
    using AT = typename Pol::AT;
    auto pack_bf16x2 = [](float lo, float hi) { return Pol::pack2(lo, hi); };
    constexpr int H = SPLIT_H, NTH = H / 16, KSH = H / 32;
    constexpr int NT1 = NTH / P;           // l1 n-tiles per member
    constexpr int KP = SW / NT1;           // l1 K-parts (waves per l1 n-tile)
    constexpr int KS1 = KSH / KP;          // l1 k-steps per wave
    constexpr int HS = H / P;              // features per member slice
    constexpr int KS2 = HS / 32;           // l2 k-steps per member
    constexpr int NOC = 16 * NO;
    constexpr int ST = SW * 64;
    static_assert(NT1 * KP == SW && KS2 >= 1 && 4 * SW == NTH, "split geometry");
    constexpr int pad = 16;                // bf16 elements (32 B) of row padding
    constexpr int ldh = H + pad;           // u1 row stride (bf16)
    constexpr int lda0 = KSI * 32 + pad;   // a0 row stride (bf16)
    constexpr int ldp = HS + 4;            // l1 partial row stride (fp32)
    static_assert(P == 8, "the member sum is a 3-level lane butterfly");

    const SampleArgs& a = sa.a;
    const int b = blockIdx.x;
    const int g = (b / (8 * P)) * 8 + b % 8, c = (b / 8) % P;
    if (g >= sa.G) return;                 // whole workgroup: no barrier is skipped
    XPHASE_START;
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int row0 = g * 16;
    const MlpLayout& L = a.L;
    constexpr int XD = 4 * XQ;
    const int SD = a.SD, TD = a.TD, K = a.K, KF = a.KF;
    constexpr int NV = 16 * XD;            // coordinates of a 16-env eps block
    constexpr int NVW = NV / SW;           // per wave: 2 XD (a multiple of 8)
    constexpr int KW = XQ;                 // sweep loads per lane: NVW * P / 64 = XD / 4

    // ---- LDS carve (all offsets multiples of 16 B) ----
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    size_t o = 0;
    AT* a0 = (AT*)(smem + o); o += dppo_align16(2 * 16 * lda0);
    AT* u1 = (AT*)(smem + o); o += dppo_align16(2 * 16 * ldh);
    float* p1 = (float*)(smem + o); o += dppo_align16(4 * KP * 16 * ldp);
    float* part = (float*)(smem + o); o += dppo_align16(4 * SW * NV);      // [wave][16 x XD]
    int* xfail = (int*)(smem + o); o += 16;                // [0] exchange failure, [1] exchange mode
    float* xs = (float*)(smem + o); o += dppo_align16(4 * 16 * XD);
    float* st = (float*)(smem + o); o += dppo_align16(4 * 16 * SD);
    float* temb = (float*)(smem + o); o += dppo_align16(4 * K * TD);
    float* sch = (float*)(smem + o); o += dppo_align16(4 * K * DPPO_SCHED_COLS);
    float* bias = (float*)(smem + o); o += dppo_align16(4 * 2 * (3 * H + NOC));
    float* zt = (float*)(smem + o); o += dppo_align16(4 * K * 16 * XD);
    u32x4* stage = (u32x4*)(smem + o); o += (size_t)SW * 2 * NO * 1024;

    // ---- resident weight fragments (one actor at a time) ----
    const __amdgpu_buffer_rsrc_t rs_base = packed_rsrc(a.packed_base), rs_ft = packed_rsrc(a.packed_ft);
    auto W = [&](int ft, int seg) { return wsrc(ft ? rs_ft : rs_base, L.off[seg]); };
    const int t1 = wave % NT1, kp = wave / NT1;
    u32x4 rin[KSI][4], rl1[KS1], rl2[KS2][4], rout[2][NO];
    auto load_in = [&](int ft) {
#pragma unroll
        for (int ks = 0; ks < KSI; ++ks)
#pragma unroll
            for (int n = 0; n < 4; ++n) rin[ks][n] = load_bfrag_c(W(ft, SEG_W_IN), KSI, 4 * wave + n, ks, lane);
    };
    auto load_l1 = [&](int ft) {
#pragma unroll
        for (int j = 0; j < KS1; ++j) rl1[j] = load_bfrag_c(W(ft, SEG_W_L1), KSH, NT1 * c + t1, kp * KS1 + j, lane);
    };
    auto load_l2 = [&](int ft) {
#pragma unroll
        for (int s = 0; s < KS2; ++s)
#pragma unroll
            for (int n = 0; n < 4; ++n) rl2[s][n] = load_bfrag_c(W(ft, SEG_W_L2), KSH, 4 * wave + n, c * KS2 + s, lane);
    };
    auto load_out = [&](int ft) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int n = 0; n < NO; ++n) rout[s][n] = load_bfrag_c(W(ft, SEG_W_OUT), KSH, n, 2 * wave + s, lane);
    };
    // re-order the out-Dense fragments to the transposed-result k-slot order (slot_feature), once
    // per actor, through this wave's own LDS staging area (one wave's LDS ops complete in order)
    auto permute_out = [&]() {
        u32x4* stg = stage + wave * 2 * NO * 64;
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int n = 0; n < NO; ++n) stg[(s * NO + n) * 64 + lane] = rout[s][n];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int j = lane >> 4, q = lane & 15;
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int n = 0; n < NO; ++n) {
                const uint16_t* src = (const uint16_t*)(stg + (s * NO + n) * 64);
                uint32_t w[4];
#pragma unroll
                for (int e2 = 0; e2 < 4; ++e2) {
                    const int f0 = slot_feature(j, 2 * e2), f1 = slot_feature(j, 2 * e2 + 1);
                    const uint32_t lo = src[(16 * (f0 >> 3) + q) * 8 + (f0 & 7)];
                    const uint32_t hi = src[(16 * (f1 >> 3) + q) * 8 + (f1 & 7)];
                    w[e2] = lo | (hi << 16);
                }
                rout[s][n] = u32x4{w[0], w[1], w[2], w[3]};
            }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };

    // announce this member's XCD (sc1 granule, tag = seq << 6: step tags are seq << 6 | i + 1)
    uint64_t* const xann = sa.xbuf + XANN + (size_t)g * P;
    const uint32_t ann_tag = sa.seq << 6;
    if (tid == 0)
        __hip_atomic_store(xann + c, ((uint64_t)ann_tag << 32) | (uint32_t)xcc_id(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    const int ft0 = __builtin_amdgcn_readfirstlane(K - 1 < KF ? 1 : 0);
    load_in(ft0); load_l1(ft0); load_l2(ft0); load_out(ft0);
    int cur = ft0;

    // ---- prologue: biases, time embeddings, schedule, noise (as sampler.hip) ----
    const int NB4 = 2 * (3 * H + NOC) / 4;
    auto bias_src = [&](int i4) {
        const int w = i4 / ((3 * H + NOC) / 4), j = 4 * (i4 % ((3 * H + NOC) / 4));
        const uint8_t* PK = w ? a.packed_ft : a.packed_base;
        const int seg = j < H ? SEG_B_IN : (j < 2 * H ? SEG_B_L1 : (j < 3 * H ? SEG_B_L2 : SEG_B_OUT));
        const int jj = j < 3 * H ? j % H : j - 3 * H;
        return (const float4*)(PK + L.off[seg]) + jj / 4;
    };
    for (int i4 = tid; i4 < NB4; i4 += ST) ((float4*)bias)[i4] = *bias_src(i4);
    for (int i = tid; i < K * TD; i += ST)
        temb[i] = ((const float*)((i / TD < KF ? a.packed_ft : a.packed_base) + L.off[SEG_TEMB]))[i];
    for (int i = tid; i < K * DPPO_SCHED_COLS; i += ST) sch[i] = a.sched[i];
    const int XG = (XD + 3) / 4;
    for (int it = tid; it < (K + 1) * 16 * XG; it += ST) {
        const int step = it / (16 * XG), r = (it / XG) % 16, gq = it % XG, row = row0 + r;
        float z[4];
        if (step == K && a.x_T) {
#pragma unroll
            for (int k = 0; k < 4; ++k) z[k] = (row < a.E && 4 * gq + k < XD) ? a.x_T[(size_t)row * XD + 4 * gq + k] : 0.f;
        } else if (INJ && step < K) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                z[k] = (row < a.E && 4 * gq + k < XD) ? a.noise[((size_t)step * a.E + row) * XD + 4 * gq + k] : 0.f;
        } else {
            philox_normal4(a.seed, (uint32_t)gq, (uint32_t)(a.env_offset + row), (uint32_t)step, a.call_id, z);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int q = 4 * gq + k;
            if (q >= XD) break;
            if (step < K) {
                zt[(step * 16 + r) * XD + q] = fminf(fmaxf(z[k], -a.randn_clip), a.randn_clip);
            } else {
                xs[r * XD + q] = z[k];
                if (KF == K && c == 0 && a.chains && row < a.E) store_out(a.chains + ((size_t)row * (KF + 1) + 0) * XD + q, z[k]);
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);                     // vmcnt(0): the resident set has landed
    permute_out();
    // the group's exchange mode from the members' announcements (bounded like the exchange): every
    // member sees the same P words, so all agree; a timeout selects the placement-independent form
    if (wave == 0) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 10000000ull;   // 100 ms
        uint64_t v = ((uint64_t)ann_tag << 32);
        bool ok = false;
        for (;;) {
            if (lane < P) v = __hip_atomic_load(xann + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__all(lane >= P || (uint32_t)(v >> 32) == ann_tag)) { ok = true; break; }
            if (__builtin_amdgcn_s_memrealtime() > t_end) break;
        }
        const int x0 = __builtin_amdgcn_readfirstlane((int)(uint32_t)v);
        const bool one_xcd = ok && !sa.force_shared && __all(lane >= P || (int)(uint32_t)v == x0);
        if (lane == 0) xfail[1] = one_xcd ? 1 + x0 : 0;
#ifdef DPPO_SAMPLER_TIMING
        if (lane == 0 && c == 0) atomicAdd(&dppo_split_xmode_groups[one_xcd ? 1 : 0], 1u);
#endif
    }
    // pre-enqueued rollout step: wait for the host's observation (bounded, as sampler.hip)
    // everything that does not need the observation is done before its wait: a0's x / temb /
    // padding columns and the exchange-failure flag (xs, x_T, comes from the noise loop above)
    __syncthreads();
    const int k1w = KSI * 32;
    for (int idx = tid; idx < 16 * k1w; idx += ST) {
        const int r = idx / k1w, cc = idx % k1w;
        if (cc >= XD + TD && cc < a.IN) continue;              // state columns: after the wait
        const float v = cc < XD ? xs[r * XD + cc] : (cc < XD + TD ? temb[(K - 1) * TD + cc - XD] : 0.f);
        a0[r * lda0 + cc] = Pol::cvt(v);
    }
    if (tid == 0) *xfail = 0;
    XPHASE(7);                                              // timing builds: phase 7 = prologue before the wait
    // after the wait each thread writes the state columns of the entries it read itself (the tagged
    // load and the go path map entry i to thread i mod ST), so one barrier ends the prologue
    if (a.cond_tagged) {
        sampler_load_state_tagged<ST>(a, row0, st, c == 0, tid);
        XPHASE(8);                                          // phase 8 = the wait for the tagged observation
        for (int i = tid; i < 16 * SD; i += ST) {
            const int r = i / SD, cc = i % SD, row = row0 + r;
            a0[r * lda0 + XD + TD + cc] = Pol::cvt(st[i]);
            if (a.cond_out && c == 0 && row < a.E) store_out(a.cond_out + (size_t)row * SD + cc, st[i]);
        }
    } else {
        if (a.go) {
            if (tid == 0) {
                const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 400000000ull;   // 100 MHz: 4 s
#if DPPO_SPLIT_SIGNAL >= 1
                while (__hip_atomic_load(a.go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < a.go_value) {
#else
                while (__hip_atomic_load(a.go, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < a.go_value) {
#endif
                    __builtin_amdgcn_s_sleep(8);
                    if (__builtin_amdgcn_s_memrealtime() > t_end) {
                        if (c == 0) __hip_atomic_fetch_or(a.done, 0x80000000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        break;
                    }
                }
#if DPPO_SPLIT_SIGNAL >= 1
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");    // one system acquire after the match
#endif
            }
            __syncthreads();
        }
        XPHASE(8);                                              // phase 8 = the wait for go
        for (int i = tid; i < 16 * SD; i += ST) {
            const int r = i / SD, cc = i % SD, row = row0 + r;
            const float v = row < a.E ? a.cond[(size_t)row * SD + cc] : 0.f;
            st[i] = v;
            a0[r * lda0 + XD + TD + cc] = Pol::cvt(v);
            if (a.cond_out && c == 0 && row < a.E) store_out(a.cond_out + (size_t)row * SD + cc, v);
        }
    }
    __syncthreads();
    const int env = lane & 15, jq = lane >> 4;
    // exchange region of this group: its XCD's own (L2-local, sc0 stores) or the shared one (sc1)
    const int xmode = __builtin_amdgcn_readfirstlane(xfail[1]);
    uint64_t* const xregion = sa.xbuf + (size_t)xmode * XREGION;
    XPHASE(0);
    for (int i = 0; i < K; ++i) {
        XSTEP(i);
        const int t = K - 1 - i;
        const int PK = __builtin_amdgcn_readfirstlane(t < KF ? 1 : 0);
        // the actor switch (t = K'-1, once per launch): the step before reloaded each layer's
        // fragments right after their last use, so only the out-Dense re-order is left here
        const int PKn = __builtin_amdgcn_readfirstlane(t >= 1 && t - 1 < KF ? 1 : 0);
        const bool pre = t >= 1 && PKn != PK;             // this step is the last of its actor
        if (PK != cur) {
            __builtin_amdgcn_s_waitcnt(0x0F70);
            permute_out();
            cur = PK;
        }
        XPHASE(1);
        const float* bb = bias + PK * (3 * H + NOC);
        // ---- in-Dense (transposed): h1 features 16(4w+n) + 4jq + r of env; no activation (mlp.py:144)
        f32x4 h1[4];
        {
            u32x4 af[KSI];
#pragma unroll
            for (int ks = 0; ks < KSI; ++ks) af[ks] = lds_afrag<Pol>(a0, lda0, 0, ks, lane);
            // this wave's in-Dense and l2 biases, read with the fragments (not between the chains)
            f32x4 bin[4], bl2[4];
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                bin[n] = *(const f32x4*)(bb + 16 * (4 * wave + n) + 4 * jq);
                bl2[n] = *(const f32x4*)(bb + 2 * H + 16 * (4 * wave + n) + 4 * jq);
            }
            // k-step outer: four independent accumulator chains in flight (n-outer made hipcc
            // finish each tile's chain and its relu/pack/store before issuing the next)
#pragma unroll
            for (int n = 0; n < 4; ++n) zero_acc(h1[n]);
#pragma unroll
            for (int ks = 0; ks < KSI; ++ks)
#pragma unroll
                for (int n = 0; n < 4; ++n) h1[n] = Pol::mma(rin[ks][n], af[ks], h1[n]);
            if (pre) load_in(PKn);
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const int f = 16 * (4 * wave + n) + 4 * jq;
                h1[n] += bin[n];
                u32x2 pk;
                pk[0] = pack_bf16x2(fmaxf(h1[n][0], 0.f), fmaxf(h1[n][1], 0.f));
                pk[1] = pack_bf16x2(fmaxf(h1[n][2], 0.f), fmaxf(h1[n][3], 0.f));
                *(u32x2*)(u1 + env * ldh + f) = pk;
            }
            // the residual term member 0 adds to its l2 partial: h1 + b_l2 (mlp.py:206)
#pragma unroll
            for (int n = 0; n < 4; ++n) h1[n] += bl2[n];
        }
        XPHASE(11);
        lds_sync();
        XPHASE(2);
        // ---- l1 (transposed): this member's output columns, K split over KP waves
        {
            f32x4 acc0, acc1;
            zero_acc(acc0); zero_acc(acc1);
            const f32x4 bl1 = *(const f32x4*)(bb + H + HS * c + 16 * t1 + 4 * jq);
            u32x4 bfr[KS1];                    // every fragment read in flight before the chains
#pragma unroll
            for (int j = 0; j < KS1; ++j) bfr[j] = lds_afrag<Pol>(u1, ldh, 0, kp * KS1 + j, lane);
#pragma unroll
            for (int j = 0; j < KS1; ++j) {
                if (j & 1) acc1 = Pol::mma(rl1[j], bfr[j], acc1);
                else acc0 = Pol::mma(rl1[j], bfr[j], acc0);
            }
            if (pre) load_l1(PKn);
            f32x4 s = acc0 + acc1;
            if (kp == 0) s += bl1;                 // the l1 bias rides on K-part 0
            *(f32x4*)(p1 + (kp * 16 + env) * ldp + 16 * t1 + 4 * jq) = s;
        }
        XPHASE(12);
        lds_sync();
        XPHASE(3);
        // ---- l2 (transposed) over this member's K-slice: u2 = bf16 relu(h2 + b_l1) (mlp.py:202-206)
        f32x4 h3[4];
        {
            u32x4 u2[KS2];
#pragma unroll
            for (int s = 0; s < KS2; ++s) {
                const int k0 = 32 * s + 8 * jq;
                f32x4 v0 = *(const f32x4*)(p1 + env * ldp + k0);          // K-part 0 (+ bias)
                f32x4 v1 = *(const f32x4*)(p1 + env * ldp + k0 + 4);
#pragma unroll
                for (int q = 1; q < KP; ++q) {
                    v0 += *(const f32x4*)(p1 + (q * 16 + env) * ldp + k0);
                    v1 += *(const f32x4*)(p1 + (q * 16 + env) * ldp + k0 + 4);
                }
                u2[s] = u32x4{pack_bf16x2(fmaxf(v0[0], 0.f), fmaxf(v0[1], 0.f)),
                              pack_bf16x2(fmaxf(v0[2], 0.f), fmaxf(v0[3], 0.f)),
                              pack_bf16x2(fmaxf(v1[0], 0.f), fmaxf(v1[1], 0.f)),
                              pack_bf16x2(fmaxf(v1[2], 0.f), fmaxf(v1[3], 0.f))};
            }
#pragma unroll
            for (int n = 0; n < 4; ++n) zero_acc(h3[n]);
#pragma unroll
            for (int s = 0; s < KS2; ++s)
#pragma unroll
                for (int n = 0; n < 4; ++n) h3[n] = Pol::mma(rl2[s][n], u2[s], h3[n]);
            if (pre) load_l2(PKn);
            if (c == 0) {                                    // + b_l2 + h1 (residual), once per group
#pragma unroll
                for (int n = 0; n < 4; ++n) h3[n] += h1[n];
            }
        }
        XPHASE(13);
        // ---- out-Dense partial (transposed) from this wave's own h3 registers: k-step s covers
        //      h3 tiles 2s, 2s+1 in slot_feature order; hi/lo bf16 split keeps h3 fp32-accurate
        {
            f32x4 po[NO], pl[NO];              // hi and lo products: two independent chains
#pragma unroll
            for (int n = 0; n < NO; ++n) { zero_acc(po[n]); zero_acc(pl[n]); }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                float hv[8];
#pragma unroll
                for (int e = 0; e < 4; ++e) { hv[e] = h3[2 * s][e]; hv[4 + e] = h3[2 * s + 1][e]; }
                u32x4 hi, lo;
#pragma unroll
                for (int e2 = 0; e2 < 4; ++e2) {
                    const float x0 = hv[2 * e2], x1 = hv[2 * e2 + 1];
                    hi[e2] = pack_bf16x2(x0, x1);
                    const float r0 = Pol::lo2f(hi[e2]), r1 = Pol::hi2f(hi[e2]);
                    lo[e2] = pack_bf16x2(x0 - r0, x1 - r1);
                }
#pragma unroll
                for (int n = 0; n < NO; ++n) {
                    po[n] = Pol::mma(rout[s][n], hi, po[n]);
                    pl[n] = Pol::mma(rout[s][n], lo, pl[n]);
                }
            }
#pragma unroll
            for (int n = 0; n < NO; ++n) po[n] += pl[n];
            if (pre) load_out(PKn);
#pragma unroll
            for (int n = 0; n < NO; ++n)
                if (16 * n + 4 * jq < XD) *(f32x4*)(part + wave * NV + env * XD + 16 * n + 4 * jq) = po[n];
        }
        XPHASE(14);
        lds_sync();
        XPHASE(4);
        // ---- exchange + DDPM epilogue. Wave w owns coordinates [w*NVW, (w+1)*NVW) of the 16 x XD
        //      eps block: it sums the 8 wave partials of them and publishes that slice, sweeps the
        //      slice from all P members (lane = 8 * slot + member), adds the members with a fixed
        //      xor-butterfly (bit-identical on every member) and runs the fp32 DDPM epilogue
        //      (diffusion_vpg.py:198-243, 301-320) for them. No workgroup barrier in between.
        {
            const uint32_t tag = (sa.seq << 6) | (uint32_t)(i + 1);
            uint64_t* xb = xregion + ((size_t)((i & 1) * sa.G + g) * P) * NV;
            const int vw = wave * NVW;
            if (lane < NVW) {
                float sum = part[vw + lane];
#pragma unroll
                for (int w = 1; w < SW; ++w) sum += part[w * NV + vw + lane];
                const uint64_t gr = ((uint64_t)tag << 32) | __float_as_uint(sum);
                if (xmode)   // one XCD: the line stays in its L2, where the peers' sc1 loads read it
                    __hip_atomic_store(xb + (size_t)c * NV + vw + lane, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                else
                    __hip_atomic_store(xb + (size_t)c * NV + vw + lane, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            XPHASE(15);
            // the next step's time embedding into a0 while the members arrive (a0 was last read by
            // this step's in-Dense, two barriers ago)
            if (t > 0 && lane < 16 * TD / SW) {
                const int e = wave * (16 * TD / SW) + lane, r = e / TD, cc = e % TD;
                a0[r * lda0 + XD + cc] = Pol::cvt(temb[(t - 1) * TD + cc]);
            }
            const int m = lane & 7, sl = lane >> 3;
            // this lane's epilogue inputs, read while the members arrive
            const int ve = vw + sl + 8 * (m < KW ? m : 0), re = ve / XD, qe = ve % XD;
            const float* sc = sch + t * DPPO_SCHED_COLS;
            const float c0 = sc[0], c1 = sc[1], c2 = sc[2], c3 = sc[3];
            float sd = expf(0.5f * sc[4]);
            // eval noise rule of the table row (include/dppo.h: DDPM t = 0 or any DDIM row -> 0;
            // other DDPM rows clip at 1e-3; diffusion_vpg.py:303-315)
            if (a.deterministic && sc[6] != 0.f) sd = 0.f;
            else if (a.deterministic) sd = fminf(fmaxf(sd, sc[5]), 1e6f);
            else sd = fminf(fmaxf(sd, a.min_std), 1e6f);
            const float xe = xs[ve], ze = zt[i * 16 * XD + ve], be = bb[3 * H + qe];
            const uint64_t* src = xb + (size_t)m * NV + vw + sl;
            const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 10000000ull;   // 100 ms
            float val[KW];
            bool failed = false;
            auto poll = [&](uint64_t (&x)[KW]) {
#pragma unroll
                for (int k = 0; k < KW; ++k) x[k] = __hip_atomic_load(src + 8 * k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            };
            auto arrived = [&](const uint64_t (&x)[KW]) {
                bool ok = true;
#pragma unroll
                for (int k = 0; k < KW; ++k) ok &= (uint32_t)(x[k] >> 32) == tag;
                if (!__all(ok)) return false;
#pragma unroll
                for (int k = 0; k < KW; ++k) val[k] = __uint_as_float((uint32_t)x[k]);
                return true;
            };
#if DPPO_SPLIT_POLL >= 2
            // two sweeps in flight: the next is issued before the previous one is checked, so a
            // granule is seen about half an L2 round trip after it lands instead of a whole one
            uint64_t xa[KW], xc[KW];
            poll(xa);
            for (;;) {
                bool got = false;
#pragma unroll 1
                for (int r = 0; r < 16 && !got; ++r) {
                    poll(xc);
                    got = arrived(xa);
                    if (got) break;
                    poll(xa);
                    got = arrived(xc);
                }
                if (got) break;
                if (__builtin_amdgcn_s_memrealtime() > t_end) {
                    failed = true;
                    if (lane == 0) {
                        *xfail = 1;
                        __hip_atomic_store(sa.xfail_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                    break;
                }
            }
#else
            uint64_t xa[KW];
            for (;;) {
                poll(xa);
                if (arrived(xa)) break;
#if DPPO_SPLIT_POLL_SLEEP > 0
                __builtin_amdgcn_s_sleep(DPPO_SPLIT_POLL_SLEEP);
#endif
                if (__builtin_amdgcn_s_memrealtime() > t_end) {
                    failed = true;
                    if (lane == 0) {
                        *xfail = 1;
                        __hip_atomic_store(sa.xfail_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                    break;
                }
            }
#endif
            XPHASE(5);
            // member sum over the 8 lanes of a slot in DPP (no LDS crossbar): xor 1 and xor 2 inside
            // the quad, then the half-row mirror pairs each lane with the other quad. Every lane
            // adds the same two partial sums (a + b == b + a), so all 8 hold the same bits
#pragma unroll
            for (int k = 0; k < KW; ++k) {
                val[k] += dpp_f32<0xB1>(val[k]);     // quad_perm [1,0,3,2]
                val[k] += dpp_f32<0x4E>(val[k]);     // quad_perm [2,3,0,1]
                val[k] += dpp_f32<0x141>(val[k]);    // row_half_mirror
            }
            // lane (slot sl, member m) finishes coordinate sl + 8m when m < KW
            if (m < KW) {
                float ep = val[0];
#pragma unroll
                for (int k = 1; k < KW; ++k) ep = m == k ? val[k] : ep;
                const int v = ve, r = re, q = qe, row = row0 + r;
                ep += be;
                const float x = xe;
                float y = ddpm_post(c0, c1, c2, c3, sd, x, ep, ze);   // (:198-242, :301-320)
                if (a.final_clip > 0.f && i == K - 1) y = fminf(fmaxf(y, -a.final_clip), a.final_clip);
                if (failed) y = __builtin_nanf("");
                xs[v] = y;
                a0[r * lda0 + q] = Pol::cvt(y);
                if (c == 0 && row < a.E) {
                    if (a.chains && t <= KF) store_out(a.chains + ((size_t)row * (KF + 1) + (KF - t)) * XD + q, y);
                    if (i == K - 1) {
                        store_out(a.actions + (size_t)row * XD + q, y);
                        if (a.actions_tagged)   // the action is its own flag: one aligned 8-B store
                            __hip_atomic_store(a.actions_tagged + (size_t)row * XD + q,
                                               ((uint64_t)a.cond_tag << 32) | __float_as_uint(y), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
                        else if (a.actions_host) a.actions_host[(size_t)row * XD + q] = y;
                    }
                }
            }
        }
        lds_sync();
        XPHASE(6);
    }
    XPHASE(9);                                              // phase 9 = loop end -> done signal
    if (c == 0 && a.done) {   // publish: every writer's stores reach the system before the counter moves
        __threadfence_system();
        __syncthreads();
        if (tid == 0) {
            if (*xfail) __hip_atomic_fetch_or(a.done, 0x80000000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_fetch_add(a.done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    XPHASE(10);                                             // phase 10 = the done signal (member 0)
}

// ------------------------------------------------------------------------------------------------
// P = 2 (default) or 4 members per 16-env group (DPPO_SPLIT_P=8 selects the kernel above). Fewer
// members mean a cheaper exchange (tools/xchg_probe2.hip, sc0 one-XCD granules at 16 envs: P = 2
// 0.59 us per step, 4 0.98, 8 1.55) and less arrival skew, for more l1 MFMAs per wave. Member c
// keeps 1/P of l1 in registers (P = 2: 128 of 228 VGPRs), written below for P = 4:
//   in-Dense   W_in rows [x ; state] only (K = XD + SD <= 32 KX); the time part b_in + W_in^T
//              t_emb(t) is the pack step's TIN table (dppo_layout.h), the MFMA accumulator's start
//   l1         output columns [128c, 128c+128): wave w owns n-tile w over ALL 512 inputs, so its
//              result is final (b_l1 is the accumulator's start): a = relu(h2), rounded as the
//              reference's l2 input
//   l2 + out   folded (mlp.py:186-206: the residual block is linear from the l2 product to the
//              out-Dense): eps = W_out^T h1 + M^T a + B_OUT2 with M = W_l2 W_out, packed per actor
//              (SEG_FOLD, hi/lo pairs). The member's partial eps is one MFMA per out tile on the l1
//              result straight from registers (its 4 features per lane are the MFMA's k-slots,
//              repeated against M's hi and lo halves), plus its share of the residual term: the
//              in-Dense tiles w*NTI + r*P + c (h1 hi/lo against SEG_ROUT). No l2 GEMM, no l2
//              weights resident, no LDS round trip or barrier between l1 and the exchange.
// so no wave adds a bias or a residual outside an MFMA, and no wave re-sums l1 partials.
// PM = members per group: 2 (the default, DPPO_S4_P: 1/2 of l1 per member, 2 l1 n-tiles per wave,
// a 2-member exchange; possible once l2 is folded away) or 4
template <class Pol, int XQ, int KX, bool INJ, int SWV, int PM = 4>
__global__ __launch_bounds__(SWV * 64) void sample_split4_kernel(SplitArgs sa) {
    constexpr int P = PM;
    static_assert(P == 2 || P == 4, "members per group");
    constexpr int NO = (4 * XQ + 15) / 16;
    using AT = typename Pol::AT;
    // TWO: 2-byte operands (bf16 / fp16: the fold and residual as hi/lo pairs in one 16x16x32 MFMA); else
    // fp32 (r06, P = 4: the l1 slice is 256 KB of fp32, 128 VGPRs of fragments per lane as bf16's at P = 2;
    // 16x16x4 MFMAs, the fold from RT_FOLD and the residual from W_OUT, exact fp32 operands)
    constexpr bool TWO = sizeof(AT) == 2;
    constexpr int KGP = Pol::KG;
    auto pack_bf16x2 = [](float lo, float hi) {
        if constexpr (TWO) return Pol::pack2(lo, hi);
        else return 0u;
    };
    constexpr int H = SPLIT_H, KSH = H / KGP;
    constexpr int HS = H / P;              // features per member slice (128)
    constexpr int SW = SWV;                // waves per member: 8 (2 per SIMD) or 4 (1 per SIMD)
    constexpr int NTI = 32 / SW;           // in-Dense n-tiles per wave
    constexpr int NL1 = (HS / 16) / SW;    // l1 n-tiles of the member slice per wave
    constexpr int NR = NTI / P;            // in-Dense tiles per wave whose residual term this member adds
    static_assert(NL1 * SW == HS / 16 && NTI * SW == 32 && NTI % P == 0, "split geometry");
    constexpr int NOC = 16 * NO;
    constexpr int ST = SW * 64;
    constexpr int pad = 16;
    constexpr int ldh = H + pad;           // u1 row stride (2-byte elements)
    constexpr int lda0 = KX * KGP + pad;   // a0 row stride
    constexpr int XD = 4 * XQ;
    constexpr int NV = 16 * XD;            // coordinates of a 16-env eps block
    constexpr int NVW = NV / SW;           // per wave: 2 XD
    constexpr int SL = 64 / P;             // sweep slots per wave (lane = P * slot + member)
    constexpr int KW = (NVW + SL - 1) / SL;  // sweep loads per lane
    static_assert(KW <= P, "the finishing lanes are the members' lanes");
    constexpr int NB = H + NOC;            // per-actor bias floats: b_l1 | B_OUT2
    // TIN rows in LDS: all K (hopper's KX = 1), or a 2-row ring refilled one step ahead by LDS-DMA
    // (KX = 2, walker2d / halfcheetah: the K rows' 40 KB on top of the 2-k-step in-Dense fragments
    // would exceed the CU's 160 KB, split4_lds_bytes)
    constexpr bool TRING = KX == 2 || !TWO;

    const SampleArgs& a = sa.a;
    // dual: set 0 runs the base actor's steps (t >= K'), set 1 the fine-tuned actor's (t < K'), each
    // with its actor resident for the whole launch; set 0 hands x to set 1 once. Without it, one
    // set runs every step and reloads the resident fragments at the switch (~5 us per launch)
    const int per_set = 8 * P * ((sa.G + 7) / 8);
    const int set = sa.dual ? (int)blockIdx.x / per_set : 0;
    const int b = (int)blockIdx.x - set * per_set;
    const int g = (b / (8 * P)) * 8 + b % 8, c = (b / 8) % P;
    if (g >= sa.G) return;                 // whole workgroup: no barrier is skipped
    const int gx = g + set * sa.G, GX = sa.G * (sa.dual ? 2 : 1);   // group index in the exchange regions
    XPHASE_START;
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int row0 = g * 16;
    const MlpLayout& L = a.L;
    const int SD = a.SD, K = a.K, KF = a.KF;
    const int KSX = packed_ksteps(XD + SD, KGP);  // k-step stride of the W_XS image
    const int i0 = sa.dual && set == 1 ? K - KF : 0, i1 = sa.dual && set == 0 ? K - KF : K;   // steps of this set

    // ---- LDS carve (all offsets multiples of 16 B) ----
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    size_t o = 0;
    AT* a0 = (AT*)(smem + o); o += dppo_align16(sizeof(AT) * 16 * lda0);
    AT* u1 = (AT*)(smem + o); o += dppo_align16(sizeof(AT) * 16 * ldh);
    float* part = (float*)(smem + o); o += dppo_align16(4 * SW * NV);      // [wave][16 x XD]
    int* xfail = (int*)(smem + o); o += 16;                // [0] exchange failure, [1] exchange mode
    float* xs = (float*)(smem + o); o += dppo_align16(4 * 16 * XD);
    float* st = (float*)(smem + o); o += dppo_align16(4 * 16 * SD);
    float* tin = (float*)(smem + o); o += dppo_align16(4 * (TRING ? 2 : K) * H);
    float* sch = (float*)(smem + o); o += dppo_align16(4 * K * DPPO_SCHED_COLS);
    float* bias = (float*)(smem + o); o += dppo_align16(4 * 2 * NB);
    float* zt = (float*)(smem + o); o += dppo_align16(4 * K * 16 * XD);
    u32x4* wxs = (u32x4*)(smem + o); o += (size_t)SW * NTI * KX * 1024;   // [wave][n][ks] in-Dense fragments
    // TRING: row t of the actor that runs it (fine-tuned below K'), as 2 KB of LDS-DMA by waves 0 and 1
    // (lane l's 16 B at slot + 16 l); waited for by the issuing wave's vmcnt(0) and published by a barrier
    auto tin_dma = [&](int tr, int slot) {
        if (wave < H / 256) {
            const uint8_t* src = (tr < KF ? a.packed_ft : a.packed_base) + L.off[SEG_TIN] + (size_t)tr * H * 4 + 1024 * wave + 16 * lane;
            __builtin_amdgcn_global_load_lds((void*)src, (__attribute__((address_space(3))) void*)(tin + slot * H + 256 * wave), 16, 0, 0);
        }
    };

    // ---- resident weight fragments (one actor at a time): l1 and the folded out-Dense in
    //      registers; the in-Dense fragments in this wave's own LDS ----
    const __amdgpu_buffer_rsrc_t rs_base = packed_rsrc(a.packed_base), rs_ft = packed_rsrc(a.packed_ft);
    auto W = [&](int ft, int seg) { return wsrc(ft ? rs_ft : rs_base, L.off[seg]); };
    u32x4 rl1[NL1][KSH], rfold[NL1][NO], rres[NR][NO];
    // LDS-DMA of one 1 KiB fragment (lane l's 16 B land at dst + 16 l); wave-private destinations,
    // consumed only after this wave's vmcnt(0)
    auto dma_frag = [&](int ft, int seg, int KS, int ntile, int ks, u32x4* dst) {
        const uint8_t* src = (ft ? a.packed_ft : a.packed_base) + L.off[seg] + ((size_t)(ntile * KS + ks) << 10) + 16 * lane;
        __builtin_amdgcn_global_load_lds((void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    };
    auto load_in = [&](int ft) {
#pragma unroll
        for (int ks = 0; ks < KX; ++ks)
#pragma unroll
            for (int n = 0; n < NTI; ++n) dma_frag(ft, SEG_W_XS, KSX, NTI * wave + n, ks, wxs + ((wave * NTI + n) * KX + ks) * 64);
    };
    auto load_l1 = [&](int ft) {
#pragma unroll
        for (int t = 0; t < NL1; ++t)
#pragma unroll
            for (int j = 0; j < KSH; ++j) rl1[t][j] = load_bfrag_c(W(ft, SEG_W_L1), KSH, (HS / 16) * c + NL1 * wave + t, j, lane);
    };
    auto load_fold = [&](int ft) {
        if constexpr (TWO) {   // FOLD / ROUT: [feature tile][out tile] hi/lo fragments
#pragma unroll
            for (int tt = 0; tt < NL1; ++tt)
#pragma unroll
                for (int n = 0; n < NO; ++n) rfold[tt][n] = load_bfrag_c(W(ft, SEG_FOLD), NO, (HS / 16) * c + NL1 * wave + tt, n, lane);
#pragma unroll
            for (int r = 0; r < NR; ++r)
#pragma unroll
                for (int n = 0; n < NO; ++n) rres[r][n] = load_bfrag_c(W(ft, SEG_ROUT), NO, NTI * wave + r * P + c, n, lane);
        } else {               // fp32: M (RT_FOLD) and W_out (W_OUT) as packed [K = H][N = out]: a 16-feature
                               // tile is one k-step
#pragma unroll
            for (int tt = 0; tt < NL1; ++tt)
#pragma unroll
                for (int n = 0; n < NO; ++n) rfold[tt][n] = load_bfrag_c(W(ft, SEG_RT_FOLD), L.ks_h, n, (HS / 16) * c + NL1 * wave + tt, lane);
#pragma unroll
            for (int r = 0; r < NR; ++r)
#pragma unroll
                for (int n = 0; n < NO; ++n) rres[r][n] = load_bfrag_c(W(ft, SEG_W_OUT), L.ks_h, n, NTI * wave + r * P + c, lane);
        }
    };

    // announce this member's XCD (sc1 granule, tag = seq << 6: step tags are seq << 6 | i + 1)
    uint64_t* const xann = sa.xbuf + XANN + (size_t)gx * P;
    const uint32_t ann_tag = sa.seq << 6;
    if (tid == 0)
        __hip_atomic_store(xann + c, ((uint64_t)ann_tag << 32) | (uint32_t)xcc_id(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    const int ft0 = __builtin_amdgcn_readfirstlane(sa.dual ? set : (K - 1 < KF ? 1 : 0));
    load_in(ft0); load_l1(ft0); load_fold(ft0);
    int cur = ft0;

    // ---- prologue: biases, in-Dense time tables, schedule, noise ----
    for (int i4 = tid; i4 < 2 * NB / 4; i4 += ST) {
        const int w = i4 / (NB / 4), j = 4 * (i4 % (NB / 4));
        const uint8_t* PK = w ? a.packed_ft : a.packed_base;
        ((float4*)bias)[i4] = j < H ? *((const float4*)(PK + L.off[SEG_B_L1]) + j / 4)
                                    : *((const float4*)(PK + L.off[SEG_B_OUT2]) + (j - H) / 4);
    }
    // TIN row t of the actor that runs step t (base for t >= K', fine-tuned below)
    if constexpr (TRING) {
        tin_dma(K - 1 - i0, i0 & 1);   // the set's first step; later rows one step ahead
    } else {
        for (int i4 = tid; i4 < K * H / 4; i4 += ST) {
            const int t = 4 * i4 / H;
            ((float4*)tin)[i4] = ((const float4*)((t < KF ? a.packed_ft : a.packed_base) + L.off[SEG_TIN]))[i4];
        }
    }
    // per-step epilogue constants [i][c0 c1 c2 c3 sd]: schedule row t = K-1-i and the noise rule
    // (include/dppo.h: eval DDPM t = 0 or any DDIM row -> 0; other DDPM rows clip at 1e-3; train:
    // min_std; diffusion_vpg.py:303-315)
    for (int i = tid; i < K; i += ST) {
        const float* sc = a.sched + (K - 1 - i) * DPPO_SCHED_COLS;
        float sd = expf(0.5f * sc[4]);
        if (a.deterministic && sc[6] != 0.f) sd = 0.f;
        else if (a.deterministic) sd = fminf(fmaxf(sd, sc[5]), 1e6f);
        else sd = fminf(fmaxf(sd, a.min_std), 1e6f);
        float* e = sch + i * DPPO_SCHED_COLS;
        e[0] = sc[0]; e[1] = sc[1]; e[2] = sc[2]; e[3] = sc[3]; e[4] = sd;
    }
    const int XG = (XD + 3) / 4;
    for (int it = tid; it < (K + 1) * 16 * XG; it += ST) {
        const int step = it / (16 * XG), r = (it / XG) % 16, gq = it % XG, row = row0 + r;
        float z[4];
        if (step == K && a.x_T) {
#pragma unroll
            for (int k = 0; k < 4; ++k) z[k] = (row < a.E && 4 * gq + k < XD) ? a.x_T[(size_t)row * XD + 4 * gq + k] : 0.f;
        } else if (INJ && step < K) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                z[k] = (row < a.E && 4 * gq + k < XD) ? a.noise[((size_t)step * a.E + row) * XD + 4 * gq + k] : 0.f;
        } else {
            philox_normal4(a.seed, (uint32_t)gq, (uint32_t)(a.env_offset + row), (uint32_t)step, a.call_id, z);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int q = 4 * gq + k;
            if (q >= XD) break;
            if (step < K) {
                zt[(step * 16 + r) * XD + q] = fminf(fmaxf(z[k], -a.randn_clip), a.randn_clip);
            } else {
                xs[r * XD + q] = z[k];
                if (KF == K && c == 0 && a.chains && row < a.E) store_out(a.chains + ((size_t)row * (KF + 1) + 0) * XD + q, z[k]);
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);                     // vmcnt(0): the resident set has landed
    // the group's exchange mode from the members' announcements (bounded like the exchange): every
    // member sees the same P words, so all agree; a timeout selects the placement-independent form
    if (wave == 0) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 10000000ull;   // 100 ms
        uint64_t v = ((uint64_t)ann_tag << 32);
        bool ok = false;
        for (;;) {
            if (lane < P) v = __hip_atomic_load(xann + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__all(lane >= P || (uint32_t)(v >> 32) == ann_tag)) { ok = true; break; }
            if (__builtin_amdgcn_s_memrealtime() > t_end) break;
        }
        const int x0 = __builtin_amdgcn_readfirstlane((int)(uint32_t)v);
        const bool one_xcd = ok && !sa.force_shared && __all(lane >= P || (int)(uint32_t)v == x0);
        if (lane == 0) xfail[1] = one_xcd ? 1 + x0 : 0;
#ifdef DPPO_SAMPLER_TIMING
        if (lane == 0 && c == 0) atomicAdd(&dppo_split_xmode_groups[one_xcd ? 1 : 0], 1u);
#endif
    }
    __syncthreads();
    // a0 = [x | state | 0]: everything but the state columns before the observation wait
    constexpr int k1w = KX * KGP;
    for (int idx = tid; idx < 16 * k1w; idx += ST) {
        const int r = idx / k1w, cc = idx % k1w;
        if (cc >= XD && cc < XD + SD) continue;              // state columns: after the wait
        a0[r * lda0 + cc] = Pol::cvt(cc < XD ? xs[r * XD + cc] : 0.f);
    }
    if (tid == 0) *xfail = 0;
    XPHASE(7);
    if (a.cond_tagged) {
        sampler_load_state_tagged<ST>(a, row0, st, c == 0, tid);
        XPHASE(8);
        for (int i = tid; i < 16 * SD; i += ST) {
            const int r = i / SD, cc = i % SD, row = row0 + r;
            a0[r * lda0 + XD + cc] = Pol::cvt(st[i]);
            if (a.cond_out && c == 0 && row < a.E) store_out(a.cond_out + (size_t)row * SD + cc, st[i]);
        }
    } else {
        if (a.go) {
            if (tid == 0) {
                const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 400000000ull;   // 100 MHz: 4 s
                while (__hip_atomic_load(a.go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < a.go_value) {
                    __builtin_amdgcn_s_sleep(8);
                    if (__builtin_amdgcn_s_memrealtime() > t_end) {
                        if (c == 0) __hip_atomic_fetch_or(a.done, 0x80000000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        break;
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");    // one system acquire after the match
            }
            __syncthreads();
        }
        XPHASE(8);
        for (int i = tid; i < 16 * SD; i += ST) {
            const int r = i / SD, cc = i % SD, row = row0 + r;
            const float v = row < a.E ? a.cond[(size_t)row * SD + cc] : 0.f;
            st[i] = v;
            a0[r * lda0 + XD + cc] = Pol::cvt(v);
            if (a.cond_out && c == 0 && row < a.E) store_out(a.cond_out + (size_t)row * SD + cc, v);
        }
    }
    __syncthreads();
    uint64_t* const xh = sa.xbuf + XHOFF + (size_t)g * XMAX_NV;     // dual: x after the base actor's steps
    const uint32_t htag = (sa.seq << 6) | 63u;
    if (sa.dual && set == 1) {
        // the base set waits for the observation first, so this wait is bounded like that one (4 s)
        // plus margin; a timeout leaves x NaN and is flagged like an exchange failure
        if (tid < NV) {
            const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 500000000ull;   // 5 s
            uint64_t v;
            bool ok = true;
            for (;;) {
                v = __hip_atomic_load(xh + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)(v >> 32) == htag) break;
                if (__builtin_amdgcn_s_memrealtime() > t_end) { ok = false; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            xs[tid] = ok ? __uint_as_float((uint32_t)v) : __builtin_nanf("");
            if (!ok) {
                *xfail = 1;
                __hip_atomic_store(sa.xfail_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        __syncthreads();
        for (int idx = tid; idx < NV; idx += ST) a0[(idx / XD) * lda0 + idx % XD] = Pol::cvt(xs[idx]);
        __syncthreads();
    }
    const int env = lane & 15, jq = lane >> 4;
    const int xmode = __builtin_amdgcn_readfirstlane(xfail[1]);
    uint64_t* const xregion = sa.xbuf + (size_t)xmode * XREGION;
    // this lane's exchange/epilogue coordinate (launch-constant): lane (slot sl, member m) finishes
    // coordinate sl + SL m of its wave's slice
    const int xm = lane & (P - 1), xsl = lane / P;
    const bool fin = xm < KW && xsl + SL * xm < NVW;
    const int ve = wave * NVW + (fin ? xsl + SL * xm : 0), re = ve / XD, qe = ve % XD;
    XPHASE(0);
    for (int i = i0; i < i1; ++i) {
        XSTEP(i);
        const int t = K - 1 - i;
        const int PK = __builtin_amdgcn_readfirstlane(sa.dual ? cur : (t < KF ? 1 : 0));
        const int PKn = __builtin_amdgcn_readfirstlane(t >= 1 && t - 1 < KF ? 1 : 0);
        const bool pre = !sa.dual && t >= 1 && PKn != PK;   // this step is the last of its actor
        if (PK != cur) {
            __builtin_amdgcn_s_waitcnt(0x0F70);
            cur = PK;
        }
        XPHASE(1);
        const float* bb = bias + PK * NB;
        // this step's epilogue inputs, read with the in-Dense operands (none depends on this step)
        const f32x4 ec = *(const f32x4*)(sch + i * DPPO_SCHED_COLS);      // c0 c1 c2 c3
        const float esd = sch[i * DPPO_SCHED_COLS + 4];
        const float xe = xs[ve], ze = zt[i * 16 * XD + ve], be = bb[H + qe];
        // ---- in-Dense (transposed): h1 = TIN[t] + W_xs^T [x; state]; no activation (mlp.py:144)
        f32x4 h1[NTI];
        {
            u32x4 af[KX], wf[KX][NTI];
#pragma unroll
            for (int ks = 0; ks < KX; ++ks) af[ks] = lds_afrag<Pol>(a0, lda0, 0, ks, lane);
#pragma unroll
            for (int n = 0; n < NTI; ++n) h1[n] = *(const f32x4*)(tin + (TRING ? (i & 1) : t) * H + 16 * (NTI * wave + n) + 4 * jq);
#pragma unroll
            for (int n = 0; n < NTI; ++n) wf[0][n] = wxs[((wave * NTI + n) * KX + 0) * 64 + lane];
            // one LDS round trip for all of them (KX = 2: the second k-step's operands in a second
            // round trip after the first k-step's MFMAs, which keeps the walker2d form within 256 VGPRs
            // — all at once it spilled the epilogue's output addresses to scratch)
#if DPPO_S4_INREADY
            asm volatile("" ::"v"(af[0]), "v"(h1[0]), "v"(h1[1]), "v"(h1[2]), "v"(h1[3]), "v"(wf[0][0]), "v"(wf[0][1]),
                         "v"(wf[0][2]), "v"(wf[0][3]));
            if constexpr (NTI == 8)
                asm volatile("" ::"v"(h1[NTI - 4]), "v"(h1[NTI - 3]), "v"(h1[NTI - 2]), "v"(h1[NTI - 1]), "v"(wf[0][NTI - 4]),
                             "v"(wf[0][NTI - 3]), "v"(wf[0][NTI - 2]), "v"(wf[0][NTI - 1]));
#endif
#if DPPO_S4_EPIEARLY
            asm volatile("" ::"v"(ec), "v"(esd), "v"(xe), "v"(ze), "v"(be));
#endif
#pragma unroll
            for (int n = 0; n < NTI; ++n) h1[n] = Pol::mma(wf[0][n], af[0], h1[n]);
            if constexpr (KX == 2) {
#pragma unroll
                for (int n = 0; n < NTI; ++n) wf[1][n] = wxs[((wave * NTI + n) * KX + 1) * 64 + lane];
#if DPPO_S4_INREADY
                asm volatile("" ::"v"(af[1]), "v"(wf[1][0]), "v"(wf[1][1]), "v"(wf[1][2]), "v"(wf[1][3]));
                if constexpr (NTI == 8)
                    asm volatile("" ::"v"(wf[1][NTI - 4]), "v"(wf[1][NTI - 3]), "v"(wf[1][NTI - 2]), "v"(wf[1][NTI - 1]));
#endif
#pragma unroll
                for (int n = 0; n < NTI; ++n) h1[n] = Pol::mma(wf[1][n], af[1], h1[n]);
            }
            if (pre) load_in(PKn);
            if constexpr (TRING)   // the next step's row into the other slot (last read in step i - 1)
                if (i + 1 < i1) tin_dma(t - 1, (i + 1) & 1);
#pragma unroll
            for (int n = 0; n < NTI; ++n) {
                const int f = 16 * (NTI * wave + n) + 4 * jq;
                if constexpr (TWO) {
                    u32x2 pk;
                    pk[0] = pack_bf16x2(relu_f(h1[n][0]), relu_f(h1[n][1]));
                    pk[1] = pack_bf16x2(relu_f(h1[n][2]), relu_f(h1[n][3]));
                    *(u32x2*)(u1 + env * ldh + f) = pk;
                } else {
                    *(f32x4*)(u1 + env * ldh + f) = f32x4{relu_f(h1[n][0]), relu_f(h1[n][1]), relu_f(h1[n][2]), relu_f(h1[n][3])};
                }
            }
        }
        // the residual term W_out^T h1 of this member's in-Dense tiles (h1 as a hi/lo pair against
        // ROUT's repeated W_out), issued under the barrier
        f32x4 po[NO];
#pragma unroll
        for (int n = 0; n < NO; ++n) zero_acc(po[n]);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            f32x4 hv = h1[r * P];
#pragma unroll
            for (int q = 1; q < P; ++q)
                if (c == q) hv = h1[r * P + q];
            u32x4 bh;
            if constexpr (TWO) {
                bh[0] = pack_bf16x2(hv[0], hv[1]);
                bh[1] = pack_bf16x2(hv[2], hv[3]);
                bh[2] = pack_bf16x2(hv[0] - Pol::lo2f(bh[0]), hv[1] - Pol::hi2f(bh[0]));
                bh[3] = pack_bf16x2(hv[2] - Pol::lo2f(bh[1]), hv[3] - Pol::hi2f(bh[1]));
            } else {
                bh = __builtin_bit_cast(u32x4, hv);   // h1's 4 features as the k-slots: exact
            }
#pragma unroll
            for (int n = 0; n < NO; ++n) po[n] = Pol::mma(rres[r][n], bh, po[n]);
        }
        XPHASE(11);
#if DPPO_PROBE_NOSYNC != 1   // timing probe only (wrong actions): drop the in-Dense barrier
        lds_sync();
#endif
        XPHASE(2);
        // ---- l1 (transposed): n-tile `wave` of this member's output columns over all 512 inputs,
        //      from b_l1; a = relu(h2) feeds the folded l2 + out-Dense (mlp.py:202-206)
        {
            f32x4 acc[NL1];
#pragma unroll
            for (int tt = 0; tt < NL1; ++tt) acc[tt] = *(const f32x4*)(bb + HS * c + 16 * (NL1 * wave + tt) + 4 * jq);
            u32x4 fb[KSH];
#pragma unroll
            for (int j = 0; j < KSH; ++j) fb[j] = lds_afrag<Pol>(u1, ldh, 0, j, lane);
#pragma unroll
            for (int j = 0; j < KSH; ++j)
#pragma unroll
                for (int tt = 0; tt < NL1; ++tt) acc[tt] = Pol::mma(rl1[tt][j], fb[j], acc[tt]);
            // schedule: the bias and L1D fragment reads first, then one read per MFMA, so L1D reads
            // stay in flight ahead of the chain (left alone, hipcc issued read -> wait -> MFMA)
            constexpr int L1D = DPPO_S4_L1D, MPC = TWO ? 1 : 4;   // hardware MFMAs per Pol::mma
            __builtin_amdgcn_sched_group_barrier(0x100, L1D + NL1, 0);
#pragma unroll
            for (int j = 0; j < KSH - L1D; ++j) {
                __builtin_amdgcn_sched_group_barrier(0x008, NL1 * MPC, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, NL1 * MPC * L1D, 0);
            if (pre) load_l1(PKn);
            // folded l2 + out-Dense: a = relu(h2) rounded once, its 4 features per lane as k-slots
            // 0-3 and again as 4-7, against M's hi and lo halves
#pragma unroll
            for (int tt = 0; tt < NL1; ++tt) {
                u32x4 ba;
                if constexpr (TWO) {
                    ba[0] = pack_bf16x2(relu_f(acc[tt][0]), relu_f(acc[tt][1]));
                    ba[1] = pack_bf16x2(relu_f(acc[tt][2]), relu_f(acc[tt][3]));
                    ba[2] = ba[0];
                    ba[3] = ba[1];
                } else {
                    ba = __builtin_bit_cast(u32x4, f32x4{relu_f(acc[tt][0]), relu_f(acc[tt][1]), relu_f(acc[tt][2]),
                                                         relu_f(acc[tt][3])});
                }
#pragma unroll
                for (int n = 0; n < NO; ++n) po[n] = Pol::mma(rfold[tt][n], ba, po[n]);
            }
            if (pre) load_fold(PKn);
#pragma unroll
            for (int n = 0; n < NO; ++n)
                if (16 * n + 4 * jq < XD) *(f32x4*)(part + wave * NV + env * XD + 16 * n + 4 * jq) = po[n];
        }
        XPHASE(14);
#if DPPO_PROBE_NOSYNC != 2   // timing probe only (wrong actions): drop the partial-sum barrier
        lds_sync();
#endif
        XPHASE(4);
        // ---- exchange + DDPM epilogue (as the P = 8 kernel; lane = P * slot + member, the member
        //      sum is log2 P DPP levels inside the quad)
        {
            const uint32_t tag = (sa.seq << 6) | (uint32_t)(i + 1);
            uint64_t* xb = xregion + ((size_t)((i & 1) * GX + gx) * P) * NV;
            const int vw = wave * NVW;
            if (lane < NVW) {
                float pp[SW];
#pragma unroll
                for (int w = 0; w < SW; ++w) pp[w] = part[w * NV + vw + lane];
#if DPPO_S4_PUBREADY
                asm volatile("" ::"v"(pp[0]), "v"(pp[1]), "v"(pp[2]), "v"(pp[3]));
                if constexpr (SW == 8) asm volatile("" ::"v"(pp[SW - 4]), "v"(pp[SW - 3]), "v"(pp[SW - 2]), "v"(pp[SW - 1]));
#endif
                float sum = pp[0];
#pragma unroll
                for (int w = 1; w < SW; ++w) sum += pp[w];
                const uint64_t gr = ((uint64_t)tag << 32) | __float_as_uint(sum);
                if (xmode)   // one XCD: the line stays in its L2, where the peers' sc1 loads read it
                    __hip_atomic_store(xb + (size_t)c * NV + vw + lane, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                else
                    __hip_atomic_store(xb + (size_t)c * NV + vw + lane, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            XPHASE(15);
            const float c0 = ec[0], c1 = ec[1], c2 = ec[2], c3 = ec[3], sd = esd;
            const int m = xm, sl = xsl;
            const uint64_t* src = xb + (size_t)m * NV + vw;
            const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 10000000ull;   // 100 ms
            float val[KW];
            bool failed = false;
            uint64_t xa[KW];
            for (;;) {
#pragma unroll
                for (int k = 0; k < KW; ++k) {
                    const int v = sl + SL * k < NVW ? sl + SL * k : NVW - 1;   // clamped lanes re-read a valid granule
                    xa[k] = __hip_atomic_load(src + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                bool ok = true;
#pragma unroll
                for (int k = 0; k < KW; ++k) ok &= (uint32_t)(xa[k] >> 32) == tag;
#ifdef DPPO_SPLIT_NOXCHG
                ok = true;   // timing probe only: one sweep, no wait for the peers (wrong actions)
#endif
                if (__all(ok)) break;
                if (__builtin_amdgcn_s_memrealtime() > t_end) {
                    failed = true;
                    if (lane == 0) {
                        *xfail = 1;
                        __hip_atomic_store(sa.xfail_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                    break;
                }
            }
#pragma unroll
            for (int k = 0; k < KW; ++k) val[k] = __uint_as_float((uint32_t)xa[k]);
            // TRING: the next TIN row (issued before the poll's loads, so their vmcnt(0) already covered
            // it) has landed before this wave reaches the step-end barrier
            if constexpr (TRING)
                if (wave < H / 256) __builtin_amdgcn_s_waitcnt(0x0F70);
            XPHASE(5);
            // member sum: xor 1 (then xor 2) inside the quad; every lane adds the same two partial
            // sums, so all P hold the same bits
#pragma unroll
            for (int k = 0; k < KW; ++k) {
                val[k] += dpp_f32<0xB1>(val[k]);     // quad_perm [1,0,3,2]
                if constexpr (P == 4) val[k] += dpp_f32<0x4E>(val[k]);     // quad_perm [2,3,0,1]
            }
            if (fin) {
                float ep = val[0];
#pragma unroll
                for (int k = 1; k < KW; ++k) ep = m == k ? val[k] : ep;
                const int v = ve, r = re, q = qe, row = row0 + r;
                ep += be;
                const float x = xe;
                float y = ddpm_post(c0, c1, c2, c3, sd, x, ep, ze);   // (:198-242, :301-320)
                if (a.final_clip > 0.f && i == K - 1) y = fminf(fmaxf(y, -a.final_clip), a.final_clip);
                if (failed) y = __builtin_nanf("");
                xs[v] = y;
                a0[r * lda0 + q] = Pol::cvt(y);
                if (c == 0 && row < a.E) {
                    if (a.chains && t <= KF) store_out(a.chains + ((size_t)row * (KF + 1) + (KF - t)) * XD + q, y);
                    if (i == K - 1) {
                        store_out(a.actions + (size_t)row * XD + q, y);
                        if (a.actions_tagged)
                            __hip_atomic_store(a.actions_tagged + (size_t)row * XD + q,
                                               ((uint64_t)a.cond_tag << 32) | __float_as_uint(y), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
                        else if (a.actions_host) a.actions_host[(size_t)row * XD + q] = y;
                    }
                }
            }
        }
#if DPPO_PROBE_NOSYNC != 3   // timing probe only (wrong actions): drop the step-end barrier
        lds_sync();
#endif
        XPHASE(6);
    }
    XPHASE(9);
    if (sa.dual && set == 0) {
        // hand x to the fine-tuned set (member 0 of the group: every member holds the same bits)
        if (c == 0 && tid < NV)
            __hip_atomic_store(xh + tid, ((uint64_t)htag << 32) | __float_as_uint(xs[tid]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (c == 0 && tid == 0 && a.done && *xfail)
            __hip_atomic_fetch_or(a.done, 0x80000000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    if (c == 0 && a.done) {
        __threadfence_system();
        __syncthreads();
        if (tid == 0) {
            if (*xfail) __hip_atomic_fetch_or(a.done, 0x80000000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_fetch_add(a.done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    XPHASE(10);
}

// =================================================================================================
// The PAIR kernel (default at >= 32 envs for 2-byte operands when one member set holds one actor):
// the folded 2-member split of sample_split4_kernel, with every member pair running TWO 16-env tiles
// (A, B) half a denoising step apart. Per tile a step is a dependent chain
//     in-Dense -> barrier -> l1 + fold -> barrier -> publish -> [cross-CU exchange] -> epilogue
// whose exchange (an L2 round trip between the 2 CUs, ~0.6 us) left the MFMA pipes idle in the
// one-tile kernel. Here one tile's exchange is in flight while the other tile's l1 runs on the
// same resident weights, in four barrier intervals per step of both tiles:
//     1: publish A(i)  ; in-Dense B(i)
//     2: l1 B(i)       [first poll of A(i) issued half-way through its MFMAs] ; sweep + epilogue A(i)
//     3: publish B(i)  ; in-Dense A(i+1)
//     4: l1 A(i+1)     [first poll of B(i) half-way] ; sweep + epilogue B(i)
// so each exchange overlaps (the other tile's in-Dense + a barrier + its l1). Twice the MFMAs per CU
// per step against no exposed exchange: at 64 envs 8 CUs instead of 16 (4 pairs x 2 members, two
// member sets). Numerics are the one-tile kernel's, operation for operation (same fragments, same
// accumulation order, same fixed member order in the exchange sum): the actions are bit-identical.
// Each member set holds one actor for the whole launch (dual sets, or K' = K / K' = 0).
template <class Pol, int XQ, int KX, bool INJ>
__global__ __launch_bounds__(512) void sample_pair_kernel(SplitArgs sa) {
    constexpr int P = 2, SW = 8;
    constexpr int NO = (4 * XQ + 15) / 16;
    using AT = typename Pol::AT;
    auto pack2 = [](float lo, float hi) { return Pol::pack2(lo, hi); };
    constexpr int H = SPLIT_H, KSH = H / 32, HS = H / P;
    constexpr int NTI = 32 / SW;           // in-Dense n-tiles per wave
    constexpr int NL1 = (HS / 16) / SW;    // l1 n-tiles of the member slice per wave
    constexpr int NR = NTI / P;            // in-Dense tiles per wave whose residual term this member adds
    constexpr int NOC = 16 * NO, ST = SW * 64, pad = 16, ldh = H + pad, lda0 = KX * 32 + pad;
    constexpr int XD = 4 * XQ, NV = 16 * XD, NVW = NV / SW, SL = 64 / P, KW = (NVW + SL - 1) / SL;
    static_assert(KW <= P && NL1 * SW == HS / 16 && NTI % P == 0, "pair geometry");
    constexpr int NB = H + NOC;
    constexpr int L1D = DPPO_S4_L1D;

    const SampleArgs& a = sa.a;
    const int G2 = (sa.G + 1) >> 1;                       // member pairs (two 16-env tiles each)
    const int per_set = 8 * P * ((G2 + 7) / 8);
    const int set = sa.dual ? (int)blockIdx.x / per_set : 0;
    const int b = (int)blockIdx.x - set * per_set;
    const int g2 = (b / (8 * P)) * 8 + b % 8, c = (b / 8) % P;
    if (g2 >= G2) return;                                 // whole workgroup: no barrier is skipped
    const int GT = 2 * G2, GX = GT * (sa.dual ? 2 : 1);   // tile slots of the exchange regions
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const MlpLayout& L = a.L;
    const int SD = a.SD, K = a.K, KF = a.KF;
    const int KSX = packed_ksteps(XD + SD, 32);
    const int i0 = sa.dual && set == 1 ? K - KF : 0, i1 = sa.dual && set == 0 ? K - KF : K;
    const int NS = i1 - i0;
    // the one actor of this set: dual -> set; otherwise K' = K (all fine-tuned) or K' = 0
    const int FT = __builtin_amdgcn_readfirstlane(sa.dual ? set : (KF > 0 ? 1 : 0));
    const int row00 = 32 * g2;

    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    size_t o = 0;
    AT* a0 = (AT*)(smem + o); o += dppo_align16(2 * 2 * 16 * lda0);        // [tile][16][lda0]
    AT* u1 = (AT*)(smem + o); o += dppo_align16(2 * 2 * 16 * ldh);         // [tile][16][ldh]
    float* part = (float*)(smem + o); o += dppo_align16(4 * 2 * SW * NV);  // [tile][wave][16 x XD]
    int* xfail = (int*)(smem + o); o += 16;
    float* xs = (float*)(smem + o); o += dppo_align16(4 * 2 * NV);         // [tile][16 x XD]
    float* st = (float*)(smem + o); o += dppo_align16(4 * 32 * SD);
    float* tin = (float*)(smem + o); o += dppo_align16((size_t)4 * NS * H); // this set's step rows
    float* sch = (float*)(smem + o); o += dppo_align16(4 * K * DPPO_SCHED_COLS);
    float* bias = (float*)(smem + o); o += dppo_align16(4 * NB);
    float* zt = (float*)(smem + o); o += dppo_align16((size_t)4 * 2 * NS * NV);   // [tile][i - i0][NV]
    u32x4* wxs = (u32x4*)(smem + o); o += (size_t)SW * NTI * KX * 1024;

    // ---- the resident set of this set's actor ----
    const __amdgpu_buffer_rsrc_t rs = packed_rsrc(FT ? a.packed_ft : a.packed_base);
    const uint8_t* const PKD = FT ? a.packed_ft : a.packed_base;
    auto W = [&](int seg) { return wsrc(rs, L.off[seg]); };
    u32x4 rl1[NL1][KSH], rfold[NL1][NO], rres[NR][NO];
#pragma unroll
    for (int ks = 0; ks < KX; ++ks)
#pragma unroll
        for (int n = 0; n < NTI; ++n) {
            const uint8_t* src = PKD + L.off[SEG_W_XS] + ((size_t)((NTI * wave + n) * KSX + ks) << 10) + 16 * lane;
            __builtin_amdgcn_global_load_lds((void*)src, (__attribute__((address_space(3))) void*)(wxs + ((wave * NTI + n) * KX + ks) * 64),
                                             16, 0, 0);
        }
#pragma unroll
    for (int t = 0; t < NL1; ++t)
#pragma unroll
        for (int j = 0; j < KSH; ++j) rl1[t][j] = load_bfrag_c(W(SEG_W_L1), KSH, (HS / 16) * c + NL1 * wave + t, j, lane);
#pragma unroll
    for (int tt = 0; tt < NL1; ++tt)
#pragma unroll
        for (int n = 0; n < NO; ++n) rfold[tt][n] = load_bfrag_c(W(SEG_FOLD), NO, (HS / 16) * c + NL1 * wave + tt, n, lane);
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int n = 0; n < NO; ++n) rres[r][n] = load_bfrag_c(W(SEG_ROUT), NO, NTI * wave + r * P + c, n, lane);

    // announce this member's XCD (one announcement per member pair)
    uint64_t* const xann = sa.xbuf + XANN + (size_t)(g2 + set * G2) * P;
    const uint32_t ann_tag = sa.seq << 6;
    if (tid == 0)
        __hip_atomic_store(xann + c, ((uint64_t)ann_tag << 32) | (uint32_t)xcc_id(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);

    // ---- prologue: biases, this set's time rows, schedule, noise ----
    for (int i4 = tid; i4 < NB / 4; i4 += ST) {
        const int j = 4 * i4;
        ((float4*)bias)[i4] = j < H ? *((const float4*)(PKD + L.off[SEG_B_L1]) + j / 4)
                                    : *((const float4*)(PKD + L.off[SEG_B_OUT2]) + (j - H) / 4);
    }
    for (int i4 = tid; i4 < NS * H / 4; i4 += ST) {
        const int r = 4 * i4 / H, t = K - 1 - (i0 + r);
        ((float4*)tin)[i4] = ((const float4*)(PKD + L.off[SEG_TIN]))[t * (H / 4) + i4 % (H / 4)];
    }
    for (int i = tid; i < K; i += ST) {
        const float* sc = a.sched + (K - 1 - i) * DPPO_SCHED_COLS;
        float sd = expf(0.5f * sc[4]);
        if (a.deterministic && sc[6] != 0.f) sd = 0.f;
        else if (a.deterministic) sd = fminf(fmaxf(sd, sc[5]), 1e6f);
        else sd = fminf(fmaxf(sd, a.min_std), 1e6f);
        float* e = sch + i * DPPO_SCHED_COLS;
        e[0] = sc[0]; e[1] = sc[1]; e[2] = sc[2]; e[3] = sc[3]; e[4] = sd;
    }
    const int XG = (XD + 3) / 4;
    const bool need_xT = !(sa.dual && set == 1);
    for (int it = tid; it < (NS + 1) * 32 * XG; it += ST) {
        const int si = it / (32 * XG), rr = (it / XG) % 32, gq = it % XG, row = row00 + rr;
        const int step = si < NS ? i0 + si : K;          // si == NS: x_T (slot K)
        if (step == K && !need_xT) continue;
        float z[4];
        if (step == K && a.x_T) {
#pragma unroll
            for (int k = 0; k < 4; ++k) z[k] = (row < a.E && 4 * gq + k < XD) ? a.x_T[(size_t)row * XD + 4 * gq + k] : 0.f;
        } else if (INJ && step < K) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                z[k] = (row < a.E && 4 * gq + k < XD) ? a.noise[((size_t)step * a.E + row) * XD + 4 * gq + k] : 0.f;
        } else {
            philox_normal4(a.seed, (uint32_t)gq, (uint32_t)(a.env_offset + row), (uint32_t)step, a.call_id, z);
        }
        const int tau = rr >> 4, r = rr & 15;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int q = 4 * gq + k;
            if (q >= XD) break;
            if (step < K) {
                zt[(tau * NS + si) * NV + r * XD + q] = fminf(fmaxf(z[k], -a.randn_clip), a.randn_clip);
            } else {
                xs[tau * NV + r * XD + q] = z[k];
                if (KF == K && c == 0 && a.chains && row < a.E) store_out(a.chains + ((size_t)row * (KF + 1) + 0) * XD + q, z[k]);
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);                     // vmcnt(0): the resident set has landed
    if (wave == 0) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 10000000ull;   // 100 ms
        uint64_t v = ((uint64_t)ann_tag << 32);
        bool ok = false;
        for (;;) {
            if (lane < P) v = __hip_atomic_load(xann + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__all(lane >= P || (uint32_t)(v >> 32) == ann_tag)) { ok = true; break; }
            if (__builtin_amdgcn_s_memrealtime() > t_end) break;
        }
        const int x0 = __builtin_amdgcn_readfirstlane((int)(uint32_t)v);
        const bool one_xcd = ok && !sa.force_shared && __all(lane >= P || (int)(uint32_t)v == x0);
        if (lane == 0) xfail[1] = one_xcd ? 1 + x0 : 0;
    }
    __syncthreads();
    constexpr int k1w = KX * 32;
    for (int idx = tid; idx < 2 * 16 * k1w; idx += ST) {
        const int rr = idx / k1w, cc = idx % k1w, tau = rr >> 4, r = rr & 15;
        if (cc >= XD && cc < XD + SD) continue;              // state columns: after the wait
        a0[(tau * 16 + r) * lda0 + cc] = Pol::cvt(cc < XD ? xs[tau * NV + r * XD + cc] : 0.f);
    }
    if (tid == 0) *xfail = 0;
    if (a.cond_tagged) {
        sampler_load_state_tagged<ST, 32>(a, row00, st, c == 0, tid);
        for (int i = tid; i < 32 * SD; i += ST) {
            const int rr = i / SD, cc = i % SD, row = row00 + rr;
            a0[rr * lda0 + XD + cc] = Pol::cvt(st[i]);
            if (a.cond_out && c == 0 && row < a.E) store_out(a.cond_out + (size_t)row * SD + cc, st[i]);
        }
    } else {
        if (a.go) {
            if (tid == 0) {
                const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 400000000ull;   // 100 MHz: 4 s
                while (__hip_atomic_load(a.go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < a.go_value) {
                    __builtin_amdgcn_s_sleep(8);
                    if (__builtin_amdgcn_s_memrealtime() > t_end) {
                        if (c == 0) __hip_atomic_fetch_or(a.done, 0x80000000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        break;
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            }
            __syncthreads();
        }
        for (int i = tid; i < 32 * SD; i += ST) {
            const int rr = i / SD, cc = i % SD, row = row00 + rr;
            const float v = row < a.E ? a.cond[(size_t)row * SD + cc] : 0.f;
            st[i] = v;
            a0[rr * lda0 + XD + cc] = Pol::cvt(v);
            if (a.cond_out && c == 0 && row < a.E) store_out(a.cond_out + (size_t)row * SD + cc, v);
        }
    }
    __syncthreads();
    const uint32_t htag = (sa.seq << 6) | 63u;
    uint64_t* const xh = sa.xbuf + XHOFF + (size_t)(2 * g2) * XMAX_NV;   // [tile][XMAX_NV]
    if (sa.dual && set == 1) {
        if (tid < 2 * NV) {
            const int tau = tid / NV, v0 = tid % NV;
            const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 500000000ull;   // 5 s
            uint64_t v;
            bool ok = true;
            for (;;) {
                v = __hip_atomic_load(xh + tau * XMAX_NV + v0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)(v >> 32) == htag) break;
                if (__builtin_amdgcn_s_memrealtime() > t_end) { ok = false; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            xs[tid] = ok ? __uint_as_float((uint32_t)v) : __builtin_nanf("");
            if (!ok) {
                *xfail = 1;
                __hip_atomic_store(sa.xfail_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        __syncthreads();
        for (int idx = tid; idx < 2 * NV; idx += ST) {
            const int tau = idx / NV, v0 = idx % NV;
            a0[(tau * 16 + v0 / XD) * lda0 + v0 % XD] = Pol::cvt(xs[idx]);
        }
        __syncthreads();
    }

    const int env = lane & 15, jq = lane >> 4;
    const int xmode = __builtin_amdgcn_readfirstlane(xfail[1]);
    uint64_t* const xregion = sa.xbuf + (size_t)xmode * XREGION;
    const int xm = lane & (P - 1), xsl = lane / P;
    const bool fin = xm < KW && xsl + SL * xm < NVW;
    const int ve = wave * NVW + (fin ? xsl + SL * xm : 0), re = ve / XD, qe = ve % XD;
    const int vw = wave * NVW;
    const float be = bias[H + qe];
    f32x4 po[2][NO];

    // ---- the phases of one tile (tau compile-time: po[] stays in registers) ----
    auto in_dense = [&](auto tauc, int i) {
        constexpr int tau = decltype(tauc)::value;
        const AT* A0 = a0 + tau * 16 * lda0;
        AT* U1 = u1 + tau * 16 * ldh;
        f32x4 h1[NTI];
        u32x4 af[KX], wf[KX][NTI];
#pragma unroll
        for (int ks = 0; ks < KX; ++ks) af[ks] = lds_afrag<Pol>(A0, lda0, 0, ks, lane);
#pragma unroll
        for (int n = 0; n < NTI; ++n) h1[n] = *(const f32x4*)(tin + (i - i0) * H + 16 * (NTI * wave + n) + 4 * jq);
#pragma unroll
        for (int ks = 0; ks < KX; ++ks)
#pragma unroll
            for (int n = 0; n < NTI; ++n) wf[ks][n] = wxs[((wave * NTI + n) * KX + ks) * 64 + lane];
        asm volatile("" ::"v"(af[0]), "v"(h1[0]), "v"(h1[1]), "v"(h1[2]), "v"(h1[3]), "v"(wf[0][0]), "v"(wf[0][1]),
                     "v"(wf[0][2]), "v"(wf[0][3]));
        if constexpr (KX == 2)
            asm volatile("" ::"v"(af[KX - 1]), "v"(wf[KX - 1][0]), "v"(wf[KX - 1][1]), "v"(wf[KX - 1][2]), "v"(wf[KX - 1][3]));
#pragma unroll
        for (int ks = 0; ks < KX; ++ks)
#pragma unroll
            for (int n = 0; n < NTI; ++n) h1[n] = Pol::mma(wf[ks][n], af[ks], h1[n]);
#pragma unroll
        for (int n = 0; n < NTI; ++n) {
            const int f = 16 * (NTI * wave + n) + 4 * jq;
            u32x2 pk;
            pk[0] = pack2(relu_f(h1[n][0]), relu_f(h1[n][1]));
            pk[1] = pack2(relu_f(h1[n][2]), relu_f(h1[n][3]));
            *(u32x2*)(U1 + env * ldh + f) = pk;
        }
#pragma unroll
        for (int n = 0; n < NO; ++n) zero_acc(po[tau][n]);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            f32x4 hv = h1[r * P];
            if (c == 1) hv = h1[r * P + 1];
            u32x4 bh;
            bh[0] = pack2(hv[0], hv[1]);
            bh[1] = pack2(hv[2], hv[3]);
            bh[2] = pack2(hv[0] - Pol::lo2f(bh[0]), hv[1] - Pol::hi2f(bh[0]));
            bh[3] = pack2(hv[2] - Pol::lo2f(bh[1]), hv[3] - Pol::hi2f(bh[1]));
#pragma unroll
            for (int n = 0; n < NO; ++n) po[tau][n] = Pol::mma(rres[r][n], bh, po[tau][n]);
        }
    };
    // the tile's exchange granules of step i: [slot i & 1][tile][member][NV]
    auto xslot = [&](int tau, int i) {
        return xregion + ((size_t)((i & 1) * GX + set * GT + 2 * g2 + tau) * P) * NV;
    };
    // l1 + fold of tile tau; the first poll of tile pt's exchange (step pi) is issued half-way
    // through the MFMA chain (pt < 0: none) and returned in xa
    auto l1_fold = [&](auto tauc, auto ptc, int pi, uint64_t (&xa)[KW]) {
        constexpr int tau = decltype(tauc)::value, pt = decltype(ptc)::value;
        const AT* U1 = u1 + tau * 16 * ldh;
        f32x4 acc[NL1];
#pragma unroll
        for (int tt = 0; tt < NL1; ++tt) acc[tt] = *(const f32x4*)(bias + HS * c + 16 * (NL1 * wave + tt) + 4 * jq);
        u32x4 fb[KSH];
#pragma unroll
        for (int j = 0; j < KSH; ++j) fb[j] = lds_afrag<Pol>(U1, ldh, 0, j, lane);
        if constexpr (pt >= 0) {
            const uint64_t* src = xslot(pt, pi) + (size_t)xm * NV + vw;
#pragma unroll
            for (int k = 0; k < KW; ++k) {
                const int v = xsl + SL * k < NVW ? xsl + SL * k : NVW - 1;
                xa[k] = __hip_atomic_load(src + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
#pragma unroll
        for (int j = 0; j < KSH; ++j)
#pragma unroll
            for (int tt = 0; tt < NL1; ++tt) acc[tt] = Pol::mma(rl1[tt][j], fb[j], acc[tt]);
        __builtin_amdgcn_sched_group_barrier(0x100, L1D + NL1, 0);
#pragma unroll
        for (int j = 0; j < KSH - L1D; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x008, NL1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            if (pt >= 0 && j == (KSH - L1D) / 2) __builtin_amdgcn_sched_group_barrier(0x020, KW, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NL1 * L1D, 0);
#pragma unroll
        for (int tt = 0; tt < NL1; ++tt) {
            u32x4 ba;
            ba[0] = pack2(relu_f(acc[tt][0]), relu_f(acc[tt][1]));
            ba[1] = pack2(relu_f(acc[tt][2]), relu_f(acc[tt][3]));
            ba[2] = ba[0];
            ba[3] = ba[1];
#pragma unroll
            for (int n = 0; n < NO; ++n) po[tau][n] = Pol::mma(rfold[tt][n], ba, po[tau][n]);
        }
        float* PT = part + tau * SW * NV;
#pragma unroll
        for (int n = 0; n < NO; ++n)
            if (16 * n + 4 * jq < XD) *(f32x4*)(PT + wave * NV + env * XD + 16 * n + 4 * jq) = po[tau][n];
    };
    auto publish = [&](int tau, int i) {
        const uint32_t tag = (sa.seq << 6) | (uint32_t)(i + 1);
        uint64_t* xb = xslot(tau, i);
        if (lane < NVW) {
            const float* PT = part + tau * SW * NV;
            float pp[SW];
#pragma unroll
            for (int w = 0; w < SW; ++w) pp[w] = PT[w * NV + vw + lane];
            asm volatile("" ::"v"(pp[0]), "v"(pp[1]), "v"(pp[2]), "v"(pp[3]), "v"(pp[4]), "v"(pp[5]), "v"(pp[6]), "v"(pp[7]));
            float sum = pp[0];
#pragma unroll
            for (int w = 1; w < SW; ++w) sum += pp[w];
            const uint64_t gr = ((uint64_t)tag << 32) | __float_as_uint(sum);
            if (xmode)
                __hip_atomic_store(xb + (size_t)c * NV + vw + lane, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            else
                __hip_atomic_store(xb + (size_t)c * NV + vw + lane, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    // finish tile tau's exchange of step i (xa: the first poll, already issued) and run its epilogue
    auto sweep_epilogue = [&](int tau, int i, uint64_t (&xa)[KW]) {
        const uint32_t tag = (sa.seq << 6) | (uint32_t)(i + 1);
        const uint64_t* src = xslot(tau, i) + (size_t)xm * NV + vw;
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 10000000ull;   // 100 ms
        bool failed = false;
        for (;;) {
            bool ok = true;
#pragma unroll
            for (int k = 0; k < KW; ++k) ok &= (uint32_t)(xa[k] >> 32) == tag;
            if (__all(ok)) break;
            if (__builtin_amdgcn_s_memrealtime() > t_end) {
                failed = true;
                if (lane == 0) {
                    *xfail = 1;
                    __hip_atomic_store(sa.xfail_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                break;
            }
#pragma unroll
            for (int k = 0; k < KW; ++k) {
                const int v = xsl + SL * k < NVW ? xsl + SL * k : NVW - 1;
                xa[k] = __hip_atomic_load(src + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        float val[KW];
#pragma unroll
        for (int k = 0; k < KW; ++k) {
            val[k] = __uint_as_float((uint32_t)xa[k]);
            val[k] += dpp_f32<0xB1>(val[k]);                // member sum: quad_perm [1,0,3,2]
        }
        if (fin) {
            const int t = K - 1 - i;
            const f32x4 ec = *(const f32x4*)(sch + i * DPPO_SCHED_COLS);
            const float sd = sch[i * DPPO_SCHED_COLS + 4];
            float* XS = xs + tau * NV;
            const float x = XS[ve], ze = zt[(tau * NS + (i - i0)) * NV + ve];
            float ep = val[0];
#pragma unroll
            for (int k = 1; k < KW; ++k) ep = xm == k ? val[k] : ep;
            ep += be;
            float y = ddpm_post(ec[0], ec[1], ec[2], ec[3], sd, x, ep, ze);   // (:198-242, :301-320)
            if (a.final_clip > 0.f && i == K - 1) y = fminf(fmaxf(y, -a.final_clip), a.final_clip);
            if (failed) y = __builtin_nanf("");
            XS[ve] = y;
            a0[(tau * 16 + re) * lda0 + qe] = Pol::cvt(y);
            // the row and its output addresses are rebuilt here every step: hoisted out of the step
            // loop, eight 64-bit addresses stayed live across it and spilled to scratch
            int row = row00 + 16 * tau + re;
            asm volatile("" : "+v"(row));
            if (c == 0 && row < a.E) {
                if (a.chains && t <= KF) store_out(a.chains + ((size_t)row * (KF + 1) + (KF - t)) * XD + qe, y);
                if (i == K - 1) {
                    store_out(a.actions + (size_t)row * XD + qe, y);
                    if (a.actions_tagged)
                        __hip_atomic_store(a.actions_tagged + (size_t)row * XD + qe,
                                           ((uint64_t)a.cond_tag << 32) | __float_as_uint(y), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
                    else if (a.actions_host) a.actions_host[(size_t)row * XD + qe] = y;
                }
            }
        }
    };
    using T0 = std::integral_constant<int, 0>;
    using T1 = std::integral_constant<int, 1>;
    using TN = std::integral_constant<int, -1>;
    uint64_t xaA[KW], xaB[KW];
#pragma unroll
    for (int k = 0; k < KW; ++k) xaA[k] = xaB[k] = 0;

    in_dense(T0{}, i0);
    lds_sync();
    l1_fold(T0{}, TN{}, 0, xaB);
    lds_sync();
    for (int i = i0; i < i1; ++i) {
        const bool more = i + 1 < i1;
        publish(0, i);                       // 1: publish A(i) ; in-Dense B(i)
        in_dense(T1{}, i);
        lds_sync();
        l1_fold(T1{}, T0{}, i, xaA);         // 2: l1 B(i) [poll A(i)] ; epilogue A(i)
        sweep_epilogue(0, i, xaA);
        lds_sync();
        publish(1, i);                       // 3: publish B(i) ; in-Dense A(i+1)
        if (more) in_dense(T0{}, i + 1);
        lds_sync();
        if (more) {                          // 4: l1 A(i+1) [poll B(i)] ; epilogue B(i)
            l1_fold(T0{}, T1{}, i, xaB);
        } else {
            const uint64_t* src = xslot(1, i) + (size_t)xm * NV + vw;
#pragma unroll
            for (int k = 0; k < KW; ++k) {
                const int v = xsl + SL * k < NVW ? xsl + SL * k : NVW - 1;
                xaB[k] = __hip_atomic_load(src + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        sweep_epilogue(1, i, xaB);
        lds_sync();
    }
    const int nreal = (row00 < a.E ? 1 : 0) + (row00 + 16 < a.E ? 1 : 0);   // 16-env tiles with envs
    if (sa.dual && set == 0) {
        if (c == 0 && tid < 2 * NV)
            __hip_atomic_store(xh + (tid / NV) * XMAX_NV + tid % NV, ((uint64_t)htag << 32) | __float_as_uint(xs[tid]),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (c == 0 && tid == 0 && a.done && *xfail)
            __hip_atomic_fetch_or(a.done, 0x80000000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    if (c == 0 && a.done) {
        __threadfence_system();
        __syncthreads();
        if (tid == 0) {
            if (*xfail) __hip_atomic_fetch_or(a.done, 0x80000000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_fetch_add(a.done, (uint32_t)nreal, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

size_t pair_lds_bytes(int XD, int SD, int K, int NS, int KX, int NO) {
    const int pad = 16, ldh = SPLIT_H + pad, lda0 = KX * 32 + pad, NV = 16 * XD;
    size_t o = 0;
    o += dppo_align16(2 * 2 * 16 * lda0);
    o += dppo_align16(2 * 2 * 16 * ldh);
    o += dppo_align16(4 * 2 * 8 * NV);
    o += 16;
    o += dppo_align16(4 * 2 * NV);
    o += dppo_align16(4 * 32 * SD);
    o += dppo_align16((size_t)4 * NS * SPLIT_H);
    o += dppo_align16(4 * K * DPPO_SCHED_COLS);
    o += dppo_align16(4 * (SPLIT_H + 16 * NO));
    o += dppo_align16((size_t)4 * 2 * NS * NV);
    o += (size_t)32 * KX * 1024;
    return o;
}

size_t split4_lds_bytes(int XD, int SD, int K, int KX, int NO, int sw, int esz = 2) {
    const int pad = 16, ldh = SPLIT_H + pad, lda0 = KX * (esz == 2 ? 32 : 16) + pad;
    size_t o = 0;
    o += dppo_align16((size_t)esz * 16 * lda0);
    o += dppo_align16((size_t)esz * 16 * ldh);
    o += dppo_align16(4 * sw * 16 * XD);
    o += 16;
    o += dppo_align16(4 * 16 * XD);
    o += dppo_align16(4 * 16 * SD);
    o += dppo_align16(4 * ((KX == 2 || esz == 4) ? 2 : K) * SPLIT_H);   // TIN: all K rows, or the 2-row ring (TRING)
    o += dppo_align16(4 * K * DPPO_SCHED_COLS);
    o += dppo_align16(4 * 2 * (SPLIT_H + 16 * NO));
    o += dppo_align16(4 * K * 16 * XD);
    o += (size_t)32 * KX * 1024;                  // sw waves x 32/sw n-tiles x KX k-steps
    (void)NO; (void)sw;
    return o;
}

size_t split_lds_bytes(int XD, int SD, int TD, int K, int KSI, int NO) {
    const int pad = 16, ldh = SPLIT_H + pad, lda0 = KSI * 32 + pad, KP = SW / (SPLIT_H / 16 / SPLIT_P);
    const int ldp = SPLIT_H / SPLIT_P + 4;
    size_t o = 0;
    o += dppo_align16(2 * 16 * lda0);
    o += dppo_align16(2 * 16 * ldh);
    o += dppo_align16(4 * KP * 16 * ldp);
    o += dppo_align16(4 * SW * 16 * XD);
    o += 16;
    o += dppo_align16(4 * 16 * XD);
    o += dppo_align16(4 * 16 * SD);
    o += dppo_align16(4 * K * TD);
    o += dppo_align16(4 * K * DPPO_SCHED_COLS);
    o += dppo_align16(4 * 2 * (3 * SPLIT_H + 16 * NO));
    o += dppo_align16(4 * K * 16 * XD);
    o += (size_t)SW * 2 * NO * 1024;
    return o;
}

__global__ void xchg_zero_kernel(uint64_t* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        __hip_atomic_store(p + i, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// exchange buffers: one per stream (launches on one stream are ordered, so they can share one).
// A slot is bound to one stream while `live`; dppo_sampler_release_stream unbinds it (the pipe that
// owned the stream is closed), and a new stream takes an unbound slot of its device first. A buffer
// is never freed: a rebound slot keeps its buffer and CONTINUES its launch sequence number, so no
// granule left in it by the previous stream can carry a tag the next launch waits for, and no
// zeroing (or device-wide synchronisation) is needed to hand it over.
struct XchgBuf {
    hipStream_t stream;
    int device;
    int live;
    uint64_t* buf;
    uint32_t seq;
    uint32_t* fail_host;   // mapped pinned word (SplitArgs::xfail_host)
    uint32_t* fail_dev;
};
std::mutex g_xmu;
XchgBuf g_xb[16];
int g_nxb = 0;
int g_cus = 0;

int xchg_for(hipStream_t s, uint64_t** buf, uint32_t* seq, uint32_t** fail_dev) {
    int dev = 0;
    DPPO_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_xmu);
    for (int i = 0; i < g_nxb; ++i)
        if (g_xb[i].live && g_xb[i].stream == s && g_xb[i].device == dev) {
            // an earlier launch on this stream lost its members' co-residency (another tenant took
            // the CUs it waited for) and wrote NaN actions: report it instead of sampling on
            if (__hip_atomic_load(g_xb[i].fail_host, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
                __hip_atomic_store(g_xb[i].fail_host, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return dppo_set_error(DPPO_EHIP, "split sampler: a launch's partial-sum exchange timed out "
                                      "(its workgroups were not all resident at once); its actions are NaN");
            }
            *buf = g_xb[i].buf;
            *seq = g_xb[i].seq = (g_xb[i].seq + 1) & 0x03FFFFFFu;
            *fail_dev = g_xb[i].fail_dev;
            return DPPO_OK;
        }
    int slot = -1;
    for (int i = 0; i < g_nxb && slot < 0; ++i)       // a released slot of this device
        if (!g_xb[i].live && g_xb[i].device == dev) slot = i;
    if (slot < 0 && g_nxb == 16) {
        // every slot is bound to a live stream (a process with more than 16 sampling streams):
        // rebind the slot of a stream with no work pending; only when every such stream is busy,
        // wait for ONE of them (never the whole device: another stream may hold a pipelined launch
        // that waits for an observation the host publishes only after this call returns)
        // (a query that is neither done nor not-ready means the stream no longer exists — its owner
        // destroyed it without dppo_sampler_release_stream: its slot is free, nothing to wait for)
        for (int i = 0; i < 16 && slot < 0; ++i) {
            if (g_xb[i].device != dev) continue;
            const hipError_t q = hipStreamQuery(g_xb[i].stream);
            if (q != hipErrorNotReady) {
                (void)hipGetLastError();
                slot = i;
            }
        }
        if (slot < 0) {
            static int next_evict = 0;
            for (int k = 0; k < 16 && slot < 0; ++k) {
                const int i = (next_evict + k) % 16;
                if (g_xb[i].device == dev) slot = i;
            }
            if (slot < 0) return dppo_set_error(DPPO_EHIP, "split sampler: no exchange buffer slot for this device");
            next_evict = (slot + 1) % 16;
            DPPO_HIP(hipStreamSynchronize(g_xb[slot].stream));
        }
    }
    if (slot >= 0) {                                    // rebind: same buffer, sequence continues
        XchgBuf& x = g_xb[slot];
        __hip_atomic_store(x.fail_host, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        x.stream = s; x.live = 1;
        x.seq = (x.seq + 1) & 0x03FFFFFFu;
        *buf = x.buf;
        *seq = x.seq;
        *fail_dev = x.fail_dev;
        return DPPO_OK;
    }
    slot = g_nxb;
    XchgBuf& x = g_xb[slot];
    const size_t n = XTOTAL;
    DPPO_HIP(hipMalloc((void**)&x.buf, sizeof(uint64_t) * n));
    DPPO_HIP(hipHostMalloc((void**)&x.fail_host, sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent));
    *x.fail_host = 0;
    DPPO_HIP(hipHostGetDevicePointer((void**)&x.fail_dev, x.fail_host, 0));
    // zeroed with write-through stores: no XCD's L2 is left holding a dirty copy of any line
    hipLaunchKernelGGL(xchg_zero_kernel, dim3(1024), dim3(256), 0, s, x.buf, n);
    DPPO_HIP(hipGetLastError());
    x.stream = s; x.device = dev; x.seq = 1; x.live = 1;
    ++g_nxb;
    *buf = x.buf;
    *seq = x.seq;
    *fail_dev = x.fail_dev;
    return DPPO_OK;
}

}  // namespace

// ABI 10: unbind the exchange buffer of `stream` (its owner is done sampling on it): waits for the
// stream's work, then leaves the buffer to the next new stream of the device
extern "C" DPPO_API int dppo_sampler_release_stream(void* stream) {
    hipStream_t s = (hipStream_t)stream;
    std::lock_guard<std::mutex> lk(g_xmu);
    for (int i = 0; i < g_nxb; ++i)
        if (g_xb[i].live && g_xb[i].stream == s) {
            DPPO_HIP(hipStreamSynchronize(s));
            g_xb[i].live = 0;
        }
    return DPPO_OK;
}

namespace {

int device_cus() {
    if (!g_cus) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
            g_cus = n;
    }
    return g_cus;
}

template <class Pol, int XQ, int KSI, bool INJ>
int launch_split_k(const SplitArgs& sa, hipStream_t s) {
    constexpr int NO = (4 * XQ + 15) / 16;
    auto k = sample_split_kernel<Pol, SPLIT_P, XQ, KSI, INJ>;
    const SampleArgs& a = sa.a;
    const size_t lds = split_lds_bytes(a.XD, a.SD, a.TD, a.K, KSI, NO);
    if (lds > 160 * 1024) return dppo_set_error(DPPO_EUNSUPPORTED, "split sampler needs %zu B of LDS", lds);
    { const int rc_ = dppo_func_lds((const void*)k, (size_t)lds); if (rc_) return rc_; }
    const int blocks = 8 * SPLIT_P * ((sa.G + 7) / 8);
    DppoKtScope kt(KT_SAMPLER, s);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(SW * 64), lds, s, sa);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

// waves per member of the P = 4 kernel. The kernel also builds with 4 (one wave per SIMD, 512
// registers: the l1 / l2 fragments partly in AGPRs, each wave two l1 n-tiles and eight in-Dense /
// l2 n-tiles): measured 63.7 vs 59.3 us per launch at 8 (no second wave to hide its latencies), so
// 8 is the default (-DDPPO_S4_WAVES=4 builds the one-wave-per-SIMD form as an A/B variant)
#ifndef DPPO_S4_WAVES
#define DPPO_S4_WAVES 8
#endif
constexpr int SPLIT4_WAVES = DPPO_S4_WAVES;
int split_waves() { return SPLIT4_WAVES; }

template <class Pol, int XQ, int KX, bool INJ, int SWV, int PM>
int launch_split4_kw(const SplitArgs& sa, hipStream_t s) {
    constexpr int NO = (4 * XQ + 15) / 16;
    // the finishing lanes are the members' lanes: a wave's 16 x XD / SWV coordinates in (64 / PM)
    // slots at most PM deep (the one-wave-per-SIMD form covers XD <= 16 at PM = 2)
    constexpr int NVW = 16 * 4 * XQ / SWV, KW = (NVW + 64 / PM - 1) / (64 / PM);
    if constexpr (KW > PM) {
        return dppo_set_error(DPPO_EUNSUPPORTED, "split sampler: %d waves per member do not cover XD = %d", SWV, 4 * XQ);
    } else {
    auto k = sample_split4_kernel<Pol, XQ, KX, INJ, SWV, PM>;
    const SampleArgs& a = sa.a;
    const size_t lds = split4_lds_bytes(a.XD, a.SD, a.K, KX, NO, SWV, (int)sizeof(typename Pol::AT));
    if (lds > 160 * 1024) return dppo_set_error(DPPO_EUNSUPPORTED, "split sampler needs %zu B of LDS", lds);
    { const int rc_ = dppo_func_lds((const void*)k, (size_t)lds); if (rc_) return rc_; }
    const int blocks = 8 * PM * ((sa.G + 7) / 8) * (sa.dual ? 2 : 1);
    DppoKtScope kt(KT_SAMPLER, s);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(SWV * 64), lds, s, sa);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
    }
}

// the pair kernel's instantiated shapes: hopper dims (XD = 12, XD + SD <= 32)
constexpr bool pair_shape_ok(int XD, int KX) { return XD == 12 && KX == 1; }

template <class Pol, int XQ, int KX, bool INJ>
int launch_pair_k(const SplitArgs& sa, hipStream_t s) {
    constexpr int NO = (4 * XQ + 15) / 16;
    auto k = sample_pair_kernel<Pol, XQ, KX, INJ>;
    const SampleArgs& a = sa.a;
    const int NS = sa.dual ? (a.K - a.KF > a.KF ? a.K - a.KF : a.KF) : a.K;
    const size_t lds = pair_lds_bytes(a.XD, a.SD, a.K, NS, KX, NO);
    if (lds > 160 * 1024) return dppo_set_error(DPPO_EUNSUPPORTED, "pair sampler needs %zu B of LDS", lds);
    { const int rc_ = dppo_func_lds((const void*)k, (size_t)lds); if (rc_) return rc_; }
    const int G2 = (sa.G + 1) / 2;
    const int blocks = 8 * 2 * ((G2 + 7) / 8) * (sa.dual ? 2 : 1);
    DppoKtScope kt(KT_SAMPLER, s);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(512), lds, s, sa);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

// members per group of the folded kernel: 2 (default: 47.2 us per bench launch), or 4 with
// -DDPPO_S4_P=4 (50.4 us; same box, tools/ab_variants.sh) — a build-time A/B knob
#ifndef DPPO_S4_P
#define DPPO_S4_P 2
#endif
constexpr int S4P = DPPO_S4_P;

template <class Pol, int XQ, int KX, bool INJ>
int launch_split4_k(const SplitArgs& sa, hipStream_t s) {
    return launch_split4_kw<Pol, XQ, KX, INJ, SPLIT4_WAVES, S4P>(sa, s);
}

// DPPO_SPLIT_P: members per 16-env group, the folded kernel (default) or 8 (the r01 kernel; A/B knob)
int split_p_choice() {
    static const int p = [] {
        const char* e = getenv("DPPO_SPLIT_P");
        return e && atoi(e) == 8 ? 8 : S4P;
    }();
    return p;
}


// the split sampler's plan for a shape: P members per 16-env group (2, 4 or 8; 0 = not taken),
// whether the two actors run on two member sets (dual), and whether each member pair runs two
// 16-env tiles (the pair kernel); blocks = workgroups of one launch
struct SplitPlan { int P; bool dual; bool pair; int blocks; };

SplitPlan split_plan(int precision, int H, int XD, int SD, int ks_in, int E, int K, int KF) {
    // fp32 (r06): the folded kernel at P = 4 members (an fp32 l1 quarter is 128 VGPRs of fragments), for
    // the instantiated width XD = 12 (hopper; other fp32 shapes stream the weights, sampler.hip)
    const bool f32 = precision == DPPO_F32;
    if ((!dppo_prec_2b(precision) && !(f32 && XD == 12)) || H != SPLIT_H || XD % 4 != 0 || XD > 32 || K > 62)
        return {0, false, false, 0};
    const int G = dppo_cdiv(E, 16);
    if (G < 1 || G > XMAX_G) return {0, false, false, 0};
    const int cus = device_cus();
    // every workgroup of the launch co-resident (one per CU: the register budget)
    auto fits = [&](int P, int sets, int groups) { return cus == 0 || sets * 8 * P * ((groups + 7) / 8) <= cus; };
    const int KX = dppo_cdiv(XD + SD, f32 ? 16 : 32);
    const int PF = f32 ? 4 : S4P;   // members per group of the folded kernel
    const bool p4 = KX <= 2 && split4_lds_bytes(XD, SD, K, KX, dppo_cdiv(XD, 16), split_waves(), f32 ? 4 : 2) <= 160 * 1024 &&
                    fits(PF, 1, G);
    if (f32) {
        static const bool dual_f = [] { const char* e = getenv("DPPO_SPLIT_DUAL"); return !e || atoi(e) != 0; }();
        const bool d = dual_f && KF > 0 && KF < K && (cus == 0 || 2 * 2 * 8 * PF * ((G + 7) / 8) <= cus);
        return p4 ? SplitPlan{PF, d, false, 8 * PF * ((G + 7) / 8) * (d ? 2 : 1)} : SplitPlan{0, false, false, 0};
    }
    const bool p8 = ks_in == 2 && fits(8, 1, G);
    static const bool dual_on = [] { const char* e = getenv("DPPO_SPLIT_DUAL"); return !e || atoi(e) != 0; }();
    // two sets only while two launches of them still fit side by side (the pipelined rollout keeps
    // the next step's launch resident while this one runs)
    const bool dual = dual_on && KF > 0 && KF < K && (cus == 0 || 2 * 2 * 8 * S4P * ((G + 7) / 8) <= cus);
    // the pair kernel: two tiles per member pair; each member set must hold one actor
    // opt-in (DPPO_SPLIT_PAIR=1): bit-identical, but measured SLOWER at 64 envs (70.0 vs 47.4 us per
    // launch, tools/r03_pair.sh): the exchange is hidden, everything else in a tile's step adds up
    static const bool pair_on = [] { const char* e = getenv("DPPO_SPLIT_PAIR"); return e && atoi(e) != 0; }();
    const int G2 = (G + 1) / 2;
    const bool pdual = dual_on && KF > 0 && KF < K && (cus == 0 || 2 * 2 * 8 * 2 * ((G2 + 7) / 8) <= cus);
    const int NS = pdual ? (K - KF > KF ? K - KF : KF) : K;
    const bool pair = pair_on && S4P == 2 && G >= 2 && pair_shape_ok(XD, KX) && (pdual || KF == K || KF == 0) &&
                      pair_lds_bytes(XD, SD, K, NS, KX, dppo_cdiv(XD, 16)) <= 160 * 1024 && fits(2, pdual ? 2 : 1, G2);
    auto blocks = [&](int P, bool d2, int groups) { return 8 * P * ((groups + 7) / 8) * (d2 ? 2 : 1); };
    if (split_p_choice() == 8)
        return p8 ? SplitPlan{8, false, false, blocks(8, false, G)}
                  : (p4 ? SplitPlan{S4P, dual, false, blocks(S4P, dual, G)} : SplitPlan{0, false, false, 0});
    if (pair) return SplitPlan{2, pdual, true, blocks(2, pdual, G2)};
    return p4 ? SplitPlan{S4P, dual, false, blocks(S4P, dual, G)}
              : (p8 ? SplitPlan{8, false, false, blocks(8, false, G)} : SplitPlan{0, false, false, 0});
}

}  // namespace

int split_members_for(int precision, int H, int XD, int SD, int ks_in, int E, int K, int KF) {
    const SplitPlan p = split_plan(precision, H, XD, SD, ks_in, E, K, KF);
    return p.P * (p.dual ? 2 : 1);
}

// dppo_sampler_plan's fields: kernel (0 weight streaming, 1 split P = 8, 2 folded split, one tile per
// group, 3 pair), members P per set, member sets, workgroups per launch
void split_plan_query(int precision, int H, int XD, int SD, int ks_in, int E, int K, int KF, int* out) {
    const SplitPlan p = split_plan(precision, H, XD, SD, ks_in, E, K, KF);
    out[0] = p.P == 0 ? 0 : (p.pair ? 3 : (p.P == 8 ? 1 : 2));
    out[1] = p.P;
    out[2] = p.P ? (p.dual ? 2 : 1) : 0;
    out[3] = p.blocks;
}

bool sample_split_supported(int precision, int H, int XD, int SD, int ks_in, int E, int K, int KF) {
    return split_members_for(precision, H, XD, SD, ks_in, E, K, KF) > 0;
}

int sampler_device_cus() { return device_cus(); }

int launch_sample_split(const SampleArgs& a, int precision, hipStream_t s) {
    const SplitPlan plan = split_plan(precision, a.H, a.XD, a.SD, a.L.ks_in, a.E, a.K, a.KF);
    const int P = plan.P;
    if (!P) return DPPO_EUNSUPPORTED;
    SplitArgs sa;
    sa.a = a;
    sa.dual = plan.dual ? 1 : 0;
    sa.G = dppo_cdiv(a.E, 16);
    static const int force_shared = [] {
        const char* e = getenv("DPPO_SPLIT_XCHG");
        return e && !strcmp(e, "shared") ? 1 : 0;
    }();
    sa.force_shared = force_shared;
    int rc = xchg_for(s, &sa.xbuf, &sa.seq, &sa.xfail_host);
    if (rc) return rc;
    const bool inj = a.noise != nullptr;
    const bool f16 = precision == DPPO_F16;
    if (precision == DPPO_F32) {   // split_plan took XD = 12 only
        if (a.XD != 12 || P != 4) return DPPO_EUNSUPPORTED;
        if (a.XD + a.SD > 16)
            return inj ? launch_split4_kw<PolicyF32, 3, 2, true, 8, 4>(sa, s) : launch_split4_kw<PolicyF32, 3, 2, false, 8, 4>(sa, s);
        return inj ? launch_split4_kw<PolicyF32, 3, 1, true, 8, 4>(sa, s) : launch_split4_kw<PolicyF32, 3, 1, false, 8, 4>(sa, s);
    }
    if (plan.pair) {
        if (f16) return inj ? launch_pair_k<PolicyF16, 3, 1, true>(sa, s) : launch_pair_k<PolicyF16, 3, 1, false>(sa, s);
        return inj ? launch_pair_k<PolicyBF16, 3, 1, true>(sa, s) : launch_pair_k<PolicyBF16, 3, 1, false>(sa, s);
    }
    if (P == S4P) {
        const bool kx2 = a.XD + a.SD > 32;
        switch (a.XD / 4) {
#define DPPO_SPLIT4_CASE(xq)                                                                                 \
    case xq:                                                                                                 \
        if (kx2) {                                                                                           \
            if (f16) return inj ? launch_split4_k<PolicyF16, xq, 2, true>(sa, s) : launch_split4_k<PolicyF16, xq, 2, false>(sa, s); \
            return inj ? launch_split4_k<PolicyBF16, xq, 2, true>(sa, s) : launch_split4_k<PolicyBF16, xq, 2, false>(sa, s); \
        }                                                                                                    \
        if (f16) return inj ? launch_split4_k<PolicyF16, xq, 1, true>(sa, s) : launch_split4_k<PolicyF16, xq, 1, false>(sa, s); \
        return inj ? launch_split4_k<PolicyBF16, xq, 1, true>(sa, s) : launch_split4_k<PolicyBF16, xq, 1, false>(sa, s);
            DPPO_SPLIT4_CASE(1) DPPO_SPLIT4_CASE(2) DPPO_SPLIT4_CASE(3) DPPO_SPLIT4_CASE(4)
            DPPO_SPLIT4_CASE(5) DPPO_SPLIT4_CASE(6) DPPO_SPLIT4_CASE(7) DPPO_SPLIT4_CASE(8)
#undef DPPO_SPLIT4_CASE
            default: return DPPO_EUNSUPPORTED;
        }
    }
    switch (a.XD / 4) {
#define DPPO_SPLIT_CASE(xq)                                                                                 \
    case xq:                                                                                                \
        if (f16) return inj ? launch_split_k<PolicyF16, xq, 2, true>(sa, s) : launch_split_k<PolicyF16, xq, 2, false>(sa, s); \
        return inj ? launch_split_k<PolicyBF16, xq, 2, true>(sa, s) : launch_split_k<PolicyBF16, xq, 2, false>(sa, s);
        DPPO_SPLIT_CASE(1) DPPO_SPLIT_CASE(2) DPPO_SPLIT_CASE(3) DPPO_SPLIT_CASE(4)
        DPPO_SPLIT_CASE(5) DPPO_SPLIT_CASE(6) DPPO_SPLIT_CASE(7) DPPO_SPLIT_CASE(8)
#undef DPPO_SPLIT_CASE
        default: return DPPO_EUNSUPPORTED;
    }
}
