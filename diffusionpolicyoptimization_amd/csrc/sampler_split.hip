// sampler_split.hip — a9: VPGDiffusion.call (model/diffusion/diffusion_vpg.py:250-339) as a
// register-resident SPLIT kernel: the sampler for <= 512 envs per GPU (bf16 / fp16 at any action width
// with XD + SD <= 64, fp32 at hopper's; every other shape streams the weights, sampler.hip).
//
// Why: the weight-streaming kernel gives each 16-env tile one CU, which must pull the whole 1.1 MB bf16
// actor through its 64 B/clk load path every denoising step (~8 us a step at 64 envs). Here each 16-env
// group is owned by P workgroups (one per CU, "members": P = 2 for 2-byte operands, 8 for fp32) and
// member c keeps 1/P of l1 in its register file for the whole launch (the 1 MB bf16 / 2 MB fp32 l1 of
// one actor: 128 VGPRs of fragments per lane either way). The l2 layer is folded into the out-Dense
// (mlp.py:186-206: the residual block is linear from the l2 product to the out-Dense):
//   eps = W_out^T h1 + M^T relu(h2) + B_OUT2,   M = W_l2 W_out,   B_OUT2 = b_out + W_out^T b_l2
// so the only cross-CU traffic of a denoising step is one exchange of 16 x XD fp32 partial eps between
// the P members, and every member then runs the same fp32 DDPM epilogue on the same sum (fixed member
// order: bit-identical x on all of them).
//
// The exchange is in-launch (MI355X_MICROARCH.md "handoff-1to1"/R2 granules): each member stores its
// partials as 8-byte {tag, value} granules and every wave sweeps its slice of the group's granules with
// agent-scope (sc1, L1-bypassing) loads until every tag matches. Tags carry a per-launch sequence
// number and the step index, so nothing is zeroed between launches; slots alternate by step parity (a
// member can be at most one step ahead of a peer). The wait is bounded (100 ms): a launch that times
// out writes NaN actions and flags bit 31 of *done. Store flavour, chosen per group at run time (never
// assumed from blockIdx):
//   * every member reads its XCD from HW_REG_XCC_ID and announces it (sc1 granule) in the prologue;
//     the members sweep the announcements and agree on the mode;
//   * all on one XCD -> "L2-local": workgroup-scope (sc0) granule stores, which keep the line in that
//     XCD's L2, where the peers' sc1 loads find it (tools/xchg_probe2.hip: P = 2 0.59 us per exchange
//     step). These granules live in a region owned by that XCD alone ([xcc][slot][G][P][NV], fixed
//     stride), so no other XCD's L2 ever holds a copy of those lines;
//   * otherwise -> write-through agent-scope (sc1) stores into the shared region, the
//     placement-independent form.
// Block -> (group, member): members of a group share blockIdx % 8 (one XCD under the observed
// round-robin placement: a speed choice only; correctness does not depend on placement).
// (r06: the r01 8-member kernel with an l2 GEMM and the r03 pair kernel — two tiles per member pair —
// both measured slower than this one, were removed; DESIGN.md §3 keeps their numbers.)
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

// timing probes (tools/variant_build.sh ... -DDPPO_PROBE_NOSYNC=k, results wrong): drop barrier k of a
// folded-kernel step (1 in-Dense, 2 partial sums, 3 step end)
#ifndef DPPO_PROBE_NOSYNC
#define DPPO_PROBE_NOSYNC 0
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

constexpr int SPLIT_P = 8;         // the most members per 16-env group (fp32); the exchange regions' stride
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



// tuning knobs of the split kernel (tools/variant_build.sh <tag> "-D..." + tools/ab_variants.sh)
#ifndef DPPO_S4_L1D
#define DPPO_S4_L1D 1        // l1: u1 fragment reads kept in flight ahead of the MFMA chain (r06, same box,
                             // 300 launches x 2: 1 46.8 / 4 47.8 / 2 47.1-47.5 / 3 47.7-47.9 / 6 47.5 / 0
                             // 58.0 us at hopper bf16; fp32 neutral; profiles/r06l_sampler_l1d_ab.txt)
#endif
#ifndef DPPO_S4_INREADY
#define DPPO_S4_INREADY 0    // 1: the in-Dense's LDS operands forced into one round trip (the r02-r05 form); r06 with
                             // l1 read-ahead 1: left to the compiler measured 46.0-46.3 vs 46.8-47.0 us at hopper
                             // bf16, -1.4 % at DDIM 512 fp16, -0.5 % walker2d 256, fp32 neutral (r06m A/B)
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

// ------------------------------------------------------------------------------------------------
// P = 2 (2-byte operands) or 4 (fp32, or -DDPPO_S4_P=4) members per 16-env group. Fewer members mean a
// cheaper exchange (tools/xchg_probe2.hip, sc0 one-XCD granules at 16 envs: P = 2 0.59 us per step, 4
// 0.98, 8 1.55) and less arrival skew, for more l1 MFMAs per wave. Member c
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
// a 2-member exchange; possible once l2 is folded away), 4, or 8 (fp32 with SWV = 4: one wave per
// SIMD, one l1 n-tile each; the member sum adds a third DPP level)
template <class Pol, int XQ, int KX, bool INJ, int SWV, int PM = 4>
__global__ __launch_bounds__(SWV * 64) void sample_split4_kernel(SplitArgs sa) {
    constexpr int P = PM;
    static_assert(P == 2 || P == 4 || P == 8, "members per group");
    constexpr int NO = (4 * XQ + 15) / 16;
    using AT = typename Pol::AT;
    // TWO: 2-byte operands (bf16 / fp16: the fold and residual as hi/lo pairs in one 16x16x32 MFMA); else
    // fp32 (r06, P = 8 on 4 waves or 4 on 8: the l1 slice is 128 VGPRs of fragments per lane as bf16's at P = 2;
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
        const bool one_xcd = ok && __all(lane >= P || (int)(uint32_t)v == x0);
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
    // fp32 at KX = 2 (hopper: XD + SD = 23 > 16): the in-Dense's second k-step reads state columns only
    // (XD <= KG), so its product is launch-constant per actor — formed once here (and again after a
    // non-dual actor switch) and added to the TIN row: 4 of the step's 16x16x4 MFMAs per in-Dense tile
    // and one LDS operand round trip fewer. (The 2-byte walker2d / halfcheetah form keeps its second
    // k-step: 16 more VGPRs spill it.)
    constexpr bool SBP = KX == 2 && !TWO;
    static_assert(!SBP || XD <= KGP, "x within the in-Dense's first k-step");
    f32x4 sb[SBP ? NTI : 1];
    auto state_part = [&]() {
        if constexpr (SBP) {
            const u32x4 af1 = lds_afrag<Pol>(a0, lda0, 0, 1, lane);
#pragma unroll
            for (int n = 0; n < NTI; ++n) {
                zero_acc(sb[n]);
                sb[n] = Pol::mma(wxs[((wave * NTI + n) * KX + 1) * 64 + lane], af1, sb[n]);
            }
        }
    };
    state_part();
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
            __builtin_amdgcn_s_waitcnt(0x0F70);   // the other actor's fragments (load_in / load_l1 / load_fold)
            cur = PK;
            state_part();
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
            constexpr int KXS = SBP ? 1 : KX;   // k-steps run per step
            u32x4 af[KXS], wf[KXS][NTI];
#pragma unroll
            for (int ks = 0; ks < KXS; ++ks) af[ks] = lds_afrag<Pol>(a0, lda0, 0, ks, lane);
#pragma unroll
            for (int n = 0; n < NTI; ++n) h1[n] = *(const f32x4*)(tin + (TRING ? (i & 1) : t) * H + 16 * (NTI * wave + n) + 4 * jq);
#pragma unroll
            for (int n = 0; n < NTI; ++n) wf[0][n] = wxs[((wave * NTI + n) * KX + 0) * 64 + lane];
            // one LDS round trip for all of them (2-byte KX = 2: the second k-step's operands in a second
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
            if constexpr (SBP)
#pragma unroll
                for (int n = 0; n < NTI; ++n) h1[n] += sb[n];
#pragma unroll
            for (int n = 0; n < NTI; ++n) h1[n] = Pol::mma(wf[0][n], af[0], h1[n]);
            if constexpr (KXS == 2) {
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
            // member sum: xor 1 (then xor 2) inside the quad, then across the two quads of 8 lanes (P = 8);
            // every lane adds the same two partial sums (a + b == b + a), so all P hold the same bits
#pragma unroll
            for (int k = 0; k < KW; ++k) {
                val[k] += dpp_f32<0xB1>(val[k]);     // quad_perm [1,0,3,2]
                if constexpr (P >= 4) val[k] += dpp_f32<0x4E>(val[k]);     // quad_perm [2,3,0,1]
                if constexpr (P == 8) val[k] += dpp_f32<0x141>(val[k]);    // row_half_mirror: lane i <-> 7 - i
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

// members per group of the folded kernel: 2 (default: 47.2 us per bench launch), or 4 with
// -DDPPO_S4_P=4 (50.4 us; same box, tools/ab_variants.sh) — a build-time A/B knob
#ifndef DPPO_S4_P
#define DPPO_S4_P 2
#endif
constexpr int S4P = DPPO_S4_P;
// fp32: P = 8 members of 4 waves (one per SIMD: the 16x16x4 MFMA's 32-cycle issue is the step's bound,
// so halving each SIMD's l1 share pays for the 8-member exchange), or P = 4 of 8 waves (-DDPPO_F32_P=4)
#ifndef DPPO_F32_P
#define DPPO_F32_P 8
#endif
constexpr int F32P = DPPO_F32_P, F32W = F32P == 8 ? 4 : 8;

template <class Pol, int XQ, int KX, bool INJ>
int launch_split4_k(const SplitArgs& sa, hipStream_t s) {
    return launch_split4_kw<Pol, XQ, KX, INJ, SPLIT4_WAVES, S4P>(sa, s);
}

// the split sampler's plan for a shape: P members per 16-env group (2 for 2-byte operands, 4 for fp32;
// 0 = not taken: the weight-streaming sampler, sampler.hip), whether the two actors run on two member
// sets (dual), blocks = workgroups of one launch. (r06: the r01 8-member kernel and the r03 pair kernel,
// both measured slower than this one, were removed; walker2d / halfcheetah run it since their TIN ring.)
struct SplitPlan { int P; bool dual; int blocks; };

SplitPlan split_plan(int precision, int H, int XD, int SD, int E, int K, int KF) {
    // fp32 (r06): the folded kernel at P = F32P members (an fp32 l1 eighth on 4 waves, or a quarter on 8, is
    // 128 VGPRs of fragments per lane), for the instantiated width XD = 12 (hopper; other fp32 shapes stream
    // the weights, sampler.hip)
    const bool f32 = precision == DPPO_F32;
    if ((!dppo_prec_2b(precision) && !(f32 && XD == 12)) || H != SPLIT_H || XD % 4 != 0 || XD > 32 || K > 62)
        return {0, false, 0};
    const int G = dppo_cdiv(E, 16);
    if (G < 1 || G > XMAX_G) return {0, false, 0};
    const int cus = device_cus();
    const int P = f32 ? F32P : S4P;   // members per group
    const int KX = dppo_cdiv(XD + SD, f32 ? 16 : 32);
    // every workgroup of the launch co-resident (one per CU: the register budget)
    if (KX > 2 || split4_lds_bytes(XD, SD, K, KX, dppo_cdiv(XD, 16), f32 ? F32W : split_waves(), f32 ? 4 : 2) > 160 * 1024 ||
        (cus && 8 * P * ((G + 7) / 8) > cus))
        return {0, false, 0};
    // two member sets (one per actor) only while two launches of them still fit side by side (the
    // pipelined rollout keeps the next step's launch resident while this one runs)
    const bool dual = KF > 0 && KF < K && (cus == 0 || 2 * 2 * 8 * P * ((G + 7) / 8) <= cus);
    return {P, dual, 8 * P * ((G + 7) / 8) * (dual ? 2 : 1)};
}

}  // namespace

int split_members_for(int precision, int H, int XD, int SD, int ks_in, int E, int K, int KF) {
    (void)ks_in;
    const SplitPlan p = split_plan(precision, H, XD, SD, E, K, KF);
    return p.P * (p.dual ? 2 : 1);
}

// dppo_sampler_plan's fields: kernel (0 weight streaming, 2 folded split; 1 and 3, the removed 8-member
// and pair kernels, are no longer returned), members P per set, member sets, workgroups per launch
void split_plan_query(int precision, int H, int XD, int SD, int ks_in, int E, int K, int KF, int* out) {
    (void)ks_in;
    const SplitPlan p = split_plan(precision, H, XD, SD, E, K, KF);
    out[0] = p.P == 0 ? 0 : 2;
    out[1] = p.P;
    out[2] = p.P ? (p.dual ? 2 : 1) : 0;
    out[3] = p.blocks;
}

bool sample_split_supported(int precision, int H, int XD, int SD, int ks_in, int E, int K, int KF) {
    return split_members_for(precision, H, XD, SD, ks_in, E, K, KF) > 0;
}

int sampler_device_cus() { return device_cus(); }

int launch_sample_split(const SampleArgs& a, int precision, hipStream_t s) {
    const SplitPlan plan = split_plan(precision, a.H, a.XD, a.SD, a.E, a.K, a.KF);
    const int P = plan.P;
    if (!P) return DPPO_EUNSUPPORTED;
    SplitArgs sa;
    sa.a = a;
    sa.dual = plan.dual ? 1 : 0;
    sa.G = dppo_cdiv(a.E, 16);
    int rc = xchg_for(s, &sa.xbuf, &sa.seq, &sa.xfail_host);
    if (rc) return rc;
    const bool inj = a.noise != nullptr;
    const bool f16 = precision == DPPO_F16;
    if (precision == DPPO_F32) {   // split_plan took XD = 12 only
        if (a.XD != 12 || P != F32P) return DPPO_EUNSUPPORTED;
        if (a.XD + a.SD > 16)
            return inj ? launch_split4_kw<PolicyF32, 3, 2, true, F32W, F32P>(sa, s)
                       : launch_split4_kw<PolicyF32, 3, 2, false, F32W, F32P>(sa, s);
        return inj ? launch_split4_kw<PolicyF32, 3, 1, true, F32W, F32P>(sa, s)
                   : launch_split4_kw<PolicyF32, 3, 1, false, F32W, F32P>(sa, s);
    }
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
