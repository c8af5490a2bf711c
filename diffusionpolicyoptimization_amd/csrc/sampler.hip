// sampler.hip — a9: VPGDiffusion.call (model/diffusion/diffusion_vpg.py:250-339), DDPM branch.
//
// One workgroup (8 waves) owns 16 env rows for ALL K denoising steps: rows are independent, so
// the K x 4 dependent GEMMs of a rollout step run without any inter-workgroup synchronisation.
// Per step: a0 = [x, t_emb(t), state] (mlp_diffusion.py:72-86) -> in-Dense -> relu -> l1 -> relu
// -> l2 + h1 (residual, mlp.py:186-206) -> out-Dense = eps; then the fused fp32 DDPM epilogue
// (diffusion_vpg.py:198-243, 301-320). Activations never leave LDS; weights stream from L2.
// The actor used at step t is actor_ft when t < K' else the frozen base actor (diffusion_vpg.py:161-180);
// the reference's always-computed base forward (:161) does not change the result and is skipped.
#include <mutex>
#include <stdlib.h>
#include <string.h>
#include "dppo_common.cuh"
#include "dppo_internal.h"
#include "dppo_sampler.h"

// phase timing for tuning builds (-DDPPO_SAMPLER_TIMING): wave 0 of every workgroup adds the
// shader-clock cycles of each phase of every denoising step (barrier waits included)
#ifdef DPPO_SAMPLER_TIMING
__device__ unsigned long long dppo_sampler_cycles[16];
#define SPHASE(k)                                                                 \
    do {                                                                          \
        if (threadIdx.x == 0) {                                                   \
            const unsigned long long now_ = __builtin_readcyclecounter();         \
            atomicAdd(&dppo_sampler_cycles[(k)], now_ - t_phase_);                \
            t_phase_ = now_;                                                      \
        }                                                                         \
    } while (0)
#define SPHASE_START unsigned long long t_phase_ = __builtin_readcyclecounter()
extern "C" DPPO_API int dppo_debug_sampler_cycles(unsigned long long* out, int reset) {
    DPPO_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(dppo_sampler_cycles), sizeof(unsigned long long) * 16));
    if (reset) {
        unsigned long long z[16] = {};
        DPPO_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dppo_sampler_cycles), z, sizeof(z)));
    }
    return DPPO_OK;
}
#else
#define SPHASE(k) do {} while (0)
#define SPHASE_START do {} while (0)
#endif

// ---- the sampler's weight stream with resident fragments ----
// A CU streams its actor's weights from L2 every denoising step, and its vector-memory path
// (64 B/clk) is what bounds the kernel. Fragments that fit in the register file
// beside the working set are loaded once per actor instead ("resident"): the in-layer, the
// out-layer and the first RK k-steps of both hidden layers. Only the rest streams through the
// QD-deep queue. A streamed segment is {W: matrix offset advanced past its resident k-steps,
// KSF: the matrix's k-step count (the n-tile stride), KS: k-steps streamed}.
struct SSeg {
    WSrc W;
    int KSF, KS;
};
struct SNext {
    SSeg s1, s2;   // the two streamed segments after the current one
};
__device__ inline SSeg sseg(WSrc W, int KSF, int k0) { return SSeg{WSrc{W.rsrc, W.off + ((uint32_t)k0 << 10)}, KSF, KSF - k0}; }

template <int KS>
__device__ inline u32x4 sfrag(WSrc W, int KSF, const SNext& nx, int ntile, int j, int lane) {
    if (j < KS) return load_bfrag_c(W, KSF, ntile, j, lane);                 // compile-time branch
    const int j1 = j - KS;
    const bool first = j1 < nx.s1.KS;                                         // wave-uniform
    return first ? load_bfrag_c(nx.s1.W, nx.s1.KSF, ntile, j1, lane)
                 : load_bfrag_c(nx.s2.W, nx.s2.KSF, ntile, j1 - nx.s1.KS, lane);
}

template <int D, int NT>
__device__ inline void squeue_prime(WQueue<D, NT>& Q, const SSeg& s0, const SNext& nx, int ntile0, int lane) {
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int j = d;
            if (j < s0.KS) Q.b[d][n] = load_bfrag_c(s0.W, s0.KSF, ntile0 + n, j, lane);
            else if (j - s0.KS < nx.s1.KS) Q.b[d][n] = load_bfrag_c(nx.s1.W, nx.s1.KSF, ntile0 + n, j - s0.KS, lane);
            else Q.b[d][n] = load_bfrag_c(nx.s2.W, nx.s2.KSF, ntile0 + n, j - s0.KS - nx.s1.KS, lane);
        }
}

// acc = A[16 rows][KSF*KG] x W[:, ntile0*16 ..): k-steps [0, RKL) from the resident fragments
// (computed first: they cover the latency of the queue's first loads after the layer barrier),
// k-steps [RKL, KSF) from the queue, which keeps D k-steps of look-ahead into the next segments.
// k-steps [RKL, RKL+LKL) come from fragments kept in LDS (lw: [LKL][NTOT n-tiles][64 lanes] x 16 B).
template <class P, int NT, int KSF, int RKL, int LKL, int NTOT, int D>
__device__ inline void gemm_res(const typename P::AT* A, int lda, WSrc Ws, const u32x4 (*res)[NT], const u32x4* lw,
                                int ntile0, f32x4 (&acc)[1][NT], int lane, WQueue<D, NT>& Q, const SNext& nx) {
    constexpr int KS = KSF - RKL - LKL;
#pragma unroll
    for (int n = 0; n < NT; ++n) zero_acc(acc[0][n]);
#pragma unroll
    for (int ks = 0; ks < RKL; ++ks) {
        const u32x4 a = lds_afrag<P>(A, lda, 0, ks, lane);
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[0][n] = P::mma(a, res[ks][n], acc[0][n]);
    }
#pragma unroll
    for (int kl = 0; kl < LKL; ++kl) {
        const u32x4 a = lds_afrag<P>(A, lda, 0, RKL + kl, lane);
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[0][n] = P::mma(a, lw[(kl * NTOT + ntile0 + n) * 64 + lane], acc[0][n]);
    }
#pragma unroll
    for (int j = 0; j < KS; ++j) {
        u32x4 c[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) c[n] = Q.b[0][n];
#pragma unroll
        for (int d = 0; d + 1 < D; ++d)
#pragma unroll
            for (int n = 0; n < NT; ++n) Q.b[d][n] = Q.b[d + 1][n];
#pragma unroll
        for (int n = 0; n < NT; ++n) Q.b[D - 1][n] = sfrag<KS>(Ws, KSF, nx, ntile0 + n, j + D, lane);
        const u32x4 a = lds_afrag<P>(A, lda, 0, RKL + LKL + j, lane);
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[0][n] = P::mma(a, c[n], acc[0][n]);
    }
}

// SW waves per workgroup, each owning NT = H/(16*SW) n-tiles of every hidden layer. RK hidden
// k-steps and (RIO) the whole in- and out-layers are resident in registers, LK more hidden
// k-steps in LDS; QD k-steps of the rest in flight.
template <class P, int NT, int NO, int KSI, bool INJ, int QD, int SW, int RK, int LK, int RIO>
__global__ __launch_bounds__(SW * 64) void sample_kernel(SampleArgs a) {
    SPHASE_START;
    using AT = typename P::AT;
    constexpr int ST = SW * 64;
    constexpr int KSH = ksh_for<P>(NT, SW);
    constexpr int NOK = KSH / SW;
    constexpr bool RIN = RIO & 1, ROUT = RIO & 2;   // in-layer / out-layer resident
    constexpr int RKI = RIN ? KSI : 0;       // resident in-layer k-steps
    constexpr int NTOT = NT * SW;            // n-tiles of a hidden layer
    static_assert(RK + LK < KSH, "at least one streamed hidden k-step");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int row0 = blockIdx.x * 16;
    const MlpLayout& L = a.L;
    const int pad = lds_pad_elems<P>();
    const int H = a.H;
    const int ldh = H + pad;
    const int k1w = L.ks_in * P::KG;
    const int lda0 = k1w + pad;
    const int XD = a.XD, SD = a.SD, TD = a.TD, K = a.K, KF = a.KF;
    const int NOC = 16 * NO;

    // ---- LDS carve (all offsets multiples of 16 B) ----
    size_t o = 0;
    AT* tA = (AT*)(smem + o); o += dppo_align16(sizeof(AT) * 16 * ldh);
    AT* tB = (AT*)(smem + o); o += dppo_align16(sizeof(AT) * 16 * ldh);
    AT* a0 = (AT*)(smem + o); o += dppo_align16(sizeof(AT) * 16 * lda0);
    float* xs = (float*)(smem + o); o += dppo_align16(4 * 16 * XD);
    float* st = (float*)(smem + o); o += dppo_align16(4 * 16 * SD);
    float* temb = (float*)(smem + o); o += dppo_align16(4 * K * TD);
    float* part = (float*)(smem + o); o += dppo_align16(4 * SW * 16 * NOC);
    float* sch = (float*)(smem + o); o += dppo_align16(4 * K * DPPO_SCHED_COLS);
    float* bias = (float*)(smem + o); o += dppo_align16(4 * 2 * (3 * H + NOC));  // [actor][in,l1,l2,out]
    float* zt = (float*)(smem + o); o += dppo_align16(4 * K * 16 * XD);           // clipped noise [i][row][q]
    u32x4* lw1 = (u32x4*)(smem + o); o += (size_t)LK * NTOT * 1024;                // LDS-resident hidden k-steps
    u32x4* lw2 = (u32x4*)(smem + o); o += (size_t)LK * NTOT * 1024;

    const int ntile0 = wave * NT;
    const __amdgpu_buffer_rsrc_t rs_base = packed_rsrc(a.packed_base), rs_ft = packed_rsrc(a.packed_ft);
    // actor selection is wave-uniform: keep it scalar (readfirstlane), or hipcc may treat the buffer
    // resource as divergent and wrap every weight load in a waterfall loop
    auto W = [&](int ft, int seg) { return wsrc(ft ? rs_ft : rs_base, L.off[seg]); };
    // the streamed segments of a denoising step: [in (unless resident)], l1[RK..], l2[RK..]
    auto s_in = [&](int ft) { return sseg(W(ft, SEG_W_IN), KSI, 0); };
    auto s_l1 = [&](int ft) { return sseg(W(ft, SEG_W_L1), KSH, RK + LK); };
    auto s_l2 = [&](int ft) { return sseg(W(ft, SEG_W_L2), KSH, RK + LK); };
    // hidden k-steps [RK, RK+LK) of both hidden layers into LDS, [k][n-tile][lane] (callers barrier)
    auto load_lds = [&](int ft) {
        const WSrc w1 = W(ft, SEG_W_L1), w2 = W(ft, SEG_W_L2);
        for (int c = tid; c < LK * NTOT * 64; c += ST) {
            const int kl = c / (NTOT * 64), nt = (c / 64) % NTOT, ln = c % 64;
            const uint32_t so = (uint32_t)(nt * KSH + RK + kl) << 10;
            lw1[c] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(w1.rsrc, ln << 4, w1.off + so, 0));
            lw2[c] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(w2.rsrc, ln << 4, w2.off + so, 0));
        }
    };

    // resident fragments of the actor in use (reloaded when the actor changes, once per launch)
    u32x4 r_in[RKI > 0 ? RKI : 1][NT], r_l1[RK > 0 ? RK : 1][NT], r_l2[RK > 0 ? RK : 1][NT];
    ORing<NOK, NO> r_out;
    auto load_resident = [&](int ft) {
#pragma unroll
        for (int k = 0; k < RKI; ++k)
#pragma unroll
            for (int n = 0; n < NT; ++n) r_in[k][n] = load_bfrag_c(W(ft, SEG_W_IN), KSI, ntile0 + n, k, lane);
#pragma unroll
        for (int k = 0; k < RK; ++k)
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                r_l1[k][n] = load_bfrag_c(W(ft, SEG_W_L1), KSH, ntile0 + n, k, lane);
                r_l2[k][n] = load_bfrag_c(W(ft, SEG_W_L2), KSH, ntile0 + n, k, lane);
            }
        if constexpr (ROUT) out_prefetch<NOK, NO, SW>(r_out, W(ft, SEG_W_OUT), L.ks_h, wave, lane);
    };
    // the weight stream starts with step 0 (t = K-1); its first loads and the resident set go out
    // before anything waits (noise, the host's observation)
    const int ft0 = __builtin_amdgcn_readfirstlane(K - 1 < KF ? 1 : 0);
    WQueue<QD, NT> R;
    if constexpr (RIN) squeue_prime(R, s_l1(ft0), SNext{s_l2(ft0), s_l1(ft0)}, ntile0, lane);
    else squeue_prime(R, s_in(ft0), SNext{s_l1(ft0), s_l2(ft0)}, ntile0, lane);
    load_resident(ft0);
    if constexpr (LK > 0) load_lds(ft0);      // made visible by the prologue's barriers
    int cur = ft0;

    // ---- prologue: schedule, biases, state, x_T, time-embedding table ----
    // All global loads go out first (16 B per lane), the Philox/Box-Muller noise is computed while
    // they are in flight, then everything lands in LDS: the prologue runs before the host's
    // observation arrives, and in a pipelined rollout it is what the env step has to cover.
    const int NB4 = 2 * (3 * H + NOC) / 4;                  // float4s of both actors' biases
    float4 bv[4];
    auto bias_src = [&](int i4) {
        const int w = i4 / ((3 * H + NOC) / 4), j = 4 * (i4 % ((3 * H + NOC) / 4));
        const uint8_t* PK = w ? a.packed_ft : a.packed_base;
        const int seg = j < H ? SEG_B_IN : (j < 2 * H ? SEG_B_L1 : (j < 3 * H ? SEG_B_L2 : SEG_B_OUT));
        const int jj = j < 3 * H ? j % H : j - 3 * H;
        return (const float4*)(PK + L.off[seg]) + jj / 4;
    };
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (tid + u * ST < NB4) bv[u] = *bias_src(tid + u * ST);
    float tv = 0.f;
    if (tid < K * TD) {
        const int t = tid / TD;
        tv = ((const float*)((t < KF ? a.packed_ft : a.packed_base) + L.off[SEG_TEMB]))[tid];
    }
    float scv = tid < K * DPPO_SCHED_COLS ? a.sched[tid] : 0.f;
    // noise: all K steps' draws up front (injected, or the Philox stream: one block gives the 4
    // normals of a group of 4 action coordinates), clipped to +-randn_clip (:319), so the
    // denoising loop carries no RNG state; slot K is x_T
    const int XG = (XD + 3) / 4;
    for (int it = tid; it < (K + 1) * 16 * XG; it += ST) {
        const int step = it / (16 * XG), r = (it / XG) % 16, g = it % XG, row = row0 + r;
        float z[4];
        if (step == K && a.x_T) {
#pragma unroll
            for (int k = 0; k < 4; ++k) z[k] = (row < a.E && 4 * g + k < XD) ? a.x_T[(size_t)row * XD + 4 * g + k] : 0.f;
        } else if (INJ && step < K) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                z[k] = (row < a.E && 4 * g + k < XD) ? a.noise[((size_t)step * a.E + row) * XD + 4 * g + k] : 0.f;
        } else {
            philox_normal4(a.seed, (uint32_t)g, (uint32_t)(a.env_offset + row), (uint32_t)step, a.call_id, z);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int q = 4 * g + k;
            if (q >= XD) break;
            if (step < K) {
                zt[(step * 16 + r) * XD + q] = fminf(fmaxf(z[k], -a.randn_clip), a.randn_clip);
            } else {
                xs[r * XD + q] = z[k];
                if (KF == K && a.chains && row < a.E) a.chains[((size_t)row * (KF + 1) + 0) * XD + q] = z[k];
            }
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (tid + u * ST < NB4) ((float4*)bias)[tid + u * ST] = bv[u];
    for (int i4 = tid + 4 * ST; i4 < NB4; i4 += ST) ((float4*)bias)[i4] = *bias_src(i4);
    // time embeddings t_emb(t) (mlp_diffusion.py:40-45) of the actor each step uses, from the
    // table the pack step derived (dppo_layout.h SEG_TEMB)
    if (tid < K * TD) temb[tid] = tv;
    for (int i = tid + ST; i < K * TD; i += ST)
        temb[i] = ((const float*)((i / TD < KF ? a.packed_ft : a.packed_base) + L.off[SEG_TEMB]))[i];
    if (tid < K * DPPO_SCHED_COLS) sch[tid] = scv;
    for (int i = tid + ST; i < K * DPPO_SCHED_COLS; i += ST) sch[i] = a.sched[i];
    // the resident set and the queue's first loads have landed by now; say so with a real wait
    // (not inline asm), or the waitcnt pass carries them into the loop as possibly in flight and
    // drains the queue before their first use in every layer
    __builtin_amdgcn_s_waitcnt(0x0F70);                     // vmcnt(0)
    // a pre-enqueued step waits here (everything above does not depend on the observation) for
    // the host to publish it; bounded: ~4 s, then the step runs on whatever is in the buffer and
    // flags the timeout in the high bit of *done so the host reports it
    if (a.cond_tagged) {
        sampler_load_state_tagged<ST>(a, row0, st, true, tid);
        for (int i = tid; i < 16 * SD; i += ST) {
            const int row = row0 + i / SD;
            if (a.cond_out && row < a.E) a.cond_out[(size_t)row * SD + i % SD] = st[i];
        }
    } else {
    if (a.go) {
        if (tid == 0) {
            const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 400000000ull;   // 100 MHz clock: 4 s
            while (__hip_atomic_load(a.go, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < a.go_value) {
                __builtin_amdgcn_s_sleep(8);
                if (__builtin_amdgcn_s_memrealtime() > t_end) {
                    __hip_atomic_fetch_or(a.done, 0x80000000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
            }
        }
        __syncthreads();
    }
    for (int i = tid; i < 16 * SD; i += ST) {
        const int r = i / SD, c = i % SD, row = row0 + r;
        const float v = row < a.E ? a.cond[(size_t)row * SD + c] : 0.f;
        st[i] = v;
        if (a.cond_out && row < a.E) a.cond_out[(size_t)row * SD + c] = v;
    }
    }
    __syncthreads();
    // a0 = [x, temb(t), state, 0-pad] for step 0 (t = K-1); later steps get x and temb from the
    // DDPM epilogue of the step before, the state part never changes
    for (int idx = tid; idx < 16 * k1w; idx += ST) {
        const int r = idx / k1w, c = idx % k1w;
        float v = 0.f;
        if (c < XD) v = xs[r * XD + c];
        else if (c < XD + TD) v = temb[(K - 1) * TD + c - XD];
        else if (c < a.IN) v = st[r * SD + c - XD - TD];
        a0[r * lda0 + c] = P::cvt(v);
    }
    __syncthreads();

    for (int i = 0; i < K; ++i) {
        SPHASE(0);
        const int t = K - 1 - i;
        const int is_ft = t < KF;
        const int PK = __builtin_amdgcn_readfirstlane(is_ft);
        const int PKn = __builtin_amdgcn_readfirstlane(t - 1 >= 0 ? (t - 1 < KF ? 1 : 0) : is_ft);
        if (PK != cur) {                                    // the actor switch (t = K'-1): once per launch
            load_resident(PK);
            if constexpr (LK > 0) load_lds(PK);
            // wait for the reload HERE (a real s_waitcnt the waitcnt pass sees, not inline asm):
            // otherwise the pass treats the resident registers as possibly in flight on every
            // iteration and drains the weight queue before their first use in each layer
            __builtin_amdgcn_s_waitcnt(0x0F70);             // vmcnt(0)
            if constexpr (LK > 0) __syncthreads();
            cur = PK;
        }
        const float* bb = bias + is_ft * (3 * H + NOC);
        ORing<NOK, NO> ob;                                 // out-layer fragments, consumed 3 layers later
        if constexpr (ROUT) ob = r_out;
        else out_prefetch<NOK, NO, SW>(ob, W(PK, SEG_W_OUT), L.ks_h, wave, lane);
        SPHASE(1);
        // b) in-Dense: h1 = a0 W_in + b_in  (no activation after the input layer, mlp.py:144)
        f32x4 h1[1][NT], acc[1][NT];
        if constexpr (RIN)
            gemm_res<P, NT, KSI, KSI, 0, NTOT, QD>(a0, lda0, W(PK, SEG_W_IN), r_in, nullptr, ntile0, h1, lane, R,
                                                   SNext{s_l1(PK), s_l2(PK)});
        else
            gemm_res<P, NT, KSI, 0, 0, NTOT, QD>(a0, lda0, s_in(PK).W, r_in, nullptr, ntile0, h1, lane, R,
                                                 SNext{s_l1(PK), s_l2(PK)});
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int col = (ntile0 + n) * 16 + ccol(lane);
            const float bv = bb[col];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                h1[0][n][r] += bv;
                tA[crow(lane, r) * ldh + col] = P::cvt(fmaxf(h1[0][n][r], 0.f));
            }
        }
        lds_sync();
        SPHASE(2);
        // c) l1: relu(h1) W_l1 + b -> relu -> tB   (pre-activation block, mlp.py:192-193,202-203)
        gemm_res<P, NT, KSH, RK, LK, NTOT, QD>(tA, ldh, s_l1(PK).W, r_l1, lw1, ntile0, acc, lane, R,
                                     RIN ? SNext{s_l2(PK), s_l1(PKn)} : SNext{s_l2(PK), s_in(PKn)});
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int col = (ntile0 + n) * 16 + ccol(lane);
            const float bv = bb[H + col];
#pragma unroll
            for (int r = 0; r < 4; ++r) tB[crow(lane, r) * ldh + col] = P::cvt(fmaxf(acc[0][n][r] + bv, 0.f));
        }
        lds_sync();
        SPHASE(3);
        // d) l2: relu(h2) W_l2 + b + h1 (residual, mlp.py:206) -> tA; the stream moves on to the
        //    next denoising step (possibly the other actor)
        gemm_res<P, NT, KSH, RK, LK, NTOT, QD>(tB, ldh, s_l2(PK).W, r_l2, lw2, ntile0, acc, lane, R,
                                     RIN ? SNext{s_l1(PKn), s_l2(PKn)} : SNext{s_in(PKn), s_l1(PKn)});
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int col = (ntile0 + n) * 16 + ccol(lane);
            const float bv = bb[2 * H + col];
#pragma unroll
            for (int r = 0; r < 4; ++r) tA[crow(lane, r) * ldh + col] = P::cvt(acc[0][n][r] + bv + h1[0][n][r]);
        }
        lds_sync();
        SPHASE(4);
        // e) out-Dense (N = XD <= 16*NO): k split over the waves, partials through LDS
        {
            f32x4 po[1][NO];
            gemm_narrow_pre<P, 1, NOK, NO, SW>(tA, ldh, ob, po, wave, lane);
#pragma unroll
            for (int n = 0; n < NO; ++n)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    part[(wave * 16 + crow(lane, r)) * NOC + n * 16 + ccol(lane)] = po[0][n][r];
        }
        lds_sync();
        SPHASE(5);
        // f) DDPM epilogue, fp32 (diffusion_vpg.py:198-243, 301-320)
        if (tid < 16 * XD) {
            const int r = tid / XD, q = tid % XD, row = row0 + r;
            float eps = bb[3 * H + q];
#pragma unroll
            for (int w = 0; w < SW; ++w) eps += part[(w * 16 + r) * NOC + q];
            const float* sc = sch + t * DPPO_SCHED_COLS;
            const float x = xs[tid];
            float sd = expf(0.5f * sc[4]);
            // eval noise rule of the table row (include/dppo.h: DDPM t = 0 or any DDIM row -> 0;
            // other DDPM rows clip at 1e-3; diffusion_vpg.py:303-315)
            if (a.deterministic && sc[6] != 0.f) sd = 0.f;
            else if (a.deterministic) sd = fminf(fmaxf(sd, sc[5]), 1e6f);
            else sd = fminf(fmaxf(sd, a.min_std), 1e6f);
            float xn = ddpm_post(sc[0], sc[1], sc[2], sc[3], sd, x, eps, zt[i * 16 * XD + tid]);   // (:198-242, :301-320)
            if (a.final_clip > 0.f && i == K - 1) xn = fminf(fmaxf(xn, -a.final_clip), a.final_clip);
            xs[tid] = xn;
            a0[r * lda0 + q] = P::cvt(xn);                      // next step's input
            if (row < a.E) {
                if (a.chains && t <= KF) a.chains[((size_t)row * (KF + 1) + (KF - t)) * XD + q] = xn;
                if (i == K - 1) {
                    a.actions[(size_t)row * XD + q] = xn;
                    if (a.actions_tagged)   // the action is its own flag: one aligned 8-B store
                        __hip_atomic_store(a.actions_tagged + (size_t)row * XD + q,
                                           ((uint64_t)a.cond_tag << 32) | __float_as_uint(xn), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
                    else if (a.actions_host) a.actions_host[(size_t)row * XD + q] = xn;
                }
            }
        } else if (t > 0) {                                     // the next step's time embedding
            for (int e = tid - 16 * XD; e < 16 * TD; e += ST - 16 * XD) {
                const int r = e / TD, c = e % TD;
                a0[r * lda0 + XD + c] = P::cvt(temb[(t - 1) * TD + c]);
            }
        }
        lds_sync();
        SPHASE(6);
    }
    if (a.done) {   // publish: every writer's stores reach the system before the counter moves
        __threadfence_system();
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(a.done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <class P>
static size_t sample_lds_bytes(const SampleArgs& a, int NO, int SW, int LK) {
    using AT = typename P::AT;
    const int pad = lds_pad_elems<P>();
    const int ldh = a.H + pad;
    const int lda0 = a.L.ks_in * P::KG + pad;
    size_t o = 0;
    o += dppo_align16(sizeof(AT) * 16 * ldh) * 2;
    o += dppo_align16(sizeof(AT) * 16 * lda0);
    o += dppo_align16(4 * 16 * a.XD);
    o += dppo_align16(4 * 16 * a.SD);
    o += dppo_align16(4 * a.K * a.TD);
    o += dppo_align16(4 * SW * 16 * 16 * NO);
    o += dppo_align16(4 * a.K * DPPO_SCHED_COLS);
    o += dppo_align16(4 * 2 * (3 * a.H + 16 * NO));
    o += dppo_align16(4 * a.K * 16 * a.XD);
    o += (size_t)2 * LK * (a.H / 16) * 1024;
    return o;
}

template <class P, int NT, int NO, int KSI, bool INJ, int QD, int SW, int RK, int LK, int RIO>
static int launch_sample_q(const SampleArgs& a, hipStream_t s) {
    if (a.L.ks_h != ksh_for<P>(NT, SW) || a.L.ks_in != KSI || a.L.ks_h % SW != 0)
        return dppo_set_error(DPPO_EUNSUPPORTED, "sampler: hidden %d not supported at this precision", a.H);
    const size_t lds = sample_lds_bytes<P>(a, NO, SW, LK);
    if (lds > 160 * 1024) return dppo_set_error(DPPO_EUNSUPPORTED, "sampler needs %zu B of LDS", lds);
    auto k = sample_kernel<P, NT, NO, KSI, INJ, QD, SW, RK, LK, RIO>;
    { const int rc_ = dppo_func_lds((const void*)k, (size_t)lds); if (rc_) return rc_; }
    DppoKtScope kt(KT_SAMPLER, s);
    hipLaunchKernelGGL(k, dim3(dppo_cdiv(a.E, 16)), dim3(SW * 64), lds, s, a);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

// Sampler selection (DPPO_SAMPLER_CFG, default "x"):
//   "x": the split register-resident kernel (sampler_split.hip) where it applies (2-byte operands,
//        H = 512, <= 512 envs), else the weight-streaming kernel below;
//   "r": the weight-streaming kernel always (8 waves, in/out layers + 2 hidden k-steps resident,
//        QD 3, for 2-byte operands at H = 512; 16 waves with nothing resident otherwise).
// (r01 measured five other resident-set geometries of the streaming kernel, "l", "m", "q", "i",
// "e", and two 16-wave ones: all slower; they were removed in r03 with the binary's size in mind.)
static char sampler_cfg() {
    static char c = [] {
        const char* e = getenv("DPPO_SAMPLER_CFG");
        return e && e[0] == 'r' ? 'r' : 'x';
    }();
    return c;
}

template <class P, int NT16, int NO, int KSI, bool INJ>
static int launch_sample_k(const SampleArgs& a, hipStream_t s) {
    if constexpr (P::KG == 32 && NT16 == 2) {   // 2-byte operands, H = 512
        return launch_sample_q<P, 4, NO, KSI, INJ, 3, 8, 2, 0, 3>(a, s);
    } else {
        return launch_sample_q<P, NT16, NO, KSI, INJ, 3, 16, 0, 0, 0>(a, s);
    }
}

template <class P, int NT, int NO, int KSI>
static int launch_sample(const SampleArgs& a, hipStream_t s) {
    if (a.noise) return launch_sample_k<P, NT, NO, KSI, true>(a, s);
    return launch_sample_k<P, NT, NO, KSI, false>(a, s);
}

template <class P>
static int dispatch_sample(const SampleArgs& a, hipStream_t s) {
    const int NT = a.H / (16 * 16);   // n-tiles per wave of the 16-wave layout
    const int NO = dppo_cdiv(a.XD, 16);
    const int KSI = a.L.ks_in;
#define DPPO_SAMPLE_CASE(nt, no, ksi) \
    if (NT == nt && NO == no && KSI == ksi) return launch_sample<P, nt, no, ksi>(a, s);
    if constexpr (P::KG == 32) {   // bf16: H = 512 (NT 2)
        DPPO_SAMPLE_CASE(2, 1, 2) DPPO_SAMPLE_CASE(2, 2, 2) DPPO_SAMPLE_CASE(2, 1, 4) DPPO_SAMPLE_CASE(2, 2, 4)
    } else {                       // fp32: H = 512 or 256
        DPPO_SAMPLE_CASE(2, 1, 4) DPPO_SAMPLE_CASE(2, 2, 4) DPPO_SAMPLE_CASE(1, 1, 4) DPPO_SAMPLE_CASE(1, 2, 4)
    }
#undef DPPO_SAMPLE_CASE
    return dppo_set_error(DPPO_EUNSUPPORTED, "sampler: hidden %d / action chunk %d / in-layer k-steps %d not instantiated",
                          a.H, a.XD, KSI);
}

// the geometry launch_sample_k picks, for dppo_sampler_stream_bytes
struct SamplerGeom { int SW, RK, LK, RIO; };
static SamplerGeom sampler_geom(int precision, int H) {
    if (dppo_prec_2b(precision) && H == 512) return {8, 2, 0, 3};
    return {16, 0, 0, 0};
}

extern "C" int dppo_sampler_stream_bytes(const dppo_dims* d, int precision, int64_t* bytes_per_tile, int* waves) {
    Dims D;
    int rc = dppo_check_dims(d, &D);
    if (rc) return rc;
    DPPO_CHECK(bytes_per_tile, "dppo_sampler_stream_bytes: null output");
    DPPO_CHECK(dppo_prec_ok(precision), "dppo_sampler_stream_bytes: bad precision %d", precision);
    const MlpLayout L = make_mlp_layout(D.IN, D.H, D.XD, D.TD, precision, D.K);
    const SamplerGeom g = sampler_geom(precision, D.H);
    const int64_t ntot = D.H / 16, no = dppo_cdiv(D.XD, 16);
    const int64_t in_f = (int64_t)L.ks_in * ntot, out_f = (int64_t)L.ks_h * no;
    const int64_t rin = (g.RIO & 1) ? in_f : 0, rout = (g.RIO & 2) ? out_f : 0;
    const int64_t per_step = (in_f - rin) + 2 * (L.ks_h - g.RK - g.LK) * ntot + (out_f - rout);
    const int64_t resident = rin + rout + 2 * (int64_t)(g.RK + g.LK) * ntot;
    const int actors = (D.KF > 0 && D.KF < D.K) ? 2 : 1;        // the resident set is reloaded at the switch
    *bytes_per_tile = ((int64_t)D.K * per_step + actors * resident) * 1024;
    if (waves) *waves = g.SW;
    return DPPO_OK;
}

static int sample_impl(const dppo_dims* d, int precision, const void* packed_base, const void* packed_ft,
                       const float* sched, const float* cond, int n_envs, const float* x_T, const float* noise,
                       uint64_t seed, uint64_t call_id, int env_offset, int deterministic,
                       float min_sampling_std, float randn_clip, float final_clip,
                       float* actions, float* chains, float* cond_out, float* actions_host, void* stream,
                       const uint32_t* go = nullptr, uint32_t go_value = 0, uint32_t* done = nullptr,
                       const uint64_t* cond_tagged = nullptr, uint32_t cond_tag = 0,
                       uint64_t* actions_tagged = nullptr) {
    Dims D;
    int rc = dppo_check_dims(d, &D);
    if (rc) return rc;
    DPPO_CHECK(n_envs >= 0, "dppo_sample: n_envs < 0");
    DPPO_CHECK(dppo_prec_ok(precision), "dppo_sample: bad precision %d", precision);
    if (n_envs == 0) return DPPO_OK;
    DPPO_CHECK(packed_base && packed_ft && sched && (cond || cond_tagged) && actions, "dppo_sample: null pointer argument");
    // tables an optimizer step deferred (DPPO_STEP_DEFER_SAMPLER_TABLES) are re-derived first, on this stream
    rc = dppo_refresh_sampler_tables(packed_ft, stream);
    if (rc) return rc;
    rc = dppo_refresh_sampler_tables(packed_base, stream);
    if (rc) return rc;
    SampleArgs a;
    a.packed_base = (const uint8_t*)packed_base;
    a.packed_ft = (const uint8_t*)packed_ft;
    a.sched = sched; a.cond = cond; a.x_T = x_T; a.noise = noise; a.actions = actions; a.chains = chains;
    a.cond_out = cond_out; a.actions_host = actions_host;
    a.go = go; a.go_value = go_value; a.done = done;
    a.cond_tagged = cond_tagged; a.cond_tag = cond_tag; a.actions_tagged = actions_tagged;
    a.seed = seed; a.call_id = (uint32_t)call_id; a.E = n_envs; a.env_offset = env_offset;
    a.deterministic = deterministic; a.min_std = min_sampling_std; a.randn_clip = randn_clip; a.final_clip = final_clip;
    a.XD = D.XD; a.SD = D.SD; a.TD = D.TD; a.H = D.H; a.K = D.K; a.KF = D.KF; a.IN = D.IN;
    a.L = make_mlp_layout(D.IN, D.H, D.XD, D.TD, precision, D.K);
    hipStream_t s = (hipStream_t)stream;
    if (sampler_cfg() == 'x') {
        rc = launch_sample_split(a, precision, s);
        if (rc != DPPO_EUNSUPPORTED) return rc;
    }
    return precision == DPPO_BF16 ? dispatch_sample<PolicyBF16>(a, s)
         : precision == DPPO_F16  ? dispatch_sample<PolicyF16>(a, s) : dispatch_sample<PolicyF32>(a, s);
}

extern "C" int dppo_sampler_layout(const dppo_dims* d, int precision, int n_envs, int* members) {
    Dims D;
    int rc = dppo_check_dims(d, &D);
    if (rc) return rc;
    DPPO_CHECK(members, "dppo_sampler_layout: null output");
    const MlpLayout L = make_mlp_layout(D.IN, D.H, D.XD, D.TD, precision, D.K);
    *members = sampler_cfg() == 'x' ? split_members_for(precision, D.H, D.XD, D.SD, L.ks_in, n_envs, D.K, D.KF) : 0;
    return DPPO_OK;
}

// The split kernel's members wait on each other inside a launch, so every active workgroup of a
// launch must be resident at once; a second launch in flight (the pipelined rollout's next step)
// must not take the CUs the first one still needs. One workgroup per CU (register budget), G * P
// active workgroups per launch. The streaming kernel has no inter-workgroup wait.
extern "C" int dppo_sampler_max_in_flight(const dppo_dims* d, int precision, int n_envs, int* launches) {
    int members = 0;
    int rc = dppo_sampler_layout(d, precision, n_envs, &members);
    if (rc) return rc;
    DPPO_CHECK(launches, "dppo_sampler_max_in_flight: null output");
    if (members == 0 || n_envs <= 0) {
        *launches = 8;
        return DPPO_OK;
    }
    Dims D;
    dppo_check_dims(d, &D);
    const MlpLayout L = make_mlp_layout(D.IN, D.H, D.XD, D.TD, precision, D.K);
    int plan[4];
    split_plan_query(precision, D.H, D.XD, D.SD, L.ks_in, n_envs, D.K, D.KF, plan);
    // the launch's own workgroup count (rounded as the launch rounds it), one per CU
    const int active = plan[3] > 0 ? plan[3] : dppo_cdiv(n_envs, 16) * members, cus = sampler_device_cus();
    *launches = cus > 0 ? (cus / active > 0 ? cus / active : 1) : 1;
    return DPPO_OK;
}

extern "C" int dppo_sampler_plan(const dppo_dims* d, int precision, int n_envs, int* plan) {
    Dims D;
    int rc = dppo_check_dims(d, &D);
    if (rc) return rc;
    DPPO_CHECK(plan, "dppo_sampler_plan: null output");
    const MlpLayout L = make_mlp_layout(D.IN, D.H, D.XD, D.TD, precision, D.K);
    if (sampler_cfg() == 'x') {
        split_plan_query(precision, D.H, D.XD, D.SD, L.ks_in, n_envs, D.K, D.KF, plan);
    } else {
        plan[0] = plan[1] = plan[2] = plan[3] = 0;
    }
    if (plan[0] == 0) plan[3] = dppo_cdiv(n_envs, 16);
    return DPPO_OK;
}

extern "C" int dppo_sample(const dppo_dims* d, int precision, const void* packed_base, const void* packed_ft,
                           const float* sched, const float* cond, int n_envs, const float* x_T, const float* noise,
                           uint64_t seed, uint64_t call_id, int env_offset, int deterministic,
                           float min_sampling_std, float randn_clip, float final_clip,
                           float* actions, float* chains, void* stream) {
    return sample_impl(d, precision, packed_base, packed_ft, sched, cond, n_envs, x_T, noise, seed, call_id, env_offset,
                       deterministic, min_sampling_std, randn_clip, final_clip, actions, chains, nullptr, nullptr,
                       stream);
}

// device address of pinned host memory (a cache: the rollout reuses the same staging buffers and
// counters every step); null if the memory is not mapped. One process-wide table under a mutex: a
// mapped pinned allocation has one device address for every device (unified addressing), so the
// entry does not depend on the calling thread or its current device; entries are never freed
// (dropping one only costs a hipHostGetDevicePointer), so no eviction waits on a device.
static void* mapped_ptr(const void* host) {
    constexpr int N = 32;
    static std::mutex mu;
    static const void* keys[N] = {};
    static void* vals[N] = {};
    static int next = 0;
    {
        std::lock_guard<std::mutex> lk(mu);
        for (int i = 0; i < N; ++i)
            if (keys[i] == host && vals[i]) return vals[i];
    }
    void* dev = nullptr;
    if (hipHostGetDevicePointer(&dev, const_cast<void*>(host), 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(mu);
    keys[next] = host; vals[next] = dev;
    next = (next + 1) % N;
    return dev;
}

// One rollout step's device work in one call (train_ppo_diffusion_agent.py:106-122): the sampler
// reads the observation straight from the mapped pinned buffer (and copies it into its rollout
// slot), writes the actions straight into the mapped pinned action buffer, and the host waits
// for the stream — no copy kernels in the step. Unmapped staging memory falls back to two
// hipMemcpyAsync around the launch.
extern "C" int dppo_sample_step(const dppo_dims* d, int precision, const void* packed_base, const void* packed_ft,
                                const float* sched, const float* cond_host, float* cond, int n_envs, uint64_t seed,
                                uint64_t call_id, int env_offset, int deterministic, float min_sampling_std,
                                float randn_clip, float final_clip, float* actions, float* actions_host,
                                float* chains, int synchronize, void* stream) {
    Dims D;
    int rc = dppo_check_dims(d, &D);
    if (rc) return rc;
    if (n_envs == 0) return DPPO_OK;
    DPPO_CHECK(cond_host && cond && actions && actions_host, "dppo_sample_step: null pointer argument");
    hipStream_t s = (hipStream_t)stream;
    const float* cond_dev_view = (const float*)mapped_ptr(cond_host);
    float* act_dev_view = (float*)mapped_ptr(actions_host);
    if (cond_dev_view && act_dev_view) {
        rc = sample_impl(d, precision, packed_base, packed_ft, sched, cond_dev_view, n_envs, nullptr, nullptr, seed,
                         call_id, env_offset, deterministic, min_sampling_std, randn_clip, final_clip, actions, chains,
                         cond, act_dev_view, stream);
        if (rc) return rc;
    } else {
        DPPO_HIP(hipMemcpyAsync(cond, cond_host, sizeof(float) * (size_t)n_envs * D.SD, hipMemcpyHostToDevice, s));
        rc = dppo_sample(d, precision, packed_base, packed_ft, sched, cond, n_envs, nullptr, nullptr, seed, call_id,
                         env_offset, deterministic, min_sampling_std, randn_clip, final_clip, actions, chains, stream);
        if (rc) return rc;
        DPPO_HIP(hipMemcpyAsync(actions_host, actions, sizeof(float) * (size_t)n_envs * D.XD, hipMemcpyDeviceToHost, s));
    }
    if (synchronize) DPPO_HIP(hipStreamSynchronize(s));
    return DPPO_OK;
}

// ---- pipelined rollout steps (see include/dppo.h) ----
extern "C" int dppo_host_alloc(size_t bytes, void** ptr) {
    DPPO_CHECK(ptr && bytes > 0, "dppo_host_alloc: bad arguments");
    DPPO_HIP(hipHostMalloc(ptr, bytes, hipHostMallocMapped | hipHostMallocCoherent));
    memset(*ptr, 0, bytes);
    return DPPO_OK;
}

// Up to 4 host-mapped -> device copies in ONE kernel launch (the rollout's reward / termination /
// first flags into the update's device buffers). hipMemcpyAsync of the same pinned buffers went through
// the SDMA path, where the second and third copies started ~0.9 ms after they were issued with the
// device idle (r03 HIP trace: rollout -> update gap 1.2-2.1 ms per iteration); a kernel reading the
// coherent mapped memory over the bus runs as soon as the stream reaches it.
struct HostCopies { const uint8_t* src[4]; uint8_t* dst[4]; size_t n[4]; };
__global__ __launch_bounds__(256) void copy_host_kernel(HostCopies c) {
    const size_t stride = (size_t)gridDim.x * 256, t0 = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (int r = 0; r < 4; ++r) {
        if (!c.n[r]) continue;
        const uint8_t* s = c.src[r];
        uint8_t* d = c.dst[r];
        const size_t n = c.n[r];
        if ((((uintptr_t)s | (uintptr_t)d) & 15) == 0) {
            const size_t n16 = n / 16;
            for (size_t i = t0; i < n16; i += stride) ((uint4*)d)[i] = ((const uint4*)s)[i];
            for (size_t i = 16 * n16 + t0; i < n; i += stride) d[i] = s[i];
        } else {
            for (size_t i = t0; i < n; i += stride) d[i] = s[i];
        }
    }
}

extern "C" int dppo_copy_from_host(int n, void* const* dst, const void* const* src_host, const size_t* bytes, void* stream) {
    DPPO_CHECK(n >= 0 && n <= 4 && (n == 0 || (dst && src_host && bytes)), "dppo_copy_from_host: bad arguments");
    HostCopies c = {};
    size_t total = 0;
    for (int i = 0; i < n; ++i) {
        DPPO_CHECK(bytes[i] == 0 || (dst[i] && src_host[i]), "dppo_copy_from_host: null range %d", i);
        c.src[i] = (const uint8_t*)mapped_ptr(src_host[i]);
        DPPO_CHECK(bytes[i] == 0 || c.src[i], "dppo_copy_from_host: source %d is not mapped host memory (dppo_host_alloc)", i);
        c.dst[i] = (uint8_t*)dst[i];
        c.n[i] = bytes[i];
        total += bytes[i];
    }
    if (total == 0) return DPPO_OK;
    const size_t blocks = (total / 16 + 255) / 256;
    hipLaunchKernelGGL(copy_host_kernel, dim3((unsigned)(blocks < 1 ? 1 : (blocks > 256 ? 256 : blocks))), dim3(256), 0,
                       (hipStream_t)stream, c);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

extern "C" int dppo_host_free(void* ptr) {
    if (ptr) DPPO_HIP(hipHostFree(ptr));
    return DPPO_OK;
}

extern "C" int dppo_rollout_enqueue(const dppo_dims* d, int precision, const void* packed_base, const void* packed_ft,
                                    const float* sched, const float* cond_host, float* cond, int n_envs, uint64_t seed,
                                    uint64_t call_id, int env_offset, int deterministic, float min_sampling_std,
                                    float randn_clip, float final_clip, float* actions, float* actions_host,
                                    float* chains, const uint32_t* go, uint32_t go_value, uint32_t* done, void* stream) {
    DPPO_CHECK(cond_host && cond && actions && actions_host && go && done, "dppo_rollout_enqueue: null pointer argument");
    const float* cond_dev = (const float*)mapped_ptr(cond_host);
    float* act_dev = (float*)mapped_ptr(actions_host);
    const uint32_t* go_dev = (const uint32_t*)mapped_ptr(go);
    uint32_t* done_dev = (uint32_t*)mapped_ptr(done);
    DPPO_CHECK(cond_dev && act_dev && go_dev && done_dev,
               "dppo_rollout_enqueue: staging buffers must come from dppo_host_alloc (mapped, coherent)");
    return sample_impl(d, precision, packed_base, packed_ft, sched, cond_dev, n_envs, nullptr, nullptr, seed, call_id,
                       env_offset, deterministic, min_sampling_std, randn_clip, final_clip, actions, chains, cond,
                       act_dev, stream, go_dev, go_value, done_dev);
}

extern "C" int dppo_rollout_enqueue_tagged(const dppo_dims* d, int precision, const void* packed_base,
                                           const void* packed_ft, const float* sched, const uint64_t* obs_tagged,
                                           float* cond, int n_envs, uint64_t seed, uint64_t call_id, int env_offset,
                                           int deterministic, float min_sampling_std, float randn_clip,
                                           float final_clip, float* actions, uint64_t* actions_tagged, float* chains,
                                           uint32_t tag, uint32_t* done, void* stream) {
    DPPO_CHECK(obs_tagged && cond && actions && actions_tagged && done,
               "dppo_rollout_enqueue_tagged: null pointer argument");
    DPPO_CHECK(tag != 0, "dppo_rollout_enqueue_tagged: tag 0 is the buffer's initial value");
    const uint64_t* obs_dev = (const uint64_t*)mapped_ptr(obs_tagged);
    uint64_t* act_dev = (uint64_t*)mapped_ptr(actions_tagged);
    uint32_t* done_dev = (uint32_t*)mapped_ptr(done);
    DPPO_CHECK(obs_dev && act_dev && done_dev,
               "dppo_rollout_enqueue_tagged: staging buffers must come from dppo_host_alloc (mapped, coherent)");
    return sample_impl(d, precision, packed_base, packed_ft, sched, nullptr, n_envs, nullptr, nullptr, seed, call_id,
                       env_offset, deterministic, min_sampling_std, randn_clip, final_clip, actions, chains, cond,
                       nullptr, stream, nullptr, 0, done_dev, obs_dev, tag, act_dev);
}
