// rowtile.hip — row-tile fused MLP kernels for the update half of the hot path.
//
// One workgroup (8 waves) owns 16*MT rows and runs a whole residual MLP on them with the
// activations in LDS and the weights streamed in fragment order (dppo_common.cuh):
//   actor, mode LOGPROB : DiffusionMLP forward + p_mean_var + Normal.log_prob epilogue
//                         (VPGDiffusion.get_logprobs, model/diffusion/diffusion_vpg.py:343-425)
//   actor, mode TRAIN   : rows gathered through the minibatch permutation
//                         (train_ppo_diffusion_agent.py:287-312) -> forward -> fused c_loss policy
//                         term and its gradient (diffusion_ppo.py:45-106) -> backward dX chain,
//                         writing feature-major activation/gradient images for the dW kernel
//   critic, mode VALUE  : CriticObs forward (model/common/critic.py:40-54)
//   critic, mode TRAIN  : forward -> v_loss gradient (diffusion_ppo.py:108-118) -> backward chain
#include <stdlib.h>
#include <type_traits>
#include <string.h>
#include "dppo_ppo.h"
#include "rowtile_common.cuh"


// weight-stream queue depth of the actor row tile (k-steps in flight per wave; tuning knob)
#ifndef DPPO_ROWTILE_QD
#define DPPO_ROWTILE_QD 3
#endif

// Phase timing for tuning builds (tools/variant_build.sh ... -DDPPO_ROWTILE_TIMING): wave 0 of
// every workgroup adds the shader-clock cycles it spent in each phase (barrier waits included).
#ifdef DPPO_ROWTILE_TIMING
__device__ unsigned long long dppo_phase_cycles[32];
#define PHASE(k)                                                                  \
    do {                                                                          \
        if (threadIdx.x == 0) {                                                   \
            const unsigned long long now_ = __builtin_readcyclecounter();         \
            atomicAdd(&dppo_phase_cycles[(k)], now_ - t_phase_);                  \
            t_phase_ = now_;                                                      \
        }                                                                         \
    } while (0)
#define PHASE_START unsigned long long t_phase_ = __builtin_readcyclecounter()
extern "C" DPPO_API int dppo_debug_phase_cycles(unsigned long long* out, int reset) {
    DPPO_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(dppo_phase_cycles), sizeof(unsigned long long) * 32));
    if (reset) {
        unsigned long long z[32] = {};
        DPPO_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dppo_phase_cycles), z, sizeof(z)));
    }
    return DPPO_OK;
}
#else
#define PHASE(k) do {} while (0)
#define PHASE_START do {} while (0)
#endif

// =============================================================================================
// actor
// =============================================================================================
template <class P, int MT>
struct ActorSmem {
    static constexpr int ROWS = 16 * MT;
    size_t tA, tB, a0, xp, xn, st, temb, sch, rn, rj, radv, rlpo, nrm, bias, total;
    __host__ __device__ ActorSmem(const ActorArgs& a) {
        using AT = typename P::AT;
        const int pad = lds_pad_elems<P>();
        const int ldh = a.H + pad, lda0 = a.L.ks_in * P::KG + pad;
        size_t o = 0;
        tA = o; o += dppo_align16(sizeof(AT) * ROWS * ldh);
        tB = o; o += dppo_align16(sizeof(AT) * ROWS * ldh);
        a0 = o; o += dppo_align16(sizeof(AT) * ROWS * lda0);
        xp = o; o += dppo_align16(4 * ROWS * a.XD);
        xn = o; o += dppo_align16(4 * ROWS * a.XD);
        st = o; o += dppo_align16(4 * ROWS * a.SD);
        temb = o; o += dppo_align16(4 * a.KF * a.TD);
        sch = o; o += dppo_align16(4 * a.KF * DPPO_SCHED_COLS);
        rn = o; o += dppo_align16(4 * ROWS);
        rj = o; o += dppo_align16(4 * ROWS);
        radv = o; o += dppo_align16(4 * ROWS);
        rlpo = o; o += dppo_align16(4 * ROWS);
        nrm = o; o += 16;
        bias = o; o += dppo_align16(4 * (3 * a.H + 16 * dppo_cdiv(a.XD, 16)));
        total = o;
    }
};

template <class P, int MT, int NT, int NO, int KSI, bool TRAIN, int WAVES>
__device__ __forceinline__ void actor_rowtile_body(const ActorArgs& a) {
    using AT = typename P::AT;
    constexpr int THREADS = 64 * WAVES;
    constexpr int ROWS = 16 * MT;
    static_assert(ROWS <= 64, "the epilogue maps one row per lane of wave 0");
    constexpr int KSH = ksh_for<P>(NT, WAVES);
    constexpr int NOK = nok_for<P>(NT);
    constexpr int KSO = 2;
    PHASE_START;   // k-steps of the transposed out layer (out dim <= 2*KG, padded even)
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const MlpLayout& L = a.L;
    const ActorSmem<P, MT> S(a);
    const int pad = lds_pad_elems<P>();
    const int ldh = a.H + pad;
    const int k1w = L.ks_in * P::KG, lda0 = k1w + pad;
    const int ktw = L.ks_out_t * P::KG;   // width of the dy tile (A operand of dh3 = dy W_out^T)
    const int XD = a.XD, SD = a.SD, TD = a.TD, KF = a.KF, IN = a.IN;
    constexpr bool train = TRAIN;
    // pretraining (ROWS_PRETRAIN) runs the TRAIN body with its own prologue rows and epilogue loss
    const bool pre = train && a.mode == ROWS_PRETRAIN;
    const int H = a.H;
    AT* tA = (AT*)(smem + S.tA);
    AT* tB = (AT*)(smem + S.tB);
    AT* a0 = (AT*)(smem + S.a0);
    float* bias = (float*)(smem + S.bias);   // [in, l1, l2][H], out[16*NO]
    float* xp = (float*)(smem + S.xp);
    float* xn = (float*)(smem + S.xn);
    float* st = (float*)(smem + S.st);
    float* temb = (float*)(smem + S.temb);
    float* sch = (float*)(smem + S.sch);
    int* rn = (int*)(smem + S.rn);
    int* rj = (int*)(smem + S.rj);
    float* radv = (float*)(smem + S.radv);   // per row: the row's advantage (train)
    float* rlpo = (float*)(smem + S.rlpo);   // per row: its old log-prob (train)
    float* nrm = (float*)(smem + S.nrm);     // advantage normalisation: mean, std + 1e-8
    float* part = (float*)(smem + S.tA);   // out-layer partials alias tA (relu(h1) is dead after L2)
    const size_t grow0 = (size_t)a.row0 + (size_t)blockIdx.x * ROWS;
    const __amdgpu_buffer_rsrc_t wsr = packed_rsrc(a.ws.base);
    const uint32_t ldm32 = (uint32_t)a.ws.ldm, grow32 = (uint32_t)grow0;

    // ---- prologue: rows, gathers, schedule, biases, time embedding for t < K' (actor_ft) ----
    // Its barriers are LDS-only (lds_sync): a __syncthreads() waits vmcnt(0), i.e. for the primed
    // weight stream and every gather, at each of the three barriers. Each LDS write below takes its
    // value from a global load the compiler waits for first, so lgkmcnt(0) + s_barrier publishes
    // it; the image stores (a0T, seg) stay in flight (only later kernels read them).
    // The weight stream starts first (its latency overlaps everything below). One thread per row
    // maps it through the minibatch permutation (Feistel cycle-walk: done once per row) and
    // fetches the row's per-sample scalars; the chains / obs gathers follow one barrier later.
    const int ntile0 = wave * NT;
    const __amdgpu_buffer_rsrc_t rs = packed_rsrc(a.packed);
    auto W = [&](int seg) { return wsrc(rs, L.off[seg]); };
    constexpr int QD = DPPO_ROWTILE_QD;   // weight k-steps in flight per wave
    WQueue<QD, NT> R;
    // the stream after L1: l1 (L2), then (train) the backward's W_out^T, M^T and l1^T
    const NextLayers after_l1 = train ? NextLayers{W(SEG_W_L1), KSH, W(SEG_T_OUT), KSO}
                                      : NextLayers{W(SEG_W_L1), KSH, W(SEG_W_L1), KSH};
    queue_prime(R, W(SEG_W_IN), KSI, after_l1, ntile0, lane);
    // Phase 1 computes only the row map, so its barrier waits on no global load: the per-row
    // advantage / old log-prob and the minibatch moments are loaded into registers here and
    // reach LDS after L1 (first read in the epilogue); parameters and gathers share phase 2.
    float pre_adv = 0.f, pre_lpo = 0.f, pre_m = 0.f, pre_s = 0.f;
    if (tid < ROWS) {
        const int64_t gr = (int64_t)grow0 + tid;
        int n = -1, j = 0;
        if (gr < a.nrows) {
            if (pre) {                         // row = sample; t = KF-1-j below, KF = K
                n = (int)gr;
                j = KF - 1 - a.tsteps[gr];
            } else if (train) {
                const uint64_t idx = minibatch_row(a.row_index, (uint64_t)(a.start + gr), a.fk);
                if (idx < a.fk.n) {   // tf.unravel_index; sample counts are < 2^32 (host-checked)
                    n = (int)((uint32_t)idx / (uint32_t)KF);
                    j = (int)((uint32_t)idx - (uint32_t)n * (uint32_t)KF);
                }
            } else {
                n = (int)((uint64_t)gr / (uint64_t)KF);
                j = (int)((uint64_t)gr - (uint64_t)n * (uint64_t)KF);
            }
        }
        rn[tid] = n; rj[tid] = j;
        if (train && !pre) {
            pre_adv = n >= 0 ? a.adv[n] : 0.f;
            pre_lpo = n >= 0 ? a.lp_old[(size_t)n * KF + j] : 0.f;
        }
    } else if (train && !pre && tid == ROWS) {   // population mean / std of the minibatch (diffusion_ppo.py:74-75)
        const double* S3 = a.adv_stats;
        const double mean = S3[1] / S3[0];
        const double var = fmax(S3[2] / S3[0] - mean * mean, 0.0);
        pre_m = (float)mean;
        pre_s = (float)(sqrt(var) + 1e-8);
    }
    lds_sync();
    // time embeddings t_emb(r TS), r < K' (mlp_diffusion.py:40-45): rows of the image's TEMB table,
    // which the fold launch after every write of the image re-derives (pack.hip rt_fold_kernel; r05's
    // in-tile derivation, three dependent phases of global reads, took 11k of a tile's cycles)
    const float* temb_img = (const float*)(a.packed + L.off[SEG_TEMB]);
    for (int i = tid; i < KF * TD; i += THREADS) temb[i] = temb_img[i];
    for (int i = tid; i < KF * DPPO_SCHED_COLS; i += THREADS) sch[i] = a.sched[i];
    for (int i = tid; i < 3 * H + 16 * NO; i += THREADS) {
        // the out-Dense bias with b_in and b_l2 folded through it (RT_BOUT: the forward runs no l2 GEMM)
        const int seg = i < H ? SEG_B_IN : (i < 2 * H ? SEG_B_L1 : (i < 3 * H ? SEG_B_L2 : SEG_RT_BOUT));
        const int j = i < 3 * H ? i % H : i - 3 * H;
        bias[i] = ((const float*)(a.packed + L.off[seg]))[j];
    }
    for (int i = tid; i < ROWS * XD; i += THREADS) {
        const int r = i / XD, q = i % XD, n = rn[r];
        float vp = 0.f, vn = 0.f;
        if (n >= 0 && pre) {
            // q_sample (diffusion.py:196-202): x_t = sqrt(ac_t) x_0 + sqrt(1 - ac_t) noise; xn keeps the noise
            const int t = KF - 1 - rj[r];
            const float z = a.noise[(size_t)n * XD + q];
            vp = a.qsched[2 * t] * a.chains[(size_t)n * XD + q] + a.qsched[2 * t + 1] * z;
            vn = z;
        } else if (n >= 0) {
            const float* c = a.chains + ((size_t)n * (KF + 1) + rj[r]) * XD + q;
            vp = c[0]; vn = c[XD];   // chains_prev = chains[:, j], chains_next = chains[:, j+1]
        }
        xp[i] = vp; xn[i] = vn;
    }
    for (int i = tid; i < ROWS * SD; i += THREADS) {
        const int r = i / SD, c = i % SD, n = rn[r];
        st[i] = n >= 0 ? a.obs[(size_t)n * SD + c] : 0.f;
    }
    lds_sync();
    // a0 = [x_prev, temb(t), state] (mlp_diffusion.py:86), t = K'-1-j (diffusion_vpg.py:456-458)
    for (int i = tid; i < ROWS * k1w; i += THREADS) {
        const int r = i / k1w, c = i % k1w;
        const int t = KF - 1 - rj[r];
        float v = 0.f;
        if (c < XD) v = xp[r * XD + c];
        else if (c < XD + TD) v = temb[t * TD + c - XD];
        else if (c < IN) v = st[r * SD + c - XD - TD];
        a0[r * lda0 + c] = P::cvt(v);
    }
    if (train) {   // a0T image (permuted row order, img_pos) and the per-row t bucket
        for (int i = tid; i < (ROWS / 8) * IN; i += THREADS) {
            const int c = i / (ROWS / 8), g = i % (ROWS / 8);
            store_img8<P>(a.ws.a0T, a.ws.ldm, grow0, c, g, [&](int r) {
                const int t = KF - 1 - rj[r];
                return c < XD ? xp[r * XD + c] : (c < XD + TD ? temb[t * TD + c - XD] : st[r * SD + c - XD - TD]);
            });
        }
        if (tid < ROWS) a.ws.seg[grow0 + img_pos(tid)] = rn[tid] >= 0 ? (int8_t)(KF - 1 - rj[tid]) : (int8_t)-1;
    }
    lds_sync();

    PHASE(0);
    f32x4 acc[MT][NT];
    // relu masks: one bit per accumulator element (64-bit for 64x64 wave tiles)
    using MaskT = typename std::conditional<(MT * NT * 4 > 32), uint64_t, uint32_t>::type;
    static_assert(MT * NT * 4 <= 64, "relu masks are at most 64-bit");
    MaskT mask1 = 0, mask2 = 0;
    // The weight stream is one QD-deep queue per wave through every layer of the kernel:
    //   in -> l1 -> [train] out^T -> M^T -> l1^T. The l2 layer never runs as a GEMM: the residual block
    //   is linear from the l2 product to the out-Dense (mlp.py:186-206), so
    //     eps  = relu(h2) M + a0 M0 + RT_BOUT,    M = W_l2 W_out, M0 = W_in W_out  (dppo_layout.h RT_*)
    //     d relu(h2) = dy M^T,                    dh3 = dy W_out^T (the residual's share of dh1)
    //   with M, M0 as 2-byte hi/lo pairs (fp32 products of the rounded weights): h3 is never formed,
    //   so it is never rounded (the oracle's round_h3=False rounding points).
    constexpr bool TWO = sizeof(AT) == 2;
    const size_t fold_mat = packed_matrix_bytes(H, XD, P::KG), fold0_mat = packed_matrix_bytes(IN, XD, P::KG);
    ORing<NOK, NO> obh, obl;              // RT_FOLD hi / lo fragments of this wave's k-steps
    u32x4 o0[2][NO];                      // RT_FOLD0 hi / lo of k-step `wave` (waves < KSI)
    // ---- L1: h1 = a0 W_in + b (no activation on the input layer) ----
    gemm_queue<P, MT, NT, KSI, QD>(a0, lda0, W(SEG_W_IN), ntile0, acc, lane, R, after_l1);
    add_bias(acc, bias, ntile0, lane);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (acc[m][n][r] > 0.f) mask1 |= MaskT(1) << ((m * NT + n) * 4 + r);
                acc[m][n][r] = fmaxf(acc[m][n][r], 0.f);
            }
    // materialise the mask now (otherwise hipcc keeps the 8*MT*NT floats alive until the backward)
    asm volatile("" : "+v"(mask1));
    store_acc_lds<P, MT, NT>(tA, ldh, ntile0, lane, acc);
    if constexpr (train) store_accT<P, MT, NT>(wsr, ws_off(a.ws, a.ws.u1T), ldm32, ntile0, grow32, lane, acc);
    lds_sync();
    PHASE(1);
    if (train && !pre) {   // loaded in the prologue, read from the epilogue on (after later barriers)
        if (tid < ROWS) { radv[tid] = pre_adv; rlpo[tid] = pre_lpo; }
        else if (tid == ROWS) { nrm[0] = pre_m; nrm[1] = pre_s; }
    }
    // ---- L2: h2 = relu(h1) W_l1 + b ----
    if constexpr (train)
        gemm_queue<P, MT, NT, KSH, QD>(tA, ldh, W(SEG_W_L1), ntile0, acc, lane, R,
                                       NextLayers{W(SEG_T_OUT), KSO, W(SEG_RT_TFOLD), KSO});
    else
        gemm_queue<P, MT, NT, KSH, QD, true, true>(tA, ldh, W(SEG_W_L1), ntile0, acc, lane, R, after_l1);
    add_bias(acc, bias + H, ntile0, lane);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (acc[m][n][r] > 0.f) mask2 |= MaskT(1) << ((m * NT + n) * 4 + r);
                acc[m][n][r] = fmaxf(acc[m][n][r], 0.f);
            }
    asm volatile("" : "+v"(mask2));
    store_acc_lds<P, MT, NT>(tB, ldh, ntile0, lane, acc);
    if constexpr (train) store_accT<P, MT, NT>(wsr, ws_off(a.ws, a.ws.u2T), ldm32, ntile0, grow32, lane, acc);
    // the folded out-Dense's fragments: fetched after the l1 result's stores (held
    // through them they pushed the 16-wave tile into spills), landing during the barrier
    out_prefetch<NOK, NO, WAVES>(obh, W(SEG_RT_FOLD), KSH, wave, lane);
    if constexpr (TWO) out_prefetch<NOK, NO, WAVES>(obl, wsrc(rs, L.off[SEG_RT_FOLD] + fold_mat), KSH, wave, lane);
    if (wave < KSI) {
#pragma unroll
        for (int n = 0; n < NO; ++n) {
            o0[0][n] = load_bfrag_c(W(SEG_RT_FOLD0), KSI, n, wave, lane);
            if constexpr (TWO) o0[1][n] = load_bfrag_c(wsrc(rs, L.off[SEG_RT_FOLD0] + fold0_mat), KSI, n, wave, lane);
        }
    }
    lds_sync();
    PHASE(2);
    // ---- L4 (folded): eps = relu(h2) M + a0 M0 + RT_BOUT; the relu(h2) k-steps dealt over the waves
    //      (NOK each), a0's KSI k-steps to waves 0..KSI-1; partials reduce through LDS ----
    {
        f32x4 po[MT][NO];
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < NO; ++n) zero_acc(po[m][n]);
#pragma unroll
        for (int i = 0; i < NOK; ++i)
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                const u32x4 av = lds_afrag<P>(tB, ldh, m, wave + WAVES * i, lane);
#pragma unroll
                for (int n = 0; n < NO; ++n) {
                    po[m][n] = P::mma(av, obh.b[i][n], po[m][n]);
                    if constexpr (TWO) po[m][n] = P::mma(av, obl.b[i][n], po[m][n]);
                }
            }
        if (wave < KSI) {
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                const u32x4 av = lds_afrag<P>(a0, lda0, m, wave, lane);
#pragma unroll
                for (int n = 0; n < NO; ++n) {
                    po[m][n] = P::mma(av, o0[0][n], po[m][n]);
                    if constexpr (TWO) po[m][n] = P::mma(av, o0[1][n], po[m][n]);
                }
            }
        }
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < NO; ++n)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    part[(wave * ROWS + m * 16 + crow(lane, r)) * (16 * NO) + n * 16 + ccol(lane)] = po[m][n][r];
    }
    lds_sync();

    PHASE(4);
    // ---- epilogue: p_mean_var + Normal.log_prob (+ c_loss policy term and its gradient) ----
    // Spread over the whole workgroup: (A) one (row, q) element per thread -> log-prob, mean,
    // clip flags into scratch in tA (h3 is dead once the out layer has run); (B) one row per lane
    // of wave 0 -> the row's mean log-prob and loss terms; (C) one (row, q) element per thread ->
    // d loss / d eps into the dy tile (A operand of the backward) and the dyT image.
    const float* bo = bias + 3 * H;            // RT_BOUT
    const int nh = min(a.hp.reward_horizon, XD / a.Da) * a.Da;                      // [:, :reward_horizon]
    float* e_lp = (float*)tB;                  // [ROWS][XD] (relu(h2) is dead once the out layer has run)
    float* e_mu = e_lp + ROWS * XD;            // [ROWS][XD]
    float* e_uc = e_mu + ROWS * XD;            // [ROWS][XD] 1 = x_recon not clipped
    float* e_dn = e_uc + ROWS * XD;            // [ROWS] d loss / d newlogprob
    auto row_sd = [&](int r) {                 // diffusion_vpg.py:473-474
        const float* sc = sch + (KF - 1 - rj[r]) * DPPO_SCHED_COLS;
        return fminf(fmaxf(expf(0.5f * sc[4]), a.hp.min_lp_std), 1e6f);
    };
    for (int idx = tid; idx < ROWS * XD && !pre; idx += THREADS) {
        const int r = idx / XD, q = idx % XD;
        const float* sc = sch + (KF - 1 - rj[r]) * DPPO_SCHED_COLS;
        const float sd = row_sd(r);
        float eps = bo[q];
#pragma unroll
        for (int w = 0; w < WAVES; ++w) eps += part[(w * ROWS + r) * (16 * NO) + q];
        const float x = xp[r * XD + q];
        float xr = sc[0] * x - sc[1] * eps;
        e_uc[idx] = fabsf(xr) <= 1.f ? 1.f : 0.f;
        xr = fminf(fmaxf(xr, -1.f), 1.f);
        const float mu = sc[2] * xr + sc[3] * x;
        const float z = (xn[r * XD + q] - mu) / sd;
        const float lp = -0.5f * z * z - logf(sd) - LOG_2PI_HALF;
        e_lp[idx] = lp;
        e_mu[idx] = mu;
        if (!train && rn[r] >= 0 && a.lp_elem) a.lp_elem[((size_t)rn[r] * KF + rj[r]) * XD + q] = lp;
    }
    lds_sync();
    PHASE(5);
    if (tid < 64 && !pre) {
        const int r = tid;
        float pg = 0.f, kl = 0.f, cf = 0.f, ra = 0.f, dnewlp = 0.f;
        if (r < ROWS) {
            const int n = rn[r], j = rj[r];
            float lpsum = 0.f;
            for (int q = 0; q < nh; ++q) lpsum += fminf(fmaxf(e_lp[r * XD + q], -5.f), 2.f);
            const float newlp = lpsum / (float)nh;
            if (!train) {
                if (n >= 0 && a.lp_mean) a.lp_mean[(size_t)n * KF + j] = newlp;
            } else if (n >= 0) {
                float A = radv[r];
                if (a.hp.norm_adv) A = (A - nrm[0]) / nrm[1];   // population std over the minibatch (:74-75)
                A *= powf(a.hp.gamma_denoising, (float)(KF - j - 1));                 // :83-86
                const float oldlp = rlpo[r];
                const float logratio = newlp - oldlp;
                const float ratio = expf(logratio);
                float cc;                                                              // :93-101
                if (KF > 1) {
                    const float tf = (float)j / (float)(KF - 1);
                    cc = a.hp.clip_coef_base + (a.hp.clip_coef - a.hp.clip_coef_base) *
                         (expf(a.hp.clip_coef_rate * tf) - 1.f) / (expf(a.hp.clip_coef_rate) - 1.f);
                } else {
                    cc = (float)j;
                }
                const float pg1 = -A * ratio;
                const float rcl = fminf(fmaxf(ratio, 1.f - cc), 1.f + cc);
                const float pg2 = -A * rcl;
                pg = fmaxf(pg1, pg2);
                kl = (ratio - 1.f) - logratio;
                cf = fabsf(ratio - 1.f) > cc ? 1.f : 0.f;
                ra = ratio;
                const bool in_r = ratio >= 1.f - cc && ratio <= 1.f + cc;
                const float dpg = (pg1 >= pg2) ? -A : (in_r ? -A : 0.f);   // tf.maximum ties -> first arg
                dnewlp = dpg * ratio * a.hp.grad_scale;
            }
            e_dn[r] = dnewlp;
        }
        if (train) {
            pg = wave_sum(pg); kl = wave_sum(kl); cf = wave_sum(cf); ra = wave_sum(ra);
            if (tid == 0) {
                atomic_add_metric(a.metrics, 0, pg);
                atomic_add_metric(a.metrics, 2, kl);
                atomic_add_metric(a.metrics, 3, cf);
                atomic_add_metric(a.metrics, 4, ra);
            }
        }
    }
    if constexpr (!train) return;
    lds_sync();
    PHASE(6);
    // d loss / d eps through clip(lp), Normal.log_prob, mu and clip(x_recon); idx -> (q, r) with r
    // fastest so the dyT image stores coalesce
    AT* dyt = a0;   // a0 tile is dead after L1; dy tile has row stride lda0
    float sq = 0.f;                      // pretrain: this thread's sum of (eps - noise)^2
    float geta = 0.f;                    // learnable DDIM eta: this thread's share of d loss / d eta
    const bool leta = a.hp.eta_unscale != 0.f;
    // 2-byte operands: columns [LOK, LOK + XD) of the dy tile repeat dy, the A operand of M^T's lo half
    // (RT_TFOLD); the dyT image and the metric sums take the first copy only
    const int LOK = rt_tfold_lok(KSO, P::KG);
    for (int idx = tid; idx < ROWS * ktw; idx += THREADS) {
        const int qa = idx / ROWS, r = idx % ROWS;
        const bool dup = TWO && qa >= LOK;
        const int q = dup ? qa - LOK : qa;
        float d = 0.f;
        if (pre) {
            // p_losses, predict_epsilon (diffusion.py:186-194): mean((eps - noise)^2)
            if (q < XD && rn[r] >= 0) {
                float eps = bo[q];
#pragma unroll
                for (int w = 0; w < WAVES; ++w) eps += part[(w * ROWS + r) * (16 * NO) + q];
                const float e = eps - xn[r * XD + q];
                if (!dup) sq += e * e;
                d = a.pre_scale * e;
            }
        } else if (q < XD && q < nh && rn[r] >= 0) {
            const int e = r * XD + q;
            const float lp = e_lp[e];
            const float sd = row_sd(r);
            const float* sc = sch + (KF - 1 - rj[r]) * DPPO_SCHED_COLS;
            const float dlp = (lp >= -5.f && lp <= 2.f) ? e_dn[r] / (float)nh : 0.f;
            const float res = xn[r * XD + q] - e_mu[e];
            const float dmu = dlp * res / (sd * sd);
            d = e_uc[e] != 0.f ? -sc[1] * sc[2] * dmu : 0.f;
            if (leta && !dup) {
                // DDIM row (include/dppo.h): mu = sqrt(abar_prev) x0 + dd eps', sigma = max(eta s, 1e-10),
                // dd = sqrt(clip(1 - abar_prev - sigma^2, 0, 1e6)); d mu / d eta = (d dd / d eta) eps' with
                // eps' = (x - sqrt(abar) x0) / sqrt(1 - abar) = (x - x0 / c0) c0 / c1, dd = c3 c1 / c0;
                // d std / d eta = s where sigma is neither clamped nor clipped (oracle ddim_eta_grad_terms)
                const float s = sc[7];
                const float sig = expf(0.5f * sc[4]);
                const float x = xp[r * XD + q];
                float eps = bo[q];   // the out-layer partials in tB are still live (as in the pretrain branch)
#pragma unroll
                for (int w = 0; w < WAVES; ++w) eps += part[(w * ROWS + r) * (16 * NO) + q];
                const float x0 = fminf(fmaxf(sc[0] * x - sc[1] * eps, -1.f), 1.f);
                const float ep2 = (x - x0 / sc[0]) * sc[0] / sc[1];
                const float dd = sc[3] * sc[1] / sc[0];
                const bool free_sig = sig > 1e-10f * 1.0001f;
                const float ddd = (dd > 0.f && free_sig) ? -sig * s / dd : 0.f;
                const float dstd = (free_sig && sig > a.hp.min_lp_std && sig < 1e6f) ? s : 0.f;
                geta += dlp * (res / (sd * sd) * ddd * ep2 + (res * res / (sd * sd * sd) - 1.f / sd) * dstd);
            }
        }
        dyt[r * lda0 + qa] = P::cvt(d);
    }
    if (pre) {
        sq = wave_sum(sq);
        if (lane == 0) atomic_add_metric(a.metrics, 0, sq);
    }
    if (leta) {   // d loss / d eta (with the loss's 1/b and loss_scale; the fp16 seed scale divided out)
        geta = wave_sum(geta);
        if (lane == 0 && geta != 0.f) atomic_add_metric(a.metrics, 8, (double)geta * (double)a.hp.eta_unscale);
    }
    lds_sync();
    for (int i = tid; i < (ROWS / 8) * XD; i += THREADS) {   // dyT image from the dy tile
        const int q = i / (ROWS / 8), g = i % (ROWS / 8);
        store_img8<P>(a.ws.dyT, a.ws.ldm, grow0, q, g, [&](int r) { return P::tof(dyt[r * lda0 + q]); });
    }
    PHASE(7);

    // ---- backward dX chain (weights continue in the same stream) ----
    // B4: dh3 = dy W_out^T (kept only in tB: B2 re-reads it from there, which frees 8*MT*NT VGPRs;
    // no image: l2's weight gradient is (u2^T dy) W_out^T, dppo_ppo.h pl2)
    gemm_queue<P, MT, NT, KSO, QD>(a0, lda0, W(SEG_T_OUT), ntile0, acc, lane, R,
                                   NextLayers{W(SEG_RT_TFOLD), KSO, W(SEG_T_L1), KSH});
    store_acc_lds<P, MT, NT>(tB, ldh, ntile0, lane, acc);
    PHASE(8);
    // B3 (folded): dh2 = (dy M^T) * relu'(h2) = (dh3 W_l2^T) * relu'(h2), from the same dy tile (its
    // repeated columns against M^T's lo half)
    gemm_queue<P, MT, NT, KSO, QD>(a0, lda0, W(SEG_RT_TFOLD), ntile0, acc, lane, R,
                                   NextLayers{W(SEG_T_L1), KSH, W(SEG_T_L1), KSH});
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (!((mask2 >> ((m * NT + n) * 4 + r)) & 1u)) acc[m][n][r] = 0.f;
    store_acc_lds<P, MT, NT>(tA, ldh, ntile0, lane, acc);
    store_accT<P, MT, NT>(wsr, ws_off(a.ws, a.ws.dh2T), ldm32, ntile0, grow32, lane, acc);
    lds_sync();
    PHASE(9);
    // B2: dh1 = dh3 + (dh2 W_l1^T) * relu'(h1)
    gemm_queue<P, MT, NT, KSH, QD, true, true>(tA, ldh, W(SEG_T_L1), ntile0, acc, lane, R,
                                               NextLayers{W(SEG_T_L1), KSH, W(SEG_T_L1), KSH});
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool on = (mask1 >> ((m * NT + n) * 4 + r)) & 1u;
                const float dh3 = P::tof(tB[(m * 16 + crow(lane, r)) * ldh + (ntile0 + n) * 16 + ccol(lane)]);
                acc[m][n][r] = dh3 + (on ? acc[m][n][r] : 0.f);
            }
    store_accT<P, MT, NT>(wsr, ws_off(a.ws, a.ws.dh1T), ldm32, ntile0, grow32, lane, acc);
    PHASE(10);
}

// =============================================================================================
// critic
// =============================================================================================
template <class P, int MT>
struct CriticSmem {
    static constexpr int ROWS = 16 * MT;
    size_t tA, tB, a0, rn, rv, bias, total;
    __host__ __device__ CriticSmem(const CriticArgs& a) {
        using AT = typename P::AT;
        const int pad = lds_pad_elems<P>();
        const int ldh = a.HC + pad;
        const int ka = (a.L.ks_in > a.L.ks_out_t ? a.L.ks_in : a.L.ks_out_t) * P::KG + pad;
        size_t o = 0;
        tA = o; o += dppo_align16(sizeof(AT) * ROWS * ldh);
        tB = o; o += dppo_align16(sizeof(AT) * ROWS * ldh);
        a0 = o; o += dppo_align16(sizeof(AT) * ROWS * ka);
        rn = o; o += dppo_align16(4 * ROWS);
        rv = o; o += dppo_align16(4 * ROWS);
        bias = o; o += dppo_align16(4 * (3 * a.HC + 16));
        total = o;
    }
};

template <class P, int MT, int NT, bool TRAIN, int WAVES>
__device__ __forceinline__ void critic_rowtile_body(const CriticArgs& a) {
    using AT = typename P::AT;
    constexpr int THREADS = 64 * WAVES;
    constexpr int ROWS = 16 * MT;
    static_assert(ROWS <= 64, "the epilogue maps one row per lane of wave 0");
    constexpr int KSH = ksh_for<P>(NT, WAVES);
    constexpr int NOK = nok_for<P>(NT);
    constexpr int KSI = 2, KSO = 2;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const MlpLayout& L = a.L;
    const CriticSmem<P, MT> S(a);
    const int pad = lds_pad_elems<P>();
    const int ldh = a.HC + pad;
    const int lda0 = (L.ks_in > L.ks_out_t ? L.ks_in : L.ks_out_t) * P::KG + pad;
    const int k1w = L.ks_in * P::KG, ktw = L.ks_out_t * P::KG;
    const int SD = a.SD;
    constexpr bool train = TRAIN;
    const int HC = a.HC;
    AT* tA = (AT*)(smem + S.tA);
    AT* tB = (AT*)(smem + S.tB);
    AT* a0 = (AT*)(smem + S.a0);
    int* rn = (int*)(smem + S.rn);
    float* bias = (float*)(smem + S.bias);
    float* part = (float*)(smem + S.tB);
    const size_t grow0 = (size_t)blockIdx.x * ROWS;
    int64_t nrows = a.nrows;
    if (train && a.crow_n) {
        // sample-weighted rows: the count is known on the device only; tiles past the 64-row
        // padded count exit (the dW launch reads images only that far, DWArgs::rows_dev)
        nrows = __builtin_amdgcn_readfirstlane(*a.crow_cnt);
        if ((int64_t)grow0 >= (nrows + 63) / 64 * 64) return;
    }
    for (int i = tid; i < 3 * HC + 16; i += THREADS) {
        const int seg = i < HC ? SEG_B_IN : (i < 2 * HC ? SEG_B_L1 : (i < 3 * HC ? SEG_B_L2 : SEG_B_OUT));
        const int j = i < 3 * HC ? i % HC : i - 3 * HC;
        bias[i] = ((const float*)(a.packed + L.off[seg]))[j];
    }
    const __amdgpu_buffer_rsrc_t wsr = packed_rsrc(a.ws.base);
    const uint32_t ldm32 = (uint32_t)a.ws.ldm, grow32 = (uint32_t)grow0;

    if (tid < ROWS) {
        const int64_t gr = (int64_t)grow0 + tid;
        int n = -1;
        if (gr < nrows) {
            if (train && a.crow_n) {
                n = a.crow_n[gr];
            } else if (train) {
                const uint64_t idx = minibatch_row(a.row_index, (uint64_t)(a.start + gr), a.fk);
                if (idx < a.fk.n) n = (int)(idx / a.KF);
            } else {
                n = (int)gr;
            }
        }
        rn[tid] = n;
    }
    lds_sync();
    for (int i = tid; i < ROWS * k1w; i += THREADS) {
        const int r = i / k1w, c = i % k1w, n = rn[r];
        a0[r * lda0 + c] = P::cvt((n >= 0 && c < SD) ? a.obs[(size_t)n * SD + c] : 0.f);
    }
    lds_sync();
    if (train) {   // csT image (permuted row order, img_pos) from the input tile
        for (int i = tid; i < (ROWS / 8) * SD; i += THREADS) {
            const int c = i / (ROWS / 8), g = i % (ROWS / 8);
            store_img8<P>(a.ws.csT, a.ws.ldm, grow0, c, g, [&](int r) { return P::tof(a0[r * lda0 + c]); });
        }
    }

    const int ntile0 = wave * NT;
    const __amdgpu_buffer_rsrc_t rs = packed_rsrc(a.packed);
    auto W = [&](int seg) { return wsrc(rs, L.off[seg]); };
    f32x4 H1[MT][NT], H2[MT][NT], acc[MT][NT];
    WRing<NT> R;
    ring_prime(R, W(SEG_W_IN), KSI, ntile0, lane);
    ORing<NOK, 1> ob;
    out_prefetch<NOK, 1, WAVES>(ob, W(SEG_W_OUT), KSH, wave, lane);
    // L1: h1 = s W_in + b
    gemm_stream<P, MT, NT, KSI>(a0, lda0, W(SEG_W_IN), ntile0, H1, lane, R, NextLayer{W(SEG_W_L1), KSH, ntile0});
    add_bias(H1, bias, ntile0, lane);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[m][n][r] = mishf(H1[m][n][r]);
    store_acc_lds<P, MT, NT>(tA, ldh, ntile0, lane, acc);
    if constexpr (train) store_accT<P, MT, NT>(wsr, ws_off(a.ws, a.ws.cu1T), ldm32, ntile0, grow32, lane, acc);
    lds_sync();
    // L2: h2 = mish(h1) W_l1 + b
    gemm_stream<P, MT, NT, KSH>(tA, ldh, W(SEG_W_L1), ntile0, H2, lane, R, NextLayer{W(SEG_W_L2), KSH, ntile0});
    add_bias(H2, bias + HC, ntile0, lane);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[m][n][r] = mishf(H2[m][n][r]);
    store_acc_lds<P, MT, NT>(tB, ldh, ntile0, lane, acc);
    if constexpr (train) store_accT<P, MT, NT>(wsr, ws_off(a.ws, a.ws.cu2T), ldm32, ntile0, grow32, lane, acc);
    lds_sync();
    // L3: h3 = mish(h2) W_l2 + b + h1
    gemm_stream<P, MT, NT, KSH>(tB, ldh, W(SEG_W_L2), ntile0, acc, lane, R,
                                train ? NextLayer{W(SEG_T_OUT), KSO, ntile0} : NextLayer{W(SEG_W_L2), KSH, ntile0});
    add_bias(acc, bias + 2 * HC, ntile0, lane);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[m][n][r] += H1[m][n][r];
    store_acc_lds<P, MT, NT>(tA, ldh, ntile0, lane, acc);
    if constexpr (train) store_accT<P, MT, NT>(wsr, ws_off(a.ws, a.ws.ch3T), ldm32, ntile0, grow32, lane, acc);
    lds_sync();
    // L4: V = h3 W_out + b
    {
        f32x4 po[MT][1];
        gemm_narrow_pre<P, MT, NOK, 1, WAVES>(tA, ldh, ob, po, wave, lane);
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) part[(wave * ROWS + m * 16 + crow(lane, r)) * 16 + ccol(lane)] = po[m][0][r];
    }
    lds_sync();
    if (wave == 0 && lane < ROWS) {
        const int r = lane, n = rn[r];
        float V = bias[3 * HC];
#pragma unroll
        for (int w = 0; w < WAVES; ++w) V += part[(w * ROWS + r) * 16];
        if (!train) {
            if (n >= 0) a.values[n] = V;
        } else {
            float vl = 0.f, dv = 0.f;
            if (n >= 0) {
                const float w = a.crow_mult ? (float)a.crow_mult[n] : 1.f;   // copies of the sample in the minibatch
                const float R = a.returns[n], diff = V - R;
                if (a.hp.clip_vloss > 0.f) {
                    // diffusion_ppo.py:110-116: 0.5 max((V-R)^2, (V_old + clip(V - V_old, -c, c) - R)^2); the
                    // gradient as TF routes it: tf.maximum's to its first argument on ties, clip_by_value's
                    // through where V - V_old lies in [-c, c] (bounds included), zero outside
                    const float c = a.hp.clip_vloss, old = a.hp.old_values[n], d = V - old;
                    const float vc = old + fminf(fmaxf(d, -c), c), dc = vc - R;
                    const float lu = diff * diff, lc = dc * dc;
                    vl = 0.5f * fmaxf(lu, lc) * w;
                    const float g = lu >= lc ? diff : ((d >= -c && d <= c) ? dc : 0.f);
                    dv = a.hp.vf_coef * g * a.hp.grad_scale * w;
                } else {
                    vl = 0.5f * diff * diff * w;                     // v_loss = 0.5 mean((V-R)^2), diffusion_ppo.py:118
                    dv = a.hp.vf_coef * diff * a.hp.grad_scale * w;  // loss = pg + vf_coef * v_loss (agent :340)
                }
            }
            for (int q = 0; q < ktw; ++q) a0[r * lda0 + q] = P::cvt(q == 0 ? dv : 0.f);
            ((AT*)a.ws.cdvT)[grow0 + img_pos(r)] = P::cvt(dv);
            vl = wave_sum(vl);
            if (lane == 0) atomic_add_metric(a.metrics, 1, vl);
        }
    }
    if constexpr (!train) return;
    lds_sync();
    // B4: dh3 = dV W_out^T (kept only in tB, re-read by B2; no image, as the actor's)
    gemm_stream<P, MT, NT, KSO>(a0, lda0, W(SEG_T_OUT), ntile0, acc, lane, R, NextLayer{W(SEG_T_L2), KSH, ntile0});
    store_acc_lds<P, MT, NT>(tB, ldh, ntile0, lane, acc);
    lds_sync();
    // B3: dh2 = (dh3 W_l2^T) * mish'(h2)
    gemm_stream<P, MT, NT, KSH>(tB, ldh, W(SEG_T_L2), ntile0, acc, lane, R, NextLayer{W(SEG_T_L1), KSH, ntile0});
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[m][n][r] *= mish_gradf(H2[m][n][r]);
    store_acc_lds<P, MT, NT>(tA, ldh, ntile0, lane, acc);
    store_accT<P, MT, NT>(wsr, ws_off(a.ws, a.ws.cdh2T), ldm32, ntile0, grow32, lane, acc);
    lds_sync();
    // B2: dh1 = dh3 + (dh2 W_l1^T) * mish'(h1)
    gemm_stream<P, MT, NT, KSH>(tA, ldh, W(SEG_T_L1), ntile0, acc, lane, R, NextLayer{W(SEG_T_L1), KSH, ntile0});
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float dh3 = P::tof(tB[(m * 16 + crow(lane, r)) * ldh + (ntile0 + n) * 16 + ccol(lane)]);
                acc[m][n][r] = dh3 + acc[m][n][r] * mish_gradf(H1[m][n][r]);
            }
    store_accT<P, MT, NT>(wsr, ws_off(a.ws, a.ws.cdh1T), ldm32, ntile0, grow32, lane, acc);
}

// Kernel entry points. The *_o4 forms cap registers at 128 (4 waves per SIMD: two 8-wave row
// tiles per CU) at the price of a few spills; which form runs is chosen per launch (row_tile_cfg).
template <class P, int MT, int NT, int NO, int KSI, bool TRAIN, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void actor_rowtile_kernel(ActorArgs a) {
    actor_rowtile_body<P, MT, NT, NO, KSI, TRAIN, WAVES>(a);
}
template <class P, int MT, int NT, int NO, int KSI, bool TRAIN, int WAVES>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(4))) void actor_rowtile_kernel_o4(ActorArgs a) {
    actor_rowtile_body<P, MT, NT, NO, KSI, TRAIN, WAVES>(a);
}
template <class P, int MT, int NT, bool TRAIN, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void critic_rowtile_kernel(CriticArgs a) {
    critic_rowtile_body<P, MT, NT, TRAIN, WAVES>(a);
}
template <class P, int MT, int NT, bool TRAIN, int WAVES>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(4))) void critic_rowtile_kernel_o4(CriticArgs a) {
    critic_rowtile_body<P, MT, NT, TRAIN, WAVES>(a);
}

// Row-tile shapes: actor 64 rows on 16 waves (2-byte operands, H = 512, XD <= 16, at least one
// round of tiles), else 32 rows on 8 waves (fp32: 16); critic 32 rows on 8 waves at occupancy 4 (the _o4
// kernel). r02 measured the alternatives (actor 32x8 at occupancy 4, 64x8; critic at occupancy 2)
// slower or equal; r03 removed them with the binary's size in mind.
struct RowTileCfg { int actor; int critic; };
static RowTileCfg row_tile_cfg() { return RowTileCfg{0, 1}; }

// =============================================================================================
// launchers
// =============================================================================================
template <class P, int MT, int NT, int NO, int KSI, bool TRAIN, int WAVES, bool O4>
static int launch_actor_t(const ActorArgs& a, hipStream_t s) {
    if (a.L.ks_in != KSI || a.L.ks_h != ksh_for<P>(NT, WAVES) || a.L.ks_out_t != 2 || a.L.ks_h != WAVES * nok_for<P>(NT))
        return dppo_set_error(DPPO_EUNSUPPORTED, "actor row tile: layout does not match the instantiation");
    const ActorSmem<P, MT> S(a);
    const int pad = lds_pad_elems<P>();
    const size_t part_bytes = (size_t)4 * WAVES * 16 * MT * 16 * NO;
    const size_t tb_bytes = sizeof(typename P::AT) * 16 * MT * (a.H + pad);
    if (part_bytes > tb_bytes) return dppo_set_error(DPPO_EUNSUPPORTED, "actor: partial buffer does not fit");
    if (S.total > 160 * 1024) return dppo_set_error(DPPO_EUNSUPPORTED, "actor row tile needs %zu B LDS", S.total);
    auto k = O4 ? actor_rowtile_kernel_o4<P, MT, NT, NO, KSI, TRAIN, WAVES> : actor_rowtile_kernel<P, MT, NT, NO, KSI, TRAIN, WAVES>;
    { const int rc_ = dppo_func_lds((const void*)k, (size_t)S.total); if (rc_) return rc_; }
    // TRAIN mode covers every row of the 64-padded feature-major images (padding rows get
    // finite activations and zero gradients), so the dW kernel never reads unwritten memory
    const int64_t all = (a.mode == ROWS_TRAIN || a.mode == ROWS_PRETRAIN) ? (int64_t)a.ws.ldm : a.nrows;
    const int64_t rows = (a.row_end > 0 ? a.row_end : all) - a.row0;
    const int64_t grid = (rows + 16 * MT - 1) / (16 * MT);
    if (grid <= 0) return DPPO_OK;
    DppoKtScope kt(a.mode == ROWS_TRAIN || a.mode == ROWS_PRETRAIN ? KT_ACTOR_TRAIN : KT_ACTOR_LOGPROB, s);
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(64 * WAVES), S.total, s, a);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

template <class P, int MT, int NT, int NO, int KSI, int WAVES, bool O4>
static int launch_actor_m(const ActorArgs& a, hipStream_t s) {
    return (a.mode == ROWS_TRAIN || a.mode == ROWS_PRETRAIN) ? launch_actor_t<P, MT, NT, NO, KSI, true, WAVES, O4>(a, s)
                                : launch_actor_t<P, MT, NT, NO, KSI, false, WAVES, O4>(a, s);
}

// bf16: 64-row tiles, 16 waves (half the weight stream per row of 32-row tiles; LDS-limited);
// fp32: 32-row tiles, 16 waves
template <class P, int MT, int WAVES, bool O4 = false>
static int dispatch_actor(const ActorArgs& a, hipStream_t s) {
    const int NT = a.H / (16 * WAVES), NO = dppo_cdiv(a.XD, 16), KSI = a.L.ks_in;
#define DPPO_ACTOR_CASE(nt, no, ksi) \
    if (NT == nt && NO == no && KSI == ksi) return launch_actor_m<P, MT, nt, no, ksi, WAVES, O4>(a, s);
    if constexpr (P::KG == 32 && WAVES == 16) {   // bf16, H = 512 on 16 waves
        DPPO_ACTOR_CASE(2, 1, 2) DPPO_ACTOR_CASE(2, 2, 2) DPPO_ACTOR_CASE(2, 1, 4) DPPO_ACTOR_CASE(2, 2, 4)
    } else if constexpr (P::KG == 32) {           // bf16, 8 waves: the in-layer is 2 k-steps up to 64 inputs, 4 up to 128
        DPPO_ACTOR_CASE(4, 1, 2) DPPO_ACTOR_CASE(4, 2, 2) DPPO_ACTOR_CASE(4, 1, 4) DPPO_ACTOR_CASE(4, 2, 4)
        DPPO_ACTOR_CASE(2, 1, 2) DPPO_ACTOR_CASE(2, 2, 2) DPPO_ACTOR_CASE(2, 1, 4) DPPO_ACTOR_CASE(2, 2, 4)
    } else {                       // fp32: 33..64 inputs -> 4 k-steps
        DPPO_ACTOR_CASE(4, 1, 4) DPPO_ACTOR_CASE(4, 2, 4) DPPO_ACTOR_CASE(2, 1, 4) DPPO_ACTOR_CASE(2, 2, 4)
    }
#undef DPPO_ACTOR_CASE
    return dppo_set_error(DPPO_EUNSUPPORTED, "actor: hidden %d / chunk %d not instantiated", a.H, a.XD);
}

static int64_t actor_device_cus() {
    static int n = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            c = 256;
        return c > 0 ? c : 256;
    }();
    return n;
}

// the 2-byte operand policies (bf16, fp16) share the tile configurations
template <class P2>
static int launch_actor_2b(const ActorArgs& a, hipStream_t s) {
    const int v = row_tile_cfg().actor;
    // (r04: a 128-row tile, one activation tile in LDS with in-place layers, 8 or 4 waves of 8 x 4 /
    // 8 x 8 accumulator tiles, ran SLOWER: 0.464 / 0.543 vs 0.421 ms per fused 50,000-row minibatch,
    // profiles/r04c_actor_tile128_ab.jsonl; register spills at 256 / 512 registers per wave and
    // unhidden LDS / weight latency at 1-2 waves per SIMD. Removed)
    // bf16, H = 512: 64-row tiles on 16 waves halve the weight stream per row of 32-row tiles; their
    // out-layer partials (16 waves x 64 rows x 16*NO) only fit the aliased LDS tile for XD <= 16
    // (walker2d / halfcheetah, XD = 24, run the 32-row tile)
    if (a.H == 512 && v == 0 && a.XD <= 16) {
        // (r05: running the short last round of 64-row tiles as twice as many 32-row tiles in a launch
        // of their own cost more than it saved, update 16.5 vs 15.5 ms per iteration: the critic's half
        // on the side stream fills the CUs that round leaves idle. Removed.)
        // a minibatch of less than one round of 64-row tiles (the per-rank share of an 8-GPU run
        // under the reference's global minibatch: 6,250 rows = 98 tiles) finishes in one tile's
        // latency either way, and a 32-row tile's is about 0.6 of a 64-row tile's (update 50.1 ->
        // 47.1 ms per iteration at 6,250-row minibatches, tools/ab_small_mb.sh)
        const int64_t rows = (a.mode == ROWS_TRAIN || a.mode == ROWS_PRETRAIN) ? (int64_t)a.ws.ldm : a.nrows;
        if ((rows + 63) / 64 < actor_device_cus()) return dispatch_actor<P2, 2, 8>(a, s);
        return dispatch_actor<P2, 4, 16>(a, s);
    }
    return dispatch_actor<P2, 2, 8>(a, s);
}

int launch_actor_rowtile(const ActorArgs& a, int precision, hipStream_t s) {
    if (precision == DPPO_BF16) return launch_actor_2b<PolicyBF16>(a, s);
    if (precision == DPPO_F16) return launch_actor_2b<PolicyF16>(a, s);
    // fp32: 32-row tiles on 16 waves (four per SIMD behind the 16x16x4 MFMA chains): update 41.5 ->
    // 40.5 ms per iteration against 8 waves (profiles/r06zz_f32_tile_16wave_ab.txt)
    return dispatch_actor<PolicyF32, 2, 16>(a, s);
}

template <class P, int MT, int NT, bool TRAIN, int WAVES, bool O4>
static int launch_critic_t(const CriticArgs& a, hipStream_t s) {
    if (a.L.ks_in != 2 || a.L.ks_h != ksh_for<P>(NT, WAVES) || a.L.ks_out_t != 2 || a.L.ks_h != WAVES * nok_for<P>(NT))
        return dppo_set_error(DPPO_EUNSUPPORTED, "critic row tile: layout does not match the instantiation");
    const CriticSmem<P, MT> S(a);
    if (S.total > 160 * 1024) return dppo_set_error(DPPO_EUNSUPPORTED, "critic row tile needs %zu B LDS", S.total);
    if ((size_t)4 * WAVES * 16 * MT * 16 > sizeof(typename P::AT) * 16 * MT * (a.HC + lds_pad_elems<P>()))
        return dppo_set_error(DPPO_EUNSUPPORTED, "critic: partial buffer does not fit");
    auto k = O4 ? critic_rowtile_kernel_o4<P, MT, NT, TRAIN, WAVES> : critic_rowtile_kernel<P, MT, NT, TRAIN, WAVES>;
    { const int rc_ = dppo_func_lds((const void*)k, (size_t)S.total); if (rc_) return rc_; }
    // TRAIN mode covers every row of the 64-padded feature-major images (padding rows get
    // finite activations and zero gradients), so the dW kernel never reads unwritten memory
    const int64_t rows = a.mode == ROWS_TRAIN ? (int64_t)a.ws.ldm : a.nrows;
    const int64_t grid = (rows + 16 * MT - 1) / (16 * MT);
    if (grid == 0) return DPPO_OK;
    DppoKtScope kt(a.mode == ROWS_TRAIN ? KT_CRITIC_TRAIN : KT_CRITIC_FWD, s);
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(64 * WAVES), S.total, s, a);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

template <class P, int MT, int WAVES, bool O4>
static int dispatch_critic(const CriticArgs& a, hipStream_t s) {
    const int NT = a.HC / (16 * WAVES);
    const bool tr = a.mode == ROWS_TRAIN;
    if (NT == 2) return tr ? launch_critic_t<P, MT, 2, true, WAVES, O4>(a, s) : launch_critic_t<P, MT, 2, false, WAVES, O4>(a, s);
    return dppo_set_error(DPPO_EUNSUPPORTED, "critic: hidden %d not instantiated", a.HC);
}

#ifndef DPPO_CRITIC_MT
#define DPPO_CRITIC_MT 2   // 16-row MFMA tiles per critic row tile (measurement knob of tuning builds)
#endif
int launch_critic_rowtile(const CriticArgs& a, int precision, hipStream_t s) {
    return precision == DPPO_BF16 ? dispatch_critic<PolicyBF16, DPPO_CRITIC_MT, 8, true>(a, s)
         : precision == DPPO_F16  ? dispatch_critic<PolicyF16, DPPO_CRITIC_MT, 8, true>(a, s)
                                  : dispatch_critic<PolicyF32, 2, 8, true>(a, s);
}

// =============================================================================================
// C ABI: old-logprob pass and value pass
// =============================================================================================
extern "C" int dppo_logprob(const dppo_dims* d, int precision, const void* packed_ft, const float* sched,
                            const float* cond, const float* chains, int n, float min_logprob_std, int reward_horizon,
                            float* lp_elem, float* lp_mean, void* stream) {
    Dims D;
    int rc = dppo_check_dims(d, &D);
    if (rc) return rc;
    DPPO_CHECK(dppo_prec_ok(precision), "bad precision %d", precision);
    DPPO_CHECK(n >= 0, "dppo_logprob: n < 0");
    if (n == 0) return DPPO_OK;
    DPPO_CHECK(packed_ft && sched && cond && chains && (lp_elem || lp_mean), "dppo_logprob: null pointer");
    DPPO_CHECK(reward_horizon >= 1, "dppo_logprob: reward_horizon < 1");
    ActorArgs a = {};
    a.packed = (const uint8_t*)packed_ft;
    a.L = make_mlp_layout(D.IN, D.H, D.XD, D.TD, precision, D.K);
    a.sched = sched; a.obs = cond; a.chains = chains;
    a.XD = D.XD; a.SD = D.SD; a.TD = D.TD; a.IN = D.IN; a.H = D.H; a.KF = D.KF; a.Da = D.Da; a.TS = D.TS;
    a.mode = ROWS_LOGPROB;
    a.nrows = (int64_t)n * D.KF;
    a.lp_elem = lp_elem; a.lp_mean = lp_mean;
    a.hp.min_lp_std = min_logprob_std;
    a.hp.reward_horizon = reward_horizon;
    return launch_actor_rowtile(a, precision, (hipStream_t)stream);
}

extern "C" int dppo_critic_forward(const dppo_dims* d, int precision, const void* packed_critic, const float* cond,
                                   int n, float* values, void* stream) {
    Dims D;
    int rc = dppo_check_dims(d, &D);
    if (rc) return rc;
    DPPO_CHECK(dppo_prec_ok(precision), "bad precision %d", precision);
    DPPO_CHECK(n >= 0, "dppo_critic_forward: n < 0");
    if (n == 0) return DPPO_OK;
    DPPO_CHECK(packed_critic && cond && values, "dppo_critic_forward: null pointer");
    CriticArgs a = {};
    a.packed = (const uint8_t*)packed_critic;
    a.L = make_mlp_layout(D.SD, D.HC, 1, 0, precision);
    a.obs = cond; a.SD = D.SD; a.HC = D.HC; a.KF = D.KF;
    a.mode = ROWS_VALUE; a.nrows = n; a.values = values;
    return launch_critic_rowtile(a, precision, (hipStream_t)stream);
}
