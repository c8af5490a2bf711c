// pack.hip — flat fp32 Keras parameters -> packed MFMA fragment images (dppo_layout.h).
// Replaces the Keras variable storage of model/common/mlp.py:95-206 (kernels are [in,out]).
#include <mutex>
#include "dppo_common.cuh"
#include "dppo_internal.h"

// Every segment of the images being re-derived — the actor's and/or the critic's — and the actor's
// time tables (TEMB, TIN, B_OUT2) in ONE launch: the images are re-derived after every optimiser
// step, on the critical path of every PPO minibatch, where each extra launch is a kernel boundary.
// A job is either a packed matrix (one thread per (ntile, ks, lane) fragment slot, 16 B each) or a
// zero-padded fp32 copy; the time-table blocks follow the job blocks.
#define PACK_MAXJ 24
struct PackJob {
    int kind;            // 0 = packed matrix, 1 = fp32 copy with zero padding, 2 = zero n 4-byte words
    int K, N, transposed;
    int k_split, k_skip; // source row of packed row k: k < k_split ? k : k + k_skip (row subsets)
    int n, npad;         // copy: valid / padded element counts
    const float* src;    // source params (already offset)
    uint8_t* dst;        // destination in the image (already offset)
    int threads;         // work items of this job
};
// the actor's time tables: blocks [0, R) TEMB rows; with 2-byte operands also blocks [R, 2R) TIN
// rows and block 2R B_OUT2 (tables = 2R + 1, else R); and nfold blocks of FOLD / ROUT fragments (one
// 16-feature tile each). Launch order: fold blocks, table blocks, then the element jobs
struct TembArgs {
    const float* params;
    FlatOffsets F;
    int TD, stride, R, XD, H, nout, tables, nfold;
    int first_table;      // table block b runs time_table_block(first_table + b): R skips the TEMB rows
    float *temb, *tin, *bout2;
    uint8_t *fold, *rout;
};
struct PackArgs {
    PackJob j[PACK_MAXJ];
    int start[PACK_MAXJ + 1];
    int njobs;
    int pack_blocks;     // blocks of the job part (256 threads each), after the time-table blocks
    TembArgs tb;
};

constexpr int PACK_THREADS = 256;

// t_emb(t) = Dense(2TD->TD)(mish(Dense(TD->2TD)(SinusoidalPosEmb(t)))) (mlp_diffusion.py:40-45,
// modules.py:4-15), one workgroup per table row; the arithmetic and its order match the oracle
// restatement. With ET = the 2-byte operand type (split-sampler tables) also TIN = b_in +
// sum_j rnd(t_emb_j) rnd(W_in[XD + j]) (each block re-derives its t_emb row) and B_OUT2 = b_out +
// sum_h b_l2[h] rnd(W_out[h]) with a fixed-order reduction (the sampler's h3 is fp32-accurate, so
// b_l2 enters the out-Dense unrounded). The first 128 threads work; all take part in barriers.
template <class ET>
__device__ void time_table_block(const TembArgs& b, int blk) {
    __shared__ float te[64];
    __shared__ float ta1[128];
    __shared__ float tr[64];
    __shared__ float red[128][33];
    const int tid = threadIdx.x;
    const float* params = b.params;
    const FlatOffsets& F = b.F;
    const int TD = b.TD, R = b.R, XD = b.XD, H = b.H;
    if (blk == 2 * R) {   // B_OUT2
        if (tid < 128) {
            float acc[32];
#pragma unroll
            for (int q = 0; q < 32; ++q) acc[q] = 0.f;
            for (int h = tid; h < H; h += 128) {
                const float bl2 = params[F.l2_b + h];
#pragma unroll
                for (int q = 0; q < 32; ++q)
                    if (q < XD) acc[q] += bl2 * (float)(ET)params[F.out_w + (size_t)h * XD + q];
            }
#pragma unroll
            for (int q = 0; q < 32; ++q) red[tid][q] = acc[q];
        }
        __syncthreads();
        if (tid < b.nout) {
            float s = tid < XD ? params[F.out_b + tid] : 0.f;
            if (tid < XD)
                for (int k = 0; k < 128; ++k) s += red[k][tid];
            b.bout2[tid] = s;
        }
        return;
    }
    const int row = blk % R, t = row * b.stride;   // row r holds t_emb(r * stride)
    if (tid < TD) te[tid] = temb_sinusoid(tid, t, TD);
    __syncthreads();
    if (tid < 2 * TD) ta1[tid] = temb_hidden(params, F.time_w1, F.time_b1, te, TD, tid);
    __syncthreads();
    if (tid < TD) {
        const float acc = temb_output(params, F.time_w2, F.time_b2, ta1, TD, tid);
        if (blk < R) b.temb[(size_t)row * TD + tid] = acc;
        tr[tid] = (float)(ET)acc;
    }
    if (blk < R) return;
    __syncthreads();
    for (int h = tid; h < H; h += PACK_THREADS) {
        float acc = params[F.in_b + h];
#pragma unroll 16                                  // the loads in flight together, not one round trip each
        for (int j = 0; j < TD; ++j) acc += tr[j] * (float)(ET)params[F.in_w + (size_t)(XD + j) * H + h];
        b.tin[(size_t)row * H + h] = acc;
    }
}

// FOLD / ROUT fragments of feature tile T (dppo_layout.h): M[f][o] = sum_j rnd(W_l2[f][j])
// rnd(W_out[j][o]) in fp32, then split into its 2-byte hi/lo pair; ROUT is rnd(W_out) rows 16T.. in
// the same fragment geometry. The tile's W_l2 rows and W_out are staged in LDS as the rounded 2-byte
// values (exact) in one round trip at hopper's out_dim <= 16 (chunks of 256 rows above);
// thread (g, f, oq) sums j-quarter g of each chunk for feature f and outs 4 oq.. (+16), so one
// broadcast read of W_l2 and one 8-B read of W_out feed 4 FMAs; the quarters are added in a fixed
// order at the end. These blocks come first in the launch (the split sampler's table refresh).
template <class ET>
__device__ void fold_block(const TembArgs& b, int T) {
    if constexpr (sizeof(ET) == 2) {
        constexpr int JMAX = 512;
        __shared__ ET fw2[16][JMAX + 8];
        __shared__ __attribute__((aligned(16))) ET wos[JMAX * 16];   // [jc][XDP]
        __shared__ float red[4][16][33];
        __shared__ float mv[16][33];
        const int tid = threadIdx.x, H = b.H, XD = b.XD, nt_out = b.nout / 16;
        const float* params = b.params;
        const FlatOffsets& F = b.F;
        const float* wo = params + F.out_w;
        const int XDP = XD <= 16 ? 16 : 32, JC = XD <= 16 ? JMAX : JMAX / 2;
        const int g = tid >> 6, fr = (tid & 63) >> 2, oq = tid & 3;
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        auto ld4 = [&](int off) {                      // 4 staged W_out values as fp32
            const u32x2 w = *(const u32x2*)(wos + off);
            return f32x4{(float)__builtin_bit_cast(ET, (uint16_t)(w[0] & 0xffffu)),
                         (float)__builtin_bit_cast(ET, (uint16_t)(w[0] >> 16)),
                         (float)__builtin_bit_cast(ET, (uint16_t)(w[1] & 0xffffu)),
                         (float)__builtin_bit_cast(ET, (uint16_t)(w[1] >> 16))};
        };
        bool whole = false;                            // W_out fully staged (one chunk)
        for (int j0 = 0; j0 < H; j0 += JC) {
            const int nj = min(JC, H - j0);
            whole = j0 == 0 && nj == H;
            __syncthreads();
            // unrolled so that 16 loads per thread are in flight (a rolled loop pays one L2
            // round trip per element)
#pragma unroll 16
            for (int i = tid; i < 16 * JC; i += PACK_THREADS) {
                const int r = i / JC, jj = i % JC, f = 16 * T + r;
                fw2[r][jj] = (ET)((jj < nj && f < H) ? params[F.l2_w + (size_t)f * H + j0 + jj] : 0.f);
            }
#pragma unroll 16
            for (int i = tid; i < JC * XDP; i += PACK_THREADS) {
                const int jj = i / XDP, o = i % XDP;
                wos[i] = (ET)((jj < nj && o < XD) ? wo[(size_t)(j0 + jj) * XD + o] : 0.f);
            }
            __syncthreads();
            const int q = JC / 4, ja = g * q;           // rows past nj are zero in both operands
            if (XDP == 32) {
#pragma unroll 4
                for (int jj = ja; jj < ja + q; ++jj) {
                    const float w = (float)fw2[fr][jj];
                    const f32x4 u = ld4(jj * 32 + 4 * oq), v = ld4(jj * 32 + 16 + 4 * oq);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        acc0[e] = fmaf(w, u[e], acc0[e]);
                        acc1[e] = fmaf(w, v[e], acc1[e]);
                    }
                }
            } else {
#pragma unroll 8
                for (int jj = ja; jj < ja + q; ++jj) {
                    const float w = (float)fw2[fr][jj];
                    const f32x4 u = ld4(jj * 16 + 4 * oq);
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc0[e] = fmaf(w, u[e], acc0[e]);
                }
            }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            red[g][fr][4 * oq + e] = acc0[e];
            red[g][fr][16 + 4 * oq + e] = acc1[e];
        }
        __syncthreads();
        for (int i = tid; i < 16 * 32; i += PACK_THREADS) {
            const int f = i >> 5, o = i & 31;
            mv[f][o] = ((red[0][f][o] + red[1][f][o]) + red[2][f][o]) + red[3][f][o];
        }
        __syncthreads();
        if (tid < 64 * nt_out) {
            const int lane = tid & 63, n = tid >> 6, o = 16 * n + (lane & 15), jq = lane >> 4;
            ET e[8], w[8];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int fl = 4 * jq + q, f = 16 * T + fl;
                const float m = o < XD ? mv[fl][o] : 0.f;
                const ET hi = (ET)m;
                e[q] = hi;
                e[4 + q] = (ET)(m - (float)hi);
                const ET wq = whole ? wos[f * XDP + o] : (ET)((o < XD && f < H) ? wo[(size_t)f * XD + o] : 0.f);
                w[q] = wq;
                w[4 + q] = wq;
            }
            const size_t idx = ((size_t)T * nt_out + n) * 64 + lane;
            reinterpret_cast<u32x4*>(b.fold)[idx] = __builtin_bit_cast(u32x4, e);
            reinterpret_cast<u32x4*>(b.rout)[idx] = __builtin_bit_cast(u32x4, w);
        }
    }
}

// The row tiles' fold (dppo_layout.h RT_*), one wave per tile, on the matrix cores from the image
// the same stream has just written (the pack launch, or a fused optimizer step): the cross-element
// products a per-element step cannot form.
//   M tile T (16 l2 inputs i): M[i][o] = sum_j rnd(W_l2[i][j]) rnd(W_out[j][o]) as 16x16 MFMA tiles whose
//     A operand is the T_L2 image's n-tile T (lane: W_l2[i][8 consecutive j]) and B the W_OUT image's
//     (lane: W_out[8 consecutive j][o]): KS_h k-steps, exact products summed in fp32 (the 2-byte
//     policies; fp32 images: the fp32 values);
//   M0 tile (16 in-Dense inputs i): the same with W_in's rows read from the fp32 parameters (i < in_dim;
//     rows up to RT_FOLD0's padded k range are zero);
//   the last block: RT_BOUT = b_out + sum_h (b_in + b_l2)[h] rnd(W_out[h][o]) (fixed-order reduction).
// The tile's M values go through LDS ([o][i]) into the RT_FOLD / RT_FOLD0 slots (hi, then lo) and the
// RT_TFOLD slots of n-tile T (hi at k = o, lo at k = LOK + o).
struct RtFoldArgs {
    uint8_t* img;
    const float* params;
    FlatOffsets F;
    size_t off_wout, off_tl2, off_fold, off_fold0, off_tfold, off_bout, off_temb;
    int H, XD, IN, nt_out, ks_h, ks_in, ks_out_t, nm, nm0;
    int TD, TS, R;        // the TEMB table's rows (row r = t_emb(r TS), r < R)
};
// one M (M0) tile: NO out tiles, the k-steps in batches of KB whose loads are all issued before the
// batch's MFMAs, with no branch inside a batch (a conditional load made hipcc wait vmcnt(0) per k-step:
// a chain of KS_h global latencies, 17 us for the launch)
template <class P, int NO, int KB, bool M0>
__device__ inline void rt_fold_tile(const RtFoldArgs& a, const __amdgpu_buffer_rsrc_t& rs, int T, int lane,
                                    float (*sm)[17]) {
    using AT = typename P::AT;
    constexpr int KG = P::KG, EPL = P::EPL;
    const WSrc wo = wsrc(rs, a.off_wout), tl2 = wsrc(rs, a.off_tl2);
    const int H = a.H, i = 16 * T + (lane & 15);
    const bool irow = i < a.IN;
    const float* wrow = a.params + a.F.in_w + (size_t)(irow ? i : 0) * H + (lane >> 4) * EPL;   // 16-B aligned
    f32x4 acc[NO];
#pragma unroll
    for (int n = 0; n < NO; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kb = 0; kb < a.ks_h; kb += KB) {
        u32x4 av[KB], bv[NO][KB];
#pragma unroll
        for (int u = 0; u < KB; ++u) {
            if constexpr (!M0) {
                av[u] = load_bfrag_c(tl2, a.ks_h, T, kb + u, lane);
            } else {   // W_in[i][8 (4) consecutive j] from the fp32 parameters, rounded as the pack rounds
                const f32x4* src = (const f32x4*)(wrow + (kb + u) * KG);
                AT e[EPL];
#pragma unroll
                for (int q = 0; q < EPL / 4; ++q) {
                    const f32x4 x = src[q];
#pragma unroll
                    for (int c = 0; c < 4; ++c) e[4 * q + c] = (AT)(irow ? x[c] : 0.f);
                }
                __builtin_memcpy(&av[u], e, 16);
            }
#pragma unroll
            for (int n = 0; n < NO; ++n) bv[n][u] = load_bfrag_c(wo, a.ks_h, n, kb + u, lane);
        }
#pragma unroll
        for (int u = 0; u < KB; ++u)
#pragma unroll
            for (int n = 0; n < NO; ++n) acc[n] = P::mma(av[u], bv[n][u], acc[n]);
    }
    // C[m = i][n = o]: lane holds i = 4 (lane >> 4) + r, o = 16 n + (lane & 15)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) sm[16 * n + (lane & 15)][4 * (lane >> 4) + r] = n < NO ? acc[n < NO ? n : 0][r] : 0.f;
}

// RT_BOUT = b_out + sum_j (b_in + b_l2)[j] rnd(W_out[j][o]): lane (o = lane & 15, group jg = lane >> 4)
// takes rnd(W_out) from the W_OUT image's fragments (its EPL consecutive j per k-step, zero past out_dim)
// and the bias sums of those j, 4 k-steps per batch of loads; the 4 groups add through two lane swaps
template <class P, int NO>
__device__ inline void rt_fold_bias(const RtFoldArgs& a, const __amdgpu_buffer_rsrc_t& rs, int lane) {
    using AT = typename P::AT;
    constexpr int KG = P::KG, EPL = P::EPL, KB = 4;
    const WSrc wo = wsrc(rs, a.off_wout);
    const int jg = lane >> 4;
    const float* bi = a.params + a.F.in_b + jg * EPL;   // 16-B aligned (host-checked offsets)
    const float* bl = a.params + a.F.l2_b + jg * EPL;
    float acc[NO];
#pragma unroll
    for (int n = 0; n < NO; ++n) acc[n] = 0.f;
    for (int kb = 0; kb < a.ks_h; kb += KB) {
        u32x4 w[NO][KB];
        f32x4 vb[KB][EPL / 4], vl[KB][EPL / 4];
#pragma unroll
        for (int u = 0; u < KB; ++u) {
#pragma unroll
            for (int n = 0; n < NO; ++n) w[n][u] = load_bfrag_c(wo, a.ks_h, n, kb + u, lane);
#pragma unroll
            for (int q = 0; q < EPL / 4; ++q) {
                vb[u][q] = *(const f32x4*)(bi + (kb + u) * KG + 4 * q);
                vl[u][q] = *(const f32x4*)(bl + (kb + u) * KG + 4 * q);
            }
        }
#pragma unroll
        for (int u = 0; u < KB; ++u)
#pragma unroll
            for (int n = 0; n < NO; ++n) {
                AT e[EPL];
                __builtin_memcpy(e, &w[n][u], 16);
#pragma unroll
                for (int q = 0; q < EPL; ++q) acc[n] = fmaf(vb[u][q / 4][q % 4] + vl[u][q / 4][q % 4], (float)e[q], acc[n]);
            }
    }
    float* bout = (float*)(a.img + a.off_bout);
#pragma unroll
    for (int n = 0; n < NO; ++n) {
        float v = acc[n];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        const int o = 16 * n + (lane & 15);
        if (lane < 16) bout[o] = o < a.XD ? a.params[a.F.out_b + o] + v : 0.f;
    }
}

template <class P>
__global__ __launch_bounds__(64) void rt_fold_kernel(RtFoldArgs a) {
    using AT = typename P::AT;
    constexpr int KG = P::KG, EPL = P::EPL;
    constexpr bool TWO = sizeof(AT) == 2;
    constexpr int NHL = TWO ? 2 : 1, NLG = 16 / EPL;
    __shared__ float sm[32][17];   // [o][i] of the tile
    const int lane = threadIdx.x, b = (int)blockIdx.x;
    const int XD = a.XD, H = a.H;
    const float* prm = a.params;
    if (b > a.nm + a.nm0) {   // TEMB row r (the row tiles read their time embeddings from the table)
        const int r = b - a.nm - a.nm0 - 1, TD = a.TD;
        float* te = &sm[0][0];          // [TD]
        float* a1 = te + 64;            // [2 TD]
        if (lane < TD) te[lane] = temb_sinusoid(lane, r * a.TS, TD);
        __syncthreads();
        if (lane < 2 * TD) a1[lane] = temb_hidden(prm, a.F.time_w1, a.F.time_b1, te, TD, lane);
        __syncthreads();
        if (lane < TD) ((float*)(a.img + a.off_temb))[(size_t)r * TD + lane] = temb_output(prm, a.F.time_w2, a.F.time_b2, a1, TD, lane);
        return;
    }
    const __amdgpu_buffer_rsrc_t rs = packed_rsrc(a.img);
    if (b == a.nm + a.nm0) {   // RT_BOUT
        if (a.nt_out > 1) rt_fold_bias<P, 2>(a, rs, lane);
        else rt_fold_bias<P, 1>(a, rs, lane);
        return;
    }
    const bool m0 = b >= a.nm;
    const int T = m0 ? b - a.nm : b;
    const int kb4 = a.ks_h % 8 ? 4 : 8;   // k-steps per batch (H = 128 / 384 with 2-byte operands: 4)
    if (m0) {
        if (a.nt_out > 1) { if (kb4 == 8) rt_fold_tile<P, 2, 8, true>(a, rs, T, lane, sm); else rt_fold_tile<P, 2, 4, true>(a, rs, T, lane, sm); }
        else { if (kb4 == 8) rt_fold_tile<P, 1, 8, true>(a, rs, T, lane, sm); else rt_fold_tile<P, 1, 4, true>(a, rs, T, lane, sm); }
    } else {
        if (a.nt_out > 1) { if (kb4 == 8) rt_fold_tile<P, 2, 8, false>(a, rs, T, lane, sm); else rt_fold_tile<P, 2, 4, false>(a, rs, T, lane, sm); }
        else { if (kb4 == 8) rt_fold_tile<P, 1, 8, false>(a, rs, T, lane, sm); else rt_fold_tile<P, 1, 4, false>(a, rs, T, lane, sm); }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // RT_FOLD / RT_FOLD0 slots of the tile: copy h, lane group lg of its k range, column c
    {
        const int KS = m0 ? a.ks_in : a.ks_h;
        uint8_t* dst = a.img + (m0 ? a.off_fold0 : a.off_fold);
        const size_t mat = (size_t)a.nt_out * KS * 64 * 16;
        const int h = lane / (NLG * 16), lgl = (lane / 16) % NLG, c = lane & 15;
        if (h < NHL) {
            const int f0 = 16 * T + lgl * EPL, ks = f0 / KG, sl = c + 16 * ((f0 % KG) / EPL);
            for (int n = 0; n < a.nt_out; ++n) {
                AT e[EPL];
#pragma unroll
                for (int q = 0; q < EPL; ++q) {
                    const float m = sm[16 * n + c][lgl * EPL + q];
                    const AT hi = (AT)m;
                    e[q] = h == 0 ? hi : (AT)(m - (float)hi);
                }
                u32x4 w;
                __builtin_memcpy(&w, e, 16);
                *reinterpret_cast<u32x4*>(dst + h * mat + (((size_t)n * KS + ks) * 64 + sl) * 16) = w;
            }
        }
    }
    if (!m0) {   // RT_TFOLD n-tile T
        const int LOK = rt_tfold_lok(a.ks_out_t, KG);
        for (int ks = 0; ks < a.ks_out_t; ++ks) {
            const int k0 = ks * KG + (lane >> 4) * EPL;
            AT e[EPL];
#pragma unroll
            for (int q = 0; q < EPL; ++q) {
                const int k = k0 + q;
                const bool lo = TWO && k >= LOK;
                const int o = lo ? k - LOK : k;
                const float m = o < XD ? sm[o][lane & 15] : 0.f;
                const AT hi = (AT)m;
                e[q] = lo ? (AT)(m - (float)hi) : hi;
            }
            u32x4 w;
            __builtin_memcpy(&w, e, 16);
            *reinterpret_cast<u32x4*>(a.img + a.off_tfold + (((size_t)T * a.ks_out_t + ks) * 64 + lane) * 16) = w;
        }
    }
}

template <int KG, int EPL, class ET = __bf16>
__global__ __launch_bounds__(PACK_THREADS) void pack_all_kernel(PackArgs a) {
    int blk = (int)blockIdx.x;                       // whole blocks take a branch: no barrier is skipped
    if (blk < a.tb.nfold) {
        fold_block<ET>(a.tb, blk);
        return;
    }
    blk -= a.tb.nfold;
    // the time-table blocks next (each a chain of dependent global round trips: the launch's long
    // pole), then the element jobs, which are one round trip each
    if (blk < a.tb.tables) {
        time_table_block<ET>(a.tb, a.tb.first_table + blk);
        return;
    }
    blk -= a.tb.tables;
    const int gid = blk * blockDim.x + threadIdx.x;
    if (gid >= a.start[a.njobs]) return;
    int ji = 0;
    while (ji + 1 < a.njobs && gid >= a.start[ji + 1]) ++ji;
    const PackJob& J = a.j[ji];
    const int t = gid - a.start[ji];
    const float* W = J.src;
    if (J.kind == 1) {
        reinterpret_cast<float*>(J.dst)[t] = t < J.n ? W[t] : 0.f;
        return;
    }
    if (J.kind == 2) {   // words [4t, 4t + 4) of the range
        uint32_t* q = reinterpret_cast<uint32_t*>(J.dst);
#pragma unroll
        for (int w = 0; w < 4; ++w)
            if (4 * t + w < J.n) q[4 * t + w] = 0u;
        return;
    }
    const int KS = packed_ksteps(J.K, KG);
    const int lane = t & 63;
    const int ks = (t >> 6) % KS;
    const int nt = (t >> 6) / KS;
    const int n = nt * 16 + (lane & 15);
    u32x4 v;
    if constexpr (EPL == 8) {
        ET e[8];                 // __bf16 or _Float16 (RNE)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int k = ks * KG + (lane >> 4) * EPL + q;
            const int kr = k < J.k_split ? k : k + J.k_skip;
            float x = 0.f;
            if (k < J.K && n < J.N) x = J.transposed ? W[(size_t)n * J.K + k] : W[(size_t)kr * J.N + n];
            e[q] = (ET)x;
        }
        v = __builtin_bit_cast(u32x4, e);
    } else {
        float e[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = ks * KG + (lane >> 4) * EPL + q;
            const int kr = k < J.k_split ? k : k + J.k_skip;   // row subsets (W_XS) as the 2-byte branch
            float x = 0.f;
            if (k < J.K && n < J.N) x = J.transposed ? W[(size_t)n * J.K + k] : W[(size_t)kr * J.N + n];
            e[q] = x;
        }
        v = __builtin_bit_cast(u32x4, e);
    }
    reinterpret_cast<u32x4*>(J.dst)[t] = v;
}

static inline uint8_t* P_out(void* p) { return (uint8_t*)p; }

// the jobs of one MLP image (and, for an actor, its time tables) appended to a
// PackArgs; returns DPPO_OK or an error code. what: PACK_ALL, PACK_UPDATE (everything but the
// split sampler's tables: W_XS, FOLD / ROUT, TIN, B_OUT2), PACK_SAMPLER (those tables only),
// PACK_SAMPLER_TEMB (those tables and the TEMB table: after a fused actor step, any precision). Every
// pack with the main jobs of an actor is followed by the row tiles' fold (launch_rt_fold).
enum { PACK_ALL = 0, PACK_UPDATE = 1, PACK_SAMPLER = 2, PACK_SAMPLER_TEMB = 3 };
#ifndef DPPO_PACK_UPDATE_TEMB
#define DPPO_PACK_UPDATE_TEMB 0   // 1: PACK_UPDATE still writes the TEMB rows (the r04 pack; A/B builds)
#endif
static int add_mlp_jobs(PackArgs& a, int in_dim, int hidden, int out_dim, int time_dim, int precision,
                        const float* params, void* packed, int temb_steps, int time_stride, int what = PACK_ALL) {
    const MlpLayout L = make_mlp_layout(in_dim, hidden, out_dim, time_dim, precision, temb_steps);
    const FlatOffsets F = make_flat_offsets(in_dim, hidden, out_dim, time_dim);
    const int KG = dppo_prec_2b(precision) ? 32 : 16;
    const bool actor = time_dim > 0;
    // the split sampler's tables (every precision since r06: fp32 runs the split kernel at P = 4, its fold
    // from RT_FOLD and its residual from W_OUT, so only the 2-byte images carry FOLD / ROUT)
    const bool split_tables = actor && L.temb_steps > 0;
    const bool main_jobs = what == PACK_ALL || what == PACK_UPDATE;
    const bool sampler_tables = split_tables && (what == PACK_ALL || what == PACK_SAMPLER || what == PACK_SAMPLER_TEMB);
    const bool temb_rows = L.temb_steps > 0 && (what != PACK_UPDATE || DPPO_PACK_UPDATE_TEMB);
    const int jobs = (main_jobs ? 11 + (actor ? 1 : 0) : 0) + (sampler_tables ? 1 : 0);
    if (a.njobs + jobs > PACK_MAXJ) return dppo_set_error(DPPO_EINVAL, "pack: too many images in one launch");
    auto mat = [&](size_t src, int K, int N, bool tr, int seg) {
        PackJob& J = a.j[a.njobs++];
        J.kind = 0; J.K = K; J.N = N; J.transposed = tr ? 1 : 0; J.src = params + src; J.dst = P_out(packed) + L.off[seg];
        J.k_split = K; J.k_skip = 0;
        J.threads = dppo_cdiv(N, 16) * packed_ksteps(K, KG) * 64;
    };
    auto cpy = [&](size_t src, int n, int npad, int seg) {
        PackJob& J = a.j[a.njobs++];
        J.kind = 1; J.n = n; J.npad = npad; J.src = params + src; J.dst = P_out(packed) + L.off[seg]; J.threads = npad;
    };
    if (main_jobs) {
        if (actor) cpy(F.time_w1, (int)(F.in_w - F.time_w1), (int)(F.in_w - F.time_w1), SEG_TIME);
        mat(F.in_w, in_dim, hidden, false, SEG_W_IN);
        cpy(F.in_b, hidden, hidden, SEG_B_IN);
        mat(F.l1_w, hidden, hidden, false, SEG_W_L1);
        cpy(F.l1_b, hidden, hidden, SEG_B_L1);
        mat(F.l2_w, hidden, hidden, false, SEG_W_L2);
        cpy(F.l2_b, hidden, hidden, SEG_B_L2);
        mat(F.out_w, hidden, out_dim, false, SEG_W_OUT);
        cpy(F.out_b, out_dim, 16 * L.nt_out, SEG_B_OUT);
        // transposed images: W^T viewed as a [K'=out][N'=in] weight, i.e. element (k', n') = W[n'][k']
        mat(F.out_w, out_dim, hidden, true, SEG_T_OUT);
        mat(F.l2_w, hidden, hidden, true, SEG_T_L2);   // the actor's: the A operand of its fold (rt_fold_kernel)
        mat(F.l1_w, hidden, hidden, true, SEG_T_L1);
    }
    if (sampler_tables) {   // split sampler: W_in rows [x ; state] (skipping the TD time-embedding rows)
        mat(F.in_w, in_dim - time_dim, hidden, false, SEG_W_XS);
        a.j[a.njobs - 1].k_split = out_dim;
        a.j[a.njobs - 1].k_skip = time_dim;
    }
    // PACK_UPDATE leaves TEMB to its consumers too: the row tiles derive their time embeddings from the
    // fp32 time MLP (rowtile.hip), the sampler's table refresh re-derives the table (r05: the TEMB
    // blocks were the pack launch's long pole on every minibatch)
    if (actor && (temb_rows || sampler_tables)) {
        if (time_dim > 64 || out_dim > 32)
            return dppo_set_error(DPPO_EUNSUPPORTED, "time table: time_dim <= 64 and out_dim <= 32");
        if (a.tb.params) return dppo_set_error(DPPO_EINVAL, "pack: one actor per launch");
        TembArgs& b = a.tb;
        b.params = params; b.F = F; b.TD = time_dim; b.stride = time_stride; b.R = L.temb_steps; b.XD = out_dim;
        b.H = hidden; b.nout = 16 * L.nt_out;
        b.temb = (float*)(P_out(packed) + L.off[SEG_TEMB]);
        b.tin = (float*)(P_out(packed) + L.off[SEG_TIN]);
        b.bout2 = (float*)(P_out(packed) + L.off[SEG_B_OUT2]);
        const bool fold2b = sampler_tables && dppo_prec_2b(precision);
        b.fold = fold2b ? P_out(packed) + L.off[SEG_FOLD] : nullptr;
        b.rout = fold2b ? P_out(packed) + L.off[SEG_ROUT] : nullptr;
        b.nfold = fold2b ? L.nt_h : 0;
        // table blocks: [0, R) TEMB rows, [R, 2R) TIN rows, 2R B_OUT2 (time_table_block)
        b.first_table = what == PACK_SAMPLER ? L.temb_steps : 0;   // PACK_SAMPLER_TEMB: the TEMB rows too
        b.tables = sampler_tables ? 2 * L.temb_steps + 1 - b.first_table : (temb_rows ? L.temb_steps : 0);
    }
    return DPPO_OK;
}

// add_mlp_jobs' main jobs (PACK_UPDATE) as element ranges of the flat parameters, same segments and
// geometry; the TEMB table is derived separately (the fused step's last workgroup)
int dppo_fuse_jobs(int in_dim, int hidden, int out_dim, int time_dim, int precision, void* packed, int temb_steps,
                   FuseJob* jobs) {
    const MlpLayout L = make_mlp_layout(in_dim, hidden, out_dim, time_dim, precision, temb_steps);
    const FlatOffsets F = make_flat_offsets(in_dim, hidden, out_dim, time_dim);
    const int KG = dppo_prec_2b(precision) ? 32 : 16;
    int n = 0;
    auto job = [&](int kind, size_t src, size_t count, int IK, int IN, int seg) {
        if (n >= FUSE_MAXJ) { n = FUSE_MAXJ + 1; return; }
        FuseJob& J = jobs[n++];
        J.kind = kind; J.IK = IK; J.IN = IN; J.KS = kind == 2 ? 0 : packed_ksteps(IK, KG);
        J.lo = (int64_t)src; J.hi = (int64_t)(src + count); J.dst = P_out(packed) + L.off[seg];
    };
    const size_t hh = (size_t)hidden * hidden, ho = (size_t)hidden * out_dim;
    if (time_dim > 0) job(2, F.time_w1, F.in_w - F.time_w1, 0, 0, SEG_TIME);
    job(0, F.in_w, (size_t)in_dim * hidden, in_dim, hidden, SEG_W_IN);
    job(2, F.in_b, hidden, 0, 0, SEG_B_IN);
    job(0, F.l1_w, hh, hidden, hidden, SEG_W_L1);
    job(1, F.l1_w, hh, hidden, hidden, SEG_T_L1);
    job(2, F.l1_b, hidden, 0, 0, SEG_B_L1);
    job(0, F.l2_w, hh, hidden, hidden, SEG_W_L2);
    job(1, F.l2_w, hh, hidden, hidden, SEG_T_L2);
    job(2, F.l2_b, hidden, 0, 0, SEG_B_L2);
    job(0, F.out_w, ho, hidden, out_dim, SEG_W_OUT);
    job(1, F.out_w, ho, out_dim, hidden, SEG_T_OUT);
    job(2, F.out_b, out_dim, 0, 0, SEG_B_OUT);
    return n <= FUSE_MAXJ ? n : -1;
}

static int launch_pack(PackArgs& a, int precision, hipStream_t s) {
    a.start[0] = 0;
    for (int i = 0; i < a.njobs; ++i) a.start[i + 1] = a.start[i] + a.j[i].threads;
    a.pack_blocks = dppo_cdiv(a.start[a.njobs], PACK_THREADS);
    const int blocks = a.tb.nfold + a.pack_blocks + a.tb.tables;
    if (blocks == 0) return DPPO_OK;
    DppoKtScope kt(KT_PACK_ALL, s);
    if (precision == DPPO_BF16)
        hipLaunchKernelGGL((pack_all_kernel<32, 8, __bf16>), dim3(blocks), dim3(PACK_THREADS), 0, s, a);
    else if (precision == DPPO_F16)
        hipLaunchKernelGGL((pack_all_kernel<32, 8, _Float16>), dim3(blocks), dim3(PACK_THREADS), 0, s, a);
    else
        hipLaunchKernelGGL((pack_all_kernel<16, 4, float>), dim3(blocks), dim3(PACK_THREADS), 0, s, a);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}


// Actor images whose split-sampler tables are stale (packed with PACK_UPDATE by an optimizer
// step that deferred them): the sampler re-derives them on its own stream before its next launch
// that reads the image (dppo_refresh_sampler_tables). The PPO row tiles never read those tables, so
// a run of minibatches packs each actor image without them and the rollout after the update pays
// for them once. Keyed by the image's address; stream order is the caller's, as for every launch.
namespace {
struct StaleTables { const void* packed; const float* params; Dims D; int precision; bool temb; };
constexpr int MAX_STALE = 32;
std::mutex g_stale_mu;
StaleTables g_stale[MAX_STALE];
int g_nstale = 0;

void clear_stale(const void* packed) {
    std::lock_guard<std::mutex> lk(g_stale_mu);
    for (int i = 0; i < g_nstale; ++i)
        if (g_stale[i].packed == packed) { g_stale[i] = g_stale[--g_nstale]; return; }
}

// the latest update of an image decides what is stale: since r05 neither a PACK_UPDATE pack nor a
// fused actor step rewrites TEMB (temb = true); the flag stays for callers that do
int mark_stale(const Dims& D, int precision, const float* params, const void* packed, bool temb) {
    std::lock_guard<std::mutex> lk(g_stale_mu);
    for (int i = 0; i < g_nstale; ++i)
        if (g_stale[i].packed == packed) { g_stale[i] = {packed, params, D, precision, temb}; return DPPO_OK; }
    if (g_nstale == MAX_STALE) return dppo_set_error(DPPO_EINVAL, "deferred sampler tables: more than %d stale images", MAX_STALE);
    g_stale[g_nstale++] = {packed, params, D, precision, temb};
    return DPPO_OK;
}
}  // namespace

// the fused step leaves the actor image's split-sampler tables stale like a PACK_UPDATE pack
int dppo_mark_tables_stale(const Dims& D, int precision, const float* actor_params, const void* packed_actor, bool temb) {
    return mark_stale(D, precision, actor_params, packed_actor, temb);
}

int dppo_pack_mlp(int in_dim, int hidden, int out_dim, int time_dim, int precision, const float* params,
                  void* packed, hipStream_t s, int temb_steps, int time_stride) {
    PackArgs a = {};
    int rc = add_mlp_jobs(a, in_dim, hidden, out_dim, time_dim, precision, params, packed, temb_steps, time_stride);
    if (rc) return rc;
    if (temb_steps > 0) clear_stale(packed);
    rc = launch_pack(a, precision, s);
    if (rc) return rc;
    return dppo_pack_rt_fold(in_dim, hidden, out_dim, time_dim, precision, params, packed, temb_steps, time_stride, s);
}

// the row tiles' fold segments of an actor image whose W_OUT / T_L2 slots are final on stream s (after
// its pack launch or a fused optimizer step): rt_fold_kernel, one wave per tile
int dppo_pack_rt_fold(int in_dim, int hidden, int out_dim, int time_dim, int precision, const float* actor_params,
                      void* packed_actor, int temb_steps, int time_stride, hipStream_t s) {
    const MlpLayout L = make_mlp_layout(in_dim, hidden, out_dim, time_dim, precision, temb_steps);
    if (time_dim <= 0) return DPPO_OK;
    if (out_dim > 32 || (dppo_prec_2b(precision) && out_dim > rt_tfold_lok(L.ks_out_t, L.KG)))
        return dppo_set_error(DPPO_EUNSUPPORTED, "row-tile fold: out_dim %d > 32", out_dim);
    const FlatOffsets F = make_flat_offsets(in_dim, hidden, out_dim, time_dim);
    if (F.in_w % 4 || F.in_b % 4 || F.l2_b % 4 || hidden % 8)
        return dppo_set_error(DPPO_EUNSUPPORTED, "row-tile fold: W_in / biases not 16-B aligned (time_dim %d)", time_dim);
    RtFoldArgs a = {};
    a.img = (uint8_t*)packed_actor; a.params = actor_params;
    a.F = make_flat_offsets(in_dim, hidden, out_dim, time_dim);
    a.off_wout = L.off[SEG_W_OUT]; a.off_tl2 = L.off[SEG_T_L2]; a.off_fold = L.off[SEG_RT_FOLD];
    a.off_fold0 = L.off[SEG_RT_FOLD0]; a.off_tfold = L.off[SEG_RT_TFOLD]; a.off_bout = L.off[SEG_RT_BOUT];
    a.H = hidden; a.XD = out_dim; a.IN = in_dim; a.nt_out = L.nt_out; a.ks_h = L.ks_h; a.ks_in = L.ks_in;
    a.ks_out_t = L.ks_out_t;
    a.nm = L.nt_h;
    a.nm0 = L.ks_in * L.KG / 16;   // RT_FOLD0's padded k range, 16 rows per tile
    // and the TEMB table (one block per row): the row tiles read their time embeddings from it
    a.off_temb = L.off[SEG_TEMB]; a.TD = time_dim; a.TS = time_stride; a.R = L.temb_steps;
    if (time_dim > 32) return dppo_set_error(DPPO_EUNSUPPORTED, "row-tile fold: time_dim %d > 32", time_dim);
    const dim3 grid(a.nm + a.nm0 + 1 + a.R);
    DppoKtScope kt(KT_PACK_ALL, s);
    if (precision == DPPO_BF16) hipLaunchKernelGGL(rt_fold_kernel<PolicyBF16>, grid, dim3(64), 0, s, a);
    else if (precision == DPPO_F16) hipLaunchKernelGGL(rt_fold_kernel<PolicyF16>, grid, dim3(64), 0, s, a);
    else hipLaunchKernelGGL(rt_fold_kernel<PolicyF32>, grid, dim3(64), 0, s, a);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

extern "C" int dppo_refresh_sampler_tables(const void* packed, void* stream) {
    if (!packed) return DPPO_OK;
    hipStream_t s = (hipStream_t)stream;
    StaleTables e;
    {
        std::lock_guard<std::mutex> lk(g_stale_mu);
        int i = 0;
        while (i < g_nstale && g_stale[i].packed != packed) ++i;
        if (i == g_nstale) return DPPO_OK;
        e = g_stale[i];
        g_stale[i] = g_stale[--g_nstale];
    }
    PackArgs a = {};
    int rc = add_mlp_jobs(a, e.D.IN, e.D.H, e.D.XD, e.D.TD, e.precision, e.params, (void*)e.packed, e.D.K, e.D.TS,
                          e.temb ? PACK_SAMPLER_TEMB : PACK_SAMPLER);
    if (rc) return rc;
    return launch_pack(a, e.precision, s);
}

int dppo_pack_models(const Dims& D, int precision, const float* actor_params, void* packed_actor,
                     const float* critic_params, void* packed_critic, hipStream_t s, bool defer_sampler_tables,
                     void* const* zero_ptrs, const size_t* zero_bytes, int n_zero) {
    PackArgs a = {};
    int rc;
    // byte ranges zeroed by the same launch (4-byte words, < 2^33 bytes each): jobs of their own
    for (int r = 0; r < n_zero; ++r) {
        if (a.njobs == PACK_MAXJ) return dppo_set_error(DPPO_EINVAL, "pack: too many jobs in one launch");
        PackJob& J = a.j[a.njobs++];
        J.kind = 2; J.dst = (uint8_t*)zero_ptrs[r]; J.n = (int)(zero_bytes[r] / 4); J.threads = (J.n + 3) / 4;
    }
    if (actor_params && packed_actor) {
        const bool defer = defer_sampler_tables && D.TD > 0;
        rc = add_mlp_jobs(a, D.IN, D.H, D.XD, D.TD, precision, actor_params, packed_actor, D.K, D.TS,
                          defer ? PACK_UPDATE : PACK_ALL);
        if (rc) return rc;
        if (defer) rc = mark_stale(D, precision, actor_params, packed_actor, !DPPO_PACK_UPDATE_TEMB);
        else clear_stale(packed_actor);   // a full pack makes a pending refresh moot
        if (rc) return rc;
    }
    if (critic_params && packed_critic) {
        rc = add_mlp_jobs(a, D.SD, D.HC, 1, 0, precision, critic_params, packed_critic, 0, 1);
        if (rc) return rc;
    }
    rc = launch_pack(a, precision, s);
    if (rc || !(actor_params && packed_actor)) return rc;
    return dppo_pack_rt_fold(D.IN, D.H, D.XD, D.TD, precision, actor_params, packed_actor, D.K, D.TS, s);
}
