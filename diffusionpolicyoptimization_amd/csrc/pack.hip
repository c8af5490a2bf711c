// pack.hip — flat fp32 Keras parameters -> packed MFMA fragment images (dppo_layout.h).
// Replaces the Keras variable storage of model/common/mlp.py:95-206 (kernels are [in,out]).
#include "dppo_common.cuh"
#include "dppo_internal.h"

// All segments of one MLP image in ONE launch (the images are re-derived after every optimiser
// step, so 12 small launches per model were ~100 us per PPO minibatch). A job is either a packed
// matrix (one thread per (ntile, ks, lane) fragment slot, 16 B each) or a zero-padded fp32 copy.
#define PACK_MAXJ 16
struct PackJob {
    int kind;            // 0 = packed matrix, 1 = fp32 copy with zero padding
    int K, N, transposed;
    int k_split, k_skip; // source row of packed row k: k < k_split ? k : k + k_skip (row subsets)
    int n, npad;         // copy: valid / padded element counts
    size_t src, dst;     // float offset in params / byte offset in the image
    int threads;         // work items of this job
};
struct PackArgs {
    PackJob j[PACK_MAXJ];
    int start[PACK_MAXJ + 1];
    int njobs;
    const float* params;
    uint8_t* out;
};

template <int KG, int EPL, class ET = __bf16>
__global__ void pack_all_kernel(PackArgs a) {
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= a.start[a.njobs]) return;
    int ji = 0;
    while (ji + 1 < a.njobs && gid >= a.start[ji + 1]) ++ji;
    const PackJob& J = a.j[ji];
    const int t = gid - a.start[ji];
    const float* W = a.params + J.src;
    if (J.kind == 1) {
        reinterpret_cast<float*>(a.out + J.dst)[t] = t < J.n ? W[t] : 0.f;
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
            float x = 0.f;
            if (k < J.K && n < J.N) x = J.transposed ? W[(size_t)n * J.K + k] : W[(size_t)k * J.N + n];
            e[q] = x;
        }
        v = __builtin_bit_cast(u32x4, e);
    }
    reinterpret_cast<u32x4*>(a.out + J.dst)[t] = v;
}

// t_emb(t) = Dense(2TD->TD)(mish(Dense(TD->2TD)(SinusoidalPosEmb(t)))) (mlp_diffusion.py:40-45,
// modules.py:4-15), one workgroup per t; the arithmetic and its order match the oracle restatement
static inline uint8_t* P_out(void* p) { return (uint8_t*)p; }

// blocks [0, R): row r of the TEMB table. With ET = the 2-byte operand type (split-sampler tables),
// also blocks [R, 2R): row r of TIN = b_in + sum_j rnd(t_emb_j) rnd(W_in[XD + j]) (each block
// re-derives its t_emb row), and block 2R: B_OUT2 = b_out + sum_h b_l2[h] rnd(W_out[h]) with a
// fixed-order reduction (the sampler's h3 is fp32-accurate, so b_l2 enters the out-Dense unrounded)
template <class ET>
__global__ __launch_bounds__(128) void temb_table_kernel(const float* __restrict__ params, FlatOffsets F, int TD,
                                                         int stride, int R, int XD, int H, float* __restrict__ temb,
                                                         float* __restrict__ tin, float* __restrict__ bout2, int nout) {
    // the sinusoid once per k (not once per (k, hidden unit)), weight loads unrolled so they issue
    // together; the sums keep the oracle's order (k ascending, then h ascending)
    __shared__ float te[64];
    __shared__ float ta1[128];
    __shared__ float tr[64];
    __shared__ float red[128][33];
    const int tid = threadIdx.x;
    if ((int)blockIdx.x == 2 * R) {   // B_OUT2
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
        __syncthreads();
        if (tid < nout) {
            float s = tid < XD ? params[F.out_b + tid] : 0.f;
            if (tid < XD)
                for (int k = 0; k < 128; ++k) s += red[k][tid];
            bout2[tid] = s;
        }
        return;
    }
    const int row = (int)blockIdx.x % R, t = row * stride;   // row r holds t_emb(r * stride)
    const int half = TD / 2;
    const float lnf = logf(10000.f) / (float)(half - 1);
    if (tid < TD) {
        const float f = expf(-(float)(tid % half) * lnf) * (float)t;
        te[tid] = tid < half ? sinf(f) : cosf(f);
    }
    __syncthreads();
    if (tid < 2 * TD) {
        float acc = params[F.time_b1 + tid];
#pragma unroll 16
        for (int k = 0; k < TD; ++k) acc += te[k] * params[F.time_w1 + k * 2 * TD + tid];
        ta1[tid] = mishf(acc);
    }
    __syncthreads();
    if (tid < TD) {
        float acc = params[F.time_b2 + tid];
#pragma unroll 16
        for (int k = 0; k < 2 * TD; ++k) acc += ta1[k] * params[F.time_w2 + k * TD + tid];
        if ((int)blockIdx.x < R) temb[(size_t)row * TD + tid] = acc;
        tr[tid] = (float)(ET)acc;
    }
    if ((int)blockIdx.x < R) return;
    __syncthreads();
    for (int h = tid; h < H; h += 128) {
        float acc = params[F.in_b + h];
        for (int j = 0; j < TD; ++j) acc += tr[j] * (float)(ET)params[F.in_w + (size_t)(XD + j) * H + h];
        tin[(size_t)row * H + h] = acc;
    }
}

int dppo_pack_mlp(int in_dim, int hidden, int out_dim, int time_dim, int precision, const float* params,
                  void* packed, hipStream_t s, int temb_steps, int time_stride) {
    const MlpLayout L = make_mlp_layout(in_dim, hidden, out_dim, time_dim, precision, temb_steps);
    const FlatOffsets F = make_flat_offsets(in_dim, hidden, out_dim, time_dim);
    const int KG = dppo_prec_2b(precision) ? 32 : 16;
    PackArgs a = {};
    auto mat = [&](size_t src, int K, int N, bool tr, int seg) {
        PackJob& J = a.j[a.njobs++];
        J.kind = 0; J.K = K; J.N = N; J.transposed = tr ? 1 : 0; J.src = src; J.dst = L.off[seg];
        J.k_split = K; J.k_skip = 0;
        J.threads = dppo_cdiv(N, 16) * packed_ksteps(K, KG) * 64;
    };
    auto cpy = [&](size_t src, int n, int npad, int seg) {
        PackJob& J = a.j[a.njobs++];
        J.kind = 1; J.n = n; J.npad = npad; J.src = src; J.dst = L.off[seg]; J.threads = npad;
    };
    if (time_dim > 0) cpy(F.time_w1, (int)(F.in_w - F.time_w1), (int)(F.in_w - F.time_w1), SEG_TIME);
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
    mat(F.l2_w, hidden, hidden, true, SEG_T_L2);
    mat(F.l1_w, hidden, hidden, true, SEG_T_L1);
    const bool split_tables = time_dim > 0 && L.temb_steps > 0 && dppo_prec_2b(precision);
    if (split_tables) {   // split sampler: W_in rows [x ; state] (skipping the TD time-embedding rows)
        mat(F.in_w, in_dim - time_dim, hidden, false, SEG_W_XS);
        a.j[a.njobs - 1].k_split = out_dim;
        a.j[a.njobs - 1].k_skip = time_dim;
    }
    for (int i = 0; i < a.njobs; ++i) a.start[i + 1] = a.start[i] + a.j[i].threads;
    a.params = params;
    a.out = (uint8_t*)packed;
    const int blocks = dppo_cdiv(a.start[a.njobs], 256);
    if (precision == DPPO_BF16)
        hipLaunchKernelGGL((pack_all_kernel<32, 8, __bf16>), dim3(blocks), dim3(256), 0, s, a);
    else if (precision == DPPO_F16)
        hipLaunchKernelGGL((pack_all_kernel<32, 8, _Float16>), dim3(blocks), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((pack_all_kernel<16, 4>), dim3(blocks), dim3(256), 0, s, a);
    DPPO_HIP(hipGetLastError());
    if (L.temb_steps > 0) {
        if (time_dim > 64 || 2 * time_dim > 128 || out_dim > 32)
            return dppo_set_error(DPPO_EUNSUPPORTED, "time table: time_dim <= 64 and out_dim <= 32");
        const int R = L.temb_steps;
        float* temb = (float*)(P_out(packed) + L.off[SEG_TEMB]);
        float* tin = (float*)(P_out(packed) + L.off[SEG_TIN]);
        float* bout2 = (float*)(P_out(packed) + L.off[SEG_B_OUT2]);
        const int nout = 16 * L.nt_out;
        if (!split_tables)
            hipLaunchKernelGGL(temb_table_kernel<float>, dim3(R), dim3(128), 0, s, params, F, time_dim, time_stride, R,
                               out_dim, hidden, temb, tin, bout2, nout);
        else if (precision == DPPO_F16)
            hipLaunchKernelGGL(temb_table_kernel<_Float16>, dim3(2 * R + 1), dim3(128), 0, s, params, F, time_dim,
                               time_stride, R, out_dim, hidden, temb, tin, bout2, nout);
        else
            hipLaunchKernelGGL(temb_table_kernel<__bf16>, dim3(2 * R + 1), dim3(128), 0, s, params, F, time_dim,
                               time_stride, R, out_dim, hidden, temb, tin, bout2, nout);
        DPPO_HIP(hipGetLastError());
    }
    return DPPO_OK;
}
