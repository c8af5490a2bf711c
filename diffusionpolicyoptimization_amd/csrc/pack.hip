// pack.hip — flat fp32 Keras parameters -> packed MFMA fragment images (dppo_layout.h).
// Replaces the Keras variable storage of model/common/mlp.py:95-206 (kernels are [in,out]).
#include "dppo_common.cuh"
#include "dppo_internal.h"

// one thread per (ntile, ks, lane) fragment slot; writes 16 B
template <int KG, int EPL>
__global__ void pack_matrix_kernel(const float* __restrict__ W, int K, int N, int transposed, uint8_t* __restrict__ out) {
    const int KS = packed_ksteps(K, KG);
    const int NTL = (N + 15) / 16;
    const int total = NTL * KS * 64;
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= total) return;
    const int lane = gid & 63;
    const int ks = (gid >> 6) % KS;
    const int nt = (gid >> 6) / KS;
    const int n = nt * 16 + (lane & 15);
    u32x4 v;
    if constexpr (EPL == 8) {
        __bf16 e[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int k = ks * KG + (lane >> 4) * EPL + q;
            float x = 0.f;
            if (k < K && n < N) x = transposed ? W[(size_t)n * K + k] : W[(size_t)k * N + n];
            e[q] = (__bf16)x;
        }
        v = __builtin_bit_cast(u32x4, e);
    } else {
        float e[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = ks * KG + (lane >> 4) * EPL + q;
            float x = 0.f;
            if (k < K && n < N) x = transposed ? W[(size_t)n * K + k] : W[(size_t)k * N + n];
            e[q] = x;
        }
        v = __builtin_bit_cast(u32x4, e);
    }
    reinterpret_cast<u32x4*>(out)[gid] = v;
}

__global__ void copy_pad_kernel(const float* __restrict__ src, int n, int npad, float* __restrict__ dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < npad) dst[i] = i < n ? src[i] : 0.f;
}

static hipError_t pack_matrix(const float* W, int K, int N, bool transposed, int precision, uint8_t* out,
                              hipStream_t s) {
    const int KG = precision == DPPO_BF16 ? 32 : 16;
    const int total = dppo_cdiv(N, 16) * packed_ksteps(K, KG) * 64;
    const int blocks = dppo_cdiv(total, 256);
    if (precision == DPPO_BF16)
        hipLaunchKernelGGL((pack_matrix_kernel<32, 8>), dim3(blocks), dim3(256), 0, s, W, K, N, transposed ? 1 : 0, out);
    else
        hipLaunchKernelGGL((pack_matrix_kernel<16, 4>), dim3(blocks), dim3(256), 0, s, W, K, N, transposed ? 1 : 0, out);
    return hipGetLastError();
}

static hipError_t copy_pad(const float* src, int n, int npad, void* dst, hipStream_t s) {
    if (npad <= 0) return hipSuccess;
    hipLaunchKernelGGL(copy_pad_kernel, dim3(dppo_cdiv(npad, 256)), dim3(256), 0, s, src, n, npad, (float*)dst);
    return hipGetLastError();
}

int dppo_pack_mlp(int in_dim, int hidden, int out_dim, int time_dim, int precision, const float* params,
                  void* packed, hipStream_t s) {
    const MlpLayout L = make_mlp_layout(in_dim, hidden, out_dim, time_dim, precision);
    const FlatOffsets F = make_flat_offsets(in_dim, hidden, out_dim, time_dim);
    uint8_t* P = (uint8_t*)packed;
    hipError_t e = hipSuccess;
#define DPPO_TRY(x) do { e = (x); if (e != hipSuccess) return dppo_hip_fail(e, #x); } while (0)
    if (time_dim > 0) {
        const int tsz = (int)(F.in_w - F.time_w1);
        DPPO_TRY(copy_pad(params + F.time_w1, tsz, tsz, P + L.off[SEG_TIME], s));
    }
    DPPO_TRY(pack_matrix(params + F.in_w, in_dim, hidden, false, precision, P + L.off[SEG_W_IN], s));
    DPPO_TRY(copy_pad(params + F.in_b, hidden, hidden, P + L.off[SEG_B_IN], s));
    DPPO_TRY(pack_matrix(params + F.l1_w, hidden, hidden, false, precision, P + L.off[SEG_W_L1], s));
    DPPO_TRY(copy_pad(params + F.l1_b, hidden, hidden, P + L.off[SEG_B_L1], s));
    DPPO_TRY(pack_matrix(params + F.l2_w, hidden, hidden, false, precision, P + L.off[SEG_W_L2], s));
    DPPO_TRY(copy_pad(params + F.l2_b, hidden, hidden, P + L.off[SEG_B_L2], s));
    DPPO_TRY(pack_matrix(params + F.out_w, hidden, out_dim, false, precision, P + L.off[SEG_W_OUT], s));
    DPPO_TRY(copy_pad(params + F.out_b, out_dim, 16 * L.nt_out, P + L.off[SEG_B_OUT], s));
    // transposed images: W^T viewed as a [K'=out][N'=in] weight, i.e. element (k', n') = W[n'][k']
    DPPO_TRY(pack_matrix(params + F.out_w, out_dim, hidden, true, precision, P + L.off[SEG_T_OUT], s));
    DPPO_TRY(pack_matrix(params + F.l2_w, hidden, hidden, true, precision, P + L.off[SEG_T_L2], s));
    DPPO_TRY(pack_matrix(params + F.l1_w, hidden, hidden, true, precision, P + L.off[SEG_T_L1], s));
#undef DPPO_TRY
    return DPPO_OK;
}
